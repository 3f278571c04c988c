#!/bin/bash
# Round 5, call x: conv5 reversed (product) vs the gate reversed with conv5 forward, vs the earlier build
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_gaterev.so rgb-d-instance-segmentation_amd/gpurun_ab_head.so --rounds 8 > $O/ab_x.txt 2>&1 || { tail -5 $O/ab_x.txt; exit 1; }
cat $O/ab_x.txt
