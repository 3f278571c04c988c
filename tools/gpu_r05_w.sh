#!/bin/bash
# Round 5, call w: conv5 over its tiles in reverse order (the gate's last-written features first).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_rev.so --rounds 8 > $O/ab_w.txt 2>&1 || { tail -5 $O/ab_w.txt; exit 1; }
cat $O/ab_w.txt
