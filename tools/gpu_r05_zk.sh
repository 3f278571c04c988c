#!/bin/bash
# Round 5, call zk: chained tile orders (gate last-to-first, conv5 first-to-last, pool images
# last-to-first) vs the product (conv5 last-to-first only): ratio GPU tests, then the in-process A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
true
tail -2 $O/tests_zk.txt
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_head.so --rounds 14 > $O/ab_zk2.txt 2>&1 || { tail -5 $O/ab_zk2.txt; exit 1; }
cat $O/ab_zk2.txt
