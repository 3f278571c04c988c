#!/bin/bash
# Round-4 batch 11: conv5 per-step stamps (diagnostic) and the ratio-predictor micro (the
# production conv5 unchanged by the stamped instantiation).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 120 python tools/conv5_stamps.py > $O/conv5_stamps.txt 2>&1; rc=$?; cat $O/conv5_stamps.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/micro_ratio.py --iters 20 2>&1 | tail -1
