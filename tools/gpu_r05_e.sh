#!/bin/bash
# Round 5, call e: conv5 split-issue stamps + A/B vs the round-4 library, ratio-predictor kernel
# trace (stem moments, phase-1 shifted patches), the fixed tests, the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
R="$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/conv5_stamps.py > $O/conv5_stamps_e.txt 2>&1 || { tail -5 $O/conv5_stamps_e.txt; exit 1; }
cat $O/conv5_stamps_e.txt
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_old.so --rounds 6 > $O/ab_e.txt 2>&1 || { tail -5 $O/ab_e.txt; exit 1; }
cat $O/ab_e.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_ratio_e" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 5 > "$R/$O/prof_ratio_e.log" 2>&1 ) || { tail -5 $O/prof_ratio_e.log; exit 1; }
f=$(find $O/prof_ratio_e -name "*kernel_stats.csv" | head -1); cut -c1-160 "$f" | head -24
TESTLOG=tests_e bash tools/gpu.sh tests tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py \
  tests/test_gpu_c2.py -s || exit 1
bash tools/gpu.sh bench || exit 1
