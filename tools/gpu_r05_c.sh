#!/bin/bash
# Round 5, call c: kernel trace of the ratio predictor (stem moments), DDP diagnostics.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_ratio" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 5 > "$R/$O/prof_ratio.log" 2>&1 ) || { tail -5 $O/prof_ratio.log; exit 1; }
f=$(find $O/prof_ratio -name "*kernel_stats.csv" | head -1); head -30 "$f"
TESTLOG=tests_c bash tools/gpu.sh tests tests/test_gpu_ddp_model.py -s || exit 1
