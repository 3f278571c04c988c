#!/bin/bash
# Kernel-trace profile of a short bench run; summary to gpurun_out/prof/run_kernel_stats.csv.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 "$@" > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
