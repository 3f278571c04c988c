#!/bin/bash
# Kernel-trace profiles of the bench with the in-tree library and with $1 (an alternative .so).
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profnew" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 > "$R/gpurun_out/profnew.log" 2>&1 || exit 1
RGBD_HIP_LIB="$R/$1" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profold" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 > "$R/gpurun_out/profold.log" 2>&1 || exit 1
echo done
