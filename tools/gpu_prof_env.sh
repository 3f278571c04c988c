#!/bin/bash
# Kernel-trace profile of a short bench run per value of an environment switch:
#   bash tools/gpu_prof_env.sh VAR v1 v2 ...   -> gpurun_out/prof_VAR_v/run_kernel_trace.csv
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
var=$1; shift
for v in "$@"; do
  export "$var=$v"; timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${var}_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --cpu-baseline 0 --inference 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_${var}_$v.log" 2>&1 || { echo "rocprof $var=$v failed $?"; exit 1; }
  echo "$var=$v done"
done
