#!/bin/bash
# Kernel-trace profile of a driver per value of an environment switch:
#   bash tools/gpu_prof_env.sh VAR "v1 v2 ..." [driver args...]
#   -> gpurun_out/prof_VAR_v/run_kernel_trace.csv   (default driver: bench.py --steps 3 --warmup 1)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
var=$1; vals=$2; shift 2
[ $# -eq 0 ] && set -- bench.py --steps 3 --warmup 1 --cpu-baseline 0 --inference 0
drv=$1; shift
for v in $vals; do
  export "$var=$v"; timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${var}_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/$drv" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/prof_${var}_$v.log" 2>&1 || { echo "rocprof $var=$v failed $?"; exit 1; }
  echo "$var=$v done"
done
