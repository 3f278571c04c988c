#!/bin/bash
# Kernel traces of tools/micro_dsam_conv.py under each "ENV=VAL ..." setting given as an argument;
# prints per-(kernel, grid) average durations of the DSAM conv kernels and the per-setting sum.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace -d "$R/gpurun_out/sweep/c$i" -o run --output-format csv -- python3 "$R/tools/micro_dsam_conv.py" --iters 5 > "$R/gpurun_out/sweep/c$i.log" 2>&1 || { echo "cfg $cfg failed"; tail -5 "$R/gpurun_out/sweep/c$i.log"; exit 1; }
  echo "== $cfg"; python3 "$R/tools/trace_by_grid.py" "$(find "$R/gpurun_out/sweep/c$i" -name '*kernel_trace.csv' | head -1)" k_ | grep -E "dsam_lds|items|plan"
done
