#!/bin/bash
# Kernel traces of tools/micro_dsam_conv.py under each RGBD_DSAM_DBG mode (one process each).
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dbg
cd /tmp && export TMPDIR=/tmp
for d in "$@"; do
  RGBD_DSAM_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace -d "$R/gpurun_out/dbg/d$d" -o run --output-format csv -- python3 "$R/tools/micro_dsam_conv.py" --iters 5 > "$R/gpurun_out/dbg/d$d.log" 2>&1 || { echo "mode $d failed"; tail -5 "$R/gpurun_out/dbg/d$d.log"; exit 1; }
  echo "== DBG=$d"; python3 "$R/tools/trace_by_grid.py" "$(find "$R/gpurun_out/dbg/d$d" -name '*kernel_trace.csv' | head -1)" k_
done
