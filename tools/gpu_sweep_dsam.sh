#!/bin/bash
# k_dsam_lds kernel times (rocprofv3 kernel trace of tools/micro_dsam_conv.py) per
# (RGBD_DSAM_KC, RGBD_DSAM_PERSIST) pair given as "kc:persist" arguments.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for cfg in "$@"; do
  kc=${cfg%%:*}; pe=${cfg##*:}
  export RGBD_DSAM_KC=$kc RGBD_DSAM_PERSIST=$pe
  d="$GRAFT_REPO_ROOT/gpurun_out/sweep_${kc}_${pe}"
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/micro_dsam_conv.py" --iters 5 > "$d.log" 2>&1 || { echo "cfg $cfg failed"; exit 1; }
  echo "== kc=$kc persist=$pe"; python3 tools/trace_by_grid.py "$d/run_kernel_trace.csv" | grep "k_dsam_lds" | cut -c1-80
done
