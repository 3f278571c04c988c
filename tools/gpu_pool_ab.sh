#!/bin/bash
# Kernel-trace A/B of the ratio predictor's pool kernels: current library vs $1 (relative path).
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/poolab
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/poolab/new" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 20 > "$R/gpurun_out/poolab/new.log" 2>&1 || { echo "new failed"; exit 1; }
RGBD_HIP_LIB="$R/$1" timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/poolab/old" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 20 > "$R/gpurun_out/poolab/old.log" 2>&1 || { echo "old failed"; exit 1; }
for v in new old; do echo "== $v"; python3 "$R/tools/trace_by_grid.py" $(find "$R/gpurun_out/poolab/$v" -name "*kernel_trace.csv") | grep -E "pool|conv3x3|gate|chain"; done
