#!/bin/bash
# PMC passes (kernel-trace only, one counter group per pass) on the ratio-predictor micro driver.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 5 > "$R/gpurun_out/pmc/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo done
