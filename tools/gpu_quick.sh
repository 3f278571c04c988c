#!/bin/bash
# Quick GPU iteration: selected GPU tests (-k expr), then the ratio micro driver under a kernel
# trace.  Each GPU step has its own time limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -k "$1" > gpurun_out/quick_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -3 gpurun_out/quick_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/quick" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 10 > "$R/gpurun_out/quick.log" 2>&1 || { echo "micro failed"; exit 1; }
grep "ratio fwd" "$R/gpurun_out/quick.log"
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/quick/run_kernel_stats.csv" 13 12
if [ -n "$2" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $2 -d "$R/gpurun_out/quickpmc" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 5 > "$R/gpurun_out/quickpmc.log" 2>&1 || { echo "pmc failed"; exit 1; }
fi
echo done
