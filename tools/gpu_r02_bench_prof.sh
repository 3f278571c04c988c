#!/bin/bash
# Bench line + a kernel-trace profile of the same step (per-grid summary for profiles/).
# Optional $1: pytest node ids to run first.  Each GPU step has its own limit; stop at failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest $1 -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_sel.log 2>&1
  rc=$?; tail -15 gpurun_out/tests_sel.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed $?"; tail -5 "$R/gpurun_out/prof.log"; exit 1; }
echo done
