#!/bin/bash
# Selected GPU tests (-k expr) then bench + kernel-trace profile; every GPU step has its own
# time limit and the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread -k "$1" > gpurun_out/check_tests.log 2>&1
rc=$?; tail -25 gpurun_out/check_tests.log; [ $rc -eq 0 ] || exit $rc
shift
bash tools/gpu_bench.sh "$@" && python3 tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv 7 24
