#!/bin/bash
# Round-4 full GPU check as the driver runs it: smoke, the whole -m gpu suite, the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${RUN:-r05}; mkdir -p $O
bash tools/gpu.sh smoke || exit 1
TESTLOG=tests_full timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests_full.log 2>&1
rc=$?; tail -5 $O/tests_full.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh bench || exit 1
