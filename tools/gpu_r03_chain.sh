#!/bin/bash
# Round-3 GPU chain: smoke, bench, rocprof of the bench step, then the new dense / Swin tests,
# then the whole GPU suite.  Test failures (pytest rc 1) do not stop the chain; a fault, abort,
# segfault or time limit (any other non-zero rc) does, and nothing else runs on the GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
step() {
  "$@"; local rc=$?
  echo "== $* -> rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping the chain"; exit $rc; fi
  return 0
}
step bash tools/gpu_r03.sh smoke
step bash tools/gpu_r03.sh bench
step bash tools/gpu_r03.sh prof
TESTLOG=new step bash tools/gpu_r03.sh tests tests/test_gpu_dense.py tests/test_gpu_swin.py
step bash tools/gpu_r03.sh tests tests --ignore=tests/test_gpu_dense.py --ignore=tests/test_gpu_swin.py
