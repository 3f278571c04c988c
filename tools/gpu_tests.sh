#!/bin/bash
# GPU test driver: each GPU step under its own timeout; stop at the first GPU failure.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests.log
exit $rc
