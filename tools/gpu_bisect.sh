#!/bin/bash
# One GPU test file under several environment settings (bisection of a run-time switch); stops at
# the first failure.  BISECT_ENVS: space-separated configs, ',' separating variables, X = none.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in ${BISECT_ENVS:-X}; do
  [ "$cfg" = "X" ] && c="" || c=${cfg//,/ }
  env $c timeout -k 10 300 python -u -m pytest $1 -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/bisect.log 2>&1
  rc=$?
  echo "$cfg rc=$rc $(tail -1 gpurun_out/bisect.log)"
  [ $rc -eq 0 ] || exit $rc
done
