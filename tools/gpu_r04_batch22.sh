#!/bin/bash
# Round-4 batch 22: MSDA kernels with branch-free tap loads (and the runs backward's slot values
# issued before its stores / atomics): MSDA + model tests, the C2 micro (per-query vs runs, random vs
# constant offsets), the full_model block.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests22 bash tools/gpu_r04.sh tests tests/test_gpu_msda.py tests/test_gpu_trainer.py || exit 1
for runs in 0 1; do for off in "" "--const-offsets"; do
  RGBD_MSDA_RUNS=$runs timeout -k 10 120 python tools/micro_msda.py $off > $O/msda22_${runs}${off}.json 2>&1 || { tail -5 $O/msda22_${runs}${off}.json; exit 1; }
  echo "runs=$runs $off: $(tail -1 $O/msda22_${runs}${off}.json)"
done; done
timeout -k 10 600 python tools/run_full_model.py > $O/full_model22.json 2> $O/full_model.err || { tail -20 $O/full_model.err; exit 1; }
cut -c1-1500 $O/full_model22.json
