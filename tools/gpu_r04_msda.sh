#!/bin/bash
# Round-4: whole-model work — run-carrying MSDA backward, colsum chunking, sort-free matched rows
# + cached targets in the loss, device constants, the captured whole-model step: parity tests,
# the C2 MSDA micro A/B (per-query vs runs; random vs initialisation-like constant offsets), the
# full_model block (eager + captured) and the eager step's kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests_msda bash tools/gpu_r04.sh tests tests/test_gpu_msda.py tests/test_gpu_dense.py tests/test_gpu_point_loss.py tests/test_gpu_model.py tests/test_gpu_trainer.py || exit 1
for runs in 0 1; do for off in "" "--const-offsets"; do
  RGBD_MSDA_RUNS=$runs timeout -k 10 120 python tools/micro_msda.py $off > $O/msda_${runs}${off}.json 2>&1 || { tail -5 $O/msda_${runs}${off}.json; exit 1; }
  echo "runs=$runs $off: $(tail -1 $O/msda_${runs}${off}.json)"
done; done
timeout -k 10 600 python tools/run_full_model.py > $O/full_model.json 2> $O/full_model.err || { tail -20 $O/full_model.err; exit 1; }
cat $O/full_model.json
bash tools/gpu_r04.sh fullprof || exit 1
