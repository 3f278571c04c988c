#!/bin/bash
# Round-4 batch 10: unsorted top-k in the loss: point-loss / trainer tests, the full_model block.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests10 bash tools/gpu_r04.sh tests tests/test_gpu_point_loss.py tests/test_gpu_trainer.py tests/test_gpu_model.py
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python tools/run_full_model.py > $O/full_model.json 2> $O/full_model.err || { tail -5 $O/full_model.err; exit 1; }
cut -c1-1200 $O/full_model.json
