#!/bin/bash
# Round-4 batch 25: point sampling with branch-free tap loads: point-loss + trainer tests, full_model.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests25 bash tools/gpu_r04.sh tests tests/test_gpu_point_loss.py tests/test_gpu_trainer.py tests/test_gpu_model.py || exit 1
timeout -k 10 600 python tools/run_full_model.py > $O/full_model25.json 2> $O/full_model.err || { tail -20 $O/full_model.err; exit 1; }
cut -c1-700 $O/full_model25.json
