#!/bin/bash
# Round-4 batch 29: split-K reduce with one 16-byte load per split: dense / conv / trainer tests,
# the full_model block.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests29 bash tools/gpu_r04.sh tests tests/test_gpu_dense.py tests/test_gpu_conv.py tests/test_gpu_trainer.py || exit 1
timeout -k 10 600 python tools/run_full_model.py > $O/full_model29.json 2> $O/full_model.err || { tail -20 $O/full_model.err; exit 1; }
cut -c1-600 $O/full_model29.json
