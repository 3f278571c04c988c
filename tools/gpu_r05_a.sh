#!/bin/bash
# Round 5, first GPU call: the tests changed this round (parity with forced reference masks,
# cast epochs on replay, world-8 DDP rehearsals, whole-model DDP), then smoke and the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
bash tools/gpu.sh smoke || exit 1
TESTLOG=tests_a bash tools/gpu.sh tests tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py \
  tests/test_gpu_bench_ddp.py tests/test_gpu_dsam_plan.py tests/test_gpu_parity.py -s || exit 1
bash tools/gpu.sh bench || exit 1
