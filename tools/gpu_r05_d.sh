#!/bin/bash
# Round 5, call d: conv5 stamps (diag build, loader/compute split), the changed GPU tests
# (AdamW bf16 shadows, replay epochs, world-8 DDP rehearsals, whole-model DDP), the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 200 python tools/conv5_stamps.py > $O/conv5_stamps_split.txt 2>&1 || { tail -5 $O/conv5_stamps_split.txt; exit 1; }
cat $O/conv5_stamps_split.txt
TESTLOG=tests_d bash tools/gpu.sh tests "tests/test_gpu_model.py::test_bf16_stem_bn_batch_stats_exact" tests/test_gpu_adamw.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py \
  tests/test_gpu_bench_ddp.py -s || exit 1
bash tools/gpu.sh bench || exit 1
