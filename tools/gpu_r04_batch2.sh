#!/bin/bash
# Round-4 batch 2: the segment-GEMM dW (hot_path.SEG_DW) — its parity tests and the hot-path
# tests that exercise it, then the bench and a kernel-trace profile.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
TESTLOG=tests2 bash tools/gpu_r04.sh tests tests/test_gpu_dsam_plan.py tests/test_gpu_parity.py tests/test_gpu_dsam_full.py tests/test_gpu_c2.py tests/test_gpu_train_graph.py tests/test_gpu_bf16_parity.py || exit 1
bash tools/gpu_r04.sh bench || exit 1
bash tools/gpu_r04.sh prof || exit 1
