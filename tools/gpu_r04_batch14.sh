#!/bin/bash
# Round-4 batch 14: 32-bit tile decode in the chain / gate kernels: chain stamps, ratio micro,
# ratio-predictor parity tests, the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 120 python tools/chain_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2 3; do timeout -k 10 120 python tools/micro_ratio.py --iters 30 2>&1 | tail -1 || exit 1; done
TESTLOG=tests14 bash tools/gpu_r04.sh tests tests/test_gpu_model.py tests/test_gpu_bf16_parity.py tests/test_gpu_c2.py tests/test_gpu_parity.py || exit 1
bash tools/gpu_r04.sh bench --full-model 0 || exit 1
