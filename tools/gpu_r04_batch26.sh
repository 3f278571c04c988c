#!/bin/bash
# Round-4 batch 26: chain kernels' next-patch loads made non-blocking: ratio parity tests, chain
# stamps, the ratio micro, three bench runs.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests26 bash tools/gpu_r04.sh tests tests/test_gpu_model.py tests/test_gpu_c2.py tests/test_gpu_bf16_parity.py tests/test_gpu_parity.py || exit 1
timeout -k 10 300 python tools/chain_stamps.py > $O/chain_stamps26.txt 2>&1 || { tail -5 $O/chain_stamps26.txt; exit 1; }
cat $O/chain_stamps26.txt
for i in 1 2; do timeout -k 10 180 python tools/micro_ratio.py 2>&1 | tail -1 || exit 1; done
bash tools/gpu_ab_env.sh RGBD_UNUSED "x"
