#!/bin/bash
# Round-4 batch 12: conv5 DMA spread A/B (RGBD_C3_SPREAD 0 / 1): per-step stamps of both, the
# ratio-predictor micro alternated 3x each, conv5 parity tests under the spread variant.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
for sp in 0 1; do
  echo "== spread=$sp"; RGBD_C3_SPREAD=$sp timeout -k 10 120 python tools/conv5_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for i in 1 2 3; do for sp in 0 1; do
  echo "spread=$sp $(RGBD_C3_SPREAD=$sp timeout -k 10 120 python tools/micro_ratio.py --iters 30 2>&1 | tail -1)" || exit 1
done; done
RGBD_C3_SPREAD=1 TESTLOG=tests12 bash tools/gpu_r04.sh tests tests/test_gpu_model.py tests/test_gpu_bf16_parity.py tests/test_gpu_c2.py
