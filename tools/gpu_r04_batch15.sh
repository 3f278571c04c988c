#!/bin/bash
# Round-4 batch 15: LDS-DMA weight-gradient GEMM (transposed fragments, split-K): dense tests, the
# GEMM micro with it on / off, the full_model block.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests15 bash tools/gpu_r04.sh tests tests/test_gpu_dense.py tests/test_gpu_trainer.py || exit 1
for tt in 0 1; do
  echo "== RGBD_GEMM_LDS_TT=$tt"
  RGBD_GEMM_LDS_TT=$tt timeout -k 10 180 python tools/micro_gemm.py 2>&1 | grep '"dW"' | cut -c1-200 || exit 1
done
timeout -k 10 600 python tools/run_full_model.py > $O/full_model.json 2> $O/full_model.err || { tail -5 $O/full_model.err; exit 1; }
cut -c1-700 $O/full_model.json
