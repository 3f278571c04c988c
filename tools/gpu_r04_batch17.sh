#!/bin/bash
# Round-4 batch 17: k_dsam_lds N tile picked by XCD: DSAM parity tests (on), bench A/B on / off.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests17 bash tools/gpu_r04.sh tests tests/test_gpu_dsam_full.py tests/test_gpu_dsam_plan.py tests/test_gpu_c2.py || exit 1
bash tools/gpu_ab_env.sh RGBD_DSAM_XCD "0 1"
