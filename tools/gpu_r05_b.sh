#!/bin/bash
# Round 5, call b: the fixed tests (B=1 mask-logit gradient, bf16 forced masks), the conv5 loader /
# compute wave split A/B against the previous build, conv5's parity tests, the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_old.so --rounds 6 > $O/ab_conv5_split.txt 2>&1 || { tail -5 $O/ab_conv5_split.txt; exit 1; }
cat $O/ab_conv5_split.txt
TESTLOG=tests_b bash tools/gpu.sh tests tests/test_gpu_ddp_model.py tests/test_gpu_c2.py "tests/test_gpu_model.py" -s || exit 1
bash tools/gpu.sh bench || exit 1
