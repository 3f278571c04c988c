#!/bin/bash
# Round-4 batch 21: k_dsam_lds multi-chunk reduction with one chunk of partial loads in flight:
# DSAM + bench-step tests, stamps, three bench runs.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests21 bash tools/gpu_r04.sh tests tests/test_gpu_dsam_full.py tests/test_gpu_dsam_plan.py tests/test_gpu_c2.py tests/test_gpu_parity.py || exit 1
timeout -k 10 300 python tools/dsam_stamps.py > $O/dsam_stamps_red.txt 2> $O/dsam_stamps.err || { tail -5 $O/dsam_stamps.err; exit 1; }
cat $O/dsam_stamps_red.txt
bash tools/gpu_ab_env.sh RGBD_UNUSED "x"
