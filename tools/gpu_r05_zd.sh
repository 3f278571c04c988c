#!/bin/bash
# Round 5, call zd: k_dsam_lds work list grouped by XCD — DSAM / parity GPU tests, then the bench
# step A/B against the previous build and the stamped per-step cycles
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_dsam_full.py tests/test_gpu_dsam_plan.py tests/test_gpu_parity.py tests/test_gpu_c2.py > $O/tests_zd.txt 2>&1 || { tail -30 $O/tests_zd.txt; exit 1; }
tail -3 $O/tests_zd.txt
timeout -k 10 300 python tools/dsam_modes.py 0 5 > $O/dsam_modes_zd.txt 2>&1 || { tail -20 $O/dsam_modes_zd.txt; exit 1; }
cat $O/dsam_modes_zd.txt
timeout -k 10 700 bash tools/gpu_ab_k5.sh - rgb-d-instance-segmentation_amd/gpurun_ab_head.so || exit 1
cp gpurun_out/ab_k5.txt $O/ab_k5_zd.txt
