#!/bin/bash
# Round 5, call v: conv5 with the A copies on the compute waves, waited for every three steps
# (ratio tests, A/B vs the earlier build, modes).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_v bash tools/gpu.sh tests tests/test_gpu_c2.py tests/test_gpu_parity.py tests/test_gpu_model.py -k "ratio or parity or stem or bf16" || exit 1
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_head.so --rounds 8 > $O/ab_v.txt 2>&1 || { tail -5 $O/ab_v.txt; exit 1; }
cat $O/ab_v.txt
timeout -k 10 300 python -u tools/conv5_modes.py 0,2,3 > $O/conv5_modes_v.txt 2>&1 || { tail -8 $O/conv5_modes_v.txt; exit 1; }
cat $O/conv5_modes_v.txt
