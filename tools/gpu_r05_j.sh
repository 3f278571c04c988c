#!/bin/bash
# Round 5, call j: conv5 with the BN sums in LDS (A/B vs HEAD) and its lockstep / fragment-stream
# costs (diagnostic modes).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_j bash tools/gpu.sh tests tests/test_gpu_c2.py tests/test_gpu_parity.py -k "ratio or parity" || exit 1
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_head.so --rounds 6 > $O/ab_j.txt 2>&1 || { tail -5 $O/ab_j.txt; exit 1; }
cat $O/ab_j.txt
timeout -k 10 300 python -u tools/conv5_modes.py > $O/conv5_modes_j.txt 2>&1 || { tail -8 $O/conv5_modes_j.txt; exit 1; }
cat $O/conv5_modes_j.txt
