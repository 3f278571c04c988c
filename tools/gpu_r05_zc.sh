#!/bin/bash
# Round 5, call zc: early dW1 fork (bitwise test + captured-step A/B); L2 hits of k_dsam_lds's
# A-only and B-only copy streams (stamped modes 1 and 2 vs 0, one PMC pass)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k joint_dw > $O/test_joint_zc.txt 2>&1 || { tail -30 $O/test_joint_zc.txt; exit 1; }
tail -3 $O/test_joint_zc.txt
timeout -k 10 300 python tools/ab_joint_dw.py --micro 0 --rounds 6 --iters 20 > $O/ab_joint_zc.txt 2>&1 || { tail -20 $O/ab_joint_zc.txt; exit 1; }
tail -2 $O/ab_joint_zc.txt
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --kernel-include-regex 'k_dsam_lds' --pmc TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/pmcm/p1" -o run --output-format csv -- python3 "$R/tools/dsam_modes.py" 0,1,2 1 > "$R/$O/pmc_modes_zc.log" 2>&1 || { tail -20 "$R/$O/pmc_modes_zc.log"; exit 1; }
python3 "$R/tools/pmc_table.py" $(find "$R/gpurun_out/pmcm/p1" -name "*counter_collection.csv") > "$R/$O/pmc_modes_zc.txt" && cat "$R/$O/pmc_modes_zc.txt"
