#!/bin/bash
# Round 5, call za: L2 hit rate of the DSAM conv / dW / pack kernels (one PMC pass on the eager
# step); which DSAMs to pack beside the ratio predictor (captured step, alternating variants)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python tools/ab_prepack.py 01 0 - --rounds 6 --steps 20 > $O/ab_prepack_za.txt 2>&1 || { tail -20 $O/ab_prepack_za.txt; exit 1; }
cat $O/ab_prepack_za.txt
bash tools/gpu_pmc_step.sh 'k_dsam_lds|k_dsam_wgrad|k_pack_codes' "TCC_HIT_sum TCC_MISS_sum" || exit 1
python3 tools/pmc_table.py $(find gpurun_out/pmcs/p1 -name '*counter_collection.csv') > $O/pmc_l2_za.txt && cat $O/pmc_l2_za.txt
