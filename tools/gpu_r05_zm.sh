#!/bin/bash
# Round 5, call zm: k_dsam_lds with its weight / input copies sourced from L2-resident blocks (the ceiling of locality work)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python tools/dsam_modes.py 0,32,64,96 5 > $O/dsam_modes_zm.txt 2>&1 || { tail -20 $O/dsam_modes_zm.txt; exit 1; }
cat $O/dsam_modes_zm.txt
