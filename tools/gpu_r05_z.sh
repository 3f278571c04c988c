#!/bin/bash
# Round 5, call z: k_dsam_lds with every copy issued by waves 4-7 vs the kernel
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python tools/dsam_modes.py 0,16 8 > $O/dsam_modes_z.txt 2>&1 || { tail -20 $O/dsam_modes_z.txt; exit 1; }
cat $O/dsam_modes_z.txt
