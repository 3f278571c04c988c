#!/bin/bash
# Round 5, call y: k_dsam_lds step cost decomposed (copies / barrier / fragment reads removed in turn)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python tools/dsam_modes.py 0,1,2,3,7,8,15 5 > $O/dsam_modes_y.txt 2>&1 || { tail -20 $O/dsam_modes_y.txt; exit 1; }
cat $O/dsam_modes_y.txt
