#!/bin/bash
# Round 5, call u: conv5 with only its B (weights) copies / only its A (input) copies removed.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u tools/conv5_modes.py 0,1,2,3 > $O/conv5_modes_u.txt 2>&1 || { tail -8 $O/conv5_modes_u.txt; exit 1; }
cat $O/conv5_modes_u.txt
