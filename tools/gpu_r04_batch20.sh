#!/bin/bash
# Round-4 batch 20: k_dsam_lds stamps with the critical workgroups' items.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python tools/dsam_stamps.py > $O/dsam_stamps_crit.txt 2> $O/dsam_stamps.err || { tail -5 $O/dsam_stamps.err; exit 1; }
cat $O/dsam_stamps_crit.txt
