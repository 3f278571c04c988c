#!/bin/bash
# Round 5, call p: gate kernel with two tiles in flight per wave (A/B vs the product build), and
# the ratio predictor's kernel trace with the reworked stem moments.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_gate2.so --rounds 8 > $O/ab_p.txt 2>&1 || { tail -5 $O/ab_p.txt; exit 1; }
cat $O/ab_p.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_ratio_p" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 5 > "$R/$O/prof_ratio_p.log" 2>&1 ) || { tail -5 $O/prof_ratio_p.log; exit 1; }
f=$(find $O/prof_ratio_p -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-120 | head -24
