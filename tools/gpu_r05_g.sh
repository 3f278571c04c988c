#!/bin/bash
# Round 5, call g: conv5 v5 (4 waves, AGPR accumulators) and the scratch-free stem lag kernel,
# A/B against the committed build, kernel trace, conv5 / ratio / DDP tests, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
R="$GRAFT_REPO_ROOT"
TESTLOG=tests_g bash tools/gpu.sh tests tests/test_gpu_c2.py tests/test_gpu_model.py tests/test_gpu_ddp_model.py -s || exit 1
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_v3.so --rounds 6 > $O/ab_g.txt 2>&1 || { tail -5 $O/ab_g.txt; exit 1; }
cat $O/ab_g.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_ratio_g" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 5 > "$R/$O/prof_ratio_g.log" 2>&1 ) || { tail -5 $O/prof_ratio_g.log; exit 1; }
f=$(find $O/prof_ratio_g -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-120 | head -24
bash tools/gpu.sh bench || exit 1
