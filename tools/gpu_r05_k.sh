#!/bin/bash
# Round 5, call k: the stem moments with the border workgroups inside the lag launch and one sums
# launch (tests, A/B vs HEAD, kernel trace of the ratio predictor), and the whole-model glue by call
# site (TorchFunctionMode ranges).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
R="$GRAFT_REPO_ROOT"
TESTLOG=tests_k bash tools/gpu.sh tests tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_c2.py tests/test_gpu_parity.py -k "stem or graph or ratio or parity" || exit 1
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_head.so --rounds 6 > $O/ab_k.txt 2>&1 || { tail -5 $O/ab_k.txt; exit 1; }
cat $O/ab_k.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_ratio_k" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 5 > "$R/$O/prof_ratio_k.log" 2>&1 ) || { tail -5 $O/prof_ratio_k.log; exit 1; }
f=$(find $O/prof_ratio_k -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-120 | head -24
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources_k.txt > $O/glue_sources_k.log 2>&1 || { tail -8 $O/glue_sources_k.log; exit 1; }
head -70 $O/glue_sources_k.txt
