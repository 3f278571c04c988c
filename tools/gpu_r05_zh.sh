#!/bin/bash
# Round 5, call zh: the ratio tail kernels with their staging loads issued together — ratio /
# decomposition / parity GPU tests, then the bench step's kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c2.py tests/test_gpu_parity.py tests/test_gpu_bf16_parity.py tests/test_gpu_dsam_full.py > $O/tests_zh.txt 2>&1 || { tail -30 $O/tests_zh.txt; exit 1; }
tail -2 $O/tests_zh.txt
R="$GRAFT_REPO_ROOT"
B="$R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/zh_prof" -o run --output-format csv -- python3 $B > "$R/$O/prof_zh.log" 2>&1 ) || { tail -5 "$R/$O/prof_zh.log"; exit 1; }
f=$(find gpurun_out/zh_prof -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" > $O/step_timeline_zh.txt && sed -n 20,32p $O/step_timeline_zh.txt && tail -1 $O/step_timeline_zh.txt
cp $(find gpurun_out/zh_prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats_zh.csv
