#!/bin/bash
# Round 5, call zj: DGGM backward's final reduction with eight tiles in flight — parity / DSAM /
# model GPU tests (incl. the joint-dW and graph bitwise checks), then the bench step's trace
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bf16_parity.py tests/test_gpu_model.py tests/test_gpu_c2.py > $O/tests_zj.txt 2>&1 || { tail -30 $O/tests_zj.txt; exit 1; }
tail -2 $O/tests_zj.txt
R="$GRAFT_REPO_ROOT"
B="$R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/zj_prof" -o run --output-format csv -- python3 $B > "$R/$O/prof_zj.log" 2>&1 ) || { tail -5 "$R/$O/prof_zj.log"; exit 1; }
f=$(find gpurun_out/zj_prof -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" > $O/step_timeline_zj.txt && grep "dggm" $O/step_timeline_zj.txt && tail -1 $O/step_timeline_zj.txt
