#!/bin/bash
# Round 5, call zf: region-code kernels with the window loop unrolled — decomposition / parity GPU
# tests, then their kernel times in the bench step (kernel trace, filtered)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dsam_full.py tests/test_gpu_dsam_plan.py tests/test_gpu_bf16_parity.py > $O/tests_zf.txt 2>&1 || { tail -30 $O/tests_zf.txt; exit 1; }
tail -2 $O/tests_zf.txt
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_codes|k_modes|k_hist' -d "$R/gpurun_out/zf_prof" -o run --output-format csv -- python3 "$R/tools/micro_dsam.py" --iters 5 > "$R/$O/prof_zf.log" 2>&1 ) || { tail -5 "$R/$O/prof_zf.log"; exit 1; }
f=$(find gpurun_out/zf_prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-6 "$f" > $O/codes_stats_zf.csv && cat $O/codes_stats_zf.csv
