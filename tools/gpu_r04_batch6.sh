#!/bin/bash
# Round-4 batch 6: the flip-aware fp32 model test + dense / trainer tests, the capture bisection
# of the whole-model step, the full_model block with plain GEMMs on the library vs on
# csrc/gemm.hip, and the eager whole-model step's kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests6 bash tools/gpu_r04.sh tests tests/test_gpu_model.py tests/test_gpu_dense.py tests/test_gpu_trainer.py tests/test_gpu_swin.py tests/test_gpu_conv.py
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python tools/debug_full_capture.py > $O/capture_debug.txt 2>&1; rc=$?
grep -E "OK|FAIL" $O/capture_debug.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python tools/run_full_model.py > $O/full_model.json 2> $O/full_model.err || { tail -5 $O/full_model.err; exit 1; }
cut -c1-900 $O/full_model.json
bash tools/gpu_r04.sh fullprof || exit 1
