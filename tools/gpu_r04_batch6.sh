#!/bin/bash
# Round-4 batch 6: the flip-aware fp32 model test, the capture bisection of the whole-model
# step, and the eager whole-model step's kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests6 bash tools/gpu_r04.sh tests tests/test_gpu_model.py::test_full_model_mask_logits_fp32
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python tools/debug_full_capture.py > $O/capture_debug.txt 2>&1; rc=$?
cat $O/capture_debug.txt | grep -E "OK|FAIL"; [ $rc -ge 124 ] && exit $rc
bash tools/gpu_r04.sh fullprof || exit 1
