#!/bin/bash
# Iteration driver: selected GPU tests (one pytest process), the DSAM micro benchmark, the bench
# line.  Each GPU step under its own limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $1 -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_sel.log 2>&1
rc=$?; tail -8 gpurun_out/tests_sel.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/micro_dsam_conv.py --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python bench.py --cpu-baseline 0 --c5-stream 0 --parity 0 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -5 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json; d = json.load(open("gpurun_out/bench.json"))
print("value", d["value"], "ms/step", d["ms_per_step"], "inf", d["inference_img_s"]); print(d["kernel_ms"]); print(d["kernels"]["k5_dsam"])
PY
