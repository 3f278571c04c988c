#!/bin/bash
# Final-tree check after the f1 attention kernels: smoke, the whole GPU suite, the whole-model
# training step A/B (fp32 and bf16 autocast).  Each GPU step under its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/tail/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/tail/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tail/gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/tail/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_full_model.py --amp 0 --steps 8 > gpurun_out/tail/full_model_fp32.json 2> gpurun_out/tail/full_model_fp32.err || exit 1
timeout -k 10 400 python -u tools/bench_full_model.py --amp 1 --steps 8 > gpurun_out/tail/full_model_amp.json 2> gpurun_out/tail/full_model_amp.err || exit 1
cat gpurun_out/tail/full_model_fp32.json gpurun_out/tail/full_model_amp.json
