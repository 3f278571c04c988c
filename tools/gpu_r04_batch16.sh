#!/bin/bash
# Round-4 batch 16: gate prefetch depth A/B (RGBD_GATE_PF=1|2): ratio parity tests under PF=2, the
# ratio micro per depth, a short bench per depth.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
RGBD_GATE_PF=2 TESTLOG=tests16 bash tools/gpu_r04.sh tests tests/test_gpu_model.py tests/test_gpu_c2.py tests/test_gpu_bf16_parity.py || exit 1
for pf in 1 2 1 2; do
  echo "== RGBD_GATE_PF=$pf"
  RGBD_GATE_PF=$pf timeout -k 10 180 python tools/micro_ratio.py 2>&1 | tail -4 || exit 1
  RGBD_GATE_PF=$pf timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_pf$pf.json 2> $O/bench_pf$pf.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_pf$pf.json'));print('bench',d['value'],d['kernels'].get('k5_dsam'))"
done
