#!/bin/bash
# Round-4 batch 31: Swin attention fragments loaded without branches; the full check (smoke, -m gpu,
# bench with the full_model block).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
bash tools/gpu_r04_full.sh || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d['kernels']['k5_dsam']['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic'],{k:d['full_model'].get(k) for k in ('eager_img_s','graph_img_s')})"
