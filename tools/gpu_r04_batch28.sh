#!/bin/bash
# Round-4 batch 28: loads without per-element branches in the chain prefetch (phases 1-2), the
# DSAM item tables and dW planning, im2col and the GEMM epilogue: the full check (smoke, -m gpu,
# bench with the full_model block), then chain / DSAM stamps and the ratio micro.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
bash tools/gpu_r04_full.sh || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d['kernels']['k5_dsam']['ms_per_step'],{k:d['full_model'].get(k) for k in ('eager_img_s','graph_img_s')})"
timeout -k 10 300 python tools/chain_stamps.py > $O/chain_stamps28.txt 2>&1 || { tail -5 $O/chain_stamps28.txt; exit 1; }
cat $O/chain_stamps28.txt
timeout -k 10 300 python tools/dsam_stamps.py > $O/dsam_stamps28.txt 2> $O/dsam_stamps.err || { tail -5 $O/dsam_stamps.err; exit 1; }
grep -E "launch|tables" $O/dsam_stamps28.txt
for i in 1 2; do timeout -k 10 180 python tools/micro_ratio.py 2>&1 | tail -1 || exit 1; done
