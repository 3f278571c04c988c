#!/bin/bash
# Round 5, call zl: the final tree's bench line three times on one box (spread of `value`)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
: > $O/bench_spread_zl.txt
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --c5-stream 0 --inference 0 --parity 0 --full-model 0 > $O/bench_zl_$k.json 2> $O/bench_zl.err || { tail -5 $O/bench_zl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_zl_$k.json'));print('run $k', d['value'], d['ms_per_step'], d['eager_img_s'], d['roofline']['frac_events'], d['kernels']['k5_dsam']['ms_per_step'])" >> $O/bench_spread_zl.txt
done
cat $O/bench_spread_zl.txt
