#!/bin/bash
# Bench value under several environment settings (A/B of run-time switches), two passes each in
# interleaved order.  BENCH_ENVS: space-separated configs, ',' separating variables, X = none.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/bench_env.txt
for pass in 1 2; do
  for cfg in ${BENCH_ENVS:-X}; do
    [ "$cfg" = "X" ] && c="" || c=${cfg//,/ }
    v=$(env $c timeout -k 10 300 python bench.py --cpu-baseline 0 --c5-stream 0 --parity 0 --inference 0 2> gpurun_out/bench_env.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['eager_img_s'])") || { echo "failed: $cfg"; tail -5 gpurun_out/bench_env.err; exit 1; }
    echo "pass $pass  $cfg  $v" | tee -a gpurun_out/bench_env.txt
  done
done
