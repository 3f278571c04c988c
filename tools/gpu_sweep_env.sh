#!/bin/bash
# bench under different tuning environments: each argument is "VAR=val[,VAR=val...]" ("-" = none)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=""
  [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 200 python bench.py --cpu-baseline 0 --c5-stream 0 --inference 0 > gpurun_out/sw_$i.json 2>/dev/null || { echo "cfg $cfg failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sw_$i.json')); k=d['kernel_ms']; print('$cfg', d['value'], k['dsam_fwd'], k['dsam_dx'], k['dsam_wgrad'])"
done
