#!/bin/bash
# Bench A/B of an environment switch on one box: alternating runs of bench.py (3 each), so DVFS /
# box differences cancel.   bash tools/gpu_ab_env.sh VAR "a b"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
var=$1; vals=$2
: > gpurun_out/ab_env.txt
for rep in 1 2 3; do
  for v in $vals; do
    env "$var=$v" timeout -k 10 300 python bench.py --cpu-baseline 0 --c5-stream 0 --parity 0 --inference 0 --full-model 0 > gpurun_out/ab_env.json 2> gpurun_out/ab_env.err || { echo "bench failed"; tail -5 gpurun_out/ab_env.err; exit 1; }
    python - "$var=$v" >> gpurun_out/ab_env.txt <<'PY'
import json, sys; d = json.load(open("gpurun_out/ab_env.json"))
k = d["kernel_ms"]
print(sys.argv[1], "value", d["value"], "conv5", k["rp_conv3x3"], "dsam fwd/dx/dw", k.get("dsam_fwd"), k.get("dsam_dx"), k.get("dsam_wgrad"), "k5", d.get("kernels", {}).get("k5_dsam", {}).get("ms_per_step"), "eager", d.get("eager_img_s"))
PY
  done
done
cat gpurun_out/ab_env.txt
