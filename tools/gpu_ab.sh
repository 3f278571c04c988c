#!/bin/bash
# A/B bench of two library builds on one box: $1 = the alternative .so (relative to the repo).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --c5-stream 0 --inference 0 --parity 0 > gpurun_out/ab_new$i.json 2>/dev/null || exit 1
  RGBD_HIP_LIB="$GRAFT_REPO_ROOT/$1" timeout -k 10 200 python bench.py --cpu-baseline 0 --c5-stream 0 --inference 0 --parity 0 > gpurun_out/ab_old$i.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for tag in ("new1", "old1", "new2", "old2"):
    d = json.load(open(f"gpurun_out/ab_{tag}.json"))
    print(tag, d["value"], d["kernel_ms"]["rp_conv3x3"], d["kernel_ms"]["rp_chain"])
PY
