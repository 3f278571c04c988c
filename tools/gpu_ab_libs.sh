#!/bin/bash
# A/B bench of several library builds on one box (alternating, 2 rounds): args = .so paths
# relative to the repo ("-" = the in-tree build).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/ab_libs.txt
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset RGBD_HIP_LIB; else export RGBD_HIP_LIB="$GRAFT_REPO_ROOT/$lib"; fi
    timeout -k 10 200 python bench.py --cpu-baseline 0 --c5-stream 0 --inference 0 --parity 0 --full-model 0 > gpurun_out/ab_libs.json 2> gpurun_out/ab_libs.err || { echo "bench failed: $lib"; tail -5 gpurun_out/ab_libs.err; exit 1; }
    python3 - "$lib" >> gpurun_out/ab_libs.txt <<'PY'
import json, sys; d = json.load(open("gpurun_out/ab_libs.json")); k = d["kernel_ms"]
print(f"{sys.argv[1]:32s} value {d['value']:8.1f} conv5 {k['rp_conv3x3']:.4f} chain {k['rp_chain']:.4f} dggm_fwd {k['dggm_fwd']:.4f} dggm_bwd {k['dggm_bwd']:.4f}")
PY
  done
done
unset RGBD_HIP_LIB
cat gpurun_out/ab_libs.txt
