#!/bin/bash
# A/B of library builds on the bench step (graph value, eager per-leg K5 timers): args = .so
# paths relative to the repo ("-" = the in-tree build); 3 alternating rounds, one process each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/ab_k5.txt
for rep in 1 2 3; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset RGBD_HIP_LIB; else export RGBD_HIP_LIB="$GRAFT_REPO_ROOT/$lib"; fi
    timeout -k 10 200 python bench.py --cpu-baseline 0 --c5-stream 0 --inference 0 --parity 0 --full-model 0 > gpurun_out/ab_k5.json 2> gpurun_out/ab_k5.err || { echo "bench failed: $lib"; tail -5 gpurun_out/ab_k5.err; exit 1; }
    python3 - "$lib" >> gpurun_out/ab_k5.txt <<'PY'
import json, sys; d = json.load(open("gpurun_out/ab_k5.json")); k = d["kernel_ms"]
print(f"{sys.argv[1]:32s} value {d['value']:8.1f} ms/step {d['ms_per_step']:.4f} k5 {d['kernels']['k5_dsam'].get('ms_per_step', 0):.4f} "
      f"fwd {k['dsam_fwd']:.4f} dx {k['dsam_dx']:.4f} wgrad {k['dsam_wgrad']:.4f}")
PY
  done
done
unset RGBD_HIP_LIB
cat gpurun_out/ab_k5.txt
