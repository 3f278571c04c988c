#!/bin/bash
# DSAM kernel knob sweep on the micro benchmark (each run under its own limit; stop at failure).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/dsam_sweep.txt
CFGS=${DSAM_SWEEP:-"X RGBD_DSAM_KC=1 RGBD_DSAM_DBG=1 RGBD_DSAM_DBG=2"}
for cfg in $CFGS; do
  [ "$cfg" = "X" ] && cfg=""
  cfg=${cfg//,/ }
  echo "== $cfg" >> gpurun_out/dsam_sweep.txt
  env $cfg timeout -k 10 120 python tools/micro_dsam_conv.py --iters 20 >> gpurun_out/dsam_sweep.txt 2>&1 || { echo "failed: $cfg"; cat gpurun_out/dsam_sweep.txt; exit 1; }
done
cat gpurun_out/dsam_sweep.txt
