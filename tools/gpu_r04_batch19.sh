#!/bin/bash
# Round-4 batch 19: k_dsam_lds chunks per step (RGBD_DSAM_KC=3|2, ring depth 2|3; 1 is refused
# for the 768-channel dX): stamps per setting, bench A/B.  (DSAM + bench-step tests passed
# under both settings in the previous call: gpurun_out/r04/tests19_kc{3,2}.log)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
for kc in 3 2; do
  echo "== RGBD_DSAM_KC=$kc"
  RGBD_DSAM_KC=$kc timeout -k 10 300 python tools/dsam_stamps.py > $O/dsam_stamps_kc$kc.txt 2> $O/dsam_stamps.err || { tail -5 $O/dsam_stamps.err; exit 1; }
  cat $O/dsam_stamps_kc$kc.txt
done
bash tools/gpu_ab_env.sh RGBD_DSAM_KC "3 2"
