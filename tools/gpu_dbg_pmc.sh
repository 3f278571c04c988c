#!/bin/bash
# PMC passes on tools/micro_dsam_conv.py under RGBD_DSAM_DBG=$1, kernels matching $2; remaining
# args = counter groups (one pass each, own time limit).
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dbgpmc
cd /tmp && export TMPDIR=/tmp
d="$1"; filt="$2"; shift 2
i=0
for grp in "$@"; do
  i=$((i+1))
  RGBD_DSAM_DBG=$d timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$filt" --pmc $grp -d "$R/gpurun_out/dbgpmc/d${d}p$i" -o run --output-format csv -- python3 "$R/tools/micro_dsam_conv.py" --iters 3 > "$R/gpurun_out/dbgpmc/d${d}p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/dbgpmc/d${d}p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_table.py" $(find "$R/gpurun_out/dbgpmc" -path "*d${d}p*" -name "*counter_collection.csv")
