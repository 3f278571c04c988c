#!/bin/bash
# PMC passes over a micro driver, restricted to kernels matching a regex:
#   bash tools/gpu_pmc_driver.sh tools/micro_ratio.py 'k_rp_chain' "SQ_WAVE_CYCLES SQ_WAIT_ANY" ...
# One quoted counter group per pass (kernel-trace only); each pass has its own hard limit.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmcd; mkdir -p gpurun_out/pmcd
cd /tmp && export TMPDIR=/tmp
drv="$1"; filt="$2"; shift 2
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$filt" --pmc $grp -d "$R/gpurun_out/pmcd/p$i" -o run --output-format csv -- python3 "$R/$drv" --iters 2 > "$R/gpurun_out/pmcd/p$i.log" 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 "$R/gpurun_out/pmcd/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_table.py" $(find "$R/gpurun_out/pmcd" -name "*counter_collection.csv")
