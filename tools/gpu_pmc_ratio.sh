#!/bin/bash
# PMC passes over the ratio predictor (tools/micro_ratio.py, train mode, bench shape) restricted
# to kernels matching $1; remaining args = counter groups (one quoted group per pass, each within
# the per-block slot limits).  Each pass has its own limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmcr; mkdir -p gpurun_out/pmcr
cd /tmp && export TMPDIR=/tmp
filt="$1"; shift
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$filt" --pmc $grp -d "$R/gpurun_out/pmcr/p$i" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 3 > "$R/gpurun_out/pmcr/p$i.log" 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 "$R/gpurun_out/pmcr/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_table.py" $(find "$R/gpurun_out/pmcr" -name "*counter_collection.csv")
