#!/bin/bash
# PMC passes restricted to kernels matching $1 over the bench step (tools/micro_dsam.py);
# remaining args = counter groups (one quoted group per pass).  Each pass has its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmck
cd /tmp && export TMPDIR=/tmp
filt="$1"; shift
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$filt" --pmc $grp -d "$R/gpurun_out/pmck/p$i" -o run --output-format csv -- python3 "$R/tools/micro_dsam.py" --iters 2 > "$R/gpurun_out/pmck/p$i.log" 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 "$R/gpurun_out/pmck/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_table.py" $(find "$R/gpurun_out/pmck" -name "*counter_collection.csv")
