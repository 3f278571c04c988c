#!/bin/bash
# PMC passes (kernel-trace only, one counter group per pass) on the full-step micro driver,
# restricted to kernels matching $1 (regex).  Each pass has its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmcs
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
filt="$1"; shift
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "$filt" --pmc $grp -d "$R/gpurun_out/pmcs/p$i" -o run --output-format csv -- python3 "$R/tools/micro_dsam.py" --iters 2 > "$R/gpurun_out/pmcs/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$R/gpurun_out/pmcs/p$i.log"; exit 1; }
done
echo done
