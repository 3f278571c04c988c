#!/bin/bash
# HBM-traffic / MFMA-busy PMC passes over the bench's full train step (tools/micro_dsam.py),
# kernel-trace only, one counter group per pass (MI355X_MICROARCH.md "rocprofv3 PMC slots":
# FETCH_SIZE and WRITE_SIZE cannot share a pass).  Each pass has its own time limit; the chain
# stops at the first failure.  Summarise with tools/traffic_table.py.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/traffic
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/traffic/counters.txt" 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/traffic/p$i" -o run --output-format csv -- python3 "$R/tools/micro_dsam.py" --iters 2 > "$R/gpurun_out/traffic/p$i.log" 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 "$R/gpurun_out/traffic/p$i.log"; exit 1; }
done
# f1 mask-predictor kernels at the C2 shape
j=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  j=$((j+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/traffic/m$j" -o run --output-format csv -- python3 "$R/tools/micro_mask.py" --iters 2 --no-torch > "$R/gpurun_out/traffic/m$j.log" 2>&1 || { echo "mask pmc pass $j ($grp) failed"; tail -5 "$R/gpurun_out/traffic/m$j.log"; exit 1; }
done
echo done
