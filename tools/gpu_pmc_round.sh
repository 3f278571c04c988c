#!/bin/bash
# PMC passes (kernel trace only, one counter group per pass, each pass its own time limit;
# MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE in separate passes).
#   ratio:  the ratio predictor (tools/micro_ratio.py, train mode, bench shape) — conv5, chain,
#           gate, pool: HBM bytes, MFMA busy, wave-state counters.
#   dsam:   the hot path's K5 legs (tools/micro_dsam.py, the bench's step): the same counters.
#   step:   the bench's default step itself (bench.py, short run): every kernel of the step.
# Tables: tools/traffic_table.py -> gpurun_out/<run>/pmc_<which>.json (+ pmc_table.py text).
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${RUN:-r05}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run_pass() {  # which driver-args group-index counters...
  local which=$1 drv=$2 idx=$3; shift 3
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$O/pmc_$which/p$idx" -o run --output-format csv -- python3 $drv > "$O/pmc_$which/p$idx.log" 2>&1 \
    || { echo "pmc $which pass $idx ($*) failed"; tail -5 "$O/pmc_$which/p$idx.log"; return 1; }
}
for which in "$@"; do
  case "$which" in
    ratio) drv="$R/tools/micro_ratio.py --iters 3" ;;
    dsam)  drv="$R/tools/micro_dsam.py --iters 2" ;;
    step)  drv="$R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0" ;;
    *) echo "unknown $which"; exit 2 ;;
  esac
  rm -rf "$O/pmc_$which"; mkdir -p "$O/pmc_$which"
  run_pass "$which" "$drv" 1 FETCH_SIZE || exit 1
  run_pass "$which" "$drv" 2 WRITE_SIZE || exit 1
  run_pass "$which" "$drv" 3 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
  run_pass "$which" "$drv" 4 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS || exit 1
  python3 "$R/tools/traffic_table.py" "$O/pmc_$which" "$O/pmc_$which.json" > "$O/pmc_$which.txt" 2>&1 || exit 1
  python3 "$R/tools/pmc_table.py" $(find "$O/pmc_$which" -name "*counter_collection.csv") >> "$O/pmc_$which.txt" 2>&1
done
echo done
