#!/bin/bash
# Round-end evidence of the tree as it stands (everything under gpurun_out/$RUN/ev):
#   smoke, the whole -m gpu suite, the default bench (the driver's commands);
#   rocprofv3 --kernel-trace --stats of the bench step (5 steps) + the step timeline / ranking;
#   PMC passes over the bench step, one counter group per pass (HBM bytes, MFMA busy, wave states).
# Every GPU step has its own time limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${RUN:-r05}/ev"; mkdir -p "$O"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread -p no:cacheprovider > "$O/tests_full.log" 2>&1
rc=$?; tail -3 "$O/tests_full.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['events_avg_us'],d['kernels']['k5_dsam']['ms_per_step'])"
B="$R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 $B > "$O/prof.log" 2>&1 ) || { tail -5 "$O/prof.log"; exit 1; }
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/step_timeline.py" "$f" > "$O/step_timeline.txt" || exit 1
python3 "$R/tools/step_kernel_ranking.py" "$f" > "$O/step_ranking.txt" || exit 1
tail -1 "$O/step_timeline.txt"
pass() {  # idx counters...
  local idx=$1; shift
  mkdir -p "$O/pmc/p$idx"
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$O/pmc/p$idx" -o run --output-format csv -- python3 $B > "$O/pmc/p$idx.log" 2>&1 ) \
    || { echo "pmc pass $idx ($*) failed"; tail -5 "$O/pmc/p$idx.log"; return 1; }
}
pass 1 FETCH_SIZE || exit 1
pass 2 WRITE_SIZE || exit 1
pass 3 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
pass 4 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS || exit 1
python3 "$R/tools/traffic_table.py" "$O/pmc" "$O/pmc_traffic.json" > "$O/pmc_table.txt" 2>&1 || exit 1
python3 "$R/tools/pmc_table.py" $(find "$O/pmc" -name "*counter_collection.csv") >> "$O/pmc_table.txt" 2>&1
echo evidence done
