#!/bin/bash
# Round 5, call f: PMC of the stem-moment lag kernel, the whole GPU suite, smoke, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
R="$GRAFT_REPO_ROOT"
rm -rf $O/pmc_lag; mkdir -p $O/pmc_lag
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "k_stem" -d "$R/$O/pmc_lag" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 2 > "$R/$O/pmc_lag.log" 2>&1 ) || { tail -5 $O/pmc_lag.log; exit 1; }
python3 tools/pmc_table.py $(find $O/pmc_lag -name "*counter_collection.csv") > $O/pmc_lag.txt 2>&1; head -30 $O/pmc_lag.txt
bash tools/gpu_full.sh || exit 1
