#!/bin/bash
# Round-2 evidence run: bench line, kernel-trace profile of the bench step, and the PMC passes
# (HBM bytes, MFMA busy, instruction mix) over the same step (tools/micro_dsam.py), one counter
# group per pass.  Each GPU step under its own limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/full
timeout -k 10 600 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/full/bench.err; exit 1; }
cat gpurun_out/full/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/full/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 > "$R/gpurun_out/full/prof.log" 2>&1 || { echo "rocprof failed $?"; tail -5 "$R/gpurun_out/full/prof.log"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/full/p$i" -o run --output-format csv -- python3 "$R/tools/micro_dsam.py" --iters 2 > "$R/gpurun_out/full/p$i.log" 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 "$R/gpurun_out/full/p$i.log"; exit 1; }
done
echo done
