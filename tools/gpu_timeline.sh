#!/bin/bash
# Kernel trace of the bench step (graph replay last) and the per-step timeline of its last step.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 > "$R/gpurun_out/tl/prof.log" 2>&1 || { echo "rocprof failed $?"; tail -5 "$R/gpurun_out/tl/prof.log"; exit 1; }
f=$(find "$R/gpurun_out/tl/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/step_timeline.py" "$f" > "$R/gpurun_out/tl/timeline.txt"
n=$(python3 - "$f" <<'PY'
import csv,sys
print(sum(1 for r in csv.DictReader(open(sys.argv[1])) if 'k_prep_pass1_q' in r['Kernel_Name']))
PY
)
python3 "$R/tools/step_timeline.py" "$f" k_prep_pass1_q 1 > "$R/gpurun_out/tl/timeline_eager.txt"
tail -3 "$R/gpurun_out/tl/timeline.txt"; tail -1 "$R/gpurun_out/tl/timeline_eager.txt"; echo "markers $n"
