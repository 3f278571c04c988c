#!/bin/bash
# The bench step under rocprofv3 --kernel-trace --stats only (no tests, no PMC passes) and its
# step timeline (tools/step_timeline.py): gpurun_out/r06/$TAG/step_timeline.txt.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r06/${TAG:-qt}"; mkdir -p "$O"
B="$R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 $B > "$O/prof.log" 2>&1 ) || { tail -5 "$O/prof.log"; exit 1; }
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/step_timeline.py" "$f" > "$O/step_timeline.txt" || exit 1
tail -1 "$O/step_timeline.txt"
