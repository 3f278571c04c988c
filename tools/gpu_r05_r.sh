#!/bin/bash
# Round 5, call r: the eager step (what N > 1 runs) under the kernel trace — where the GPU waits
# for the host.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r05"; mkdir -p $O
B="$R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0 --graph 0"
timeout -k 10 300 python $B > $O/bench_eager.json 2> $O/bench_eager.err || { tail -5 $O/bench_eager.err; exit 1; }
cat $O/bench_eager.json | head -c 400; echo
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_eager" -o run --output-format csv -- python3 $B > "$O/prof_eager.log" 2>&1 ) || { tail -5 "$O/prof_eager.log"; exit 1; }
f=$(find "$O/prof_eager" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/step_timeline.py" "$f" > "$O/step_timeline_eager.txt" || exit 1
tail -1 "$O/step_timeline_eager.txt"
