#!/bin/bash
# bench + kernel-trace profile; every GPU step has its own time limit and the chain stops at
# the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
