#!/bin/bash
# GPU driver.  Stages (arguments, in order): smoke | tests [pytest args...] | bench | prof.
#   tests: the GPU suite (or the given test selection) without -x, so one call reports every
#          failure; a hang ends at the per-test timeout.
#   bench: bench.py default run (the driver's command).
#   prof:  rocprofv3 kernel trace + stats of a short bench run.
# Every GPU step has its own time limit; the chain stops at the first failing stage.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/${RUN:-r05}
O="$R/gpurun_out/${RUN:-r05}"
stage="$1"; shift
case "$stage" in
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
    rc=$?; tail -2 "$O/smoke.log"; exit $rc ;;
  tests)
    log="$O/${TESTLOG:-tests}.log"
    timeout -k 10 1000 python -u -m pytest -m gpu -q -rfP --timeout 400 --timeout-method thread -p no:cacheprovider "${@:-tests}" > "$log" 2>&1
    rc=$?; tail -25 "$log"; exit $rc ;;
  bench)
    timeout -k 10 600 python bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
    rc=$?; cat "$O/bench.json"; [ $rc -eq 0 ] || tail -20 "$O/bench.err"; exit $rc ;;
  prof)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0 "$@" > "$O/prof.log" 2>&1
    rc=$?; tail -3 "$O/prof.log"; exit $rc ;;
  fullprof)  # the whole drop-in model's training step (tools/bench_full_model.py) under the kernel trace
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/fullprof" -o run --output-format csv -- python3 "$R/tools/bench_full_model.py" --arms hip --steps 3 "$@" > "$O/fullprof.log" 2>&1
    rc=$?; tail -3 "$O/fullprof.log"; exit $rc ;;
  full)  # the whole drop-in model's step, both arms, no profiler
    timeout -k 10 500 python tools/bench_full_model.py "$@" > "$O/full.json" 2> "$O/full.err"
    rc=$?; cat "$O/full.json"; [ $rc -eq 0 ] || tail -20 "$O/full.err"; exit $rc ;;
  *) echo "unknown stage $stage"; exit 2 ;;
esac
