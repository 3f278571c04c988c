#!/bin/bash
# Round-2 GPU check: host facts, the GPU test suite (new C2 / DDP tests first, one pytest
# process), then the default bench line.  Every GPU step under its own time limit; the chain
# stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP_NUM_THREADS', os.environ.get('OMP_NUM_THREADS'))" > gpurun_out/host.txt
timeout -k 10 1000 python -u -m pytest tests/test_gpu_c2.py tests/test_gpu_bench_ddp.py tests -m gpu -v --maxfail=6 \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/gpu_tests.log
tail -40 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "$1" = "tests-only" ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
