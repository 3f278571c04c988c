#!/bin/bash
# Round-4 batch 7: colsum micro, graph-guard GPU tests, the full_model block (eager + captured).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 120 python tools/micro_colsum.py > $O/micro_colsum.jsonl 2>&1; rc=$?; cat $O/micro_colsum.jsonl; [ $rc -ne 0 ] && exit $rc
TESTLOG=tests7 bash tools/gpu_r04.sh tests tests/test_graph_guard.py tests/test_gpu_dense.py::test_colsum
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python tools/run_full_model.py > $O/full_model.json 2> $O/full_model.err || { tail -5 $O/full_model.err; exit 1; }
cut -c1-1500 $O/full_model.json
