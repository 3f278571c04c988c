#!/bin/bash
# hipGraphLaunch fork/join reproducers (tools/graph_fork_repro.cpp, tools/graph_fork_torch.py):
# every mode after 20 prior graphs, each run under its own time limit; stops at the first fault.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in 0 1 2 3; do
  timeout -k 10 60 tools/bin/graph_fork_repro $m 20 3 > gpurun_out/repro_c_$m.log 2>&1
  rc=$?; echo "hip mode $m rc=$rc: $(tail -1 gpurun_out/repro_c_$m.log)"; [ $rc -eq 0 ] || exit $rc
done
for m in 0 1 2; do
  timeout -k 10 120 python tools/graph_fork_torch.py $m 20 > gpurun_out/repro_t_$m.log 2>&1
  rc=$?; echo "torch mode $m rc=$rc: $(tail -1 gpurun_out/repro_t_$m.log)"; [ $rc -eq 0 ] || exit $rc
done
