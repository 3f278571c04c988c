#!/bin/bash
# Round 5, call s: host time of the eager step (cProfile), what N > 1 runs.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u tools/prof_host.py > $O/prof_host.txt 2>&1 || { tail -8 $O/prof_host.txt; exit 1; }
head -70 $O/prof_host.txt
