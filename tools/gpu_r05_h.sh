#!/bin/bash
# Round 5, call h: where k_stem_lag's time goes (stamps, diagnostic build) and where the whole-model
# step's torch glue comes from (profiler call sites).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 240 python -u tools/stem_lag_stamps.py > $O/stem_lag_stamps.txt 2>&1 || { tail -8 $O/stem_lag_stamps.txt; exit 1; }
cat $O/stem_lag_stamps.txt
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources.txt > $O/glue_sources.log 2>&1 || { tail -8 $O/glue_sources.log; exit 1; }
head -50 $O/glue_sources.txt
