#!/bin/bash
# Round-4 batch 23: the whole model's eager step under the kernel trace (current tree), ranked.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
bash tools/gpu_r04.sh fullprof || exit 1
f=$(ls $O/fullprof/*/run_kernel_trace.csv $O/fullprof/run_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(find $O/fullprof -name '*kernel_trace.csv' | head -1)
python tools/step_kernel_ranking.py "$f" k_prep_pass1_q 60 > $O/full_model_ranking23.txt && cut -c1-150 $O/full_model_ranking23.txt
