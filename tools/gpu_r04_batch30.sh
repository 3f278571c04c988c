#!/bin/bash
# Round-4 batch 30 (final-tree evidence, as batch 9): the bench line + its kernel trace, the PMC
# passes over the bench step, the whole-model step's kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
bash tools/gpu_r04.sh bench || exit 1
bash tools/gpu_r04.sh prof || exit 1
bash tools/gpu_r04_pmc.sh step || exit 1
tail -45 $O/pmc_step.txt | head -12
bash tools/gpu_r04.sh fullprof || exit 1
