#!/bin/bash
# Round-4 batch 3: the whole drop-in model's step under the kernel trace (where its 80 ms go).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
bash tools/gpu_r04.sh fullprof || exit 1
