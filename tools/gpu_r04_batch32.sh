#!/bin/bash
# Round-4 batch 32: torch-op attribution of the whole model's glue (tools/full_model_ops.py).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python tools/full_model_ops.py > $O/full_model_ops.txt 2> $O/full_model_ops.err || { tail -20 $O/full_model_ops.err; exit 1; }
cut -c1-260 $O/full_model_ops.txt | head -120
