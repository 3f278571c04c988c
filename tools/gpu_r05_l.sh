#!/bin/bash
# Round 5, call l: fused residual add + LayerNorm and the HIP class head in the whole model (dense /
# model / graph / DDP tests, whole-model step before (HEAD lib not applicable: Python change) and
# the glue by call site after).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_l bash tools/gpu.sh tests tests/test_gpu_dense.py tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py tests/test_gpu_parity.py || exit 1
timeout -k 10 600 python -u tools/run_full_model.py > $O/full_model_l.json 2> $O/full_model_l.err || { tail -5 $O/full_model_l.err; exit 1; }
cat $O/full_model_l.json
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources_l.txt > $O/glue_sources_l.log 2>&1 || { tail -8 $O/glue_sources_l.log; exit 1; }
head -40 $O/glue_sources_l.txt; tail -1 $O/glue_sources_l.txt
