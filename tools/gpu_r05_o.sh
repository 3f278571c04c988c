#!/bin/bash
# Round 5, call o: clamp folded into the fused norm, bf16 dr from the norm backward, no materialised twin gradient,
# deformable-attention sampling locations in one kernel
# (tests, whole-model step, glue by call site).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_o bash tools/gpu.sh tests tests/test_gpu_dense.py tests/test_gpu_point_loss.py tests/test_gpu_lsap.py tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py tests/test_gpu_parity.py tests/test_gpu_msda.py || exit 1
timeout -k 10 600 python -u tools/run_full_model.py > $O/full_model_o.json 2> $O/full_model_o.err || { tail -5 $O/full_model_o.err; exit 1; }
cat $O/full_model_o.json
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources_o.txt > $O/glue_sources_o.log 2>&1 || { tail -8 $O/glue_sources_o.log; exit 1; }
head -40 $O/glue_sources_o.txt; tail -1 $O/glue_sources_o.txt
