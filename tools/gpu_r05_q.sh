#!/bin/bash
# Round 5, call q: the decoder memory (level embedding + permute) in one kernel each way
# (tests, whole-model step, glue by call site).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_q bash tools/gpu.sh tests tests/test_gpu_mask_predictor.py tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py tests/test_gpu_parity.py || exit 1
timeout -k 10 600 python -u tools/run_full_model.py > $O/full_model_q.json 2> $O/full_model_q.err || { tail -5 $O/full_model_q.err; exit 1; }
cat $O/full_model_q.json
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources_q.txt > $O/glue_sources_q.log 2>&1 || { tail -8 $O/glue_sources_q.log; exit 1; }
head -30 $O/glue_sources_q.txt; tail -1 $O/glue_sources_q.txt
