#!/bin/bash
# Round 5, call m: batched matcher / loss_labels, cast-once rows, fused add+LN bf16 twin
# (tests, whole-model step, glue by call site).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_m bash tools/gpu.sh tests tests/test_gpu_dense.py tests/test_gpu_point_loss.py tests/test_gpu_lsap.py tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py tests/test_gpu_parity.py || exit 1
timeout -k 10 600 python -u tools/run_full_model.py > $O/full_model_m.json 2> $O/full_model_m.err || { tail -5 $O/full_model_m.err; exit 1; }
cat $O/full_model_m.json
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources_m.txt > $O/glue_sources_m.log 2>&1 || { tail -8 $O/glue_sources_m.log; exit 1; }
head -40 $O/glue_sources_m.txt; tail -1 $O/glue_sources_m.txt
