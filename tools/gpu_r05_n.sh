#!/bin/bash
# Round 5, call n: top-k kernel, bf16-rounded float32 dX store, batched matcher
# (tests, whole-model step, glue by call site).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_n bash tools/gpu.sh tests tests/test_gpu_dense.py tests/test_gpu_point_loss.py tests/test_gpu_lsap.py tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_ddp_model.py tests/test_gpu_parity.py || exit 1
timeout -k 10 600 python -u tools/run_full_model.py > $O/full_model_n.json 2> $O/full_model_n.err || { tail -5 $O/full_model_n.err; exit 1; }
cat $O/full_model_n.json
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources_n.txt > $O/glue_sources_n.log 2>&1 || { tail -8 $O/glue_sources_n.log; exit 1; }
head -40 $O/glue_sources_n.txt; tail -1 $O/glue_sources_n.txt
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_bsplit.so --rounds 6 > $O/ab_n.txt 2>&1 || { tail -5 $O/ab_n.txt; exit 1; }
cat $O/ab_n.txt
