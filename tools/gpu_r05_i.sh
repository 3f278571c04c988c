#!/bin/bash
# Round 5, call i: k_stem_lag with the parallel wave reduction (tests, A/B vs HEAD, stamps), conv5 with
# its in-loop copies dropped (timing only), and the whole-model glue by call site.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_i bash tools/gpu.sh tests tests/test_gpu_model.py tests/test_gpu_train_graph.py tests/test_gpu_c2.py tests/test_gpu_parity.py -k "stem or graph or ratio or parity" || exit 1
timeout -k 10 300 python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_head.so --rounds 6 > $O/ab_i.txt 2>&1 || { tail -5 $O/ab_i.txt; exit 1; }
cat $O/ab_i.txt
timeout -k 10 240 python -u tools/stem_lag_stamps.py > $O/stem_lag_stamps_i.txt 2>&1 || { tail -8 $O/stem_lag_stamps_i.txt; exit 1; }
cat $O/stem_lag_stamps_i.txt
timeout -k 10 300 python -u tools/conv5_modes.py > $O/conv5_modes.txt 2>&1 || { tail -8 $O/conv5_modes.txt; exit 1; }
cat $O/conv5_modes.txt
timeout -k 10 420 python -u tools/glue_sources.py $O/glue_sources_i.txt > $O/glue_sources_i.log 2>&1 || { tail -8 $O/glue_sources_i.log; exit 1; }
head -60 $O/glue_sources_i.txt
