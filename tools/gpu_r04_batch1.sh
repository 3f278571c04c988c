#!/bin/bash
# Round-4 first measurement batch: changed GPU tests, the conv5 schedule A/B (RGBD_C3_SCHED 0/1/2),
# the bench line, a kernel-trace profile and the PMC passes of the bench step.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
bash tools/gpu_r04.sh tests tests/test_graph_guard.py tests/test_gpu_adamw.py tests/test_gpu_train_graph.py tests/test_gpu_bf16_parity.py tests/test_gpu_bench_ddp.py tests/test_gpu_c2.py tests/test_gpu_metrics.py tests/test_gpu_conv.py || exit 1
timeout -k 10 400 python tools/ab_env_ratio.py RGBD_C3_SCHED 0 1 2 --rounds 6 > gpurun_out/r04/ab_c3.txt 2>&1 || { tail -20 gpurun_out/r04/ab_c3.txt; exit 1; }
cat gpurun_out/r04/ab_c3.txt
bash tools/gpu_r04.sh bench || exit 1
bash tools/gpu_r04.sh prof || exit 1
bash tools/gpu_r04_pmc.sh dsam || exit 1
