#!/bin/bash
# Round-4 batch 27: chain phases 1-2 next-patch loads through a buffer descriptor (no per-element
# waits) and k_dsam_lds's tile code sets in two 16-byte loads: ratio + DSAM parity tests, chain and
# DSAM stamps, the ratio micro, three bench runs.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests27 bash tools/gpu_r04.sh tests tests/test_gpu_model.py tests/test_gpu_c2.py tests/test_gpu_bf16_parity.py tests/test_gpu_parity.py tests/test_gpu_dsam_full.py tests/test_gpu_dsam_plan.py || exit 1
timeout -k 10 300 python tools/chain_stamps.py > $O/chain_stamps27.txt 2>&1 || { tail -5 $O/chain_stamps27.txt; exit 1; }
cat $O/chain_stamps27.txt
timeout -k 10 300 python tools/dsam_stamps.py > $O/dsam_stamps27.txt 2> $O/dsam_stamps.err || { tail -5 $O/dsam_stamps.err; exit 1; }
grep -E "launch|tables" $O/dsam_stamps27.txt
for i in 1 2; do timeout -k 10 180 python tools/micro_ratio.py 2>&1 | tail -1 || exit 1; done
bash tools/gpu_ab_env.sh RGBD_UNUSED "x"
