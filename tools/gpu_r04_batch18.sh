#!/bin/bash
# Round-4 batch 18: k_dsam_lds per-item stamps (diagnostic instantiation) + the DSAM tests.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests18 bash tools/gpu_r04.sh tests tests/test_gpu_dsam_full.py tests/test_gpu_dsam_plan.py || exit 1
timeout -k 10 300 python tools/dsam_stamps.py > $O/dsam_stamps.txt 2> $O/dsam_stamps.err || { tail -5 $O/dsam_stamps.err; exit 1; }
cat $O/dsam_stamps.txt
