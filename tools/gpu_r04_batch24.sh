#!/bin/bash
# Round-4 batch 24: MSDA runs backward with buffer-descriptor tap loads (207 vs 236 VGPRs): MSDA
# tests, the C2 micro (runs, constant / random offsets), the full_model block.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests24 bash tools/gpu_r04.sh tests tests/test_gpu_msda.py || exit 1
for off in "--const-offsets" "" "--const-offsets"; do
  timeout -k 10 120 python tools/micro_msda.py $off > $O/msda24.json 2>&1 || { tail -5 $O/msda24.json; exit 1; }
  echo "runs=1 $off: $(tail -1 $O/msda24.json)"
done
timeout -k 10 600 python tools/run_full_model.py > $O/full_model24.json 2> $O/full_model.err || { tail -20 $O/full_model.err; exit 1; }
cut -c1-700 $O/full_model24.json
