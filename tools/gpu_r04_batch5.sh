#!/bin/bash
# Round-4 batch 5: the dW fold per (o, 32-channel chunk), the whole-model changes (run-carrying
# MSDA backward, colsum chunking, loss gathers, device constants, captured whole-model step):
# their tests, the MSDA micro A/B, the bench + its kernel trace, the full_model block.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests5 bash tools/gpu_r04.sh tests tests/test_gpu_dsam_plan.py tests/test_gpu_parity.py tests/test_gpu_dsam_full.py tests/test_gpu_msda.py tests/test_gpu_dense.py tests/test_gpu_point_loss.py tests/test_gpu_model.py tests/test_gpu_trainer.py
rc=$?; [ $rc -ge 124 ] && exit $rc   # assertion failures are reported, crashes / time limits stop here
for nc in 0 1; do
  RGBD_DIAG_NOCONV=$nc timeout -k 10 200 python tools/diag_g5.py > $O/diag_g5_noconv$nc.txt 2>&1 || { tail -5 $O/diag_g5_noconv$nc.txt; exit 1; }
  echo "noconv=$nc"; grep -E "^1 (sw|bb|mask)" $O/diag_g5_noconv$nc.txt
done
for runs in 0 1; do for off in "" "--const-offsets"; do
  RGBD_MSDA_RUNS=$runs timeout -k 10 120 python tools/micro_msda.py $off > $O/msda_${runs}${off}.json 2>&1 || { tail -5 $O/msda_${runs}${off}.json; exit 1; }
  echo "runs=$runs $off: $(tail -1 $O/msda_${runs}${off}.json)"
done; done
for lds in 0 1; do
  RGBD_GEMM_LDS=$lds timeout -k 10 180 python tools/micro_gemm.py > $O/micro_gemm_lds$lds.jsonl 2>&1 || { tail -5 $O/micro_gemm_lds$lds.jsonl; exit 1; }
done
cat $O/micro_gemm_lds1.jsonl
bash tools/gpu_r04.sh bench --full-model 0 || exit 1
bash tools/gpu_r04.sh prof || exit 1
timeout -k 10 600 python tools/run_full_model.py > $O/full_model.json 2> $O/full_model.err || { tail -20 $O/full_model.err; exit 1; }
cat $O/full_model.json
