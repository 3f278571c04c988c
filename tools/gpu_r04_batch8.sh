#!/bin/bash
# Round-4 batch 8: GEMM LDS-DMA variants A/B (RGBD_GEMM_LDS 0 / 1 / 2), point-loss + dense
# tests (bf16 sampling, every GEMM path), the full_model block (eager + captured).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04; mkdir -p $O
TESTLOG=tests8 bash tools/gpu_r04.sh tests tests/test_gpu_point_loss.py tests/test_gpu_dense.py
rc=$?; [ $rc -ge 124 ] && exit $rc
for lds in 0 1 2; do
  RGBD_GEMM_LDS=$lds timeout -k 10 180 python tools/micro_gemm.py > $O/micro_gemm_v$lds.jsonl 2>&1 || { tail -5 $O/micro_gemm_v$lds.jsonl; exit 1; }
done
python3 - <<'PY'
import json
rows = {}
for v in (0, 1, 2):
    for l in open(f"gpurun_out/r04/micro_gemm_v{v}.jsonl"):
        if l.startswith("{"):
            d = json.loads(l); rows.setdefault((d["shape"], d["case"]), {})[v] = d["ours_us"]; rows[(d["shape"], d["case"])]["lib"] = d["hipblaslt_us"]
for k, r in rows.items():
    print(k, r)
PY
for lds in 1 2; do
  RGBD_GEMM_LDS=$lds timeout -k 10 600 python tools/run_full_model.py > $O/full_model_v$lds.json 2> $O/full_model_v$lds.err || { tail -5 $O/full_model_v$lds.err; exit 1; }
  echo "lds=$lds"; cut -c1-700 $O/full_model_v$lds.json
done
