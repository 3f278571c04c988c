#!/bin/bash
# Round-6 iteration run: the tests named by -k "$1" (each GPU step under its own time limit; the
# chain stops at the first failure), then optionally the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
O="$GRAFT_REPO_ROOT/gpurun_out/r06/${TAG:-x}"; mkdir -p "$O"
timeout -k 10 ${TT:-900} python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 400 --timeout-method thread $PY -k "$1" > "$O/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$O/tests.log" | tail -3; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" "$O/tests.log" | head; exit $rc; }
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py $BENCH > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'],d['kernels']['k5_dsam']['ms_per_step'],d.get('inference_img_s'))"
fi
