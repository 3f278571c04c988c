#!/bin/bash
# Round-6 kernel iteration: the tests named by -k "$1" (stop at the first failure), then an
# interleaved A/B of the in-tree library against $AB (a .so path relative to the repo) on the
# ratio predictor (tools/ab_ratio.py), then optionally the default bench line ($BENCH = its args).
cd "$GRAFT_REPO_ROOT" || exit 1
O="$GRAFT_REPO_ROOT/gpurun_out/r06/${TAG:-x}"; mkdir -p "$O"
if [ -n "$1" ]; then
  timeout -k 10 ${TT:-600} python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k "$1" > "$O/tests.log" 2>&1
  rc=$?; grep -E "passed|failed|error" "$O/tests.log" | tail -3; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" "$O/tests.log" | head -20; exit $rc; }
fi
if [ -n "$AB" ]; then
  timeout -k 10 300 python tools/ab_ratio.py $AB --rounds ${ROUNDS:-6} > "$O/ab.txt" 2>&1 || { tail -20 "$O/ab.txt"; exit 1; }
  tail -3 "$O/ab.txt"
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py $BENCH > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline'].get('events_avg_us'),d['kernels']['k5_dsam']['ms_per_step'],d.get('inference_img_s'))"
fi
