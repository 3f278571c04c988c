#!/bin/bash
# conv5 v4 stamps ($1 = the stamped build) after an optional A/B ($AB)
cd "$GRAFT_REPO_ROOT" || exit 1
O="$GRAFT_REPO_ROOT/gpurun_out/r06/${TAG:-x}"; mkdir -p "$O"
if [ -n "$AB" ]; then
  timeout -k 10 300 python tools/ab_ratio.py $AB --rounds ${ROUNDS:-5} > "$O/ab.txt" 2>&1 || { tail -20 "$O/ab.txt"; exit 1; }
fi
timeout -k 10 200 python tools/conv5_stamps.py "$1" > "$O/stamps.txt" 2>&1 || { tail -20 "$O/stamps.txt"; exit 1; }
