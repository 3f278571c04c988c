#!/bin/bash
# tools/micro_dsam_conv.py under each "ENV=VAL ENV=VAL" setting given as an argument
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/micro_dsam_conv.py --iters 20 || exit 1
done
