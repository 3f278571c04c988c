#!/bin/bash
# Round 5, call ze: order of prepare()'s side-stream launches (captured step, alternating)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python tools/ab_hotpath_knob.py PREPARE_ORDER modes,nhwc,packs packs,modes,nhwc modes,packs,nhwc --rounds 6 --steps 20 > $O/ab_order_ze.txt 2>&1 || { tail -20 $O/ab_order_ze.txt; exit 1; }
tail -3 $O/ab_order_ze.txt
