#!/bin/bash
# Round 5, call zb: per-CU copy throughput, LDS-DMA vs register loads, from L2 / MALL / HBM
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 120 tools/bin/dma_bw > $O/dma_bw_zb.txt 2>&1 || { cat $O/dma_bw_zb.txt; exit 1; }
cat $O/dma_bw_zb.txt
