#!/bin/bash
# Round-4 batch 13: chain-kernel per-tile stamps (diagnostic).
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 python tools/chain_stamps.py 2>&1 | grep -v amdgpu.ids
