#!/bin/bash
# Round 5, call zn: final library build — smoke and the ratio / model / parity GPU tests
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_zn.log 2>&1 || { tail -5 $O/smoke_zn.log; exit 1; }
tail -1 $O/smoke_zn.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c2.py tests/test_gpu_model.py tests/test_gpu_parity.py > $O/tests_zn.txt 2>&1 || { tail -30 $O/tests_zn.txt; exit 1; }
tail -2 $O/tests_zn.txt
