#!/bin/bash
# Round 5, call t: the launcher / DDP tests with the re-timed eager line, a world-2 gloo bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
TESTLOG=tests_t bash tools/gpu.sh tests tests/test_gpu_bench_ddp.py || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --cpu-baseline 0 --inference 0 --c5-stream 0 --parity 0 --full-model 0 > $O/bench_w2.json 2> $O/bench_w2.err || { tail -5 $O/bench_w2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_w2.json'));print(d['value'], d['eager_img_s'], d['scaling_baseline_img_s'])"
