"""Micro driver for kernel-level profiling: the bench's full train step (same shapes/data),
run --iters times after warmup; use under rocprofv3 with a kernel filter."""
import argparse, os, sys, time
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, 'tests/golden')]
import torch
import bench
ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
args = bench.parse([])
ctx = bench.build(args, torch.device("cuda"))
step = bench.make_step(ctx, 1)
for _ in range(3):
    step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.iters):
    step()
torch.cuda.synchronize()
print(f"step {(time.perf_counter() - t) / a.iters * 1e3:.3f} ms")
