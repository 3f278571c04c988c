"""Host time of the eager training step (what N > 1 runs): cProfile over 10 steps of bench.py's
default step (B = 8, 640x480, bf16, no graph), the enqueue time per step with the GPU drained
first (host only) and the step time; prints the functions with the most own time."""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

args = bench.parse(["--steps", "10", "--graph", "0"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ctx = bench.build(args, dev, 0)
step = bench.make_step(ctx, 1)
for _ in range(3):
    step()
torch.cuda.synchronize()
enq = []
for _ in range(5):  # host enqueue time of one step with an idle GPU queue
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    enq.append(time.perf_counter() - t0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    step()
torch.cuda.synchronize()
per = (time.perf_counter() - t0) / 10
print(f"eager step {per * 1e3:.3f} ms; host enqueue per step {min(enq) * 1e3:.3f} ms (min of 5), "
      f"{sorted(enq)[2] * 1e3:.3f} ms (median)")
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    step()
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
print(s.getvalue()[:9000])
