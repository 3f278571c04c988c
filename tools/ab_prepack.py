"""Which DSAMs' filters to pack beside the ratio predictor (hot_path.PREPACK): the bench's
captured train step (B = 8, 640x480, bf16) built once per variant (the variant is baked into its
graph at capture), then the variants' graphs replayed in alternating rounds; prints the median
ms per step per variant.  Variants are digit strings ("01" = PREPACK (0, 1), "0", "-" = none).

    python tools/ab_prepack.py 01 0 - --rounds 6 --steps 20
"""
import argparse
import os
import statistics
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
import torch  # noqa: E402

import bench  # noqa: E402
from rgbd_amd import hot_path  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()

args = bench.parse([])
ctx = bench.build(args, torch.device("cuda"))
steps = {}
for v in a.variants:
    hot_path.PREPACK = tuple(int(c) for c in v if c != "-")
    st = bench.make_step(ctx, 1, graph=True)
    for _ in range(3):
        st()  # capture + warm-up under this variant
    torch.cuda.synchronize()
    steps[v] = st
res = {v: [] for v in a.variants}
for rnd in range(a.rounds):
    for v in a.variants:
        dt = bench.timed(steps[v], a.steps, 2, 1)
        res[v].append(1e3 * dt / a.steps)
for v in a.variants:
    print(f"PREPACK {v:4s}: {statistics.median(res[v]):.4f} ms/step (min {min(res[v]):.4f}, "
          f"max {max(res[v]):.4f}, {a.rounds} rounds x {a.steps} steps)")
