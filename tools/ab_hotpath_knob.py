"""A/B of a hot_path module setting on the bench's captured train step (B = 8, 640x480, bf16): one
graph per value (the setting is read while the step is captured), replayed in alternating rounds;
prints the median ms per step per value.  Tuple settings take comma-separated values ("-" = empty):

    python tools/ab_hotpath_knob.py PREPACK 0,1 0 -

(profiles/r05_v2/ab_order_ze.txt came from a temporary PREPARE_ORDER tuple in prepare(): the
order of its side-stream launches; the current order measured fastest and the knob was removed.)
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
ap.add_argument("name")
ap.add_argument("values", nargs="+")
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()


def parse(v, like):
    if isinstance(like, tuple):
        items = [] if v == "-" else v.split(",")
        return tuple(type(like[0])(x) if like else x for x in items) if like else tuple(items)
    return type(like)(v)


default = getattr(hot_path, a.name)
args = bench.parse([])
ctx = bench.build(args, torch.device("cuda"))
steps = {}
for v in a.values:
    setattr(hot_path, a.name, parse(v, default))
    st = bench.make_step(ctx, 1, graph=True)
    for _ in range(3):
        st()  # capture + warm-up under this value
    torch.cuda.synchronize()
    steps[v] = st
setattr(hot_path, a.name, default)
res = {v: [] for v in a.values}
for rnd in range(a.rounds):
    for v in a.values:
        res[v].append(1e3 * bench.timed(steps[v], a.steps, 2, 1) / a.steps)
for v in a.values:
    print(f"{a.name} {v:24s}: {statistics.median(res[v]):.4f} ms/step (min {min(res[v]):.4f}, "
          f"max {max(res[v]):.4f}, {a.rounds} rounds x {a.steps} steps)")
