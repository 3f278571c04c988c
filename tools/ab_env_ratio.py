"""In-process A/B of a development environment switch on the ratio predictor (train mode, bench
shape B=8 640x480 bf16): rounds alternate the switch's values, each round runs --iters forwards
per value; per-kernel times from the library's HIP-event timers.  Prints medians per value and
the max |ratio| difference between the values' outputs (the same input and dropout stream).

    python tools/ab_env_ratio.py RGBD_C3_SCHED 0 1 --rounds 8
"""
import argparse
import ctypes
import os
import statistics
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import _lib, init as winit, synthetic  # noqa: E402
from rgbd_amd.modules import EnhancedDepthImageRatioPredictor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("var")
ap.add_argument("vals", nargs="+")
ap.add_argument("--rounds", type=int, default=8)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()

L = _lib.lib()
m = EnhancedDepthImageRatioPredictor(3)
winit.init_deterministic(m, prefix="model.pixel_level_module.ratio_predictor.")
m.compute_dtype = torch.bfloat16
m = m.cuda().train()
planes, _, _ = synthetic.make_batch(3, 8, 480, 640)
d = torch.from_numpy(planes[:, 3:6].copy()).cuda()
names = ["rp_conv3x3", "rp_chain"]
res = {v: {n: [] for n in names + ["total"]} for v in a.vals}
outs = {}
for rnd in range(a.rounds + 1):
    for v in a.vals:
        os.environ[a.var] = v
        # the same dropout stream per value: reset the device counter
        if hasattr(m, "_rgbd_dropout_ctr"):
            m._rgbd_dropout_ctr.zero_()
        with torch.no_grad():
            outs[v] = m(d).float().clone()
        for _ in range(2):
            m(d)
        torch.cuda.synchronize()
        L.rgbd_timing_enable(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            m(d)
        e1.record()
        torch.cuda.synchronize()
        cnt = ctypes.c_int(0)
        for n in names:
            ms = L.rgbd_timing_read(n.encode(), ctypes.byref(cnt))
            if rnd:
                res[v][n].append(ms / max(cnt.value, 1))
        L.rgbd_timing_enable(0)
        if rnd:
            res[v]["total"].append(e0.elapsed_time(e1) / a.iters)
base = a.vals[0]
for v in a.vals:
    med = {n: statistics.median(x) for n, x in res[v].items()}
    diff = float((outs[v] - outs[base]).abs().max())
    print(f"{a.var}={v}: " + " ".join(f"{n} {t:.4f} ms" for n, t in med.items()) + f"  max|ratio - {base}| {diff:.3g}",
          flush=True)
