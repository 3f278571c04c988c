"""A/B of two library builds on the ratio predictor (train mode, bench shape), interleaved in one
process so both see the same device and clock state: per round, --iters forwards with each
library; per-kernel times from each library's own HIP-event timing.  Prints medians.

    python tools/ab_ratio.py rgb-d-instance-segmentation_amd/gpurun_ab_old.so --rounds 8
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
ap.add_argument("others", nargs="+")
ap.add_argument("--rounds", type=int, default=8)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()

new = _lib.lib()
libs = {"new": new}
for other in a.others:
    h = ctypes.CDLL(os.path.join(_R, other))
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(h, name):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
    libs[os.path.basename(other)] = h

m = EnhancedDepthImageRatioPredictor(3)
winit.init_deterministic(m, prefix="model.pixel_level_module.ratio_predictor.")
m.compute_dtype = torch.bfloat16
m = m.cuda().train()
planes, _, _ = synthetic.make_batch(3, 8, 480, 640)
d = torch.from_numpy(planes[:, 3:6].copy()).cuda()
names = ["rp_conv3x3", "rp_chain"]
res = {k: {n: [] for n in names + ["total"]} for k in libs}
for rnd in range(a.rounds + 1):
    for tag, L in libs.items():
        _lib._lib = L
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
                res[tag][n].append(ms / max(cnt.value, 1))
        L.rgbd_timing_enable(0)
        if rnd:
            res[tag]["total"].append(e0.elapsed_time(e1) / a.iters)
# same inputs, eval mode (deterministic): every build must give the in-tree build's ratio bitwise
m.eval()
outs = {}
for tag, L in libs.items():
    _lib._lib = L
    outs[tag] = m(d).cpu()
_lib._lib = new
m.train()
for tag in libs:
    print(tag, "ratio==new:", bool(torch.equal(outs[tag], outs["new"])), "  ".join(f"{n} {statistics.median(v):.4f} ms (min {min(v):.4f})" for n, v in res[tag].items()))
