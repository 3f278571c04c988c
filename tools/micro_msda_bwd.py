"""The pixel decoder's MSDA backward (k_msda_bwd_runs) at C2's shapes (B 8, levels 60x80 / 30x40 /
15x20, 8 heads x 32 channels, 3 levels x 4 points, queries = the three levels' pixels) with
sampling locations as the initialised model draws them (each query's reference point plus small
per-head / per-point offsets: neighbouring queries sample neighbouring cells), device time by HIP
events; builds to compare are given as paths (RGBD_HIP_LIB style), interleaved (diagnostic)."""
import ctypes
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
shapes = [(60, 80), (30, 40), (15, 20)]
B, NH, D, L, P = 8, 8, 32, 3, 4
S = sum(h * w for h, w in shapes)
Q = S
g = torch.Generator(device=dev).manual_seed(0)
value = torch.randn((B, S, NH, D), generator=g, device=dev).to(torch.bfloat16)
ref = []
for h, w in shapes:
    ys, xs = torch.meshgrid((torch.arange(h, device=dev) + 0.5) / h, (torch.arange(w, device=dev) + 0.5) / w, indexing="ij")
    ref.append(torch.stack([xs.reshape(-1), ys.reshape(-1)], -1))
ref = torch.cat(ref)  # [Q, 2]
off = (torch.randn((NH, L, P, 2), generator=g, device=dev) * 0.02)
loc = (ref[None, :, None, None, None, :] + off[None, None]).expand(B, Q, NH, L, P, 2).contiguous().float()
attw = torch.softmax(torch.randn((B, Q, NH, L * P), generator=g, device=dev), -1).view(B, Q, NH, L, P).contiguous()
gout = torch.randn((B, Q, NH * D), generator=g, device=dev).to(torch.bfloat16)
libs = {"in-tree": _lib.lib()}
for path in sys.argv[1:]:
    h = ctypes.CDLL(os.path.join(_R, path))
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(h, name):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
    libs[os.path.basename(path)] = h
times = {k: [] for k in libs}
outs = {}
for rnd in range(6):
    for k, L_ in libs.items():
        _lib._lib = L_
        for _ in range(2):
            r = ops.msda_backward(value, shapes, loc, attw, gout)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            r = ops.msda_backward(value, shapes, loc, attw, gout)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 5 * 1e3)
        outs[k] = [t.clone() for t in r]
ref_out = outs["in-tree"]
for k, ts in times.items():
    d = max(float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(outs[k], ref_out))
    print(f"{k}: median {sorted(ts)[len(ts) // 2]:8.1f} us  (min {min(ts):8.1f})  max rel diff vs in-tree {d:.2e}")
