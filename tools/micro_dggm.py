"""Micro benchmark of the DGGM fused fwd / bwd entry points at the bench's four scales (B=8,
640x480, bf16), each timed with CUDA events over --iters calls (RGBD_DGGM_DBG=1: constant
gates, to price the gate resampling)."""
import argparse, os, sys
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import torch
import _rgbd_import  # noqa: F401
from rgbd_amd import ops
ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda")
B, H, W = 8, 480, 640
g = torch.Generator(device=dev)
g.manual_seed(0)
pv = torch.rand((B, 10, H, W), generator=g, device=dev)
pv[:, 9] = (pv[:, 9] > 0.3).float()
res = []
for k, (C, h, w) in enumerate([(96, 120, 160), (192, 60, 80), (384, 30, 40), (768, 15, 20)]):
    col = torch.randn((B, C, h, w), generator=g, device=dev).bfloat16()
    cp1 = torch.randn((B, C, h, w), generator=g, device=dev).bfloat16()
    wt = torch.randn((C, 3, 1, 1), generator=g, device=dev)
    bs = torch.randn((C,), generator=g, device=dev)
    fns = {f"fwd{k}": lambda: ops.dggm_fuse_fwd(cp1, col, pv, wt, bs),
           f"bwd{k}": lambda: ops.dggm_fuse_bwd(col, pv, wt, bs)}
    for name, fn in fns.items():
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(f"{name} {e0.elapsed_time(e1) / a.iters * 1e3:.1f}us")
print(f"DBG={os.environ.get('RGBD_DGGM_DBG', '0')}: " + "  ".join(res))
