"""Micro benchmark: HipAdamW (csrc/adamw.hip) vs torch.optim.AdamW(fused=True) on the hot path's
parameter groups (bench workload: dsam2 = 13.3 M fp32 parameters; dsam1 + dsam0 + DGGM = 4.1 M).
Prints us per step and the HBM rate at 28 bytes per parameter (p, g, m, v read; p, m, v written)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual  # noqa: E402
from rgbd_amd.optim import HipAdamW  # noqa: E402

dev = torch.device("cuda")
mods = [DSAModule(ci, co).to(dev) for ci, co in [(96, 192), (192, 384), (384, 768)]]
dg = DepthGradientInjectionResidual([96, 192, 384, 768], 3).to(dev)
groups = {"dsam2": list(mods[2].parameters()),
          "dsam1+dsam0+dggm": list(mods[1].parameters()) + list(mods[0].parameters()) + list(dg.parameters())}
for name, ps in groups.items():
    for p in ps:
        p.grad = torch.randn_like(p)
    n = sum(p.numel() for p in ps)
    res = {"group": name, "params": n}
    for arm, opt in (("hip", HipAdamW(ps, lr=1e-5)), ("torch_fused", torch.optim.AdamW(ps, lr=1e-5, fused=True))):
        for _ in range(3):
            opt.step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            opt.step()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        res[arm + "_us"] = round(us, 1)
        res[arm + "_TBs"] = round(28 * n / us / 1e6, 2)
    print(json.dumps(res), flush=True)
