"""How many region codes a k_dsam_lds tile meets per live tap at the bench's workload (diagnostic):
one eager bench step with ops.dsam_plan wrapped, then each forward / dX leg's code sets
(the head of its plan buffer: tmasks[(class * ntiles0 + tile) * 16 + tap], u16) are read back.
Prints per leg: K steps (tap x chunk group x code) and the distinct (tap, chunk group) input
blocks those steps copy — the input copies a kernel sharing one block across its codes would
make."""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import _rgbd_import  # noqa: E402,F401
from rgbd_amd import ops  # noqa: E402

LD_BM = 128
rec = []
orig = ops.dsam_plan


def wrapped(legs):
    plans = orig(legs)
    rec.extend(zip(legs, plans))
    return plans


ops.dsam_plan = wrapped
args = bench.parse([])
dev = torch.device("cuda:0")
ctx = bench.build(args, dev)
step = bench.make_step(ctx, 1)
step()
torch.cuda.synchronize()


def ld_kc(C):
    return 3 if C % 96 == 0 else (2 if C % 64 == 0 else 1)


for (kind, code, ci, co), plan in rec:
    if kind not in (ops.LEG_FWD, ops.LEG_DX):
        continue
    B, h, w = code.shape
    tr = kind == ops.LEG_DX
    Ho, Wo = (h, w) if tr else ((h + 1) // 2, (w + 1) // 2)
    C = co if tr else ci
    Hc0, Wc0 = ((Ho + 1) // 2, (Wo + 1) // 2) if tr else (Ho, Wo)
    blk = ((Hc0 + 7) // 8 * 8) * ((Wc0 + 15) // 16 * 16)
    linear = Hc0 * Wc0 * 100 < 85 * blk
    nt = -(-(B * Hc0 * Wc0) // LD_BM) if linear else B * (-(-Hc0 // 8)) * (-(-Wc0 // 16))
    ncls = 4 if tr else 1
    tm = plan[: ncls * nt * 32].cpu().numpy().view(np.uint16).reshape(ncls, nt, 16)[:, :, :9]
    pop = np.vectorize(lambda v: bin(int(v)).count("1"))(tm)
    ncg = C // (32 * ld_kc(C))
    steps = int(pop.sum()) * ncg
    groups = int((tm != 0).sum()) * ncg
    name = "dX" if tr else "fwd"
    print(f"{name:3s} {ci}->{co} in {h}x{w}: tiles {ncls}x{nt}, steps {steps}, input blocks {groups} "
          f"({groups / max(steps, 1):.3f} of the steps), codes per live tap {steps / max(groups, 1):.3f}")
