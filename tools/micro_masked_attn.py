"""Times the masked cross-attention (f1) of one decoder-layer call: torch's nn.MultiheadAttention
math path vs the HIP module, forward and forward+backward, at the three pixel-decoder levels of
the C1 / C2 inputs (Q = 100 queries, 8 heads, hidden 256)."""
import os
import sys
from pathlib import Path

import torch
from torch import nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _rgbd_import  # noqa: E402,F401
from rgbd_amd import masked_attention  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    torch.manual_seed(0)
    ref = nn.MultiheadAttention(256, 8, 0.0).cuda()
    hip = nn.MultiheadAttention(256, 8, 0.0).cuda()
    hip.load_state_dict(ref.state_dict())
    masked_attention.install_module(hip)
    cfgs = ((8, 300), (8, 1200), (8, 4800), (1, 1200), (1, 4800), (1, 19200))
    if os.environ.get("MA_CFG"):  # e.g. MA_CFG=8x4800 (one configuration, for a kernel trace)
        cfgs = (tuple(int(x) for x in os.environ["MA_CFG"].split("x")),)
    for B, L in cfgs:
        q = torch.randn(100, B, 256, device="cuda", requires_grad=True)
        v = torch.randn(L, B, 256, device="cuda", requires_grad=True)
        k = (v.detach() + 1).requires_grad_()
        m = torch.rand(B * 8, 100, L, device="cuda") < 0.6
        g = torch.randn(100, B, 256, device="cuda")
        row = []
        for mod in (ref, hip):
            f = lambda: mod(q, k, v, attn_mask=m)  # noqa: E731
            fb = lambda: mod(q, k, v, attn_mask=m)[0].backward(g)  # noqa: E731
            row += [timed(f), timed(fb)]
        print(f"B={B} L={L:6d}  torch fwd {row[0]:8.1f} us  fwd+bwd {row[1]:8.1f} us | "
              f"hip fwd {row[2]:8.1f} us  fwd+bwd {row[3]:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
