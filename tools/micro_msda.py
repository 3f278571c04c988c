"""Time the fused deformable-attention kernels against the reference's pure-torch
multi_scale_deformable_attention (transformers 5.15, grid_sample per level) at the C2 pixel-decoder
shape: B=8, levels 60x80 / 30x40 / 15x20 (S = Q = 6300), 8 heads x 32, 4 points."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import deform_attn  # noqa: E402
from transformers.models.mask2former.modeling_mask2former import multi_scale_deformable_attention as hf  # noqa: E402


def t_us(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    dev = "cuda"
    B, shapes, NH, D, P = 8, [(60, 80), (30, 40), (15, 20)], 8, 32, 4
    S = sum(h * w for h, w in shapes)
    g = torch.Generator(device=dev).manual_seed(0)
    value = torch.randn((B, S, NH, D), generator=g, device=dev).requires_grad_(True)
    # encoder-like locations: each query (a value pixel) samples its own neighbourhood on every
    # level (reference point = its centre, offsets ~ N(0, 2 px) of the sampled level)
    refs = []
    for H, W in shapes:
        ys, xs = torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev), indexing="ij")
        refs.append(torch.stack([(xs.reshape(-1) + 0.5) / W, (ys.reshape(-1) + 0.5) / H], -1))
    ref = torch.cat(refs)
    norm = torch.tensor([[w, h] for h, w in shapes], device=dev, dtype=torch.float32)
    if "--const-offsets" in sys.argv:  # the MSDeformAttn initialisation: one offset per (head, level, point)
        off = (torch.randn((1, 1, NH, 3, P, 2), generator=g, device=dev) * 2.0).expand(B, S, NH, 3, P, 2)
    else:
        off = torch.randn((B, S, NH, 3, P, 2), generator=g, device=dev) * 2.0
    loc = (ref[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]).requires_grad_(True)
    attw = torch.softmax(torch.randn((B, S, NH, 3 * P), generator=g, device=dev), -1).view(B, S, NH, 3, P)
    attw.requires_grad_(True)
    go = torch.randn((B, S, NH * D), generator=g, device=dev)
    res = {"offsets": "const" if "--const-offsets" in sys.argv else "random"}
    for name, fn in (("hip", deform_attn.multi_scale_deformable_attention), ("hf_grid_sample", hf)):
        with torch.no_grad():
            res[name + "_fwd_us"] = t_us(lambda: fn(value, shapes, loc, attw))

        def fb():
            out = fn(value, shapes, loc, attw)
            torch.autograd.grad(out, (value, loc, attw), go)
        res[name + "_fwd_bwd_us"] = t_us(fb)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
