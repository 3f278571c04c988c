"""Micro benchmark of the bf16 DSAM conv entry points at the bench's shapes (B=8, 640x480):
packing, forward of dsam0/1/2, dW, and dX of dsam1/2, each timed with CUDA events over a graph of
--iters calls."""
import argparse, os, sys
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import torch
import _rgbd_import  # noqa: F401
from rgbd_amd import ops, synthetic
ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda")
B, H, W = 8, 480, 640
planes, _, _ = synthetic.make_batch(3, B, H, W)
d3 = torch.from_numpy(planes[:, 3:6]).to(dev)
sizes = [(120, 160), (60, 80), (30, 40)]
codes, info = ops.edsam_decompose(d3, torch.full((B,), 0.2, device=dev), sizes)
masks = ops.dsam_code_masks(codes)
g = torch.Generator(device=dev)
g.manual_seed(0)
res = []
for k, (ci, co) in enumerate([(96, 192), (192, 384), (384, 768)]):
    h, w = sizes[k]
    cw = torch.randn((4, co, ci, 3, 3), generator=g, device=dev) * 0.02
    pw = torch.randn((co, ci, 3, 3), generator=g, device=dev) * 0.02
    wf, wb = ops.dsam_pack(cw, pw, torch.bfloat16, code_mask=masks[k:k + 1])
    x = torch.randn((B, h, w, ci), generator=g, device=dev).bfloat16()
    b4 = torch.zeros((4, co), device=dev)
    resid = torch.randn((B, co, (h + 1) // 2, (w + 1) // 2), generator=g, device=dev).bfloat16()
    resid_nhwc = ops.nchw_to_nhwc(resid)
    gy = torch.randn((B, (h + 1) // 2, (w + 1) // 2, co), generator=g, device=dev).bfloat16()
    gin = torch.randn((B, ci, h, w), generator=g, device=dev).bfloat16()
    fns = {f"pack{k}": lambda: ops.dsam_pack(cw, pw, torch.bfloat16, code_mask=masks[k:k + 1], want_bwd=k > 0),
           f"fwd{k}": lambda: ops.dsam_fwd(x, codes[k], info, wf, b4, residual=resid, want_nhwc=(k < 2)),
           f"fwdh{k}": lambda: ops.dsam_fwd_nhwc(x, codes[k], info, wf, b4, residual_nhwc=resid_nhwc),
           f"dw{k}": lambda: ops.dsam_bwd_weight(None, x, codes[k], info, gout_nhwc=gy)}
    if k > 0:
        fns[f"dx{k}"] = lambda: ops.dsam_bwd_data(gy, codes[k], wb, gin, want_nhwc=True)
        gin_nhwc = ops.nchw_to_nhwc(gin)
        fns[f"dxh{k}"] = lambda: ops.dsam_bwd_data(gy, codes[k], wb, None, want_nhwc=True, want_nchw=False, cin=ci,
                                                   gin_nhwc=gin_nhwc)
    for name, fn in fns.items():
        # captured into a graph (iters calls) so host launch cost does not set the rate
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for _ in range(a.iters):
                fn()
        gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        res.append(f"{name} {e0.elapsed_time(e1) / a.iters * 1e3:.1f}us")
        del gr
print("  ".join(res))
