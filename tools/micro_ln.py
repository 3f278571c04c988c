"""Micro benchmark: the HIP LayerNorm (csrc/layernorm.hip via rgbd_amd.dense.layer_norm) forward and
backward against torch's on the row shapes of the drop-in model at C2 (B = 8, 640x480): Swin-T
stages 1-4 (f32 residual stream under autocast), the pixel decoder's encoder layers (50 400 x 256)
and the masked-attention decoder (100 queries x 8 x 256).  One JSON line per shape: kernel
time of forward + backward (HIP events around 20 iterations) and the HBM bytes moved
(x, y, dy, dx once)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense  # noqa: E402

dev = torch.device("cuda")
SHAPES = [("swin1", 153600, 96), ("swin2", 38400, 192), ("swin3", 9600, 384), ("swin4", 2400, 768),
          ("pixdec", 50400, 256), ("decoder", 800, 256)]


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3  # us


for name, M, C in SHAPES:
    ln = torch.nn.LayerNorm(C).to(dev)
    x = torch.randn((M, C), device=dev).requires_grad_()
    gy = torch.randn((M, C), device=dev)

    def ours():
        y = dense.layer_norm(x, ln)
        y.backward(gy)

    def lib():
        y = torch.nn.functional.layer_norm(x, (C,), ln.weight, ln.bias, ln.eps)
        y.backward(gy)

    t_ours, t_lib = timeit(ours), timeit(lib)
    nbytes = 5 * M * C * 4  # x + y (fwd), x + dy + dx (bwd)
    print(json.dumps({"shape": name, "rows": M, "C": C, "ours_us": round(t_ours, 1), "torch_us": round(t_lib, 1),
                      "ours_TBs": round(nbytes / t_ours / 1e6, 2)}), flush=True)
