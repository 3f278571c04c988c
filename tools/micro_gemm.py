"""Micro benchmark: the HIP GEMM family (csrc/gemm.hip via rgbd_amd.dense.gemm) against torch's
library GEMM (hipBLASLt) on the dense-layer shapes of the drop-in model at C2 (B = 8, 640x480):
pixel-decoder encoder layers (50 400 tokens: fc1 256->1024, fc2 1024->256, the 256->256
projections), Swin-T stage 1 (153 600 tokens: qkv 96->288, MLP 96->384->96), each in its
forward (0,0), dX (0,1) and dW (1,1) layout, bf16.  Prints one JSON line per shape with the
kernel time (HIP events around 20 launches), the algorithmic bytes (A + B + C once) and FLOPs."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense  # noqa: E402

dev = torch.device("cuda")
dt = torch.bfloat16
SHAPES = [  # (name, tokens M, in K, out N)
    ("pd_fc1", 50400, 256, 1024), ("pd_fc2", 50400, 1024, 256), ("pd_proj", 50400, 256, 256),
    ("swin1_qkv", 153600, 96, 288), ("swin1_fc1", 153600, 96, 384), ("swin1_fc2", 153600, 384, 96),
]


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


for name, M, K, N in SHAPES:
    x = torch.randn((M, K), device=dev, dtype=dt)
    w = torch.randn((N, K), device=dev, dtype=dt)
    gy = torch.randn((M, N), device=dev, dtype=dt)
    cases = {
        "fwd": (lambda: dense.gemm(x, w, 0, 0, M, N, K), lambda: x @ w.t(), (M * K + N * K + M * N) * 2),
        "dX": (lambda: dense.gemm(gy, w, 0, 1, M, K, N), lambda: gy @ w, (M * N + N * K + M * K) * 2),
        # dX as the backward now runs it: the weight transposed (included), then the (0, 0) layout
        "dX_t": (lambda: dense._dx(gy, w, M, K, N), lambda: gy @ w, (M * N + N * K + M * K) * 2),
        "dW": (lambda: dense.gemm(gy, x, 1, 1, N, K, M, c_f32=True), lambda: gy.t() @ x,
               (M * N + M * K) * 2 + N * K * 4),
    }
    for case, (ours, lib, nbytes) in cases.items():
        t_ours, t_lib = timeit(ours), timeit(lib)
        flop = 2.0 * M * N * K
        print(json.dumps({"shape": name, "case": case, "M": M, "K": K, "N": N, "ours_us": round(t_ours, 1),
                          "hipblaslt_us": round(t_lib, 1), "ours_TBs": round(nbytes / t_ours / 1e6, 2),
                          "ours_TFLOPs": round(flop / t_ours / 1e6, 1), "lib_TFLOPs": round(flop / t_lib / 1e6, 1)}),
              flush=True)
