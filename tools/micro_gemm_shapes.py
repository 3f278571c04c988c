"""The whole model's large-M GEMM shapes on the HIP GEMM (dense.gemm) against torch's (hipBLASLt)
for the same product, device time by HIP events over back-to-back launches (diagnostic)."""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense  # noqa: E402

dev = torch.device("cuda")
shapes = [(50400, 1024, 256), (50400, 256, 256), (50400, 256, 1024), (50400, 192, 256), (38400, 256, 256),
          (50400, 96, 256)]
n = 20
for M, N, K in shapes:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    res = {}
    for name, fn in (("hip", lambda: dense.gemm(x, w, 0, 0, M, N, K, bias=b)),
                     ("torch", lambda: torch.nn.functional.linear(x, w, b.to(torch.bfloat16)))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / n * 1e3
    fl = 2.0 * M * N * K
    by = (M * K + N * K + M * N) * 2
    print(f"M {M} N {N} K {K}: hip {res['hip']:7.1f} us ({fl / res['hip'] / 1e6:5.0f} TF/s, {by / res['hip'] / 1e3:5.0f} GB/s)"
          f"  torch {res['torch']:7.1f} us ({fl / res['torch'] / 1e6:5.0f} TF/s)")
