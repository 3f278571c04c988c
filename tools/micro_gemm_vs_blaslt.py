"""The whole model's GEMM shapes (tools/gemm_shapes.py) on the HIP GEMM (dense.gemm, bf16 operands,
float32 or bf16 C as the model calls it) against torch.matmul (hipBLASLt) on the same operands,
device time by HIP events over back-to-back launches (diagnostic)."""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense  # noqa: E402

dev = torch.device("cuda")
# (M, N, K, a_t, b_t, batch, C float32?) from tools/gemm_shapes.py's whole-model table
shapes = [(256, 256, 800, 1, 1, 1, 1), (50400, 1024, 256, 0, 0, 1, 0), (800, 256, 256, 0, 0, 1, 0),
          (256, 256, 50400, 1, 1, 1, 1), (800, 256, 256, 0, 1, 1, 1), (50400, 256, 256, 0, 0, 1, 0),
          (800, 256, 256, 0, 1, 1, 0), (50400, 256, 1024, 0, 0, 1, 0), (1024, 256, 50400, 1, 1, 1, 1),
          (96, 256, 50400, 1, 1, 1, 1), (256, 1024, 50400, 1, 1, 1, 1), (50400, 256, 1024, 0, 1, 1, 1),
          (50400, 256, 256, 0, 1, 1, 1), (800, 256, 2048, 0, 1, 1, 1), (800, 2048, 256, 0, 0, 1, 0)]
n = 20
for M, N, K, at, bt, batch, cf in shapes:
    A = torch.randn((K, M) if at else (M, K), device=dev).to(torch.bfloat16)
    Bm = torch.randn((K, N) if bt else (N, K), device=dev).to(torch.bfloat16)
    oa = A.t() if at else A
    ob = Bm if bt else Bm.t()
    res = {}
    for name, fn in (("hip", lambda: dense.gemm(A, Bm, at, bt, M, N, K, c_f32=bool(cf))),
                     ("blaslt", lambda: torch.matmul(oa, ob).float() if cf else torch.matmul(oa, ob))):
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
    print(f"M {M:6d} N {N:5d} K {K:6d} at {at} bt {bt} c32 {cf}: hip {res['hip']:7.1f} us  blaslt {res['blaslt']:7.1f} us"
          f"  ratio {res['hip'] / res['blaslt']:.2f}")
