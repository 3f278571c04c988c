"""A/B of library builds on the whole model's small and medium GEMM shapes (diagnostic): dense.gemm
with each library in turn (interleaved rounds, HIP events around a HIP-graph replay of n calls:
device time, not the host's launch rate), median
microseconds per call, and whether each build's result equals the in-tree build's bitwise.

    python tools/micro_gemm_ab.py rgb-d-instance-segmentation_amd/gpurun_ab_x.so
"""
import ctypes
import os
import statistics
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import _lib, dense  # noqa: E402

dev = torch.device("cuda")
new = _lib.lib()
libs = {"new": new}
for other in [v for v in sys.argv[1:] if not v.startswith("--")]:
    h = ctypes.CDLL(os.path.join(_R, other))
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(h, name):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
    libs[os.path.basename(other)] = h

# (M, N, K, a_t, b_t, c_f32, dtype): the decoder's (100 queries x 8 images = 800 rows) products,
# their weight gradients (K = 800 tokens) and a few pixel-decoder / Swin shapes
shapes = [(800, 256, 256, 0, 0, 0, torch.bfloat16), (800, 256, 256, 0, 1, 1, torch.bfloat16),
          (256, 256, 800, 1, 1, 1, torch.bfloat16), (800, 2048, 256, 0, 0, 0, torch.bfloat16),
          (800, 256, 2048, 0, 1, 1, torch.bfloat16), (2048, 256, 800, 1, 1, 1, torch.bfloat16),
          (800, 49, 256, 0, 0, 0, torch.bfloat16), (49, 256, 800, 1, 1, 1, torch.bfloat16),
          (2400, 256, 256, 0, 0, 0, torch.bfloat16), (9600, 256, 256, 0, 0, 0, torch.bfloat16),
          (256, 256, 2400, 1, 1, 1, torch.bfloat16), (800, 256, 256, 0, 1, 1, torch.float32)]
if "--big" in sys.argv:  # the pixel decoder's / Swin's many-tile forward products, with bias
    sys.argv.remove("--big")
    shapes = [(50400, 1024, 256, 0, 0, 0, torch.bfloat16), (50400, 256, 256, 0, 0, 0, torch.bfloat16),
              (50400, 256, 1024, 0, 0, 0, torch.bfloat16), (50400, 192, 256, 0, 0, 0, torch.bfloat16),
              (38400, 256, 256, 0, 0, 0, torch.bfloat16), (50400, 256, 256, 0, 0, 1, torch.bfloat16),
              (153600, 384, 96, 0, 0, 0, torch.bfloat16)]
n, rounds = 20, 5
for M, N, K, at, bt, cf, dt in shapes:
    A = torch.randn((K, M) if at else (M, K), device=dev).to(dt)
    Bm = torch.randn((K, N) if bt else (N, K), device=dev).to(dt)
    bias = torch.randn(N, device=dev) if M >= 38400 else None
    times = {k: [] for k in libs}
    outs, graphs = {}, {}
    for rnd in range(rounds + 1):
        for tag, L in libs.items():
            _lib._lib = L
            fn = lambda: dense.gemm(A, Bm, at, bt, M, N, K, c_f32=bool(cf), bias=bias)  # noqa: E731
            outs[tag] = fn()
            torch.cuda.synchronize()
            if rnd == 0:  # the n calls captured once per build: replays time the device alone
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(n):
                        fn()
                graphs[tag] = g
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graphs[tag].replay()
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                times[tag].append(e0.elapsed_time(e1) * 1000 / n)
    _lib._lib = new
    row = "  ".join(f"{k} {statistics.median(v):7.1f} us{'' if torch.equal(outs[k], outs['new']) else ' (DIFFERS)'}"
                    for k, v in times.items())
    print(f"M {M:5d} N {N:5d} K {K:5d} at {at} bt {bt} c32 {cf} {str(dt)[6:]:8s}: {row}", flush=True)
