"""Micro benchmark: rgbd_colsum (the dense layers' bias gradients, csrc/gemm.hip k_colsum) against
torch's column sum on the whole model's shapes (pixel decoder 50 400 tokens x 256 / 1024,
decoder queries 800 x 256 / 2048, Swin stage 1 153 600 x 96), bf16 in, float32 out."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense  # noqa: E402


def timeit(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for rows, N in [(50400, 256), (50400, 1024), (800, 256), (800, 2048), (153600, 96)]:
    y = torch.randn((rows, N), device="cuda", dtype=torch.bfloat16)
    ours = timeit(lambda: dense.colsum(y))
    lib = timeit(lambda: y.float().sum(0))
    err = float((dense.colsum(y) - y.double().sum(0)).abs().max())
    print(json.dumps({"rows": rows, "N": N, "ours_us": round(ours, 1), "torch_us": round(lib, 1),
                      "GBs": round(rows * N * 2 / ours / 1e3, 1), "max_err": err}), flush=True)
