"""Micro-benchmark of the f1 mask-predictor kernels at the C2 shape (B=8, Q=100, C=256, mask
features 120x160 of a 640x480 input) against torch.einsum (library GEMM) and the torch
interpolate/sigmoid/repeat chain.  Prints one JSON line per kernel."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import ops  # noqa: E402


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-torch", action="store_true", help="skip the torch reference timings (PMC passes)")
    args = ap.parse_args()
    global timeit
    _t = timeit
    timeit = lambda fn: _t(fn, iters=args.iters, warm=min(5, args.iters))  # noqa: E731
    B, Q, C, H, W = 8, 100, 256, 120, 160
    P = H * W
    for dt in (torch.bfloat16, torch.float32):
        es = 2 if dt == torch.bfloat16 else 4
        emb = torch.randn((B, Q, C), device="cuda").to(dt)
        pix = torch.randn((B, C, H, W), device="cuda").to(dt)
        t_hip = timeit(lambda: ops.mask_logits(emb, pix))
        t_ref = 0.0 if args.no_torch else timeit(lambda: torch.einsum("bqc,bchw->bqhw", emb, pix))
        nbytes = B * P * (C + Q) * es + B * Q * C * es
        print(json.dumps({"kernel": "k_mask_logits", "dtype": str(dt), "us": round(t_hip, 2),
                          "GB/s": round(nbytes / t_hip / 1e3, 1), "frac_hbm": round(nbytes / t_hip / 1e3 / 8000, 3),
                          "torch_einsum_us": round(t_ref, 2), "alg_bytes": nbytes}))
        logits = torch.randn((B, Q, H, W), device="cuda").to(dt)
        for size in [(60, 80), (30, 40), (15, 20)]:
            t_hip = timeit(lambda: ops.mask_attention(logits, size, 8))
            t_ref = 0.0 if args.no_torch else timeit(lambda: (F.interpolate(logits, size=size, mode="bilinear", align_corners=False)
                                    .sigmoid().flatten(2).unsqueeze(1).repeat(1, 8, 1, 1).flatten(0, 1) < 0.5).bool())
            print(json.dumps({"kernel": "k_mask_attention", "dtype": str(dt), "target": size, "us": round(t_hip, 2),
                              "torch_us": round(t_ref, 2)}))


if __name__ == "__main__":
    main()
