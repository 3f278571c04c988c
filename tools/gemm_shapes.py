"""Which HIP GEMM shapes the whole drop-in model's bf16 training step spends its time in
(diagnostic): bench.full_model's model (B = 8, 640x480), two warm-up steps, then one eager step with
every dense.gemm call bracketed by HIP events on its stream; per (M, N, K, a_t, b_t, batch, c dtype)
the calls, device time, TFLOP/s and the minimum HBM bytes (A, B, C once) per second."""
import os
import sys
from collections import defaultdict

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense, init as winit, ops, synthetic  # noqa: E402
from rgbd_amd.config import standard_config  # noqa: E402
from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation  # noqa: E402
from rgbd_amd.optim import HF_TRAINER_ADAMW, HipAdamW  # noqa: E402

dev = torch.device("cuda")
B, H, W = 8, 480, 640
scenes = [synthetic.make_scene(synthetic.scene_seed(4, i), H, W) for i in range(B)]
depth = torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(dev)
rgb = torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).contiguous().to(dev)
mask_labels = [torch.from_numpy(s["masks"].astype(np.float32)).to(dev) for s in scenes]
class_labels = [torch.from_numpy(s["classes"]).to(dev) for s in scenes]
torch.manual_seed(0)
m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
winit.init_deterministic(m)
m.set_compute_dtype(torch.bfloat16).to(dev).train()
opt = HipAdamW([p for p in m.parameters() if p.requires_grad], **HF_TRAINER_ADAMW)


def step():
    pv = ops.assemble_pixel_values(depth, rgb)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(pixel_values=pv, mask_labels=mask_labels, class_labels=class_labels)
    out.loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)


for _ in range(2):
    step()
torch.cuda.synchronize()
rec = []
orig = dense.gemm


def timed_gemm(A, Bm, a_t, b_t, M, N, K, *args, **kw):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    out = orig(A, Bm, a_t, b_t, M, N, K, *args, **kw)
    e1.record(s)
    rec.append(((M, N, K, int(a_t), int(b_t), kw.get("batch", 1), str(out.dtype).split(".")[-1], A.element_size()),
                e0, e1))
    return out


dense.gemm = timed_gemm
step()
torch.cuda.synchronize()
agg = defaultdict(lambda: [0, 0.0])
for key, e0, e1 in rec:
    agg[key][0] += 1
    agg[key][1] += e0.elapsed_time(e1) * 1e3
tot = sum(v[1] for v in agg.values())
print(f"{len(rec)} gemm calls, {tot / 1e3:.2f} ms")
print("   us total  calls   us/call  TF/s   GB/s  (M, N, K, a_t, b_t, batch, C dtype, A bytes/elt)")
for key, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    M, N, K, _, _, bt, cdt, es = key
    fl = 2.0 * M * N * K * bt * n
    by = (M * K + N * K) * es * bt * n + M * N * bt * n * (4 if cdt == "float32" else 2)
    print(f"{us:10.1f} {n:6d} {us / n:9.1f} {fl / us / 1e6:6.0f} {by / us / 1e3:6.0f}  {key}")
