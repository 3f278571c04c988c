"""Which torch ops the whole drop-in model's bf16 training step spends its glue time in (diagnostic):
the hip arm of tools/bench_full_model.py (B = 8, 640x480), two warm-up steps, then one step under
torch.profiler with input shapes and Python stacks; prints the top ops by self device time grouped
by input shape, and the call sites (5 frames) of the largest elementwise adds and copies."""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import init as winit, ops, synthetic  # noqa: E402
from rgbd_amd.config import standard_config  # noqa: E402
from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation  # noqa: E402

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
opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-5, fused=True)


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
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
key = "self_device_time_total"
try:
    print(prof.key_averages(group_by_input_shape=True).table(sort_by=key, row_limit=25, max_name_column_width=40,
                                                            max_shapes_column_width=70))
except Exception:  # older naming
    key = "self_cuda_time_total"
    print(prof.key_averages(group_by_input_shape=True).table(sort_by=key, row_limit=25, max_name_column_width=40,
                                                            max_shapes_column_width=70))
ka = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ka if e.key in ("aten::add_", "aten::add", "aten::copy_", "aten::to", "aten::_to_copy")]
rows.sort(key=lambda e: -getattr(e, key))
for e in rows[:12]:
    print(f"{e.key:16s} {getattr(e, key) / 1e3:8.2f} ms  x{e.count}")
    for fr in e.stack[:6]:
        print("      ", fr)
