"""Where the whole-model step's torch glue comes from (diagnostic): one eager bf16 training step of
bench.full_model's model under torch.profiler with stacks and shapes, and for every aten op with
device time (copies, adds, fills, index ops, ...) the call site that issued it — the innermost
line of this repository or transformers for forward ops (a TorchFunctionMode wraps each call in
a record_function: this torch build records no Python stacks), the autograd node for backward ops —
with its launches, device time and input shapes.  Writes the table to argv[1] (default stdout)."""
import os
import re
import sys
from collections import defaultdict

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402
from torch.profiler import ProfilerActivity, profile, record_function  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import init as winit, ops, synthetic  # noqa: E402
from rgbd_amd.config import standard_config  # noqa: E402
from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation  # noqa: E402
from rgbd_amd.optim import HF_TRAINER_ADAMW, HipAdamW  # noqa: E402

B, H, W = 8, 480, 640
dev = torch.device("cuda:0")
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


for _ in range(3):
    step()
torch.cuda.synchronize()
OURS = ("rgb-d-instance-segmentation_amd", "rgbd_amd", "transformers/", "bench.py")


class SiteMode(TorchFunctionMode):
    """Wraps every torch function called from this repository or transformers (forward) in a
    record_function named after the calling line, so the profiler's tree carries the call site
    (this torch build records no Python stacks)."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        f = sys._getframe(1)
        while f is not None:
            fn = f.f_code.co_filename
            if any(o in fn for o in OURS) and "/tools/" not in fn:
                short = re.sub(r"^.*?(rgb-d-instance-segmentation_amd|transformers)/", "", fn)
                with record_function(f"@{short}:{f.f_lineno}"):
                    return func(*args, **kwargs)
            f = f.f_back
        return func(*args, **kwargs)


def step_sited():
    pv = ops.assemble_pixel_values(depth, rgb)
    with SiteMode(), torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(pixel_values=pv, mask_labels=mask_labels, class_labels=class_labels)
    out.loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)


step_sited()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step_sited()
    torch.cuda.synchronize()

GLUE = ("aten::copy_", "aten::add", "aten::add_", "aten::mul", "aten::mul_", "aten::fill_", "aten::zero_",
        "aten::index", "aten::index_put_", "aten::cat", "aten::where", "aten::clamp", "aten::sub", "aten::div",
        "aten::sum", "aten::mean", "aten::addcmul_", "aten::masked_fill_", "aten::sigmoid", "aten::relu",
        "aten::threshold_backward", "aten::gt", "aten::lt", "aten::ne", "aten::eq", "aten::neg", "aten::exp",
        "aten::pow", "aten::sqrt", "aten::_softmax", "aten::_softmax_backward_data", "aten::topk", "aten::sort",
        "aten::gather", "aten::scatter_add_", "aten::nonzero", "aten::bmm", "aten::mm", "aten::addmm",
        "aten::grid_sampler_2d", "aten::grid_sampler_2d_backward", "aten::upsample_bilinear2d",
        "aten::upsample_bilinear2d_backward", "aten::binary_cross_entropy_with_logits", "aten::clone",
        "aten::contiguous", "aten::_to_copy", "aten::to", "aten::linalg_vector_norm", "aten::max", "aten::min")


def site(ev):
    """The autograd node of a backward op; for a forward op the innermost call-site range."""
    p = ev
    while p is not None:
        if p.name.startswith("autograd::engine::evaluate_function"):
            return "bwd " + p.name.split(": ", 1)[-1]
        if p.name.startswith("@"):
            return p.name[1:]
        p = p.cpu_parent
    return "(no call site)"


def device_us(ev):
    """device time of the kernels this op launched itself (not its children's)."""
    t = getattr(ev, "self_device_time_total", None)
    return t if t is not None else ev.self_cuda_time_total


tot = defaultdict(float)
cnt = defaultdict(int)
shp = {}
events = prof.events()
for ev in events:
    if ev.name not in GLUE:
        continue
    # the op that launched the kernels: skip ops whose time is a child op's (aten::to -> copy_)
    us = device_us(ev)
    if us <= 0:
        continue
    key = (ev.name, site(ev))
    tot[key] += us
    cnt[key] += 1
    shp.setdefault(key, str(ev.input_shapes)[:70])
lines = [f"{'us':>9} {'n':>4}  op / call site / first input shapes"]
for key, us in sorted(tot.items(), key=lambda kv: -kv[1])[:90]:
    lines.append(f"{us:9.1f} {cnt[key]:4d}  {key[0]:26s} {key[1]}  {shp[key]}")
lines.append(f"total glue {sum(tot.values()) / 1e3:.2f} ms over {sum(cnt.values())} ops")
out = "\n".join(lines)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        f.write(out + "\n")
print(out)
