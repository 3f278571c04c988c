"""Which part of the whole-model training step breaks HIP-graph capture: capture, in order,
(a) the forward without labels, (b) the forward with labels (loss, matcher), (c) forward +
backward, (d) forward + backward + optimizer, each after eager warm-up, in the default
("global") capture mode and then in "relaxed" mode; prints one line per attempt."""
import sys
import traceback
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import init as winit, ops, synthetic  # noqa: E402
from rgbd_amd.config import standard_config  # noqa: E402
from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation  # noqa: E402
from rgbd_amd.optim import HF_TRAINER_ADAMW, HipAdamW  # noqa: E402

dev = torch.device("cuda")
B, H, W = 2, 480, 640
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


def fwd(labels):
    pv = ops.assemble_pixel_values(depth, rgb)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        if labels:
            return m(pixel_values=pv, mask_labels=mask_labels, class_labels=class_labels).loss
        return m(pixel_values=pv).masks_queries_logits


stages = {
    "a_forward": lambda: fwd(False),
    "b_forward_loss": lambda: fwd(True),
    "c_fwd_bwd": lambda: fwd(True).backward(),
    "d_fwd_bwd_opt": lambda: (fwd(True).backward(), opt.step()),
}
for mode in ("global", "relaxed"):
    for name, fn in stages.items():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        try:
            with torch.cuda.stream(s):
                for _ in range(2):
                    fn()
                    opt.zero_grad(set_to_none=True)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                fn()
            g.replay()
            torch.cuda.synchronize()
            print(f"{mode:8s} {name:16s} OK", flush=True)
            del g
        except Exception as e:
            tb = traceback.format_exc().strip().splitlines()
            where = [ln for ln in tb if "rgb-d-instance-segmentation_amd" in ln or "transformers" in ln][-3:]
            print(f"{mode:8s} {name:16s} FAIL {repr(e)[:160]} | {' || '.join(x.strip() for x in where)}", flush=True)
            torch.cuda.synchronize()
        opt.zero_grad(set_to_none=True)
