"""Whole-model training step of the drop-in CustomMask2FormerForUniversalSegmentation (v0.4.0,
Swin-T, 48 labels) at 640x480 on one MI355X: forward with labels (loss incl. the Hungarian
matcher and 9 auxiliary outputs), backward, AdamW.  Synthetic NYUv2-shaped scenes (rectangle
instances), random-init weights.  Two arms on the same weights and inputs:
  hip   — hot path (bf16 MFMA) + f1 mask predictor + f2 deformable attention + f3 matcher on HIP
  hf    — hot path (bf16 MFMA), the f1/f2/f3 modules as the installed Hugging Face code
with the HF parts in float32 or under torch.autocast(bfloat16) (--amp).  Prints one JSON line."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--amp", type=int, default=1)
    ap.add_argument("--arms", default="hip,hf")
    args = ap.parse_args()
    from rgbd_amd import (deform_attn, dense, init as winit, mask_predictor, masked_attention, point_loss, ops, swin,
                          synthetic)
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    dev = torch.device("cuda")
    B, H, W = args.batch, args.height, args.width
    scenes = [synthetic.make_scene(synthetic.scene_seed(4, i), H, W) for i in range(B)]
    depth = torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(dev)
    rgb = torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).contiguous().to(dev)
    mask_labels = [torch.from_numpy(s["masks"].astype(np.float32)).to(dev) for s in scenes]
    class_labels = [torch.from_numpy(s["classes"]).to(dev) for s in scenes]
    res = {"batch": B, "shape": f"{W}x{H}", "amp_bf16": bool(args.amp)}
    for ai, arm in enumerate(args.arms.split(",")):
        torch.manual_seed(0)
        m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
        winit.init_deterministic(m)
        m.set_compute_dtype(torch.bfloat16).to(dev).train()
        if arm == "hf":
            mask_predictor.uninstall(m)
            masked_attention.uninstall(m)
            deform_attn.uninstall(m)
            point_loss.uninstall(m)
            dense.uninstall(m)
            swin.uninstall(m)
        if arm == "hip_nogn":  # A/B: the pixel decoder's GroupNorms back on torch
            for mod in m.modules():
                if type(mod) is dense.HipGroupNorm:
                    mod.__dict__.pop("_fused_relu", None)
                    mod.__class__ = torch.nn.GroupNorm
                elif type(mod) is dense._FusedReLU:
                    mod.__class__ = torch.nn.ReLU
        opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-5, fused=True)

        def step():
            pv = ops.assemble_pixel_values(depth, rgb)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bool(args.amp)):
                out = m(pixel_values=pv, mask_labels=mask_labels, class_labels=class_labels)
            out.loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            return out.loss
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        key = arm if arm not in res else f"{arm}_{ai}"
        res[key] = {"img_s": round(B / dt, 2), "ms_per_step": round(dt * 1e3, 1), "loss": round(float(loss.detach()), 4)}
        del m, opt
        torch.cuda.empty_cache()
    if "hip" in res and "hf" in res:
        res["speedup_hip_vs_hf_modules"] = round(res["hip"]["img_s"] / res["hf"]["img_s"], 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
