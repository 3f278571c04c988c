"""Diagnostic: which installed HIP component moves the whole model's bf16 loss.  The drop-in
model at 640x480 B=8 in eval mode (no dropout / DropPath draws) with labels: the loss and the
final mask / class logits under torch.autocast(bfloat16) with every HIP component installed,
then with one component family at a time swapped back to the HF module, against the HF-module
model in float32."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def main():
    from rgbd_amd import (deform_attn, dense, init as winit, mask_predictor, masked_attention, ops, point_loss,
                          swin, synthetic)
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    dev = torch.device("cuda")
    B, H, W = 8, 480, 640
    scenes = [synthetic.make_scene(synthetic.scene_seed(4, i), H, W) for i in range(B)]
    depth = torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(dev)
    rgb = torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).contiguous().to(dev)
    mask_labels = [torch.from_numpy(s["masks"].astype(np.float32)).to(dev) for s in scenes]
    class_labels = [torch.from_numpy(s["classes"]).to(dev) for s in scenes]
    m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
    winit.init_deterministic(m)
    m.set_compute_dtype(torch.bfloat16).to(dev).eval()
    pv = ops.assemble_pixel_values(depth, rgb)
    fams = {"dense": (dense.install, dense.uninstall), "swin": (swin.install, swin.uninstall),
            "masked_attn": (masked_attention.install, masked_attention.uninstall),
            "deform": (deform_attn.install, deform_attn.uninstall),
            "mask_pred": (mask_predictor.install, mask_predictor.uninstall),
            "point_loss": (point_loss.install, point_loss.uninstall)}

    def run(amp):
        torch.manual_seed(0)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = m(pixel_values=pv, mask_labels=mask_labels, class_labels=class_labels)
        return float(out.loss), out.masks_queries_logits.float(), out.class_queries_logits.float()

    def set_all(on):
        for name, (ins, unins) in fams.items():
            (ins if on else unins)(m)
    set_all(False)
    ref = run(False)
    print(f"HF modules float32: loss {ref[0]:.4f}")
    hf16 = run(True)
    print(f"HF modules bf16:    loss {hf16[0]:.4f}  masks {rel(hf16[1], ref[1]):.3g} classes {rel(hf16[2], ref[2]):.3g}")
    set_all(True)
    r = run(False)
    print(f"all HIP float32:    loss {r[0]:.4f}  masks {rel(r[1], ref[1]):.3g} classes {rel(r[2], ref[2]):.3g}")
    r = run(True)
    print(f"all HIP bf16:       loss {r[0]:.4f}  masks {rel(r[1], ref[1]):.3g} classes {rel(r[2], ref[2]):.3g}")
    for name, (ins, unins) in fams.items():
        set_all(True)
        unins(m)
        if name == "dense":
            swin.uninstall(m)  # the Swin layer class uses the dense kernels
        r = run(True)
        print(f"bf16 without {name:11s} loss {r[0]:.4f}  masks {rel(r[1], ref[1]):.3g} classes {rel(r[2], ref[2]):.3g}")
    for name, (ins, unins) in fams.items():
        set_all(False)
        ins(m)
        r = run(True)
        print(f"bf16 only {name:14s} loss {r[0]:.4f}  masks {rel(r[1], ref[1]):.3g} classes {rel(r[2], ref[2]):.3g}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def train_bisect():
    """Per-step training losses (bf16 autocast, train mode, AdamW lr 1e-5) with every HIP family
    installed, none, and each family alone removed: which one changes the trajectory."""
    from rgbd_amd import (deform_attn, dense, init as winit, mask_predictor, masked_attention, ops, point_loss,
                          swin, synthetic)
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    dev = torch.device("cuda")
    B, H, W = 8, 480, 640
    scenes = [synthetic.make_scene(synthetic.scene_seed(4, i), H, W) for i in range(B)]
    depth = torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(dev)
    rgb = torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).contiguous().to(dev)
    mask_labels = [torch.from_numpy(s["masks"].astype(np.float32)).to(dev) for s in scenes]
    class_labels = [torch.from_numpy(s["classes"]).to(dev) for s in scenes]
    fams = {"dense": (dense.install, dense.uninstall), "swin": (swin.install, swin.uninstall),
            "masked_attn": (masked_attention.install, masked_attention.uninstall),
            "deform": (deform_attn.install, deform_attn.uninstall),
            "mask_pred": (mask_predictor.install, mask_predictor.uninstall),
            "point_loss": (point_loss.install, point_loss.uninstall)}
    configs = [("all", set(fams)), ("none", set())] + [(f"all-{k}", set(fams) - {k}) for k in fams]
    for name, on in configs:
        torch.manual_seed(0)
        m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
        winit.init_deterministic(m)
        m.set_compute_dtype(torch.bfloat16).to(dev).train()
        for k, (ins, unins) in fams.items():
            if k not in on:
                unins(m)
        opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-5, fused=True)
        losses = []
        for _ in range(5):
            pv = ops.assemble_pixel_values(depth, rgb)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(pixel_values=pv, mask_labels=mask_labels, class_labels=class_labels)
            out.loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            losses.append(round(float(out.loss), 3))
        print(f"train {name:18s} losses {losses}", flush=True)
        del m, opt
        torch.cuda.empty_cache()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "train":
    train_bisect()
