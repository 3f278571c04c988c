"""Oracle for the v0.4.0 pixel-level-module body between the Swin encoder and the pixel
decoder (custom_model.py:324-355), PyTorch-CPU fp32 + numpy.

Inputs are the Swin colour feature maps (outside the path, Q1: detached) and the
10-channel pixel_values.  ``ratios`` may be injected (SURVEY §7 hard part (v)); otherwise
they are computed by the ratio-predictor oracle.
"""
import numpy as np
import torch

from . import edsam, ratio as ratio_mod, dggm as dggm_mod

DSAM_CH = [(96, 192), (192, 384), (384, 768)]


def split_params(sd: dict, prefix: str = ""):
    """Pick the hot-path tensors out of a state_dict keyed like the reference module."""
    rp = {k[len(prefix + "ratio_predictor."):]: v for k, v in sd.items()
          if k.startswith(prefix + "ratio_predictor.")}
    dsam = []
    for k in range(3):
        pre = f"{prefix}dsam{k}."
        dsam.append(dict(
            conv_w=torch.stack([sd[f"{pre}conv_layers.{i}.weight"] for i in range(4)]),
            conv_b=torch.stack([sd[f"{pre}conv_layers.{i}.bias"] for i in range(4)]),
            proj_w=sd[f"{pre}rgb_projection.weight"]))
    pre = prefix + "depth_gradient_injection.depth_enhancement_layers."
    dg_w = [sd[f"{pre}{i}.0.weight"] for i in range(4)]
    dg_b = [sd[f"{pre}{i}.0.bias"] for i in range(4)]
    return rp, dsam, dg_w, dg_b


def hot_path_forward(colors, pixel_values, sd, prefix="", ratios=None, training=False):
    """Returns (backbone_features list, ratios [B,1], decompositions list)."""
    depth = pixel_values[:, 3:6]
    gdepth = pixel_values[:, 6:9]
    gmask = pixel_values[:, 9:10]
    rp, dsam, dg_w, dg_b = split_params(sd, prefix)
    cp1 = [c.detach().clone() for c in colors]                      # :332
    cp2 = [c.detach().clone() for c in colors]                      # :333
    if ratios is None:
        ratios = ratio_mod.ratio_forward(depth, rp, training=training)  # :336
    decs = [edsam.decompose(depth[b].numpy(), float(ratios[b, 0].item()))
            for b in range(depth.shape[0])]
    for k in range(3):                                              # :339-352
        outs = [edsam.dsam_forward(cp1[k][b:b + 1], decs[b]["code"], decs[b]["n_masks"],
                                   **dsam[k]) for b in range(depth.shape[0])]
        cp1[k + 1] += torch.cat(outs, dim=0)
    cp2 = dggm_mod.dggm_forward(cp2, gdepth, gmask, dg_w, dg_b)      # :354
    return [a + b for a, b in zip(cp1, cp2)], ratios, decs          # :355
