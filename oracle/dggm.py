"""Oracle for DepthGradientInjectionResidual.forward, PyTorch-CPU fp32.

custom_model.py:1204-1269: per scale i,
  out_i = color_i + ReLU(Conv1x1_i(bilinear(grad -> h_i,w_i) * nearest(mask -> h_i,w_i)))
(``None`` grad or mask -> passthrough, :1263-1265).
"""
import torch.nn.functional as F


def dggm_forward(colors, grad, mask, weights, biases):
    if grad is None or mask is None:
        return list(colors)
    out = []
    for c, w, b in zip(colors, weights, biases):
        h, wd = c.shape[2:]
        g = F.interpolate(grad, size=(h, wd), mode="bilinear", align_corners=False)
        m = F.interpolate(mask, size=(h, wd), mode="nearest")
        out.append(c + F.relu(F.conv2d(g * m, w, b)))
    return out
