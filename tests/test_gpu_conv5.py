"""conv5 on its own: feature_extractor[0:4] of the ratio predictor (3x3 conv 128->256, BatchNorm,
ReLU, AdaptiveAvgPool(4); custom_model.py:1412-1416) as the bf16 kernels leave it in the ratio
workspace (`rgbd_ratio_pooled_offset`), against float64 arithmetic on the same bf16 gated
features (`rgbd_ratio_features_offset`) and bf16-rounded conv5 weights.

The kernels' contract, restated here: the conv accumulates in float32; train-mode batch statistics
are taken over the float32 conv outputs (bias included); BN + ReLU act on the conv outputs rounded
to bf16 (what the unfused path stores as y), in float32 (mul, add, max), and the pool averages.
Cases cover every route: train with the half-tile pool (480x640) and the generic pool (240x320,
ragged 90x125), eval with BN + ReLU + pool fused into conv5's epilogue (240x320, 64x128, C5's
1280x720) and eval through y (ragged 90x125, 64x96).  Tolerance: rtol 2e-4 / atol 1e-5 of the
largest pooled value — float32 vs float64 accumulation moves a y value across a bf16 rounding
boundary for ~1e-4 of the elements, one ulp each, averaged over a pool bin; an indexing slip
(a wrong tap, channel quarter, bin or tile) is off by orders of magnitude."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_inputs as gi
from checkers import ratio_ws
from rgbd_amd import init as winit

pytestmark = pytest.mark.gpu
DEV = "cuda"
PRE = "model.pixel_level_module.ratio_predictor."


def _module():
    from rgbd_amd.modules import EnhancedDepthImageRatioPredictor
    m = EnhancedDepthImageRatioPredictor(3)
    winit.init_deterministic(m, prefix=PRE)
    m.compute_dtype = torch.bfloat16
    return m


@pytest.mark.parametrize("B,H,W,training", [
    (2, 480, 640, True), (2, 240, 320, True), (2, 90, 125, True),
    (2, 240, 320, False), (2, 64, 128, False), (1, 720, 1280, False), (2, 90, 125, False), (2, 64, 96, False)])
def test_bf16_conv5_bn_relu_pool(B, H, W, training):
    from rgbd_amd import _lib, ops
    pv = gi.pixel_values(21, B, H, W)
    m = _module()
    fe = m.feature_extractor
    bn = fe[1]
    # distinct running statistics, so that eval mode's affine is not the identity
    g = torch.Generator().manual_seed(5)
    bn.running_mean.copy_(torch.randn(256, generator=g) * 0.05)
    bn.running_var.copy_(torch.rand(256, generator=g) * 0.5 + 0.5)
    run_mean, run_var = bn.running_mean.clone().double(), bn.running_var.clone().double()
    m = m.to(DEV).train(training)
    x = torch.from_numpy(pv).to(DEV)[:, 3:6]
    with torch.no_grad():
        m(x)
    torch.cuda.synchronize()
    L = _lib.lib()
    ws = ops._workspace(x.device, L.rgbd_ratio_workspace_size(1, B, H, W), "ratio")
    off = L.rgbd_ratio_features_offset(1, B, H, W)
    assert ratio_ws.ratio_pad_is_zero(ws, off, B, H, W)  # conv5's halo reads zeros outside the image
    xin = ratio_ws.ratio_features_bf16(ws, off, B, H, W).double().cpu()
    poff = L.rgbd_ratio_pooled_offset(1, B, H, W)
    got = ws[poff:poff + B * 256 * 16 * 4].view(torch.float32).reshape(B, 256, 4, 4).double().cpu()

    conv = fe[0]
    w5 = conv.weight.detach().cpu().to(torch.bfloat16).double()
    yf = F.conv2d(xin, w5, conv.bias.detach().cpu().double(), padding=1)
    if training:
        mean = yf.mean((0, 2, 3)).float()
        var = yf.var((0, 2, 3), unbiased=False).float()
    else:
        mean, var = run_mean.float(), run_var.float()
    gamma, beta = bn.weight.detach().cpu().float(), bn.bias.detach().cpu().float()
    sc = gamma / torch.sqrt(var + 1e-5)
    sh = beta - mean * sc
    yb = yf.float().to(torch.bfloat16).float()
    z = torch.clamp_min(yb * sc[None, :, None, None] + sh[None, :, None, None], 0.0)
    ref = F.adaptive_avg_pool2d(z.double(), 4)
    scale = float(ref.abs().max())
    assert scale > 1e-3
    d = (got - ref).abs()
    bad = d > 2e-4 * ref.abs() + 1e-5 * scale
    print(f"{B}x{H}x{W} train={training}: max |d| {float(d.max()):.3g} (scale {scale:.3g}), {int(bad.sum())} bad")
    assert not bool(bad.any()), (float(d.max()), scale, np.argwhere(bad.numpy())[:5].tolist())
