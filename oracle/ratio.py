"""Oracle for EnhancedDepthImageRatioPredictor, PyTorch-CPU fp32.

Restates custom_model.py:1363-1487 functionally on a parameter dict keyed like the
reference state_dict (``scale1_conv.0.weight``, ``scale1_conv.1.running_mean`` ...).
``training=False`` uses BN running stats (the parity mode, SURVEY §7 hard part (v));
``training=True`` uses batch statistics and no dropout (dropout is stochastic, Q15).
"""
import torch
import torch.nn.functional as F

EPS = 1e-5


def _bn(x, p, pre, training):
    return F.batch_norm(x, p[pre + ".running_mean"].clone(), p[pre + ".running_var"].clone(),
                        p[pre + ".weight"], p[pre + ".bias"], training=training, eps=EPS)


def _cbr(x, p, pre, pad, training):
    y = F.conv2d(x, p[pre + ".0.weight"], p[pre + ".0.bias"], padding=pad)
    return F.relu(_bn(y, p, pre + ".1", training))


def ratio_forward(depth: torch.Tensor, p: dict, training: bool = False, return_logit: bool = False) -> torch.Tensor:
    """depth [B,3,H,W] f32 -> ratio [B,1] f32 in [0.01, 0.5] (custom_model.py:1444-1487);
    ``return_logit``: the pre-sigmoid output of fc_layers.8 instead (test instrumentation)."""
    s1 = _cbr(depth, p, "scale1_conv", 1, training)                       # :1458
    s2 = _cbr(depth, p, "scale2_conv", 2, training)                       # :1459
    s3 = _cbr(depth, p, "scale3_conv", 3, training)                       # :1460
    ms = torch.cat([s1, s2, s3], dim=1)                                   # :1463
    fu = _cbr(ms, p, "feature_fusion", 0, training)                       # :1466
    a = F.relu(F.conv2d(fu, p["attention.0.weight"], p["attention.0.bias"]))
    a = torch.sigmoid(F.conv2d(a, p["attention.2.weight"], p["attention.2.bias"]))  # :1469
    at = fu * a                                                           # :1470
    e = F.conv2d(at, p["feature_extractor.0.weight"], p["feature_extractor.0.bias"], padding=1)
    e = F.relu(_bn(e, p, "feature_extractor.1", training))
    e = F.adaptive_avg_pool2d(e, 4)                                       # :1416
    e = F.conv2d(e, p["feature_extractor.4.weight"], p["feature_extractor.4.bias"], padding=1)
    e = F.relu(_bn(e, p, "feature_extractor.5", training))               # :1418-1420
    g = F.adaptive_avg_pool2d(e, 1).squeeze(-1).squeeze(-1)               # :1476-1479
    h = F.relu(F.linear(g, p["fc_layers.0.weight"], p["fc_layers.0.bias"]))
    h = F.relu(F.linear(h, p["fc_layers.3.weight"], p["fc_layers.3.bias"]))
    h = F.relu(F.linear(h, p["fc_layers.6.weight"], p["fc_layers.6.bias"]))
    raw = F.linear(h, p["fc_layers.8.weight"], p["fc_layers.8.bias"])     # :1482
    if return_logit:
        return raw
    return 0.01 + (0.5 - 0.01) * torch.sigmoid(raw)                       # :1485


def ratio_forward_modules(m, depth):
    """Same forward through the nn.Module tree of an (identically keyed) module on the CPU —
    the plain PyTorch fp32 reference used to check train-mode BatchNorm running-stat updates
    (Dropout modules are skipped so the comparison is deterministic)."""
    s = torch.cat([m.scale1_conv(depth), m.scale2_conv(depth), m.scale3_conv(depth)], dim=1)
    f = m.feature_fusion(s)
    e = m.feature_extractor(f * m.attention(f))
    g = F.adaptive_avg_pool2d(e, 1).flatten(1)
    fc = m.fc_layers
    h = fc[8](fc[7](fc[6](fc[4](fc[3](fc[1](fc[0](g)))))))
    return 0.01 + (0.5 - 0.01) * torch.sigmoid(h)
