"""Where the bf16 ratio error comes from (CPU, the oracle's float32 math): the spread-head
ratio predictor (tests/test_gpu_bf16_parity.py) at 240x320, B=6, with one thing at a time rounded
to bf16 — each weight group, the depth input, each stored activation — against the exact run.
r03 result: weight rounding dominates (each group +-3e-4..8e-4 in the ratio, partly cancelling:
4.2e-4 together), the depth input 9e-5, the stored activations <= 6e-6 each."""
import sys, torch, numpy as np
sys.path.insert(0, '/root/repo'); import _rgbd_import
import torch.nn.functional as F
from oracle import ratio as ro
from rgbd_amd import init as winit, synthetic
from rgbd_amd.modules import EnhancedDepthImageRatioPredictor
torch.set_num_threads(8)
H, W, B = 240, 320, 6
pv = np.stack([np.concatenate([synthetic.rgbd_planes(synthetic.make_scene(synthetic.scene_seed(2, i), H, W))]) for i in range(B)])
d = torch.from_numpy(pv)[:, 3:6].float()
m = EnhancedDepthImageRatioPredictor(3); winit.init_deterministic(m, prefix="model.pixel_level_module.ratio_predictor.")
p = {k: v.clone() for k, v in m.state_dict().items()}
with torch.no_grad():
    z = ro.ratio_forward(d, p, return_logit=True).double().reshape(-1)
a = 4.0 / float(z.max() - z.min()); c = -a * float(z.mean())
p["fc_layers.8.weight"] = p["fc_layers.8.weight"] * a; p["fc_layers.8.bias"] = p["fc_layers.8.bias"] * a + c
bf = lambda t: t.to(torch.bfloat16).float()
def run(wq=False, aq=set()):
    sel = (lambda k: True) if wq is True else (lambda k: bool(wq) and k.startswith(wq))
    q = {k: (bf(v) if sel(k) and k.endswith("weight") and v.dim() == 4 else v) for k, v in p.items()}
    def cbr(x, pre, pad):
        y = F.conv2d(bf(x) if "in" in aq else x, q[pre+".0.weight"], q[pre+".0.bias"], padding=pad)
        return F.relu(ro._bn(y, q, pre+".1", False))
    s1 = cbr(d, "scale1_conv", 1); s2 = cbr(d, "scale2_conv", 2); s3 = cbr(d, "scale3_conv", 3)
    ms = torch.cat([s1, s2, s3], 1)
    if "stem" in aq: ms = bf(ms)
    fu = cbr(ms, "feature_fusion", 0)
    if "fus" in aq: fu = bf(fu)
    at = F.relu(F.conv2d(fu, q["attention.0.weight"], q["attention.0.bias"]))
    at = torch.sigmoid(F.conv2d(at, q["attention.2.weight"], q["attention.2.bias"]))
    x = fu * at
    if "att" in aq: x = bf(x)
    e = F.conv2d(x, q["feature_extractor.0.weight"], q["feature_extractor.0.bias"], padding=1)
    if "y" in aq: e = bf(e)
    e = F.relu(ro._bn(e, q, "feature_extractor.1", False))
    e = F.adaptive_avg_pool2d(e, 4)
    e = F.conv2d(e, q["feature_extractor.4.weight"], q["feature_extractor.4.bias"], padding=1)
    e = F.relu(ro._bn(e, q, "feature_extractor.5", False))
    g = F.adaptive_avg_pool2d(e, 1).flatten(1)
    h = F.relu(F.linear(g, q["fc_layers.0.weight"], q["fc_layers.0.bias"]))
    h = F.relu(F.linear(h, q["fc_layers.3.weight"], q["fc_layers.3.bias"]))
    h = F.relu(F.linear(h, q["fc_layers.6.weight"], q["fc_layers.6.bias"]))
    raw = F.linear(h, q["fc_layers.8.weight"], q["fc_layers.8.bias"])
    return (0.01 + 0.49 * torch.sigmoid(raw)).reshape(-1)
with torch.no_grad():
    r0 = run()
    for name, kw in [("weights", dict(wq=True)), ("w scale", dict(wq="scale")), ("w fusion", dict(wq="feature_fusion")),
                     ("w attention", dict(wq="attention")), ("w conv5", dict(wq="feature_extractor.0")),
                     ("w tail", dict(wq="feature_extractor.4")), ("input", dict(aq={"in"})), ("stem", dict(aq={"stem"})), ("fus", dict(aq={"fus"})),
                     ("att", dict(aq={"att"})), ("y", dict(aq={"y"})), ("all acts", dict(aq={"in","stem","fus","att","y"})),
                     ("everything", dict(wq=True, aq={"in","stem","fus","att","y"}))]:
        r = run(**kw)
        print(f"{name:12s} max|dr| {float((r - r0).abs().max()):.2e}")
