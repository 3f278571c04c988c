import sys, numpy as np, torch
sys.path[:0] = ['.', 'tests/golden']
import _rgbd_import, golden_inputs as gi
from rgbd_amd import init as winit
from rgbd_amd.config import standard_config
from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
g5 = np.load('tests/golden/g5_model.npz')
m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
winit.init_deterministic(m)
import os
if os.environ.get("RGBD_DIAG_NOCONV") == "1":  # the f2 convolutions back on torch (A/B)
    from rgbd_amd.conv import HipConv2d
    for mod in m.modules():
        if type(mod) is HipConv2d:
            mod.__class__ = torch.nn.Conv2d
m = m.cuda().eval()
plm = m.model.pixel_level_module
caps = {}
plm.decoder.register_forward_pre_hook(lambda mod, a: caps.__setitem__("bb", [t.detach().clone() for t in a[0]]))
plm.encoder.register_forward_hook(lambda mod, i, o: caps.__setitem__("sw", [t.detach().clone() for t in o.feature_maps]))
ref_ratio = torch.from_numpy(g5["ratio"]).cuda()
plm.ratio_predictor.register_forward_hook(lambda mod, inp, out: ref_ratio.clone())
pv = torch.from_numpy(gi.pixel_values(1, 1, 240, 320)).cuda()
for rep in range(2):
    torch.backends.cudnn.allow_tf32 = rep == 0
    torch.backends.cuda.matmul.allow_tf32 = False
    with torch.no_grad():
        out = m(pixel_values=pv)
    for tag in ("sw", "bb"):
        for k in range(4):
            t = caps[tag][k].float().cpu().numpy().ravel()
            e = np.abs(t[g5[f"{tag}{k}_idx"]] - g5[f"{tag}{k}_val"]).max()
            print(rep, tag, k, f"max|err|={e:.3g} max|ref|={np.abs(g5[f'{tag}{k}_val']).max():.3g} sumdiff={(t.astype(np.float64).sum()-float(g5[f'{tag}{k}_sum'])):.3g}")
    ml = out.masks_queries_logits.cpu().numpy()
    print(rep, "mask logits max err", np.abs(ml - g5["mask_logits"]).max(), "max|ref|", np.abs(g5["mask_logits"]).max())
    print(rep, "class logits max err", np.abs(out.class_queries_logits.cpu().numpy() - g5["class_logits"]).max())
print("rep0: cudnn.allow_tf32=True, rep1: False")
