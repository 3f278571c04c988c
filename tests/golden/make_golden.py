"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE itself.

Runs only in the build container (``/root/reference`` does not exist on the GPU box):

    python tests/golden/make_golden.py

The reference is imported read-only with the two in-process shims SURVEY.md §8(c)
documents (no file of the reference is modified or copied):
  1. ``sys.modules['cv2']`` = empty module: custom_model.py:6 / data_process.py:18 import
     cv2, but the v0.4.0 model path never calls it;
  2. ``transformers.utils.backbone_utils.load_backbone`` aliased to the transformers 5.15
     location (custom_model.py:13 expects the 4.47 one).
Weights come from the deterministic generator (rgbd_amd.init); inputs from the seeded
synthetic-scene generator (rgbd_amd.synthetic).  Each fixture stores inputs (or the
sha256 of regenerated inputs) and the reference's outputs.

Fixtures (SURVEY.md §8(c) "Golden vectors"):
  g1_decompose.npz   a2 + a5-a8: grey, histogram, modes, windows, region codes, pooled codes
  g2_dsam.npz        a4: DSAModule forward at reduced channels (8->16, 16->32)
  g3_dggm.npz        a9: DepthGradientInjectionResidual forward at channels [4,8,16,32]
  g4_ratio.npz       a3: EnhancedDepthImageRatioPredictor eval at 240x320, B=2
  g5_model.npz       a1+a12: full model eval forward at 320x240 (ratio, logits, sampled features)
  g6_grads.npz       one loss.backward() at 320x240 B=2 (eval mode): loss + terms, the loss's
                     torch.rand draws (sha256), matches, attention masks, sampled gradients of
                     every grad-receiving parameter (make_golden.py g6)
  g8_resize.npz      a11 for frames not at model resolution: the processor's resize (PIL)
  g9_attn_masks.npz  the masked-attention decoder's attention masks at G5 / G7's inputs: per
                     mask-predictor call the reference's binarised mask (bit-packed, one head:
                     the heads repeat it) and its near-threshold pre-binarisation logits
"""
import hashlib
import json
import sys
import types
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
import _rgbd_import  # noqa: E402,F401  (registers rgbd_amd)
from rgbd_amd import init as winit, synthetic  # noqa: E402
from oracle import dggm_pre  # noqa: E402

OUT = Path(__file__).resolve().parent
REF = "/root/reference"


def import_reference():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    import transformers.utils.backbone_utils as bu
    from transformers.backbone_utils import load_backbone
    bu.load_backbone = load_backbone
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import mask2former.utils.custom_model as cm
    return cm


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ----------------------------------------------------------------------------- inputs
def decomposition_cases():
    """List of (name, depth3 f32 [3,H,W], ratio).  Regenerated identically by the tests."""
    return golden_inputs.decomposition_cases()


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    cm = import_reference()
    gray = cm.CustomMask2FormerPixelLevelModule.to_grayscale

    # ------------------------------------------------------------------ G1
    cases = golden_inputs.decomposition_cases()
    dsam = cm.DSAModule(8, 16)
    rec = {"names": [], "shapes": [], "ratios": [], "input_sha": [], "n_modes": [],
           "centers": [], "peak_hist": [], "windows": [], "hist": [], "edges": [],
           "grey_sha": [], "code": [], "pooled": [], "error": []}
    for name, d3, r in cases:
        H, W = d3.shape[1:]
        g = gray(None, torch.from_numpy(d3))
        gnp = g.squeeze().cpu().detach().numpy()
        rec["names"].append(name); rec["shapes"].append((H, W)); rec["ratios"].append(r)
        rec["input_sha"].append(sha(d3)); rec["grey_sha"].append(sha(gnp))
        try:
            hist, edges = dsam._calculate_depth_histogram(gnp)
        except ValueError as e:
            rec["error"].append(str(e))
            for k in ("n_modes", "centers", "peak_hist", "windows", "hist", "edges", "code", "pooled"):
                rec[k].append(None)
            continue
        rec["error"].append("")
        modes = dsam._select_depth_distribution_modes(hist, edges, num_modes=3)
        if modes:
            wins = dsam._define_depth_interval_windows(modes, window_size_ratio=r)
            masks = dsam._generate_depth_region_masks(gnp, wins)
        else:
            wins = []
            masks = [np.zeros_like(gnp, dtype=bool)] * 4
        code = np.zeros((H, W), np.uint8)
        for i, m in enumerate(masks):
            code |= m.astype(np.uint8) << i
        pooled = []
        for (oh, ow) in golden_inputs.pool_sizes(H, W):
            pc = np.zeros((oh, ow), np.uint8)
            for i, m in enumerate(masks):
                t = torch.from_numpy(m).float()[None, None]
                pm = F.adaptive_max_pool2d(t, (oh, ow))[0, 0].numpy()
                pc |= (pm > 0).astype(np.uint8) << i
            pooled.append(pc)
        rec["n_modes"].append(len(modes)); rec["centers"].append(np.array(modes, np.float32))
        rec["peak_hist"].append(np.array([0], np.int64))
        rec["windows"].append(np.array([[float(a), float(b)] for a, b in wins], np.float64).reshape(-1, 2))
        rec["hist"].append(hist.astype(np.int64)); rec["edges"].append(edges.astype(np.float32))
        rec["code"].append(code); rec["pooled"].append(pooled)
    save_g1(rec)

    # ------------------------------------------------------------------ G2
    g2 = {}
    for tag, (cin, cout) in {"a": (8, 16), "b": (16, 32)}.items():
        mod = cm.DSAModule(cin, cout)
        winit.init_deterministic(mod, prefix=f"g2.{tag}.")
        for ci, case_idx in enumerate(golden_inputs.G2_CASES):
            name, d3, r = cases[case_idx]
            H, W = d3.shape[1:]
            h, w = (H + 3) // 4, (W + 3) // 4
            x = golden_inputs.feature(f"g2.{tag}.{ci}", (1, cin, h, w))
            g = gray(None, torch.from_numpy(d3))
            with torch.no_grad():
                y = mod(torch.from_numpy(x), g, r)
            g2[f"{tag}_{ci}_x"] = x
            g2[f"{tag}_{ci}_y"] = y.numpy()
            g2[f"{tag}_{ci}_case"] = np.array(case_idx)
    np.savez_compressed(OUT / "g2_dsam.npz", **g2)

    # ------------------------------------------------------------------ G3
    mod = cm.DepthGradientInjectionResidual([4, 8, 16, 32], 3)
    winit.init_deterministic(mod, prefix="g3.")
    H, W = 64, 96
    planes = np.stack([dggm_pre.dggm_planes(synthetic.make_scene(9000 + b, H, W)["depth_u8"])
                       for b in range(2)])
    grad, mask = planes[:, 0:3], planes[:, 3:4]
    cols = [golden_inputs.feature(f"g3.c{i}", (2, c, (H + s - 1) // s, (W + s - 1) // s))
            for i, (c, s) in enumerate(zip([4, 8, 16, 32], [4, 8, 16, 32]))]
    with torch.no_grad():
        outs = mod([torch.from_numpy(c) for c in cols], torch.from_numpy(grad), torch.from_numpy(mask))
    g3 = {"grad": grad, "mask": mask}
    for i in range(4):
        g3[f"color{i}"] = cols[i]
        g3[f"out{i}"] = outs[i].numpy()
    np.savez_compressed(OUT / "g3_dggm.npz", **g3)

    # ------------------------------------------------------------------ G4
    rp = cm.EnhancedDepthImageRatioPredictor(3)
    winit.init_deterministic(rp, prefix="model.pixel_level_module.ratio_predictor.")
    rp.eval()
    pv = golden_inputs.pixel_values(4, 2, 240, 320)
    feats = {}
    rp.feature_extractor[3].register_forward_hook(lambda m, i, o: feats.__setitem__("pool4", o))
    with torch.no_grad():
        ratio = rp(torch.from_numpy(pv[:, 3:6]))
    np.savez_compressed(OUT / "g4_ratio.npz", ratio=ratio.numpy(), pool4=feats["pool4"].numpy(),
                        input_sha=np.array(sha(pv)))

    # ------------------------------------------------------------------ G5 / G6
    model = build_model(cm)
    pv = golden_inputs.pixel_values(1, 1, 240, 320)
    caps = {}
    plm = model.model.pixel_level_module
    plm.ratio_predictor.register_forward_hook(lambda m, i, o: caps.__setitem__("ratio", o.detach().clone()))
    plm.decoder.register_forward_pre_hook(lambda m, a: caps.__setitem__("bb", [t.detach().clone() for t in a[0]]))
    plm.encoder.register_forward_hook(lambda m, i, o: caps.__setitem__("sw", [t.detach().clone() for t in o.feature_maps]))
    model.eval()
    with torch.no_grad():
        out = model(pixel_values=torch.from_numpy(pv))
    g5 = {"input_sha": np.array(sha(pv)), "ratio": caps["ratio"].numpy(),
          "class_logits": out.class_queries_logits.numpy(),
          "mask_logits": out.masks_queries_logits.numpy()}
    for k in range(4):
        for tag, lst in (("bb", caps["bb"]), ("sw", caps["sw"])):
            t = lst[k].numpy().ravel()
            idx = golden_inputs.sample_index(f"g5.{tag}{k}", t.size, 4096)
            g5[f"{tag}{k}_idx"] = idx
            g5[f"{tag}{k}_val"] = t[idx]
            g5[f"{tag}{k}_sum"] = np.array(t.astype(np.float64).sum())
            g5[f"{tag}{k}_abs"] = np.array(np.abs(t.astype(np.float64)).sum())
    np.savez_compressed(OUT / "g5_model.npz", **g5)

    g6_fixture(model)

    # ------------------------------------------------------------------ G7 (C2 shape)
    pv7 = golden_inputs.pixel_values(7, 1, 480, 640)
    caps.clear()
    with torch.no_grad():
        out = model(pixel_values=torch.from_numpy(pv7))
    g7 = {"input_sha": np.array(sha(pv7)), "ratio": caps["ratio"].numpy(),
          "class_logits": out.class_queries_logits.numpy()}
    ml = out.masks_queries_logits.numpy().ravel()
    idx = golden_inputs.sample_index("g7.mask", ml.size, 1 << 16)
    g7.update(mask_idx=idx, mask_val=ml[idx], mask_sum=np.array(ml.astype(np.float64).sum()),
              mask_abs=np.array(np.abs(ml.astype(np.float64)).sum()), mask_shape=np.array(out.masks_queries_logits.shape))
    for k in range(4):
        t = caps["bb"][k].numpy().ravel()
        idx = golden_inputs.sample_index(f"g7.bb{k}", t.size, 8192)
        g7[f"bb{k}_idx"] = idx
        g7[f"bb{k}_val"] = t[idx]
        g7[f"bb{k}_sum"] = np.array(t.astype(np.float64).sum())
    np.savez_compressed(OUT / "g7_model640.npz", **g7)

    processor_fixture()
    print("golden fixtures written to", OUT)

class RandRecorder(torch.overrides.TorchFunctionMode):
    """Records every torch.rand call of the reference's matcher and loss (the importance-sampled
    points, modeling_mask2former.py:455, :705, :721): shape and sha256 of the values, so the GPU
    test can replay the same draws from a CPU generator with the same seed and prove it did."""

    def __init__(self):
        super().__init__()
        self.calls = []

    def __torch_function__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if func is torch.rand:
            self.calls.append((tuple(out.shape), sha(out.numpy())))
        return out


def record_attn_masks(model, tag, calls, out):
    """The binarised attention mask of every mask-predictor call (one head per image: the heads
    repeat it), bit-packed [B][Q][L], and the interpolated logits within 2e-2 of the threshold."""
    for c, (logits, attn, size) in enumerate(calls):
        B = logits.shape[0]
        nh = attn.shape[0] // B
        a = attn.view(B, nh, *attn.shape[1:])
        assert bool((a == a[:, :1]).all()), "heads differ"
        a0 = a[:, 0].numpy()  # [B, Q, L]
        val = F.interpolate(logits, size=size, mode="bilinear", align_corners=False).flatten(2).numpy()
        assert np.array_equal(a0, val < 0) or np.array_equal(a0, 1 / (1 + np.exp(-val)) < 0.5)
        near = np.flatnonzero(np.abs(val.ravel()) < 2e-2)
        out[f"{tag}_c{c}_shape"] = np.array(a0.shape if B > 1 else a0.shape[1:])
        out[f"{tag}_c{c}_size"] = np.array(size)
        out[f"{tag}_c{c}_bits"] = np.packbits(a0.ravel())
        out[f"{tag}_c{c}_near_idx"] = near.astype(np.int64)
        out[f"{tag}_c{c}_near_val"] = val.ravel()[near].astype(np.float32)
    out[f"{tag}_ncalls"] = np.array(len(calls))


def g6_fixture(model):
    """G6: one loss.backward() of the whole model at 320x240, B=2, eval mode (no dropout, no drop
    path, no layer drop: the only random numbers are the loss's point draws, torch.manual_seed(1234)):
      * the loss and each of its 30 terms (3 per output, final + 9 auxiliary);
      * every torch.rand draw (shape + sha256, RandRecorder) for the GPU test's replay;
      * the ratio (injected on the GPU: it feeds discrete window decisions), the matched indices of
        every matcher call and the attention masks of every mask-predictor call (tag g6);
      * per grad-receiving parameter: norm, sum and sampled values (1 024 for the hot path's
        DSAM / DGGM parameters, 256 for the rest) at golden_inputs.sample_index positions."""
    pv2 = golden_inputs.pixel_values(6, 2, 240, 320)
    labels = golden_inputs.labels(6, 2, 240, 320)
    model.eval()
    model.zero_grad()
    caps, attn_calls, matches, terms = {}, [], [], {}
    plm = model.model.pixel_level_module
    hooks = [plm.ratio_predictor.register_forward_hook(lambda m, i, o: caps.__setitem__("ratio", o.detach().clone())),
             model.model.transformer_module.decoder.mask_predictor.register_forward_hook(
                 lambda m, inp, out: attn_calls.append((out[0].detach().clone(), out[1].detach().clone(), inp[2]))),
             model.criterion.matcher.register_forward_hook(
                 lambda m, inp, out: matches.append([(np.asarray(i), np.asarray(j)) for i, j in out]))]
    get_loss = model.get_loss

    def get_loss_rec(loss_dict):
        terms.update({k: float(v.detach()) for k, v in loss_dict.items()})
        return get_loss(loss_dict)
    model.get_loss = get_loss_rec
    rec = RandRecorder()
    torch.manual_seed(1234)  # the loss samples points with torch.rand (importance sampling)
    try:
        with rec:
            out = model(pixel_values=torch.from_numpy(pv2),
                        mask_labels=[torch.from_numpy(m) for m in labels[0]],
                        class_labels=[torch.from_numpy(c) for c in labels[1]])
    finally:
        for h in hooks:
            h.remove()
        del model.get_loss
    out.loss.backward()
    g6 = {"input_sha": np.array(sha(pv2)), "loss": np.array(out.loss.item()), "ratio": caps["ratio"].numpy(),
          "rand_seed": np.array(1234), "rand_shapes": np.array([str(list(s)) for s, _ in rec.calls]),
          "rand_sha": np.array([h for _, h in rec.calls]),
          "term_names": np.array(sorted(terms)), "term_vals": np.array([terms[k] for k in sorted(terms)])}
    g6["match_calls"] = np.array(len(matches))
    for c, per_img in enumerate(matches):
        for b, (i, j) in enumerate(per_img):
            g6[f"match_{c}_{b}"] = np.stack([i, j]).astype(np.int64)
    record_attn_masks(model, "g6", attn_calls, g6)
    names, hot = [], []
    for n, p in model.named_parameters():
        if p.grad is None:
            if ".dsam" in n or "depth_gradient_injection" in n:
                raise AssertionError(f"{n}: no gradient")
            continue
        if "ratio_predictor" in n or "pixel_level_module.encoder." in n:
            raise AssertionError(f"unexpected grad on {n} (Q1/Q2)")
        names.append(n)
        is_hot = ".dsam" in n or "depth_gradient_injection" in n
        hot.append(is_hot)
        g = p.grad.numpy().ravel()
        idx = golden_inputs.sample_index("g6." + n, g.size, 1024 if is_hot else 256)
        g6[n + "|norm"] = np.array(float(np.linalg.norm(g.astype(np.float64))))
        g6[n + "|sum"] = np.array(float(g.astype(np.float64).sum()))
        g6[n + "|idx"] = idx
        g6[n + "|val"] = g[idx]
    g6["names"] = np.array([n for n, h in zip(names, hot) if h])  # the hot path's (DSAM / DGGM)
    g6["all_names"] = np.array(names)                               # every grad-receiving parameter
    np.savez_compressed(OUT / "g6_grads.npz", **g6)
    model.zero_grad()
    return g6


def reference_processor(h, w):
    """The image processor finetuning.py:72-80 builds from the reference's checkpoint directory
    (do_resize, size = image_height x image_width, do_reduce_labels False, ignore_index 0 as in
    mask2former/config.json).  transformers 5.15's AutoImageProcessor needs torchvision, which is
    absent; the numpy ("PIL") backend is the processor transformers 4.47 — the version the
    reference's checkpoints were written with — instantiates by default."""
    from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
    cfg = json.loads(Path(f"{REF}/mask2former/checkpoints/standard/preprocessor_config.json").read_text())
    for k in ("image_processor_type", "_max_size", "reduce_labels", "num_labels"):
        cfg.pop(k, None)
    cfg.update(do_resize=True, size={"height": h, "width": w}, do_reduce_labels=False, ignore_index=0)
    return Mask2FormerImageProcessorPil(**cfg)


def processor_fixture():
    """G0 (a11): channels 0:6 of pixel_values and the label tensors exactly as
    map_10channel_case2 gets them from the processor (dataloader.py:405-423)."""
    g0 = {}
    # every u8 value in every channel (8 copies each, a different permutation per channel)
    base = np.tile(np.arange(256, dtype=np.uint8), 8).reshape(32, 64)
    rng = np.random.default_rng(11)
    lut_img = np.stack([base, rng.permutation(base.ravel()).reshape(32, 64), base[::-1, ::-1]], axis=-1)
    g0["lut_rgb_u8"] = lut_img
    g0["lut_out"] = reference_processor(32, 64)(images=[lut_img], return_tensors="np")["pixel_values"][0]
    for tag, (H, W) in {"small": (64, 96), "c2": (480, 640)}.items():
        sc = synthetic.make_scene(synthetic.scene_seed(70, 0), H, W)
        inst, inst2sem = golden_inputs.instance_map(sc)
        depth_rgb = np.stack([sc["depth_u8"]] * 3, axis=-1)  # PIL convert('L') -> convert('RGB')
        mi = reference_processor(H, W)(images=[sc["rgb_u8"], depth_rgb], segmentation_maps=[inst, inst],
                                        instance_id_to_semantic_id=inst2sem, return_tensors="np")
        pv6 = mi["pixel_values"].reshape(-1, H, W)                     # dataloader.py:417-418
        masks, classes = np.asarray(mi["mask_labels"][0]), np.asarray(mi["class_labels"][0])
        g0[f"{tag}_pv6_sha"] = np.array(sha(pv6.astype(np.float32)))
        g0[f"{tag}_masks_sha"] = np.array(sha(masks.astype(np.float32)))
        g0[f"{tag}_masks_shape"] = np.array(masks.shape)
        g0[f"{tag}_classes"] = classes.astype(np.int64)
        if tag == "small":
            g0["small_pv6"] = pv6.astype(np.float32)
            g0["small_masks"] = masks.astype(np.float32)
    np.savez_compressed(OUT / "g0_processor.npz", **g0)


def build_model(cm):
    """Reference model on the restated config (rgbd_amd.config), after checking that the
    restatement builds exactly the parameter shapes of the reference's standard config."""
    from rgbd_amd.config import standard_config
    ref_cfg = cm.CustomConfig.from_pretrained(f"{REF}/mask2former/checkpoints/standard",
                                              **golden_inputs.label_kwargs())
    cfg = standard_config(48)
    model = cm.CustomMask2FormerForUniversalSegmentation(cfg, version="0.4.0")
    ref_model = cm.CustomMask2FormerForUniversalSegmentation(ref_cfg, version="0.4.0")
    a = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    b = {k: tuple(v.shape) for k, v in ref_model.state_dict().items()}
    assert a == b, "restated config differs from checkpoints/standard/config.json"
    assert cfg.backbone_config.drop_path_rate == ref_cfg.backbone_config.drop_path_rate
    del ref_model
    winit.init_deterministic(model)
    return model


def attn_mask_fixture(cm):
    """G9: every mask-predictor call of the reference model at G5's (320x240) and G7's (640x480)
    inputs — the attention mask the HF decoder feeds the next layer (sigmoid(interpolated logits)
    < 0.5, modeling_mask2former.py:2048-2055) bit-packed for one head, and the interpolated
    logits within 2e-2 of the threshold (index + value) — so a run can (i) force the reference's
    masks into every decoder layer and measure pure arithmetic error, (ii) count and explain
    flipped bits without the reference on the GPU box."""
    model = build_model(cm).eval()
    calls = []
    mp = model.model.transformer_module.decoder.mask_predictor
    h = mp.register_forward_hook(lambda m, inp, out: calls.append((out[0].detach().clone(), out[1].detach().clone(),
                                                                  inp[2])))
    g9 = {}
    for tag, (cid, H, W) in {"g5": (1, 240, 320), "g7": (7, 480, 640)}.items():
        pv = golden_inputs.pixel_values(cid, 1, H, W)
        calls.clear()
        with torch.no_grad():
            out = model(pixel_values=torch.from_numpy(pv))
        g9[f"{tag}_input_sha"] = np.array(sha(pv))
        g9[f"{tag}_ncalls"] = np.array(len(calls))
        ml = out.masks_queries_logits.numpy()
        g9[f"{tag}_mask_sum"] = np.array(ml.astype(np.float64).sum())
        for c, (logits, attn, size) in enumerate(calls):
            nh = attn.shape[0] // logits.shape[0]
            a = attn.view(logits.shape[0], nh, *attn.shape[1:])
            assert bool((a == a[:, :1]).all()), "heads differ"
            a0 = a[0, 0].numpy()  # [Q, L] (B = 1)
            val = F.interpolate(logits, size=size, mode="bilinear", align_corners=False).flatten(2)[0].numpy()
            assert np.array_equal(a0, val < 0) or np.array_equal(a0, 1 / (1 + np.exp(-val)) < 0.5)
            near = np.flatnonzero(np.abs(val.ravel()) < 2e-2)
            g9[f"{tag}_c{c}_shape"] = np.array(a0.shape)
            g9[f"{tag}_c{c}_size"] = np.array(size)
            g9[f"{tag}_c{c}_bits"] = np.packbits(a0.ravel())
            g9[f"{tag}_c{c}_near_idx"] = near.astype(np.int64)
            g9[f"{tag}_c{c}_near_val"] = val.ravel()[near].astype(np.float32)
    h.remove()
    np.savez_compressed(OUT / "g9_attn_masks.npz", **g9)


def save_g1(rec):
    out = {"names": np.array(rec["names"]), "shapes": np.array(rec["shapes"]),
           "ratios": np.array(rec["ratios"], np.float64), "input_sha": np.array(rec["input_sha"]),
           "grey_sha": np.array(rec["grey_sha"]), "error": np.array(rec["error"])}
    for i in range(len(rec["names"])):
        if rec["error"][i]:
            continue
        out[f"{i}_n_modes"] = np.array(rec["n_modes"][i])
        out[f"{i}_centers"] = rec["centers"][i]
        out[f"{i}_windows"] = rec["windows"][i]
        out[f"{i}_hist"] = rec["hist"][i]
        out[f"{i}_edges"] = rec["edges"][i]
        out[f"{i}_code"] = rec["code"][i]
        for s, pc in enumerate(rec["pooled"][i]):
            out[f"{i}_pooled{s}"] = pc
    np.savez_compressed(OUT / "g1_decompose.npz", **out)


def resize_fixture():
    """G8 (a11, frames NOT at model resolution): the reference's image processor resizing a
    scene to a square size (its PIL BILINEAR for the colour and depth-as-RGB images, NEAREST
    for the instance map, then rescale + normalise + binary masks), as map_10channel_case2 calls
    it (dataloader.py:405-410).  cv2.resize (:414) is absent here and not pinned."""
    g8 = {}
    for tag, (H, W, S) in {"small": (48, 80, 64), "c2": (480, 640, 320)}.items():
        sc = synthetic.make_scene(synthetic.scene_seed(71, 0), H, W)
        inst, inst2sem = golden_inputs.instance_map(sc)
        depth_rgb = np.stack([sc["depth_u8"]] * 3, axis=-1)
        mi = reference_processor(S, S)(images=[sc["rgb_u8"], depth_rgb], segmentation_maps=[inst, inst],
                                        instance_id_to_semantic_id=inst2sem, return_tensors="np")
        pv6 = mi["pixel_values"].reshape(-1, S, S).astype(np.float32)
        masks, classes = np.asarray(mi["mask_labels"][0]).astype(np.float32), np.asarray(mi["class_labels"][0])
        g8[f"{tag}_size"] = np.array([H, W, S])
        g8[f"{tag}_pv6_sha"] = np.array(sha(pv6))
        g8[f"{tag}_masks_sha"] = np.array(sha(masks))
        g8[f"{tag}_masks_shape"] = np.array(masks.shape)
        g8[f"{tag}_classes"] = classes.astype(np.int64)
        if tag == "small":
            g8["small_pv6"] = pv6
            g8["small_masks"] = masks
    np.savez_compressed(OUT / "g8_resize.npz", **g8)


if __name__ == "__main__":
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    import golden_inputs  # noqa: E402
    if len(sys.argv) > 1 and sys.argv[1] == "resize":
        resize_fixture()
    elif len(sys.argv) > 1 and sys.argv[1] == "g6":
        torch.manual_seed(0)
        torch.set_num_threads(8)
        g6_fixture(build_model(import_reference()))
    elif len(sys.argv) > 1 and sys.argv[1] == "attn":
        torch.manual_seed(0)
        torch.set_num_threads(8)
        attn_mask_fixture(import_reference())
    else:
        main()
        resize_fixture()
