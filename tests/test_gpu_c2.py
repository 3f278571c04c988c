"""The C2 / bench configuration (640x480) pinned on the GPU:

* K1's channels 0:6 against the reference's image processor (g0_processor.npz, made from
  Mask2FormerImageProcessor by tests/golden/make_golden.py): bit-exact, every u8 value;
* the full drop-in model at 640x480 in float32 against the reference CPU run G7: mask-logit
  max-abs-err <= 1e-3 (BASELINE.json's metric at the configuration it names);
* the bench's exact training step (640x480, B=8, bf16, ratio predictor in train mode) against
  the oracle: the 4 backbone features, every DSAM / DGGM parameter gradient and the ratio
  predictor's BatchNorm running statistics at the stated bf16 tolerances;
* the reference's error convention at the module boundary: a degenerate depth histogram raises
  ValueError (numpy inside DSAModule._calculate_depth_histogram, custom_model.py:715-717)."""
import copy
import hashlib
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

import golden_inputs as gi
from oracle import dggm_pre, hot_path as hot_o, ratio as ratio_o
from rgbd_amd import init as winit, synthetic

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
REPO = Path(__file__).resolve().parents[1]
BF16_REL = 3e-2


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_assemble_matches_image_processor(golden):
    from rgbd_amd import ops
    g0 = golden("g0_processor")
    img = g0["lut_rgb_u8"]                                  # every u8 value in each channel
    depth = np.ascontiguousarray(img[..., 1])
    pv = ops.assemble_pixel_values(torch.from_numpy(depth[None]).to(DEV),
                                   torch.from_numpy(img[None]).contiguous().to(DEV)).cpu().numpy()[0]
    np.testing.assert_array_equal(_bits(pv[0:3]), _bits(g0["lut_out"]))
    for c in range(3):  # depth-as-RGB: the processor's value of channel c for the depth byte
        exp = synthetic.normalize_u8(np.stack([depth] * 3))[c]
        np.testing.assert_array_equal(_bits(pv[3 + c]), _bits(exp))
    lut = {}
    for c in range(3):
        for v, o in zip(img[..., c].ravel(), g0["lut_out"][c].ravel()):
            lut[(c, int(v))] = o
    for c in range(3):
        got = pv[3 + c].ravel()
        np.testing.assert_array_equal(_bits(got), _bits(np.array([lut[(c, int(v))] for v in depth.ravel()])))
    for tag, (H, W) in {"small": (64, 96), "c2": (480, 640)}.items():
        sc = synthetic.make_scene(synthetic.scene_seed(70, 0), H, W)
        pv = ops.assemble_pixel_values(torch.from_numpy(sc["depth_u8"][None]).to(DEV),
                                       torch.from_numpy(sc["rgb_u8"][None]).contiguous().to(DEV)).cpu().numpy()[0]
        assert hashlib.sha256(np.ascontiguousarray(pv[0:6]).tobytes()).hexdigest() == str(g0[f"{tag}_pv6_sha"]), tag


def _full_model(dtype=torch.float32):
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
    winit.init_deterministic(m)
    return m.set_compute_dtype(dtype).to(DEV)


def test_full_model_mask_logits_640x480_fp32(golden):
    """BASELINE.json: mask logits within 1e-3 of the reference at 640x480.  The input is
    assembled on the GPU (K1) from the scene's u8 planes — its sha256 equals the fixture's."""
    from rgbd_amd import ops
    g7 = golden("g7_model640")
    sc = synthetic.make_scene(synthetic.scene_seed(7, 0), 480, 640)
    pv = ops.assemble_pixel_values(torch.from_numpy(sc["depth_u8"][None]).to(DEV),
                                   torch.from_numpy(sc["rgb_u8"][None]).contiguous().to(DEV))
    assert hashlib.sha256(pv.cpu().numpy().tobytes()).hexdigest() == str(g7["input_sha"])
    m = _full_model().eval()
    plm = m.model.pixel_level_module
    with torch.no_grad():
        r = plm.ratio_predictor(pv[:, 3:6])
    np.testing.assert_allclose(r.cpu().numpy(), g7["ratio"], rtol=1e-5)
    with torch.no_grad():
        out_e2e = m(pixel_values=pv)
    ref_ratio = torch.from_numpy(g7["ratio"]).to(DEV)
    h = plm.ratio_predictor.register_forward_hook(lambda mod, inp, out: ref_ratio.clone())
    try:
        with torch.no_grad():
            out = m(pixel_values=pv)
    finally:
        h.remove()
    idx = g7["mask_idx"]
    assert tuple(out.masks_queries_logits.shape) == tuple(g7["mask_shape"])
    err = float(np.abs(out.masks_queries_logits.cpu().numpy().ravel()[idx] - g7["mask_val"]).max())
    e2e = float(np.abs(out_e2e.masks_queries_logits.cpu().numpy().ravel()[idx] - g7["mask_val"]).max())
    print(f"640x480 mask-logit max-abs-err (fp32): reference ratio injected {err:.3g}, end to end {e2e:.3g}")
    assert err <= 1e-3
    assert e2e <= 1e-3
    np.testing.assert_allclose(out.class_queries_logits.cpu().numpy(), g7["class_logits"], atol=1e-3)


def test_bench_train_step_640x480_b8_vs_oracle():
    """bench.py's timed step, as timed (K1 -> ratio predictor train mode -> K3 -> K5 x3 -> K2, then
    the backward), against the oracle on the same inputs.  The ratio comes out of the train-mode
    predictor with dropout (stochastic, Q15), so the oracle is fed the GPU's ratio; the predictor
    itself is checked through its BatchNorm running statistics (batch statistics of the 8 images)."""
    sys.path.insert(0, str(REPO))
    import bench
    torch.set_num_threads(16)
    args = bench.parse([])
    assert (args.batch, args.height, args.width, args.dtype) == (8, 480, 640, "bf16")
    ctx = bench.build(args, DEV)
    rp_cpu = copy.deepcopy(ctx["rp"]).cpu().train()
    cap = {}
    ctx["rp"].register_forward_hook(lambda mod, inp, out: cap.update(pv=inp[0].detach().clone(), ratio=out.detach().clone()))
    fb, _, _, _ = bench.make_parts(ctx, 1)
    feats = fb()
    torch.cuda.synchronize()
    # K1 in the step: bit-exact planes
    B = args.batch
    pv = np.stack([np.concatenate([synthetic.rgbd_planes(s), dggm_pre.dggm_planes(s["depth_u8"])])
                   for s in ctx["scenes"]])
    np.testing.assert_array_equal(_bits(cap["pv"].cpu().numpy()), _bits(pv[:, 3:6]))
    # ratio predictor, train mode: running statistics after the step's forward
    with torch.no_grad():
        ratio_o.ratio_forward_modules(rp_cpu, torch.from_numpy(pv[:, 3:6]))
    got = {k: v.cpu() for k, v in ctx["rp"].state_dict().items()}
    for k, v in rp_cpu.state_dict().items():
        if "running_mean" in k:
            d = (got[k] - v).abs().max().item()
            assert d <= 2e-2 * max(1.0, v.abs().max().item()), (k, d)
        if "running_var" in k:
            rel = ((got[k] - v).abs() / v.abs().clamp_min(1e-6)).max().item()
            assert rel <= 5e-2, (k, rel)
        if "num_batches_tracked" in k:
            assert int(got[k]) == int(v)
    ratio = cap["ratio"].cpu()
    assert ratio.shape == (B, 1) and bool(((ratio >= 0.01) & (ratio <= 0.5)).all())
    # hot path forward + backward vs the oracle fed the same ratio
    sd = {}
    for k, m in enumerate(ctx["dsams"]):
        for kk, v in m.state_dict().items():
            sd[f"dsam{k}.{kk}"] = v.detach().float().cpu().clone().requires_grad_(True)
    for kk, v in ctx["dg"].state_dict().items():
        sd[f"depth_gradient_injection.{kk}"] = v.detach().float().cpu().clone().requires_grad_(True)
    colors = [c.float().cpu() for c in ctx["colors"]]
    ref, _, decs = hot_o.hot_path_forward(colors, torch.from_numpy(pv), sd, ratios=ratio)
    torch.autograd.backward(ref, [g.float().cpu() for g in ctx["gouts"]])
    for k in range(4):
        a, e = feats[k].detach().float().cpu().numpy(), ref[k].detach().numpy()
        rel = np.abs(a - e).max() / np.abs(e).max()
        assert rel < BF16_REL, f"feature {k}: {rel}"
    named = {}
    for k, m in enumerate(ctx["dsams"]):
        for n, p in m.named_parameters():
            named[f"dsam{k}.{n}"] = p
    for n, p in ctx["dg"].named_parameters():
        named[f"depth_gradient_injection.{n}"] = p
    assert len(named) == 35
    for n, p in named.items():
        a, e = p.grad.float().cpu().numpy(), sd[n].grad.numpy()
        scale = max(float(np.abs(e).max()), 1e-6)
        err = np.abs(a - e).max() / scale
        mean_err = np.abs(a - e).mean() / max(float(np.abs(e).mean()), 1e-12)
        assert err < BF16_REL and mean_err < 1e-2, f"{n}: max rel {err:.3g}, mean rel {mean_err:.3g}"
    assert all(d["n_masks"] >= 1 for d in decs)


@pytest.mark.parametrize("case", ["all_nan", "tiny_range"])
def test_degenerate_depth_raises_value_error(case):
    """The drop-in model's forward raises the reference's ValueError (not a silent zero-mask
    decomposition) when the depth histogram range is non-finite or too narrow for 512 bins."""
    m = _full_model().eval()
    pv = torch.from_numpy(gi.pixel_values(1, 1, 64, 96)).to(DEV)
    if case == "all_nan":
        pv[:, 3:6] = float("nan")
    else:
        pv[:, 3:6] = 1.0
        pv[:, 3:6, 0, 0] = float(np.nextafter(np.float32(1.0), np.float32(2.0)))
    with torch.no_grad(), pytest.raises(ValueError):
        m(pixel_values=pv)
    torch.cuda.synchronize()


def test_instance_labels_match_image_processor(golden):
    """a11 labels on the device (rgbd_amd.data.instance_labels) against the processor's own
    mask_labels / class_labels (g0_processor.npz), plus a batch with an all-background map."""
    from oracle import labels as labels_o
    from rgbd_amd import data
    g0 = golden("g0_processor")
    for tag, (H, W) in {"small": (64, 96), "c2": (480, 640)}.items():
        sc = synthetic.make_scene(synthetic.scene_seed(70, 0), H, W)
        inst, table = gi.instance_map(sc)
        masks, classes = data.instance_labels(torch.from_numpy(inst[None]).to(DEV), [table])
        m = masks[0].cpu().numpy()
        assert tuple(m.shape) == tuple(g0[f"{tag}_masks_shape"])
        assert hashlib.sha256(np.ascontiguousarray(m).tobytes()).hexdigest() == str(g0[f"{tag}_masks_sha"]), tag
        np.testing.assert_array_equal(classes[0].cpu().numpy(), g0[f"{tag}_classes"])
    scenes = [synthetic.make_scene(synthetic.scene_seed(71, i), 48, 80) for i in range(3)]
    maps, tables = zip(*[gi.instance_map(s) for s in scenes])
    maps = np.stack(maps)
    maps[1] = 0                                            # background only -> no instance
    out = data.map_10channel(torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).to(DEV),
                             torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(DEV),
                             torch.from_numpy(maps).to(DEV), list(tables))
    for b in range(3):
        em, ec = labels_o.instance_labels(maps[b], tables[b], ignore_index=0)
        np.testing.assert_array_equal(out["mask_labels"][b].cpu().numpy(), em)
        np.testing.assert_array_equal(out["class_labels"][b].cpu().numpy(), ec)
    assert out["mask_labels"][1].shape[0] == 0
    batch = data.collate_fn_v2([{k: (v[b] if k == "pixel_values" else v[b]) for k, v in out.items()}
                                for b in range(3)])
    assert tuple(batch["pixel_values"].shape) == (3, 10, 48, 80) and len(batch["mask_labels"]) == 3
