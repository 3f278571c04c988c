"""K4 ratio predictor and the whole drop-in model on the GPU against the golden vectors
generated from the reference (G4, G5, G6).  G5's mask logits carry the north-star metric:
max |mask logit - reference| <= 1e-3 in float32 mode."""
import copy
import hashlib

import numpy as np
import pytest
import torch

import golden_inputs as gi
from checkers import ratio_ws
from oracle import ratio as ratio_o
from rgbd_amd import deform_attn, init as winit, mask_predictor, masked_attention

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF16_UNFORCED_REL_TOL = 4.2e-2  # G5 bf16 hot path, own attention masks: 2x the measured 2.11e-2
# G6 (whole-model gradients vs the reference), non-zero-class tensors: the CPU oracle (the reference
# HF stages around the restated hot path) reaches norm 8.8e-5, sample L2 1.3e-3, max 1.4e-2 rms
G6_NORM_REL, G6_SAMPLE_L2, G6_SAMPLE_MAX = 1e-4, 5e-3, 5e-2
PRE = "model.pixel_level_module.ratio_predictor."


def _ratio_module(dtype=torch.float32):
    from rgbd_amd.modules import EnhancedDepthImageRatioPredictor
    m = EnhancedDepthImageRatioPredictor(3)
    winit.init_deterministic(m, prefix=PRE)
    m.compute_dtype = dtype
    return m


def test_ratio_predictor_eval_golden(golden):
    g4 = golden("g4_ratio")
    pv = gi.pixel_values(4, 2, 240, 320)
    assert hashlib.sha256(pv.tobytes()).hexdigest() == str(g4["input_sha"])
    m = _ratio_module().to(DEV).eval()
    r = m(torch.from_numpy(pv).to(DEV)[:, 3:6]).cpu().numpy()
    np.testing.assert_allclose(r, g4["ratio"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("H,W", [(90, 125), (64, 96)])
def test_ratio_predictor_eval_bf16_ragged(H, W):
    """bf16 eval ratio on shapes with partial conv tiles / overlapping pool regions vs the fp32
    CPU module tree (same bf16 tolerance as the golden case)."""
    pv = gi.pixel_values(5, 2, H, W)
    m_cpu = _ratio_module().eval()
    m = copy.deepcopy(m_cpu)
    m.compute_dtype = torch.bfloat16
    m = m.to(DEV).eval()
    r = m(torch.from_numpy(pv).to(DEV)[:, 3:6]).cpu().numpy()
    with torch.no_grad():
        ref = ratio_o.ratio_forward_modules(m_cpu, torch.from_numpy(pv[:, 3:6]))
    np.testing.assert_allclose(r, np.asarray(ref, dtype=np.float32).reshape(r.shape), atol=5e-3)


@pytest.mark.parametrize("B", [1, 11])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ratio_predictor_eval_batch_over_eight(dtype, B):
    """Eval ratio at B = 11 (the fused tail's second, partial group of eight images) and B = 1
    against the fp32 CPU module tree: 1e-5 in fp32, the stated bf16 tolerance in bf16."""
    pv = gi.pixel_values(6, B, 64, 96)
    m_cpu = _ratio_module().eval()
    m = copy.deepcopy(m_cpu)
    m.compute_dtype = dtype
    m = m.to(DEV).eval()
    r = m(torch.from_numpy(pv).to(DEV)[:, 3:6]).cpu().numpy()
    with torch.no_grad():
        ref = np.asarray(ratio_o.ratio_forward_modules(m_cpu, torch.from_numpy(pv[:, 3:6])), dtype=np.float32)
    if dtype == torch.float32:
        np.testing.assert_allclose(r, ref.reshape(r.shape), rtol=1e-5, atol=1e-6)
    else:
        np.testing.assert_allclose(r, ref.reshape(r.shape), atol=5e-3)


def test_ratio_predictor_eval_bf16(golden):
    g4 = golden("g4_ratio")
    pv = gi.pixel_values(4, 2, 240, 320)
    m = _ratio_module(torch.bfloat16).to(DEV).eval()
    r = m(torch.from_numpy(pv).to(DEV)[:, 3:6]).cpu().numpy()
    np.testing.assert_allclose(r, g4["ratio"], atol=5e-3)  # stated bf16 tolerance on the ratio


@pytest.mark.parametrize("H,W,B", [(240, 320, 3), (96, 128, 3), (64, 96, 11), (64, 96, 1)])
def test_ratio_predictor_train_batchnorm(H, W, B):
    """Train mode: batch-statistics BatchNorm; every running stat updated like torch.  B = 11:
    the fused tail conv + BN stages its pooled maps eight images at a time (two groups, the second
    partial)."""
    pv = gi.pixel_values(8, B, H, W)
    m_cpu = _ratio_module().train()
    m = copy.deepcopy(m_cpu).to(DEV).train()
    m(torch.from_numpy(pv).to(DEV)[:, 3:6])
    with torch.no_grad():
        ratio_o.ratio_forward_modules(m_cpu, torch.from_numpy(pv[:, 3:6]))
    got = {k: v.cpu() for k, v in m.state_dict().items()}
    for k, v in m_cpu.state_dict().items():
        if "running" in k:
            np.testing.assert_allclose(got[k].numpy(), v.numpy(), rtol=2e-4, atol=2e-5, err_msg=k)
        if "num_batches_tracked" in k:
            assert int(got[k]) == int(v)


def _full_model(dtype=torch.float32):
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
    winit.init_deterministic(m)
    return m.set_compute_dtype(dtype).to(DEV)


@pytest.mark.parametrize("H,W", [(240, 320), (90, 125)])
def test_bf16_train_mode_batchnorm_stats(H, W):
    """The bf16 chain/conv5 kernels (LDS-resident weights, LDS-DMA conv5) in train mode: running
    stats of all six BN layers within bf16 tolerance of the PyTorch-CPU fp32 module tree.  90x125
    leaves partial 8x32 conv tiles and overlapping adaptive-pool regions."""
    pv = gi.pixel_values(8, 2, H, W)
    m_cpu = _ratio_module().train()
    m = copy.deepcopy(m_cpu)
    m.compute_dtype = torch.bfloat16
    m = m.to(DEV).train()
    r = m(torch.from_numpy(pv).to(DEV)[:, 3:6])
    assert torch.isfinite(r).all() and float(r.min()) >= 0.01 and float(r.max()) <= 0.5
    with torch.no_grad():
        ratio_o.ratio_forward_modules(m_cpu, torch.from_numpy(pv[:, 3:6]))
    got = {k: v.cpu() for k, v in m.state_dict().items()}
    for k, v in m_cpu.state_dict().items():
        if "running_mean" in k:
            d = (got[k] - v).abs().max().item()
            assert d <= 2e-2 * max(1.0, v.abs().max().item()), (k, d)
        if "running_var" in k:
            rel = ((got[k] - v).abs() / v.abs().clamp_min(1e-6)).max().item()
            assert rel <= 5e-2, (k, rel)


@pytest.mark.parametrize("H,W", [(240, 320), (90, 125), (480, 640), (7, 9), (90, 129), (66, 130), (40, 65)])
def test_bf16_stem_bn_batch_stats_exact(H, W):
    """The stem BatchNorms' batch statistics in bf16 train mode come from the moments of the 7x7x3
    depth windows (k_stem_lag with its border workgroups / k_stem_sums / k_stem_s2 / k_stem_bn: lag correlations + border
    corrections, double), not from a pass over the stem — against float64 arithmetic on the same
    bf16-rounded depth and stem weights: batch mean to 2e-6 of the channel scale, unbiased
    variance to 2e-5 relative (read back from the running-stat update, momentum 0.1).  (7, 9):
    below the moments path's minimum size, the former statistics pass.  (90, 129), (66, 130),
    (40, 65): W % 64 in {1, 2}, where the last 64-column border chunk holds fewer than three
    columns and the right corner cells come from the chunk holding column W - 3."""
    import torch.nn.functional as F
    pv = gi.pixel_values(8, 2, H, W)[:, 3:6]
    m = _ratio_module()
    m.compute_dtype = torch.bfloat16
    m = m.to(DEV).train()
    mods = dict(m.named_modules())
    bns = [mods[f"scale{i}_conv.1"] for i in (1, 2, 3)]
    for bn in bns:
        bn.running_mean.zero_()
        bn.running_var.fill_(1.0)
    m(torch.from_numpy(pv).to(DEV))
    torch.cuda.synchronize()
    x = torch.from_numpy(pv).to(torch.bfloat16).double()
    for i, bn in enumerate(bns):
        conv = mods[f"scale{i + 1}_conv.0"]
        w = conv.weight.detach().cpu().to(torch.bfloat16).double()
        y = F.conv2d(x, w, conv.bias.detach().cpu().double(), padding=conv.padding)
        mean = y.mean((0, 2, 3))
        var = y.var((0, 2, 3), unbiased=True)
        got_mean = bn.running_mean.detach().cpu().double() / 0.1
        got_var = (bn.running_var.detach().cpu().double() - 0.9) / 0.1
        scale = float(y.abs().max())
        dm = float((got_mean - mean).abs().max())
        dv = float(((got_var - var).abs() / var.abs().clamp_min(1e-12)).max())
        print(f"stem BN {i}: mean err {dm:.3g} (scale {scale:.3g}), var rel err {dv:.3g}")
        assert dm <= 2e-6 * max(scale, 1.0), (i, dm)
        assert dv <= 2e-5, (i, dv)


@pytest.mark.parametrize("H,W", [(64, 96), (90, 125), (240, 320)])
@pytest.mark.parametrize("path", ["gate", "phase2"])
def test_bf16_train_mode_gated_features(H, W, path):
    """The train-mode gated features (fused * attention(fused), custom_model.py:1469-1470, the
    conv5 input) read from the ratio workspace, against the PyTorch-CPU fp32 module tree in
    train mode, for both bf16 routes: k_rp_gate over phase 1's stored raw fusion output (the
    default) and phase 2's stem + fusion recompute (RGBD_RATIO_F_PHASE2).  Aligned (64x96,
    240x320) and ragged (90x125) shapes.  Tolerance on the features themselves: bf16 operands
    and a bf16-stored fusion output against f32 — max |diff| <= 3e-2 of max |ref|, mean |diff|
    <= 1e-2 of mean |ref| (a fragment-order slip moves whole channel/pixel blocks and fails
    both by orders of magnitude)."""
    from rgbd_amd import _lib, ops
    B = 2
    pv = gi.pixel_values(12, B, H, W)
    m_cpu = _ratio_module().train()
    m = copy.deepcopy(m_cpu)
    m.compute_dtype = torch.bfloat16
    m.train_route = path
    m = m.to(DEV).train()
    x = torch.from_numpy(pv).to(DEV)[:, 3:6]
    m(x)
    torch.cuda.synchronize()
    L = _lib.lib()
    ws = ops._workspace(x.device, L.rgbd_ratio_workspace_size(1, B, H, W), "ratio")
    off = L.rgbd_ratio_features_offset(1, B, H, W)
    got = ratio_ws.ratio_features_bf16(ws, off, B, H, W).float().cpu()
    ref = {}
    m_cpu.feature_extractor.register_forward_pre_hook(lambda mod, a: ref.__setitem__("x", a[0].detach().clone()))
    with torch.no_grad():
        ratio_o.ratio_forward_modules(m_cpu, torch.from_numpy(pv[:, 3:6]))
    e = ref["x"]
    d = (got - e).abs()
    assert float(d.max()) <= 3e-2 * float(e.abs().max()), (path, float(d.max()), float(e.abs().max()))
    assert float(d.mean()) <= 1e-2 * float(e.abs().mean()), (path, float(d.mean()), float(e.abs().mean()))


def test_full_model_mask_logits_fp32(golden):
    """North-star parity: mask-logit max-abs-err vs the reference CPU path <= 1e-3 (fp32 mode), at
    G5 (320x240).

    Two effects outside the hot path's arithmetic are separated out:
    * the ratio feeds discrete window decisions, and a 1e-7 relative difference between our and
      torch-CPU's float32 ratio can move a pixel whose grey depth sits within that distance of a
      window bound (SURVEY §7 hard part (v)): the ratio is checked on its own (rtol 1e-5) and the
      reference ratio is injected for the logits;
    * the HF masked-attention decoder binarises sigmoid(mask) < 0.5 between layers: a logit
      within float noise of 0 flips its attention bit and moves later logits by ~1e-3.  So the
      1e-3 bound is asserted on runs with the REFERENCE's attention masks forced into every
      decoder layer (tests/golden/g9_attn_masks.npz, made by importing the reference; pinned to
      the oracle by test_oracle_attention_masks_match_g9): pure arithmetic, no binarisation —
      (i) the reference HF stages on the CPU fed with the GPU hot-path features, (ii) everything
      on the GPU.  Flips are counted separately: a flipped bit is explained only when the
      reference logit lies within bench.FLIP_EXPLAIN_FACTOR (4) x the call's measured
      pre-binarisation |delta logit| (the forced run's, at the fixture's near-threshold
      positions) — in the forced run at every call, in the unforced run at its first flipped
      call (later calls inherit that flip's consequences)."""
    import bench
    g5 = golden("g5_model")
    refm = bench.ReferenceMasks("g5")
    m = _full_model().eval()
    pv_cpu = torch.from_numpy(gi.pixel_values(1, 1, 240, 320))
    assert hashlib.sha256(pv_cpu.numpy().tobytes()).hexdigest() == refm.input_sha == str(g5["input_sha"])
    pv = pv_cpu.to(DEV)
    plm = m.model.pixel_level_module
    with torch.no_grad():
        r = plm.ratio_predictor(pv[:, 3:6])
    np.testing.assert_allclose(r.cpu().numpy(), g5["ratio"], rtol=1e-5)
    ref_ratio = torch.from_numpy(g5["ratio"]).to(DEV)
    caps = {}
    h1 = plm.ratio_predictor.register_forward_hook(lambda mod, inp, out: ref_ratio.clone())
    h2 = plm.decoder.register_forward_pre_hook(lambda mod, a: caps.__setitem__("bb", [t.detach().cpu() for t in a[0]]))
    runs = {}
    try:
        for force in (False, True):
            rec = []
            h = refm.attach(m, force, rec)
            try:
                with torch.no_grad():
                    runs[force] = (m(pixel_values=pv), rec)
            finally:
                h.remove()
    finally:
        h1.remove()
        h2.remove()
    # (i) the reference HF stages on the CPU, fed with the GPU hot-path features, masks forced
    mc = _full_model().cpu().eval()
    assert mask_predictor.uninstall(mc) == 1  # the reference HF modules are the CPU checker
    assert deform_attn.uninstall(mc) == 6
    assert masked_attention.uninstall(mc) == 9
    mc.model.pixel_level_module.hot_path_features = lambda pv_, colors, ratios=None, **kw: caps["bb"]
    calls, rec_c = [], []
    h3 = mc.model.transformer_module.decoder.mask_predictor.register_forward_hook(
        lambda mod, inp, out: calls.append((inp, out)))  # before the forcing hook: the predictor's own outputs
    h5 = refm.attach(mc, True, rec_c)
    try:
        with torch.no_grad():
            out = mc(pixel_values=pv_cpu)
    finally:
        h3.remove()
        h5.remove()
    # f1 pinned on the reference's own calls: each of the 10 mask-predictor calls of the CPU run,
    # replayed through the HIP predictor on the GPU with the same inputs
    hip_pred = m.model.transformer_module.decoder.mask_predictor
    assert isinstance(hip_pred, mask_predictor.HipMaskPredictor) and len(calls) == 10
    worst = 0.0
    for (outputs, pix_emb, size), (mask_ref, attn_ref) in calls:
        with torch.no_grad():
            mask_h, attn_h = hip_pred(outputs.to(DEV), pix_emb.to(DEV), size)
        worst = max(worst, float((mask_h.cpu() - mask_ref).abs().max()))
        val = torch.nn.functional.interpolate(mask_ref, size=size, mode="bilinear", align_corners=False).flatten(2)
        near = (val.abs() < 1e-4).unsqueeze(1).expand(-1, hip_pred.num_heads, -1, -1).flatten(0, 1)
        assert not bool(((attn_h.cpu() != attn_ref) & ~near).any())
    print(f"f1 mask predictor (HIP vs reference CPU calls): max-abs-err {worst:.3g}")
    assert worst <= 1e-4
    ref = g5["mask_logits"]
    hot = float(np.abs(out.masks_queries_logits.numpy() - ref).max())
    gpu_forced = float(np.abs(runs[True][0].masks_queries_logits.cpu().numpy() - ref).max())
    gpu = float(np.abs(runs[False][0].masks_queries_logits.cpu().numpy() - ref).max())
    forced = refm.flips(runs[True][1])
    first = refm.flips(runs[False][1], deltas=forced["deltas"], upto_first=True)
    unforced = refm.flips(runs[False][1], deltas=forced["deltas"])
    print(f"mask-logit max-abs-err (fp32, reference masks forced): hot path {hot:.3g}, everything on the GPU "
          f"{gpu_forced:.3g}; unforced {gpu:.3g} with {unforced['flips']} flipped attention bits (first at call "
          f"{first['first_call']}: {first['flips']} bits, {first['unexplained']} unexplained); forced run: "
          f"{forced['flips']} own-mask flips, max near-threshold |delta logit| {forced['max_delta_logit']:.3g}")
    assert hot <= 1e-3
    assert gpu_forced <= 1e-3
    np.testing.assert_allclose(out.class_queries_logits.numpy(), g5["class_logits"], atol=1e-3)
    np.testing.assert_allclose(runs[True][0].class_queries_logits.cpu().numpy(), g5["class_logits"], atol=1e-3)
    assert forced["unexplained"] == 0, "a bit of the model's own mask flipped away from the threshold"
    assert first["unexplained"] == 0, "the unforced run's first flipped call has a flip beyond the arithmetic"
    assert forced["max_delta_logit"] <= 1e-4
    # the unforced run IS the forced one when no bit flips; otherwise its extra error is the flips'
    assert gpu <= 1e-3 if unforced["flips"] == 0 else gpu <= 1e-2


def test_full_model_mask_logits_bf16(golden):
    """bf16 hot path (ratio predictor, DSAM, DGGM) in the float32 HF model at G5: with the
    reference's attention masks forced (G9; arithmetic only) the max relative logit error is
    within the bench line's bound (parity.bf16.tolerance_rel); the unforced run's extra error
    comes from attention bits flipped at its first flipped call within the arithmetic's reach."""
    import bench
    g5 = golden("g5_model")
    refm = bench.ReferenceMasks("g5")
    m = _full_model(torch.bfloat16).eval()
    pv = torch.from_numpy(gi.pixel_values(1, 1, 240, 320)).to(DEV)
    ref = g5["mask_logits"]
    runs = {}
    for force in (True, False):
        rec = []
        h = refm.attach(m, force, rec)
        try:
            with torch.no_grad():
                out = m(pixel_values=pv)
        finally:
            h.remove()
        runs[force] = (float(np.abs(out.masks_queries_logits.float().cpu().numpy() - ref).max() / np.abs(ref).max()),
                       rec)
    forced = refm.flips(runs[True][1])
    first = refm.flips(runs[False][1], deltas=forced["deltas"], upto_first=True)
    print(f"mask-logit max-rel-err (bf16 hot path): reference masks forced {runs[True][0]:.3g}, unforced "
          f"{runs[False][0]:.3g} (first flipped call {first['first_call']}: {first['flips']} bits, "
          f"{first['unexplained']} unexplained)")
    assert runs[True][0] < bench.BF16_LOGIT_REL_TOL  # the bench line's bound (parity.bf16.tolerance_rel)
    assert first["unexplained"] == 0
    # measured 2.11e-2 (7 flipped bits at the first flipped call, all explained): 2x headroom
    assert runs[False][0] < BF16_UNFORCED_REL_TOL


def _g6_run(m, g6, refm, force, pv, masks, classes):
    """One G6 training forward + backward of the fp32 drop-in model on the GPU with the
    reference's torch.rand draws replayed (tests/checkers/rand_replay.py) and, with ``force``,
    the reference's attention masks forced into every decoder layer (bench.ReferenceMasks "g6")."""
    from checkers.rand_replay import CpuRandReplay
    terms, matches, rec = {}, [], []
    get_loss = m.get_loss

    def get_loss_rec(loss_dict):
        terms.update({k: float(v.detach()) for k, v in loss_dict.items()})
        return get_loss(loss_dict)
    m.get_loss = get_loss_rec
    hm = m.criterion.matcher.register_forward_hook(
        lambda mod, inp, out: matches.append([(i.cpu().numpy(), j.cpu().numpy()) for i, j in out]))
    h = refm.attach(m, force, rec)
    m.zero_grad(set_to_none=True)
    rr = CpuRandReplay(int(g6["rand_seed"]))
    try:
        with rr:
            out = m(pixel_values=pv, mask_labels=[torch.from_numpy(x).to(DEV) for x in masks],
                    class_labels=[torch.from_numpy(c).to(DEV) for c in classes])
    finally:
        h.remove()
        hm.remove()
        del m.get_loss
    rr.check(g6)
    out.loss.backward()
    grads = {n: p.grad.detach().double().cpu().numpy().ravel() for n, p in m.named_parameters() if p.grad is not None}
    return float(out.loss), terms, matches, grads, rec


def test_full_model_grads_fp32(golden):
    """The whole drop-in model's training step pinned to the reference's (G6: one loss.backward()
    of the reference model at 320x240, B=2, eval mode, made by importing the reference:
    make_golden.py g6), everything on the GPU in float32.

    The reference's loss draws its sample points with torch.rand on the CPU generator; they are
    replayed here (checkers/rand_replay.py, checked call by call against the fixture's sha256).
    The ratio is compared (rtol 1e-5) and the reference's injected, as in the G5 test (a 1e-7
    ratio difference can move a pixel across a window bound).  Two runs:
    * reference attention masks forced into every decoder layer (arithmetic only): the loss
      (rtol 1e-5) and each of its 30 terms (rtol 2e-5), every matcher call's assignment
      (identical), and for EVERY grad-receiving parameter (363 tensors, 37.3 M values;
      checkers/g6_compare.py) the gradient norm (rtol G6_NORM_REL) and the fixture's sampled
      values (1 024 per DSAM / DGGM tensor, 256 per other tensor): relative L2 error
      <= G6_SAMPLE_L2, every sample within G6_SAMPLE_MAX x the tensor's rms; the nine decoder
      self-attention key biases, whose gradient is zero in exact arithmetic (the reference's is
      1e-10 of the largest rms), as negligible as the reference's;
    * the model's own masks: the same bounds when no attention bit flips; flipped bits must be
      explained by the arithmetic (bench.ReferenceMasks.flips) and the loss stays within 1e-3.
    Q1/Q2: the Swin encoder and the ratio predictor receive no gradient."""
    import bench
    g6 = golden("g6_grads")
    refm = bench.ReferenceMasks("g6")
    m = _full_model().eval()
    pv_np = gi.pixel_values(6, 2, 240, 320)
    assert hashlib.sha256(pv_np.tobytes()).hexdigest() == str(g6["input_sha"])
    pv = torch.from_numpy(pv_np).to(DEV)
    masks, classes = gi.labels(6, 2, 240, 320)
    plm = m.model.pixel_level_module
    with torch.no_grad():
        r = plm.ratio_predictor(pv[:, 3:6])
    np.testing.assert_allclose(r.cpu().numpy(), g6["ratio"], rtol=1e-5)
    ref_ratio = torch.from_numpy(g6["ratio"]).to(DEV)
    h1 = plm.ratio_predictor.register_forward_hook(lambda mod, inp, out: ref_ratio.clone())
    try:
        runs = {force: _g6_run(m, g6, refm, force, pv, masks, classes) for force in (True, False)}
    finally:
        h1.remove()
    names = [str(n) for n in g6["all_names"]]
    term_ref = dict(zip([str(k) for k in g6["term_names"]], [float(v) for v in g6["term_vals"]]))

    def compare(run):
        from checkers.g6_compare import compare_grads
        loss, terms, matches, grads, _ = run
        assert sorted(terms) == sorted(term_ref)
        assert sorted(grads) == sorted(names), set(grads) ^ set(names)
        rep = compare_grads(grads, g6)
        rep.update(loss_rel=abs(loss - float(g6["loss"])) / abs(float(g6["loss"])),
                   term_rel=max(abs(terms[k] - v) / max(abs(v), 1e-12) for k, v in term_ref.items()),
                   matches_equal=len(matches) == int(g6["match_calls"]) and all(
                       np.array_equal(np.stack([i, j]), g6[f"match_{c}_{b}"])
                       for c, per in enumerate(matches) for b, (i, j) in enumerate(per)))
        del rep["zero_class"]
        return rep

    def within(rep):
        from checkers.g6_compare import ZERO_FLOOR
        return (rep["loss_rel"] <= 1e-5 and rep["term_rel"] <= 2e-5 and rep["norm_rel"][0] <= G6_NORM_REL
                and rep["sample_l2"][0] <= G6_SAMPLE_L2 and rep["sample_max_over_rms"][0] <= G6_SAMPLE_MAX
                and rep["zero_class_worst"] <= ZERO_FLOOR)
    forced, own = compare(runs[True]), compare(runs[False])
    fl = refm.flips(runs[True][4])
    fl_own = refm.flips(runs[False][4], deltas=fl["deltas"])
    first = refm.flips(runs[False][4], deltas=fl["deltas"], upto_first=True)
    print(f"G6 forced masks: {forced}")
    print(f"G6 own masks: {own}; own-mask flips {fl_own['flips']} (first call {first['first_call']}, "
          f"{first['unexplained']} unexplained)")
    assert forced["matches_equal"]
    assert within(forced), forced
    assert fl["unexplained"] == 0 and first["unexplained"] == 0
    if fl_own["flips"] == 0:
        assert own["matches_equal"] and within(own), own
    else:
        assert own["loss_rel"] <= 1e-3, own
    for n, p in m.named_parameters():
        if "ratio_predictor" in n or "pixel_level_module.encoder." in n:
            assert p.grad is None, f"{n} must not receive gradients (Q1/Q2)"
