"""K4 ratio predictor and the whole drop-in model on the GPU against the golden vectors
generated from the reference (G4, G5, G6).  G5's mask logits carry the north-star metric:
max |mask logit - reference| <= 1e-3 in float32 mode."""
import copy
import hashlib

import numpy as np
import pytest
import torch

import golden_inputs as gi
from oracle import ratio as ratio_o
from rgbd_amd import init as winit

pytestmark = pytest.mark.gpu
DEV = "cuda"
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


def test_ratio_predictor_eval_bf16(golden):
    g4 = golden("g4_ratio")
    pv = gi.pixel_values(4, 2, 240, 320)
    m = _ratio_module(torch.bfloat16).to(DEV).eval()
    r = m(torch.from_numpy(pv).to(DEV)[:, 3:6]).cpu().numpy()
    np.testing.assert_allclose(r, g4["ratio"], atol=5e-3)  # stated bf16 tolerance on the ratio


@pytest.mark.parametrize("H,W", [(240, 320), (96, 128)])
def test_ratio_predictor_train_batchnorm(H, W):
    """Train mode: batch-statistics BatchNorm; every running stat updated like torch."""
    pv = gi.pixel_values(8, 3, H, W)
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


def test_full_model_mask_logits_fp32(golden):
    """North-star parity: mask-logit max-abs-err vs the reference CPU path <= 1e-3 (fp32 mode).

    The ratio feeds discrete window decisions: a 1e-7 relative difference between our and
    torch-CPU's float32 ratio can move a pixel whose grey depth sits within that distance of
    a window bound to the other region.  So (SURVEY §7 hard part (v)) the ratio is checked on
    its own (rtol 1e-5) and the logits are checked with the reference's ratio injected; the
    un-injected end-to-end error is asserted at the looser 1e-2."""
    g5 = golden("g5_model")
    m = _full_model().eval()
    pv = torch.from_numpy(gi.pixel_values(1, 1, 240, 320)).to(DEV)
    plm = m.model.pixel_level_module
    with torch.no_grad():
        r = plm.ratio_predictor(pv[:, 3:6])
        out_free = m(pixel_values=pv)
    np.testing.assert_allclose(r.cpu().numpy(), g5["ratio"], rtol=1e-5)
    ref_ratio = torch.from_numpy(g5["ratio"]).to(DEV)
    h = plm.ratio_predictor.register_forward_hook(lambda mod, inp, out: ref_ratio.clone())
    try:
        with torch.no_grad():
            out = m(pixel_values=pv)
    finally:
        h.remove()
    err = float(np.abs(out.masks_queries_logits.cpu().numpy() - g5["mask_logits"]).max())
    free = float(np.abs(out_free.masks_queries_logits.cpu().numpy() - g5["mask_logits"]).max())
    print(f"mask-logit max-abs-err (fp32): {err:.3g} with the reference ratio, {free:.3g} end-to-end")
    assert err <= 1e-3
    assert free <= 1e-2
    np.testing.assert_allclose(out.class_queries_logits.cpu().numpy(), g5["class_logits"], atol=1e-3)


def test_full_model_mask_logits_bf16(golden):
    g5 = golden("g5_model")
    m = _full_model(torch.bfloat16).eval()
    pv = torch.from_numpy(gi.pixel_values(1, 1, 240, 320)).to(DEV)
    with torch.no_grad():
        out = m(pixel_values=pv)
    ref = g5["mask_logits"]
    rel = float(np.abs(out.masks_queries_logits.cpu().numpy() - ref).max() / np.abs(ref).max())
    print(f"mask-logit max-rel-err (bf16 hot path) = {rel:.3g}")
    assert rel < 5e-2


def test_full_model_grads_fp32(golden):
    g6 = golden("g6_grads")
    m = _full_model().eval()
    pv = torch.from_numpy(gi.pixel_values(6, 2, 240, 320)).to(DEV)
    masks, classes = gi.labels(6, 2, 240, 320)
    torch.manual_seed(1234)
    out = m(pixel_values=pv, mask_labels=[torch.from_numpy(x).to(DEV) for x in masks],
            class_labels=[torch.from_numpy(c).to(DEV) for c in classes])
    out.loss.backward()
    named = dict(m.named_parameters())
    for n in g6["names"]:
        n = str(n)
        g = named[n].grad.float().cpu().numpy().ravel()
        ref_norm = float(g6[n + "|norm"])
        assert abs(np.linalg.norm(g.astype(np.float64)) - ref_norm) <= 2e-2 * ref_norm + 1e-9, n
    for n, p in named.items():
        if "ratio_predictor" in n or "pixel_level_module.encoder." in n:
            assert p.grad is None, f"{n} must not receive gradients (Q1/Q2)"
