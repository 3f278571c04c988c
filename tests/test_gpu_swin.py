"""f2: the Swin-T backbone with HipSwinLayer (rgbd_amd/swin.py: HIP LayerNorm, qkv / output /
MLP GEMMs with fused GELU and residual epilogues, the window-attention kernel of
csrc/swin_attn.hip) against the Hugging Face SwinBackbone with the same weights, as the reference
calls it (custom_model.py:330; forward only, its features are detached).

Inputs at BASELINE's 640x480 (every stage needs window padding: 120x160 -> 126x161 ...) and
320x240; eval and train mode (DropPath active, drop_path_rate 0.3: the same torch RNG draws in
both arms).  Bars on each of the four feature maps, relative to its max: float32 1e-4 (exact f32
MFMA products, different summation order through 12 layers), bf16 autocast 5e-2."""
import copy
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import _rgbd_import  # noqa: E402,F401

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _backbones(train):
    from transformers import SwinBackbone
    from rgbd_amd import dense, swin
    from rgbd_amd.config import standard_config
    torch.manual_seed(3)
    ref = SwinBackbone(standard_config(48).backbone_config).to(DEV)
    with torch.no_grad():  # non-trivial relative-position tables (HF initialises them to zero)
        for m in ref.modules():
            if hasattr(m, "relative_position_bias_table"):
                m.relative_position_bias_table.normal_(0, 0.5)
    ref.train(train)
    hip = copy.deepcopy(ref)
    assert swin.install(hip) == 12
    dense.install(hip)
    return ref, hip


@pytest.mark.parametrize("amp", [False, True], ids=["f32", "bf16_autocast"])
@pytest.mark.parametrize("train", [False, True], ids=["eval", "train_droppath"])
@pytest.mark.parametrize("hw", [(480, 640), (240, 320)], ids=["640x480", "320x240"])
def test_swin_backbone_matches_hf(amp, train, hw):
    """HIP arm in the given precision vs the HF backbone in float32 (the reference's arithmetic),
    and, in bf16, also vs the HF backbone under the same autocast when that arm is finite."""
    ref, hip = _backbones(train)
    x = torch.randn((2, 3, *hw), device=DEV)

    def run(m, amp_):
        torch.manual_seed(11)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp_):
            return [f.float() for f in m(x).feature_maps]
    ref32, got = run(ref, False), run(hip, amp)
    for k, f in enumerate(got):
        assert torch.isfinite(f).all(), f"HIP arm: stage {k + 1} not finite"
    tol = 5e-2 if amp else 1e-4
    for k, (a, b) in enumerate(zip(got, ref32)):
        assert a.shape == b.shape
        err = _rel(a, b)
        print(f"stage {k + 1} {tuple(a.shape)}: rel err vs HF float32 {err:.3g}")
        assert err < tol, f"stage {k + 1}"
    if amp:
        ref16 = run(ref, True)
        if all(torch.isfinite(f).all() for f in ref16):
            for k, (a, b) in enumerate(zip(got, ref16)):
                print(f"stage {k + 1}: rel err vs HF bf16 autocast {_rel(a, b):.3g}")
                assert _rel(a, b) < tol
        else:
            print("HF bf16 autocast arm not finite on this device: compared with float32 only")


def test_swin_layer_takes_hf_path_with_grad():
    """With gradients required the HIP layer runs the HF forward (the fused path is forward-only)."""
    ref, hip = _backbones(False)
    x = torch.randn((1, 3, 224, 224), device=DEV)
    a = ref(x).feature_maps[-1]
    b = hip(x).feature_maps[-1]
    assert b.requires_grad and _rel(b.detach(), a.detach()) < 1e-4
