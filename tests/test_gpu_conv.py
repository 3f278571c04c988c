"""f2: the drop-in model's remaining convolutions on the HIP GEMMs (rgbd_amd/conv.py,
csrc/conv.hip + csrc/gemm.hip) against torch.nn.functional.conv2d.

Shapes: the pixel decoder's at C2 (B=8, 640x480: 1x1 input projections at H/8..H/32 with bias,
the FPN lateral 1x1 96->256 and the 3x3 256->256 output convolution at H/4 without bias, the
1x1 mask projection), odd sizes from C5 (1280x720: 23x40 at H/32, widths not a multiple of 8),
and Swin's 4x4 stride-4 patch embedding.

Bars: im2col bit-exact against F.unfold; float32 (exact-f32 MFMA) outputs and all gradients
within 1e-4 of float64 relative to the max; bf16 under autocast against float32 torch within
2e-2 (outputs) / 3e-2 (gradients) relative to the max (bf16 operands, float32 sums)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / max(float(b.double().abs().max()), 1e-30))


@pytest.mark.parametrize("k,C,H,W", [(3, 5, 7, 13), (3, 16, 8, 16), (3, 32, 23, 40), (4, 3, 16, 24), (4, 3, 480, 640)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_im2col_bitexact_vs_unfold(k, C, H, W, dt):
    from rgbd_amd.conv import _im2col
    x = torch.randn(2, C, H, W, device=DEV).to(dt)
    got = _im2col(x, k)
    want = F.unfold(x.float(), k, padding=1 if k == 3 else 0, stride=1 if k == 3 else 4).to(dt)
    assert torch.equal(got, want)


CASES = [  # (Cin, Cout, k, bias, H, W, B)
    (768, 256, 1, True, 15, 20, 8),     # input projection, H/32 at C2
    (384, 256, 1, True, 30, 40, 8),     # H/16
    (192, 256, 1, True, 60, 80, 8),     # H/8
    (96, 256, 1, False, 120, 160, 8),   # FPN lateral at H/4
    (256, 256, 3, False, 120, 160, 8),  # FPN output convolution at H/4 (22.6 GFLOP per image)
    (256, 256, 1, True, 120, 160, 8),   # mask projection
    (768, 256, 1, True, 23, 40, 1),     # C5 H/32 (odd rows)
    (256, 256, 3, False, 23, 37, 2),    # ragged 3x3 (width not a multiple of 8)
    (3, 96, 4, True, 480, 640, 2),      # Swin patch embedding
]


def _modules(Cin, Cout, k, bias):
    from rgbd_amd.conv import HipConv2d
    torch.manual_seed(Cin * 7 + Cout + k)
    pad = 1 if k == 3 else 0
    stride = 4 if k == 4 else 1
    ref = torch.nn.Conv2d(Cin, Cout, k, stride=stride, padding=pad, bias=bias).to(DEV)
    hip = torch.nn.Conv2d(Cin, Cout, k, stride=stride, padding=pad, bias=bias).to(DEV)
    hip.load_state_dict(ref.state_dict())
    hip.__class__ = HipConv2d
    return ref, hip


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}to{c[1]}_k{c[2]}_{c[4]}x{c[5]}_b{c[6]}" for c in CASES])
def test_conv_f32_vs_float64(case):
    Cin, Cout, k, bias, H, W, B = case
    ref, hip = _modules(Cin, Cout, k, bias)
    x = torch.randn(B, Cin, H, W, device=DEV)
    x1 = x.clone().requires_grad_(True)
    y = hip(x1)
    gy = torch.randn_like(y)
    y.backward(gy)
    ref64 = ref.double()
    x2 = x.double().requires_grad_(True)
    y2 = ref64(x2)
    y2.backward(gy.double())
    assert y.dtype == torch.float32 and y.shape == y2.shape
    assert _rel(y, y2) < 1e-4
    assert _rel(x1.grad, x2.grad) < 1e-4
    assert _rel(hip.weight.grad, ref64.weight.grad) < 1e-4
    if bias:
        assert _rel(hip.bias.grad, ref64.bias.grad) < 1e-4


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", CASES[3:6] + CASES[-1:], ids=["lateral", "fpn3x3", "maskproj", "patch"])
def test_conv_bf16_autocast_vs_f32(case):
    Cin, Cout, k, bias, H, W, B = case
    ref, hip = _modules(Cin, Cout, k, bias)
    x = torch.randn(B, Cin, H, W, device=DEV)
    x1 = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = hip(x1)
    assert y.dtype == torch.bfloat16
    gy = torch.randn(y.shape, device=DEV)
    y.float().backward(gy)
    x2 = x.clone().requires_grad_(True)
    y2 = ref(x2)
    y2.backward(gy)
    print(f"{case}: out {_rel(y, y2):.2e} dx {_rel(x1.grad, x2.grad):.2e} dw {_rel(hip.weight.grad, ref.weight.grad):.2e}")
    assert _rel(y, y2) < 2e-2
    assert _rel(x1.grad, x2.grad) < 3e-2
    assert _rel(hip.weight.grad, ref.weight.grad) < 3e-2


def test_uncovered_shapes_take_torch_path():
    from rgbd_amd.conv import HipConv2d
    m = torch.nn.Conv2d(8, 8, 3, stride=2, padding=1).to(DEV)
    m.__class__ = HipConv2d
    x = torch.randn(1, 8, 9, 9, device=DEV)
    torch.testing.assert_close(m(x), F.conv2d(x, m.weight, m.bias, stride=2, padding=1))
