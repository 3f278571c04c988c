"""f2: nn.GroupNorm of the pixel decoder on the HIP kernels (csrc/groupnorm.hip, rgbd_amd.dense
HipGroupNorm) vs torch — float32 against float64 arithmetic, bf16 inputs under autocast against
torch's autocast GroupNorm (which normalises the bf16 values in float32), and the fused ReLU of
the FPN output layer (nn.Sequential(GroupNorm, ReLU)) against the unfused torch pair."""
import pytest
import torch

import _rgbd_import  # noqa: F401

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _gn(C=256, G=32, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    gn = torch.nn.GroupNorm(G, C)
    with torch.no_grad():
        gn.weight.copy_(torch.randn(C, generator=g))
        gn.bias.copy_(torch.randn(C, generator=g))
    return gn.to(DEV), g


@pytest.mark.parametrize("shape", [(2, 256, 30, 40), (8, 256, 15, 20), (1, 64, 7, 9)])
def test_groupnorm_f32_fwd_bwd(shape):
    from rgbd_amd import dense
    gn, g = _gn(C=shape[1], G=32 if shape[1] >= 32 else 8, seed=shape[2])
    hip = dense.HipGroupNorm(gn.num_groups, gn.num_channels).to(DEV)
    hip.load_state_dict(gn.state_dict())
    x = (torch.randn(shape, generator=g) * 2 + 0.5).to(DEV).requires_grad_()
    gy = torch.randn(shape, generator=g).to(DEV)
    y = hip(x)
    y.backward(gy)
    x64 = x.detach().double().requires_grad_()
    w64, b64 = gn.weight.detach().double().requires_grad_(), gn.bias.detach().double().requires_grad_()
    y64 = torch.nn.functional.group_norm(x64, gn.num_groups, w64, b64, gn.eps)
    y64.backward(gy.double())
    assert _rel(y, y64) < 1e-5
    assert _rel(x.grad, x64.grad) < 1e-4
    assert _rel(hip.weight.grad, w64.grad) < 1e-5
    assert _rel(hip.bias.grad, b64.grad) < 1e-5
    # deterministic
    x.grad = None
    hip.weight.grad = hip.bias.grad = None
    y2 = hip(x)
    assert torch.equal(y, y2)


def test_groupnorm_bf16_autocast_matches_torch():
    from rgbd_amd import dense
    gn, g = _gn(seed=3)
    hip = dense.HipGroupNorm(32, 256).to(DEV)
    hip.load_state_dict(gn.state_dict())
    x = torch.randn((4, 256, 30, 40), generator=g).to(DEV, torch.bfloat16)
    gy = torch.randn((4, 256, 30, 40), generator=g).to(DEV)
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ya, yb = hip(xa), gn(xb)
    assert ya.dtype == yb.dtype == torch.float32
    assert _rel(ya, yb) < 1e-5
    ya.backward(gy)
    yb.backward(gy)
    assert xa.grad.dtype == torch.bfloat16
    assert _rel(xa.grad, xb.grad) < 1e-2
    assert _rel(hip.weight.grad, gn.weight.grad) < 1e-4
    assert _rel(hip.bias.grad, gn.bias.grad) < 1e-4


def test_groupnorm_relu_fused_by_install():
    from rgbd_amd import dense
    gn, g = _gn(seed=7)
    ref = torch.nn.Sequential(torch.nn.Conv2d(16, 256, 1, bias=False), gn, torch.nn.ReLU()).to(DEV)
    hip = torch.nn.Sequential(torch.nn.Conv2d(16, 256, 1, bias=False), torch.nn.GroupNorm(32, 256),
                              torch.nn.ReLU()).to(DEV)
    hip.load_state_dict(ref.state_dict())
    assert dense.install(hip) == 2  # the 1x1 convolution (f2, conv.HipConv2d) and the GroupNorm
    assert type(hip[0]).__name__ == "HipConv2d"
    assert hip[1]._fused_relu and type(hip[2]).__name__ == "_FusedReLU"
    x = torch.randn((2, 16, 30, 40), generator=g).to(DEV)
    gy = torch.randn((2, 256, 30, 40), generator=g).to(DEV)
    ya, yb = hip(x), ref(x)
    assert _rel(ya, yb) < 1e-5 and float(ya.min()) >= 0.0
    ya.backward(gy)
    yb.backward(gy)
    for (na, pa), (nb, pb) in zip(hip.named_parameters(), ref.named_parameters()):
        assert _rel(pa.grad, pb.grad) < 1e-4, na
    assert dense.uninstall(hip) == 2
    assert type(hip[0]) is torch.nn.Conv2d
    assert type(hip[1]) is torch.nn.GroupNorm and type(hip[2]) is torch.nn.ReLU
    assert _rel(hip(x), yb) < 1e-5
