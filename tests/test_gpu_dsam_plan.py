"""Planning ahead (include/rgbd_hip.h rgbd_dsam_plan): every bf16 DSAM leg run with a plan made
earlier — all forward / dX legs of the three DSAMs planned by one call, the dW legs by another —
gives bitwise the outputs of the plain entry points, which plan inside the call.  Shapes: the
bench's 640x480 B=8 pyramid and a ragged one (97x131 input, odd feature sizes), region codes
from the HIP decomposition.  Reference path: custom_model.py:682-699 (DSAModule.forward); the
parity of the plain entry points themselves is test_gpu_dsam_full.py / test_gpu_parity.py."""
import pytest
import torch

import _rgbd_import  # noqa: F401
from rgbd_amd import ops, synthetic

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
CH = [(96, 192), (192, 384), (384, 768)]


def _sizes(H, W):
    s = [((H + 3) // 4, (W + 3) // 4)]
    for _ in range(2):
        s.append(((s[-1][0] + 1) // 2, (s[-1][1] + 1) // 2))
    return s


@pytest.mark.parametrize("H,W,B", [(480, 640, 8), (97, 131, 3)])
def test_planned_legs_bitwise(H, W, B):
    planes, _, _ = synthetic.make_batch(7, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    sizes = _sizes(H, W)
    codes, info = ops.edsam_decompose(d3, torch.linspace(0.05, 0.45, B, device=DEV), sizes)
    masks = ops.dsam_code_masks(codes)
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    legs = [(ops.LEG_FWD, codes[k], *CH[k]) for k in range(3)] + [(ops.LEG_DX, codes[k], *CH[k]) for k in (1, 2)]
    conv_plans = ops.dsam_plan(legs)
    dw_plans = ops.dsam_plan([(ops.LEG_DW, codes[k], *CH[k]) for k in range(3)])
    for k in range(3):
        ci, co = CH[k]
        h, w = sizes[k]
        ho, wo = (h + 1) // 2, (w + 1) // 2
        cw = torch.randn((4, co, ci, 3, 3), generator=g, device=DEV) * 0.03
        pw = torch.randn((co, ci, 3, 3), generator=g, device=DEV) * 0.03
        b4 = torch.randn((4, co), generator=g, device=DEV) * 0.1
        wf, wb = ops.dsam_pack(cw, pw, torch.bfloat16, code_mask=masks[k:k + 1])
        x = torch.randn((B, h, w, ci), generator=g, device=DEV).bfloat16()
        res = torch.randn((B, ho, wo, co), generator=g, device=DEV).bfloat16()
        gy = (torch.randn((B, ho, wo, co), generator=g, device=DEV) * 0.1).bfloat16()
        gin = torch.randn((B, h, w, ci), generator=g, device=DEV).bfloat16()
        y0 = ops.dsam_fwd_nhwc(x, codes[k], info, wf, b4, residual_nhwc=res)
        y1 = ops.dsam_fwd_nhwc(x, codes[k], info, wf, b4, residual_nhwc=res, plan=conv_plans[k])
        assert torch.equal(y0, y1), f"forward {k}"
        w0 = ops.dsam_bwd_weight(None, x, codes[k], info, gout_nhwc=gy)
        w1 = ops.dsam_bwd_weight(None, x, codes[k], info, gout_nhwc=gy, plan=dw_plans[k])
        for a, b, name in zip(w0, w1, ("dconv", "dproj", "dbias")):
            assert torch.equal(a, b), f"dW {k} {name}"
        if k > 0:
            _, d0 = ops.dsam_bwd_data(gy, codes[k], wb, None, want_nhwc=True, want_nchw=False, gin_nhwc=gin)
            _, d1 = ops.dsam_bwd_data(gy, codes[k], wb, None, want_nhwc=True, want_nchw=False, gin_nhwc=gin,
                                      plan=conv_plans[3 + (k - 1)])
            assert torch.equal(d0, d1), f"dX {k}"


def test_plan_rejects_bad_legs():
    code = torch.zeros((2, 30, 40), dtype=torch.uint8, device=DEV)
    with pytest.raises(ValueError):
        ops.dsam_plan([(7, code, 96, 192)])
    with pytest.raises(ops._lib.RgbdHipError):  # channel counts the bf16 path does not tile
        ops.dsam_plan([(ops.LEG_FWD, code, 40, 192)])


@pytest.mark.parametrize("H,W,B", [(480, 640, 8), (720, 1280, 1), (97, 131, 3), (64, 96, 2)])
def test_decompose_code_masks(H, W, B):
    """rgbd_edsam_decompose_masks: the same codes and info as the plain decomposition, and per
    scale the presence mask dsam_code_masks computes from the code planes (the Swin pyramid
    shapes take the one-launch pyramid kernel, the others the general path)."""
    planes, _, _ = synthetic.make_batch(9, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    sizes = _sizes(H, W)
    r = torch.linspace(0.05, 0.45, B, device=DEV)
    c0, i0 = ops.edsam_decompose(d3, r, sizes)
    c1, i1, m1 = ops.edsam_decompose(d3, r, sizes, code_masks=True)
    assert torch.equal(i0, i1)
    for a, b in zip(c0, c1):
        assert torch.equal(a, b)
    assert torch.equal(m1, ops.dsam_code_masks(c0))


@pytest.mark.parametrize("H,W,B,pairs", [(480, 640, 8, [(1, 0), (2, 1), (0,)]), (97, 131, 3, [(1, 0), (2, 0)])])
def test_joint_dw_bitwise(H, W, B, pairs):
    """rgbd_dsam_bwd_weight_planned_multi: the dW GEMMs of two legs in one persistent launch give
    per leg bitwise the gradients of the one-leg planned entry point (the hot path runs dsam1 and
    dsam0 this way; hot_path.JOINT_DW)."""
    planes, _, _ = synthetic.make_batch(11, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    sizes = _sizes(H, W)
    codes, info = ops.edsam_decompose(d3, torch.linspace(0.05, 0.45, B, device=DEV), sizes)
    g = torch.Generator(device=DEV)
    g.manual_seed(13)
    xs, gys = [], []
    for k in range(3):
        ci, co = CH[k]
        h, w = sizes[k]
        xs.append(torch.randn((B, h, w, ci), generator=g, device=DEV).bfloat16())
        gys.append((torch.randn((B, (h + 1) // 2, (w + 1) // 2, co), generator=g, device=DEV) * 0.1).bfloat16())
    for pair in pairs:
        plans = ops.dsam_plan([(ops.LEG_DW, codes[k], *CH[k]) for k in pair])
        got = ops.dsam_bwd_weight_multi([(gys[k], xs[k], codes[k], plans[j]) for j, k in enumerate(pair)], info)
        for j, k in enumerate(pair):
            want = ops.dsam_bwd_weight(None, xs[k], codes[k], info, gout_nhwc=gys[k])
            for a, b, name in zip(got[j], want, ("dconv", "dproj", "dbias")):
                assert torch.equal(a, b), f"joint {pair} leg {k} {name}"


def test_joint_dw_mixed_tile_shapes():
    """Legs whose output tiles differ (Cout 192 -> 6 sub-tiles, 256 -> 4) run one launch each
    behind the same entry point, with the same results."""
    B, H, W = 2, 96, 128
    planes, _, _ = synthetic.make_batch(3, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    sizes = _sizes(H, W)
    codes, info = ops.edsam_decompose(d3, torch.full((B,), 0.2, device=DEV), sizes)
    g = torch.Generator(device=DEV)
    g.manual_seed(2)
    legs = [(0, 96, 192), (1, 96, 256)]
    runs, ref = [], []
    plans = ops.dsam_plan([(ops.LEG_DW, codes[k], ci, co) for k, ci, co in legs])
    for j, (k, ci, co) in enumerate(legs):
        h, w = sizes[k]
        x = torch.randn((B, h, w, ci), generator=g, device=DEV).bfloat16()
        gy = (torch.randn((B, (h + 1) // 2, (w + 1) // 2, co), generator=g, device=DEV) * 0.1).bfloat16()
        runs.append((gy, x, codes[k], plans[j]))
        ref.append(ops.dsam_bwd_weight(None, x, codes[k], info, gout_nhwc=gy))
    got = ops.dsam_bwd_weight_multi(runs, info)
    for j in range(2):
        for a, b in zip(got[j], ref[j]):
            assert torch.equal(a, b), f"leg {j}"
