"""f2: fused multi-scale deformable attention (csrc/msda.hip) vs the reference's pure-torch
multi_scale_deformable_attention (transformers 5.15 modeling_mask2former.py:798-837, grid_sample
per level) on the same inputs, forward and all three gradients, fp32 (and bf16 value)."""
import pytest
import torch
from transformers.models.mask2former.modeling_mask2former import (
    Mask2FormerPixelDecoderEncoderMultiscaleDeformableAttention, multi_scale_deformable_attention as hf_msda)

from rgbd_amd import deform_attn, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = [
    # shapes of the C1 pixel decoder (320x240 input: /8, /16, /32), 8 heads x 32, 4 points
    (2, [(30, 40), (15, 20), (8, 10)], 8, 32, 4, 1525),
    # ragged levels, 64-wide heads, queries != value length
    (1, [(7, 9), (4, 5), (2, 3)], 4, 64, 3, 50),
    (1, [(16, 12)], 2, 16, 2, 33),
    # queries = value pixels (the encoder case)
    (2, [(30, 40), (15, 20), (8, 10)], 8, 32, 4, 1580),
    # the C5 (1280x720) pixel decoder's first two levels (90 x 160, 45 x 80)
    (1, [(90, 160), (45, 80)], 2, 32, 2, 700),
]


def _inputs(B, shapes, NH, D, P, Q, dtype=torch.float32, seed=0, spread=1.4):
    g = torch.Generator(device=DEV).manual_seed(seed)
    S = sum(h * w for h, w in shapes)
    L = len(shapes)
    value = torch.randn((B, S, NH, D), generator=g, device=DEV).to(dtype)
    # locations partly outside [0, 1] to exercise the zero padding
    loc = torch.rand((B, Q, NH, L, P, 2), generator=g, device=DEV) * spread - (spread - 1) / 2
    attw = torch.rand((B, Q, NH, L, P), generator=g, device=DEV)
    attw = attw / attw.sum(dim=(-1, -2), keepdim=True)
    return value, loc, attw


@pytest.mark.parametrize("case", CASES)
def test_msda_forward_backward_f32(case):
    B, shapes, NH, D, P, Q = case
    value, loc, attw = _inputs(B, shapes, NH, D, P, Q)
    vr, lr, ar = (t.clone().requires_grad_(True) for t in (value, loc, attw))
    vh, lh, ah = (t.clone().requires_grad_(True) for t in (value, loc, attw))
    out_r = hf_msda(vr, shapes, lr, ar)
    out_h = deform_attn.multi_scale_deformable_attention(vh, shapes, lh, ah)
    assert out_h.shape == out_r.shape
    assert float((out_h - out_r).abs().max()) < 2e-5
    go = torch.randn(out_r.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(9))
    (out_r * go).sum().backward()
    (out_h * go).sum().backward()
    for a, b, name in ((vh.grad, vr.grad, "value"), (lh.grad, lr.grad, "loc"), (ah.grad, ar.grad, "attw")):
        scale = float(b.abs().max()) + 1e-12
        err = float((a - b).abs().max()) / scale
        assert err < 1e-4, (name, err)


def _encoder_locations(B, shapes, NH, P, g, jitter=0.0):
    """Every value pixel as a query at its own reference point plus an offset per (head, level,
    point) that is the same for every query (the MSDeformAttn initialisation's grid), optionally
    jittered per query: neighbouring queries then sample shifted copies of the same cells, the
    case k_msda_bwd_runs carries contributions across."""
    refs = []
    for H, W in shapes:
        ys, xs = torch.meshgrid(torch.arange(H, device=DEV), torch.arange(W, device=DEV), indexing="ij")
        refs.append(torch.stack([(xs.reshape(-1) + 0.5) / W, (ys.reshape(-1) + 0.5) / H], -1))
    ref = torch.cat(refs)
    S, L = ref.shape[0], len(shapes)
    norm = torch.tensor([[w, h] for h, w in shapes], device=DEV, dtype=torch.float32)
    off = torch.randn((1, 1, NH, L, P, 2), generator=g, device=DEV) * 2.0
    off = off + torch.randn((B, S, NH, L, P, 2), generator=g, device=DEV) * jitter
    return ref[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]


@pytest.mark.parametrize("jitter", [0.0, 0.3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_msda_backward_carried_taps_vs_hf(jitter, dtype):
    """Encoder-shaped queries (Q = S, 3 levels x 4 points: the run-carrying backward) with
    spatially constant / jittered offsets against grid_sample's backward."""
    B, shapes, NH, D, P = 2, [(30, 40), (15, 20), (8, 10)], 8, 32, 4
    S = sum(h * w for h, w in shapes)
    g = torch.Generator(device=DEV).manual_seed(5)
    value = torch.randn((B, S, NH, D), generator=g, device=DEV).to(dtype)
    loc = _encoder_locations(B, shapes, NH, P, g, jitter)
    attw = torch.softmax(torch.randn((B, S, NH, 3 * P), generator=g, device=DEV), -1).view(B, S, NH, 3, P)
    vr, lr, ar = (t.clone().float().requires_grad_(True) for t in (value, loc, attw))
    vh, lh, ah = (t.clone().requires_grad_(True) for t in (value, loc, attw))
    go = torch.randn((B, S, NH * D), generator=g, device=DEV)
    (hf_msda(vr, shapes, lr, ar) * go).sum().backward()
    out_h = deform_attn.multi_scale_deformable_attention(vh, shapes, lh, ah)
    (out_h.float() * go).sum().backward()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for a, b, name in ((vh.grad, vr.grad, "value"), (lh.grad, lr.grad, "loc"), (ah.grad, ar.grad, "attw")):
        err = float((a.float() - b).abs().max()) / (float(b.abs().max()) + 1e-12)
        assert err < tol, (name, err)


def test_msda_bf16_value():
    B, shapes, NH, D, P, Q = CASES[0]
    value, loc, attw = _inputs(B, shapes, NH, D, P, Q, dtype=torch.bfloat16, seed=3)
    out = ops.msda_forward(value, shapes, loc, attw)
    ref = hf_msda(value.float(), shapes, loc, attw)
    assert out.dtype == torch.bfloat16
    assert float((out.float() - ref).abs().max()) <= 2.0 ** -7 * float(ref.abs().max()) + 1e-3


def test_hip_msda_module_matches_hf():
    torch.manual_seed(0)
    ref = Mask2FormerPixelDecoderEncoderMultiscaleDeformableAttention(256, 8, 3, 4).to(DEV)
    hip = Mask2FormerPixelDecoderEncoderMultiscaleDeformableAttention(256, 8, 3, 4).to(DEV)
    hip.load_state_dict(ref.state_dict())
    assert deform_attn.install(hip) == 1
    shapes = [(30, 40), (15, 20), (8, 10)]
    S = sum(h * w for h, w in shapes)
    g = torch.Generator(device=DEV).manual_seed(1)
    hs = torch.randn((2, S, 256), generator=g, device=DEV)
    pos = torch.randn((2, S, 256), generator=g, device=DEV) * 0.1
    refp = torch.rand((2, S, 3, 2), generator=g, device=DEV)
    starts = torch.tensor([0, 1200, 1500], device=DEV)
    outs = []
    for m in (ref, hip):
        x = hs.clone().requires_grad_(True)
        o, w = m(x, encoder_hidden_states=x, position_embeddings=pos, reference_points=refp,
                 spatial_shapes_list=shapes, level_start_index=starts)
        o.square().mean().backward()
        outs.append((o.detach(), w.detach(), x.grad, {n: p.grad.clone() for n, p in m.named_parameters()}))
    (o_r, w_r, gx_r, gp_r), (o_h, w_h, gx_h, gp_h) = outs
    assert float((o_h - o_r).abs().max()) < 1e-4
    assert torch.equal(w_h, w_r)
    assert float((gx_h - gx_r).abs().max()) / float(gx_r.abs().max()) < 1e-4
    for n in gp_r:
        assert float((gp_h[n] - gp_r[n]).abs().max()) / (float(gp_r[n].abs().max()) + 1e-12) < 1e-4, n


@pytest.mark.parametrize("shapes", [[(60, 80), (30, 40), (15, 20)], [(257, 515), (129, 258), (65, 129)]],
                         ids=["c1", "wide"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_msda_locations_bitwise(dt, shapes):
    """rgbd_msda_locations: ref + offsets / norm (the two-coordinate reference points, :990-994)
    with torch's dtype rules — the same bits forward, and the offsets' gradient of torch's
    expression bitwise.  "wide": level sizes above 256 that bf16 cannot hold (257, 515, 258 ...),
    which torch rounds to bf16 before dividing bf16 offsets (deform_attn.location_norm)."""
    g = torch.Generator(device=DEV).manual_seed(4)
    B, Q, NH, L, P = 2, 777, 8, 3, 4
    ref = torch.rand((B, Q, L, 2), generator=g, device=DEV)
    off = (torch.randn((B, Q, NH, L, P, 2), generator=g, device=DEV) * 3).to(dt)
    norm_l = ops.device_const([[w, h] for h, w in shapes], torch.long, DEV)
    o1 = off.clone().requires_grad_()
    want = ref[:, :, None, :, None, :] + o1 / norm_l[None, None, None, :, None, :]
    gl = torch.randn(want.shape, generator=g, device=DEV)
    want.backward(gl)
    o2 = off.clone().requires_grad_()
    norm_f = deform_attn.location_norm(shapes, dt, DEV)
    got = deform_attn.MSDALocationsFunction.apply(ref, o2, norm_f)
    got.backward(gl)
    assert got.dtype == want.dtype == torch.float32
    assert torch.equal(got, want)
    assert o2.grad.dtype == dt and torch.equal(o2.grad, o1.grad)
