"""f1: the mask predictor's einsum and attention mask (transformers 5.15
modeling_mask2former.py:2040-2056) on the HIP kernels vs PyTorch fp32 on the same inputs."""
import pytest
import torch
import torch.nn.functional as F
from transformers.models.mask2former.modeling_mask2former import Mask2FormerMaskPredictor

from rgbd_amd import mask_predictor, ops

gpu = pytest.mark.gpu
SHAPES = [(2, 100, 256, 60, 80),   # C1 mask features (320x240 input), HF num_queries / mask_feature_size
          (1, 100, 256, 120, 160),  # C2 (640x480)
          (1, 37, 64, 7, 9),        # ragged: P % 4 != 0, Q not a fragment multiple
          (2, 130, 96, 16, 12),     # two query blocks, C not a multiple of the 64-channel chunk
          (1, 5, 32, 3, 3)]


def _inputs(B, Q, C, H, W, dtype, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    emb = torch.randn((B, Q, C), generator=g, device="cuda")
    pix = torch.randn((B, C, H, W), generator=g, device="cuda")
    return emb.to(dtype), pix.to(dtype)


def _ref_attention(logits, size, heads):
    """modeling_mask2former.py:2048-2053 verbatim in torch."""
    a = F.interpolate(logits, size=size, mode="bilinear", align_corners=False)
    a = a.sigmoid().flatten(2).unsqueeze(1).repeat(1, heads, 1, 1)
    return (a.flatten(0, 1) < 0.5).bool(), F.interpolate(logits.float(), size=size, mode="bilinear",
                                                         align_corners=False).flatten(2)


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_mask_logits_f32(shape):
    emb, pix = _inputs(*shape, torch.float32)
    out = ops.mask_logits(emb, pix)
    ref = torch.einsum("bqc,bchw->bqhw", emb.double(), pix.double())
    err = float((out.double() - ref).abs().max())
    assert err <= 2e-6 * shape[2] ** 0.5 * 4, err   # exact f32 products, f32 sums of C terms


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_mask_logits_bf16(shape):
    emb, pix = _inputs(*shape, torch.bfloat16, seed=1)
    out = ops.mask_logits(emb, pix)
    ref = torch.einsum("bqc,bchw->bqhw", emb.double(), pix.double())
    # bf16 inputs exact, f32 accumulation, one bf16 rounding of the output (2^-8 relative)
    tol = ref.abs() * 2.0 ** -8 + 1e-4
    assert bool(((out.double() - ref).abs() <= tol).all())


@gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("src,dst", [((60, 80), (30, 40)), ((60, 80), (15, 20)), ((60, 80), (8, 10)),
                                     ((120, 160), (15, 20)), ((7, 9), (4, 5)), ((16, 12), (32, 24))])
def test_mask_attention_matches_torch(dtype, src, dst):
    g = torch.Generator(device="cuda").manual_seed(7)
    logits = (torch.randn((2, 11, *src), generator=g, device="cuda") * 3).to(dtype)
    logits[0, 0] = 0.0  # exact ties: sigmoid(0) = 0.5 -> False
    heads = 8
    got = ops.mask_attention(logits, dst, heads)
    ref, val = _ref_attention(logits, dst, heads)
    assert got.dtype == torch.bool and got.shape == ref.shape
    diff = got != ref
    # identical decisions except where the interpolated logit is within rounding of 0 (the two
    # sides order the four bilinear products differently)
    near = (val.abs() < 1e-5).unsqueeze(1).expand(-1, heads, -1, -1).flatten(0, 1)
    assert not bool((diff & ~near).any()), int((diff & ~near).sum())
    assert int(diff.sum()) <= int(near.sum())


@gpu
@pytest.mark.parametrize("dtype", [torch.float32])
def test_hip_mask_predictor_matches_hf(dtype):
    torch.manual_seed(0)
    ref = Mask2FormerMaskPredictor(hidden_size=256, num_heads=8, mask_feature_size=256).cuda()
    hip = Mask2FormerMaskPredictor(hidden_size=256, num_heads=8, mask_feature_size=256).cuda()
    hip.load_state_dict(ref.state_dict())
    assert mask_predictor.install(hip) == 1 and isinstance(hip, mask_predictor.HipMaskPredictor)
    assert list(hip.state_dict()) == list(ref.state_dict())
    g = torch.Generator(device="cuda").manual_seed(3)
    outputs = torch.randn((100, 2, 256), generator=g, device="cuda")
    pix = torch.randn((2, 256, 60, 80), generator=g, device="cuda")
    pix_r = pix.clone().requires_grad_(True)
    pix_h = pix.clone().requires_grad_(True)
    size = torch.Size([15, 20])
    m_r, a_r = ref(outputs, pix_r, size)
    m_h, a_h = hip(outputs, pix_h, size)
    assert m_h.shape == m_r.shape and a_h.shape == a_r.shape and a_h.dtype == a_r.dtype
    assert float((m_h - m_r).abs().max()) < 1e-4
    near = (F.interpolate(m_r.detach(), size=size, mode="bilinear", align_corners=False).flatten(2).abs() < 1e-4)
    near = near.unsqueeze(1).expand(-1, 8, -1, -1).flatten(0, 1)
    assert not bool(((a_h != a_r) & ~near).any())
    go = torch.randn(m_r.shape, generator=g, device="cuda")
    (m_r * go).sum().backward()
    (m_h * go).sum().backward()
    assert float((pix_h.grad - pix_r.grad).abs().max()) < 1e-3
    for (n, p_r), p_h in zip(ref.named_parameters(), hip.parameters()):
        scale = float(p_r.grad.abs().max()) + 1e-12
        assert float((p_h.grad - p_r.grad).abs().max()) / scale < 1e-4, n


@gpu
def test_mask_ops_reject_bad_input():
    emb, pix = _inputs(1, 4, 48, 4, 4, torch.float32)   # C % 32 != 0
    with pytest.raises(RuntimeError):
        ops.mask_logits(emb, pix)
    with pytest.raises(ValueError):
        ops.mask_logits(emb[:, :, :32], pix)
    with pytest.raises(RuntimeError):
        ops.mask_logits(emb.cpu(), pix.cpu())


@gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("B,C,H,W", [(8, 256, 60, 80), (2, 256, 15, 20), (3, 192, 7, 9)])
def test_level_memory_matches_torch(dt, B, C, H, W):
    """One level's decoder memory (input projection output + level embedding, permuted to
    [HW, B, C], :2102-2109): the values bitwise, the projection's gradient bitwise, the
    embedding's gradient (a sum over pixels and images in another order) to 1e-5."""
    g = torch.Generator(device="cuda").manual_seed(C + H)
    proj = torch.randn((B, C, H, W), generator=g, device="cuda").to(dt)
    emb = torch.randn((4, C), generator=g, device="cuda")
    p1, e1 = proj.clone().requires_grad_(), emb.clone().requires_grad_()
    want = (p1.flatten(2) + e1[2][None, :, None]).permute(2, 0, 1)
    gy = torch.randn(want.shape, generator=g, device="cuda")
    want.backward(gy)
    p2, e2 = proj.clone().requires_grad_(), emb.clone().requires_grad_()
    got = mask_predictor.level_memory(p2, e2[2])
    got.backward(gy)
    assert got.dtype == want.dtype and got.shape == want.shape and got.is_contiguous()
    assert torch.equal(got, want)
    assert p2.grad.dtype == dt and torch.equal(p2.grad, p1.grad)
    assert float((e2.grad - e1.grad).abs().max()) <= 1e-5 * float(e1.grad.abs().max())


@gpu
def test_transformer_module_matches_hf():
    """HipTransformerModule (the fused level memory) inside the installed decoder gives the HF
    module's outputs, with every parameter's gradient, on a C2-shaped call (float32)."""
    import copy
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerTransformerModule
    from rgbd_amd import dense, masked_attention
    from rgbd_amd.config import standard_config
    torch.manual_seed(3)
    cfg = standard_config(48)
    ref = Mask2FormerTransformerModule(in_features=256, config=cfg).cuda().train()
    hip = copy.deepcopy(ref)
    mask_predictor.install(hip)
    assert type(hip) is mask_predictor.HipTransformerModule
    feats = [torch.randn((2, 256, h, w), device="cuda") for h, w in ((8, 10), (15, 20), (30, 40))]
    mf = torch.randn((2, 256, 60, 80), device="cuda")
    outs = []
    for m in (ref, hip):
        fs = [f.clone().requires_grad_() for f in feats]
        o = m(fs, mf)
        loss = (sum(m_.float().square().mean() for m_ in o.masks_queries_logits)
                + sum(h.float().square().mean() for h in o.intermediate_hidden_states))
        loss.backward()
        outs.append((torch.stack([m_.detach() for m_ in o.masks_queries_logits]), [f.grad for f in fs],
                     {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    (a, fa, ga), (b, fb, gb) = outs
    assert float((a - b).abs().max()) <= 1e-5 * float(a.abs().max())
    for x, y in zip(fa, fb):
        assert float((x - y).abs().max()) <= 1e-4 * float(x.abs().max())
    assert ga.keys() == gb.keys()
    # floored at 1e-6 of the largest gradient: the self-attention key biases' gradients are zero in
    # exact arithmetic (softmax is invariant to a per-query constant) and rounding noise in both arms
    scale = max(float(v.abs().max()) for v in ga.values())
    for n in ga:
        assert float((ga[n] - gb[n]).abs().max()) <= 1e-4 * float(ga[n].abs().max()) + 1e-6 * scale, n
