"""f1: the decoder layers' masked cross-attention (transformers 5.15 modeling_mask2former.py
:1644-1650, nn.MultiheadAttention's math path) on the HIP kernels, against torch's own module with
the same parameters (fp32, same device) and a float64 restatement of the attention core."""
import math

import pytest
import torch
from torch import nn

from rgbd_amd import masked_attention

gpu = pytest.mark.gpu

# (B, Q, L): the three pixel-decoder levels at 320x240 (C1) and 640x480 (C2), ragged lengths.
SHAPES = [(2, 100, 300), (2, 100, 1200), (1, 100, 4800), (3, 37, 97), (1, 5, 1), (2, 100, 65)]


def _inputs(B, Q, L, seed=0, p_mask=0.6):
    g = torch.Generator(device="cuda").manual_seed(seed)
    query = torch.randn((Q, B, 256), generator=g, device="cuda")
    value = torch.randn((L, B, 256), generator=g, device="cuda")
    key = value + torch.randn((L, B, 256), generator=g, device="cuda")  # value + position embedding
    mask = torch.rand((B * 8, Q, L), generator=g, device="cuda") < p_mask
    # the decoder un-masks rows that would be fully masked (modeling_mask2former.py:1912-1914)
    mask[torch.where(mask.sum(-1) == mask.shape[-1])] = False
    return query, key, value, mask


def _modules(seed=0):
    torch.manual_seed(seed)
    ref = nn.MultiheadAttention(256, 8, 0.0).cuda()
    nn.init.normal_(ref.in_proj_bias, std=0.1)  # non-zero biases so the bias path is exercised
    nn.init.normal_(ref.out_proj.bias, std=0.1)
    hip = nn.MultiheadAttention(256, 8, 0.0).cuda()
    hip.load_state_dict(ref.state_dict())
    assert masked_attention.install_module(hip)
    return ref, hip


def _core64(q, k, v, mask, scale):
    """float64 restatement of F.multi_head_attention_forward's core on [Q|L, BH, 32] tensors."""
    q, k, v = (t.double().transpose(0, 1) for t in (q, k, v))
    s = torch.bmm(q * scale, k.transpose(1, 2)).masked_fill(mask, float("-inf"))
    return torch.bmm(torch.softmax(s, -1), v).transpose(0, 1)


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_core_forward_backward_vs_float64(shape):
    B, Q, L = shape
    g = torch.Generator(device="cuda").manual_seed(3)
    q = torch.randn((Q, B * 8, 32), generator=g, device="cuda", requires_grad=True)
    k = torch.randn((L, B * 8, 32), generator=g, device="cuda", requires_grad=True)
    v = torch.randn((L, B * 8, 32), generator=g, device="cuda", requires_grad=True)
    mask = torch.rand((B * 8, Q, L), generator=g, device="cuda") < 0.7
    mask[torch.where(mask.sum(-1) == L)] = False
    scale = math.sqrt(1.0 / 32)
    out = masked_attention.masked_attention(q, k, v, mask, scale)
    gout = torch.randn_like(out)
    out.backward(gout)
    q64, k64, v64 = (t.detach().double().requires_grad_() for t in (q, k, v))
    ref = _core64(q64, k64, v64, mask, scale)
    ref.backward(gout.double())
    assert float((out.double() - ref).abs().max()) <= 2e-6 * (1 + float(ref.abs().max()))
    for got, want, name in ((q.grad, q64.grad, "dq"), (k.grad, k64.grad, "dk"), (v.grad, v64.grad, "dv")):
        err = float((got.double() - want).abs().max())
        assert err <= 1e-5 * (1 + float(want.abs().max())), (name, err)


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_module_matches_torch_multihead_attention(shape):
    B, Q, L = shape
    ref, hip = _modules()
    query, key, value, mask = _inputs(B, Q, L, seed=B * Q + L)
    qs = [t.clone().requires_grad_() for t in (query, key, value)]
    qh = [t.clone().requires_grad_() for t in (query, key, value)]
    out_r, w_r = ref(*qs, attn_mask=mask, key_padding_mask=None)
    out_h, w_h = hip(*qh, attn_mask=mask, key_padding_mask=None)
    assert w_h is None and w_r is not None
    tol = 1e-5 * (1 + float(out_r.abs().max()))
    assert float((out_h - out_r).abs().max()) <= tol
    g = torch.randn_like(out_r)
    out_r.backward(g)
    out_h.backward(g)
    for a, b in zip(qs + list(ref.parameters()), qh + list(hip.parameters())):
        assert float((a.grad - b.grad).abs().max()) <= 2e-5 * (1 + float(a.grad.abs().max()))


@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_module_bf16_autocast_vs_torch(shape):
    """Under torch.autocast(bfloat16) — the bf16 configuration of the whole model — the module
    runs the kernels on the projections' bf16 q / k / v (weights None: not torch's path).  Stated
    tolerance: its error against the float32 module (outputs and every input / parameter
    gradient, max-abs relative to the max) is within 1.5x torch's own autocast error on the same
    inputs (+1e-3 slack: a handful of bf16 roundings either way)."""
    B, Q, L = shape
    ref, hip = _modules()
    query, key, value, mask = _inputs(B, Q, L, seed=7 * B + Q + L)

    def run(mod, amp):
        xs = [t.clone().requires_grad_() for t in (query, key, value)]
        mod.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out, w = mod(*xs, attn_mask=mask, key_padding_mask=None)
        g = torch.randn(out.shape, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
        out.float().backward(g)
        return out, w, [t.grad for t in xs] + [p.grad for p in mod.parameters()]
    o32, _, g32 = run(ref, False)
    ot, wt, gt = run(ref, True)
    oh, wh, gh = run(hip, True)
    assert wh is None and wt is not None and oh.dtype == ot.dtype == torch.bfloat16

    def rel(a, e):  # max-abs error relative to the max (floored: L = 1 has an exactly-zero dq)
        return float((a.float() - e).abs().max()) / max(float(e.abs().max()), 1e-3)
    et, eh = rel(ot, o32), rel(oh, o32)
    print(f"{shape}: output rel err torch-autocast {et:.3g}, hip {eh:.3g}")
    assert eh <= 1.5 * et + 1e-3
    for a, b, e in zip(gt, gh, g32):
        assert rel(b, e) <= 1.5 * rel(a, e) + 1e-3, (rel(b, e), rel(a, e))


@gpu
def test_fully_masked_row_is_nan_like_torch():
    ref, hip = _modules()
    query, key, value, mask = _inputs(1, 6, 40)
    mask[3, 2, :] = True                 # one fully masked (head, query) row
    out_r, _ = ref(query, key, value, attn_mask=mask)
    out_h, _ = hip(query, key, value, attn_mask=mask)
    assert bool(out_r[2, 0].isnan().all()) and bool(out_h[2, 0].isnan().all())
    ok = ~out_r.isnan()
    assert float((out_h[ok] - out_r[ok]).abs().max()) <= 1e-5 * (1 + float(out_r[ok].abs().max()))
    # backward (masked_attention.py docstring): the row's delta = rowsum(dO * O) is NaN, so NaN
    # reaches the gradients as in torch's backward (no silently finite gradient)
    qr = [t.clone().requires_grad_() for t in (query, key, value)]
    qh = [t.clone().requires_grad_() for t in (query, key, value)]
    out_r, _ = ref(*qr, attn_mask=mask)
    out_h, _ = hip(*qh, attn_mask=mask)
    g = torch.ones_like(out_h)
    g[2] = 0.0  # the NaN query row carries no upstream gradient
    torch.nan_to_num(out_r, nan=0.0).backward(g)
    torch.nan_to_num(out_h, nan=0.0).backward(g)
    assert not bool(qr[1].grad.isfinite().all()) and not bool(qh[1].grad.isfinite().all())


@gpu
def test_uncovered_inputs_fall_back_to_torch():
    ref, hip = _modules()
    query, key, value, mask = _inputs(1, 8, 30)
    out_r, w_r = ref(query, key, value, attn_mask=None)
    out_h, w_h = hip(query, key, value, attn_mask=None)    # no mask: torch's path, weights returned
    assert w_h is not None and torch.equal(out_h, out_r)
    hip.need_weights_output = True
    out_h, w_h = hip(query, key, value, attn_mask=mask)
    out_r, w_r = ref(query, key, value, attn_mask=mask)
    assert torch.equal(out_h, out_r) and torch.equal(w_h, w_r)


def test_install_in_decoder_layers():  # CPU: class swap only
    from transformers import Mask2FormerConfig
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerMaskedAttentionDecoder
    cfg = Mask2FormerConfig()
    dec = Mask2FormerMaskedAttentionDecoder(cfg)
    n = masked_attention.install(dec)
    assert n == cfg.decoder_layers - 1
    assert all(type(m) is masked_attention.HipMultiheadAttention for m in dec.modules()
               if isinstance(m, nn.MultiheadAttention))
    # output_attentions=True on a decoder layer: its cross-attention takes torch's path, which
    # returns the weights HF then hands back (the pre-hook install() registers)
    layer = dec.layers[0]
    masked_attention._layer_pre_hook(layer, (), {"output_attentions": True})
    assert layer.cross_attn._weights_consumed
    masked_attention._layer_pre_hook(layer, (), {"output_attentions": False})
    assert not layer.cross_attn._weights_consumed
    assert all(getattr(m, "_rgbd_attn_hook", None) is not None for m in dec.layers)
    assert masked_attention.uninstall(dec) == n
    assert all(getattr(m, "_rgbd_attn_hook", None) is None for m in dec.layers)
