"""f1: the masked cross-attention of the Mask2Former decoder layers on HIP kernels.

Reference: each ``Mask2FormerMaskedAttentionDecoderLayer`` (transformers 5.15
modeling_mask2former.py:1627-1654) calls ``nn.MultiheadAttention`` with the boolean mask the
mask predictor produced (:2048-2055) — 9 calls per forward over the three pixel-decoder levels.
torch's math path (need_weights=True, F.multi_head_attention_forward) does, per batch*head bh:
    q, k, v = linear(query / key / value, in_proj chunks)            library GEMMs
    S = (q * head_dim^-1/2) k^T + where(mask, -inf, 0); P = softmax(S); O = P v
    out = linear(O, out_proj)                                         library GEMM
``HipMultiheadAttention`` runs the projections on the HIP GEMMs (rgbd_amd/dense.py) and the masked
softmax-attention core (scores, mask, softmax, P.V and the backward) as the HIP kernels
``rgbd_masked_attn_fwd`` / ``_bwd`` (csrc/masked_attn.hip), on the projections' own
sequence-major layout (no head transposes, no [BH, Q, L] score tensor in HBM).

Differences from the torch module, by design: the attention weights (the second output) are not
materialised — HF's decoder layer calls the module with the default ``need_weights=True`` whether
or not anyone reads the weights, so the module takes torch's path (weights returned) only when
they are consumed: ``need_weights_output`` set on the module, or the decoder layer called with
``output_attentions=True`` (``install`` registers a forward pre-hook on each decoder layer that
tells its ``cross_attn`` so).  Inputs the kernels do not cover (a key padding mask, a float
mask, dropout in training, head_dim != 32, batch_first, float16) also go through torch's path
unchanged.  Under torch.autocast(bfloat16) the projections run as autocast runs them (bf16
GEMMs) and the core reads their bf16 q / k / v (float32 arithmetic, bf16 output, as torch's
autocast math path returns).
``install(model)`` swaps the class of the decoder layers' ``cross_attn`` modules in place (same
parameters, same state_dict keys).

A query row whose every key is masked: torch's softmax gives NaN for the row, and so do the
kernels (log-sum-exp +inf).  In the backward the row's delta = rowsum(dO * O) is NaN, so NaN
reaches the key gradient of that batch-head (and through it the projections' gradients), as
NaN reaches torch's (which also spreads it into dq and dv).  HF's decoder un-masks such rows
before the call (modeling_mask2former.py:2054-2055), so the model never reaches this case.
"""
import math

import torch
from torch import nn

from . import _lib
from ._lib import check
from .ops import _dtype_code, _need_cuda, _p, _stream


class MaskedAttentionFunction(torch.autograd.Function):
    """q [Q, BH, 32], k / v [L, BH, 32] float32 or bfloat16 (one dtype, contiguous), mask bool
    [BH, Q, L] -> o [Q, BH, 32] of the same dtype (float32 arithmetic either way)."""

    @staticmethod
    def forward(ctx, q, k, v, mask, scale):
        _need_cuda(q, k, v, mask)
        if not (q.dtype == k.dtype == v.dtype) or q.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("masked attention: q, k, v must share one dtype, float32 or bfloat16")
        Q, BH, hd = q.shape
        L = k.shape[0]
        out = torch.empty_like(q)
        lse = torch.empty((Q, BH), dtype=torch.float32, device=q.device)
        L_ = _lib.lib()
        ws = torch.empty((L_.rgbd_masked_attn_fwd_workspace_size(BH, Q, L),), dtype=torch.uint8, device=q.device)
        check(L_.rgbd_masked_attn_fwd(_dtype_code(q), _p(q), _p(k), _p(v), _p(mask), BH, Q, L, hd, float(scale),
                                      _p(out), _p(lse), _p(ws), _stream(q.device)), "rgbd_masked_attn_fwd")
        ctx.save_for_backward(q, k, v, mask, out, lse)
        ctx.scale = float(scale)
        return out

    @staticmethod
    def backward(ctx, gout):
        q, k, v, mask, out, lse = ctx.saved_tensors
        Q, BH, hd = q.shape
        L = k.shape[0]
        g = gout.to(q.dtype).contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        L_ = _lib.lib()
        ws = torch.empty((L_.rgbd_masked_attn_bwd_workspace_size(BH, Q, L),), dtype=torch.uint8, device=q.device)
        check(L_.rgbd_masked_attn_bwd(_dtype_code(q), _p(q), _p(k), _p(v), _p(mask), _p(out), _p(lse), _p(g), BH, Q,
                                      L, hd, ctx.scale, _p(dq), _p(dk), _p(dv), _p(ws), _stream(q.device)),
              "rgbd_masked_attn_bwd")
        return dq, dk, dv, None, None


def masked_attention(q, k, v, mask, scale):
    return MaskedAttentionFunction.apply(q.contiguous(), k.contiguous(), v.contiguous(),
                                         None if mask is None else mask.contiguous(), scale)


class HipMultiheadAttention(nn.MultiheadAttention):
    need_weights_output = False
    _weights_consumed = False  # set per call by the decoder layer's pre-hook (install)

    def _hip_ok(self, query, key, value, key_padding_mask, attn_mask, is_causal):
        E = self.embed_dim
        # float32 or bfloat16 inputs; under autocast only bfloat16 (the projections then produce
        # bf16 q / k / v, and the kernels read them as such)
        amp = torch.is_autocast_enabled("cuda")
        return (query.is_cuda and query.dtype == key.dtype == value.dtype
                and query.dtype in (torch.float32, torch.bfloat16)
                and (not amp or torch.get_autocast_dtype("cuda") == torch.bfloat16)
                and not self.batch_first and self._qkv_same_embed_dim and self.in_proj_bias is not None
                and self.bias_k is None and not self.add_zero_attn and key_padding_mask is None
                and not is_causal and E // self.num_heads == 32 and (self.dropout == 0.0 or not self.training)
                and attn_mask is not None and attn_mask.dtype == torch.bool and attn_mask.dim() == 3
                and query.dim() == 3 and key.shape == value.shape
                and tuple(attn_mask.shape) == (query.shape[1] * self.num_heads, query.shape[0], key.shape[0]))

    def forward(self, query, key, value, key_padding_mask=None, need_weights=True, attn_mask=None,
                average_attn_weights=True, is_causal=False):
        wants = need_weights and (self.need_weights_output or self._weights_consumed)
        if wants or not self._hip_ok(query, key, value, key_padding_mask, attn_mask, is_causal):
            return super().forward(query, key, value, key_padding_mask=key_padding_mask, need_weights=need_weights,
                                   attn_mask=attn_mask, average_attn_weights=average_attn_weights,
                                   is_causal=is_causal)
        Q, B, E = query.shape
        L = key.shape[0]
        H = self.num_heads
        w_q, w_k, w_v = self.in_proj_weight.chunk(3)
        b_q, b_k, b_v = self.in_proj_bias.chunk(3)
        from .dense import linear  # the projections on the HIP GEMMs (f1 dense layers)
        q = linear(query, w_q, b_q).view(Q, B * H, E // H)
        k = linear(key, w_k, b_k).view(L, B * H, E // H)
        v = linear(value, w_v, b_v).view(L, B * H, E // H)
        scale = math.sqrt(1.0 / float(E // H))  # torch's q scaling
        o = masked_attention(q, k, v, attn_mask, scale)
        out = linear(o.view(Q * B, E), self.out_proj.weight, self.out_proj.bias).view(Q, B, E)
        return out, None


def install_module(m: nn.Module) -> bool:
    """Swap one nn.MultiheadAttention for the HIP one in place (same parameters)."""
    if type(m) is not nn.MultiheadAttention:
        return False
    m.__class__ = HipMultiheadAttention
    return True


def _layer_pre_hook(layer, args, kwargs):
    """Tell the layer's cross-attention whether this call's attention weights are returned."""
    ca = layer.cross_attn
    if isinstance(ca, HipMultiheadAttention):
        ca._weights_consumed = bool(kwargs.get("output_attentions", False))
    return None


def install(model: nn.Module) -> int:
    """Swap the decoder layers' cross-attention modules for the HIP one; returns the count."""
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerMaskedAttentionDecoderLayer
    n = 0
    for m in model.modules():
        if isinstance(m, Mask2FormerMaskedAttentionDecoderLayer):
            if install_module(m.cross_attn):
                n += 1
                if getattr(m, "_rgbd_attn_hook", None) is None:
                    m._rgbd_attn_hook = m.register_forward_pre_hook(_layer_pre_hook, with_kwargs=True)
    return n


def uninstall(model: nn.Module) -> int:
    n = 0
    for m in model.modules():
        if type(m) is HipMultiheadAttention:
            m.__class__ = nn.MultiheadAttention
            m.__dict__.pop("_weights_consumed", None)
            n += 1
        hook = getattr(m, "_rgbd_attn_hook", None)
        if hook is not None:
            hook.remove()
            m._rgbd_attn_hook = None
    return n
