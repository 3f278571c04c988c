"""f2: the pixel decoder's multi-scale deformable attention on the HIP kernels.

Reference: ``Mask2FormerPixelDecoderEncoderMultiscaleDeformableAttention.forward`` and its core
``multi_scale_deformable_attention`` (transformers 5.15 modeling_mask2former.py:919-1014,
798-837): per encoder layer, value / offset / weight projections, softmax over levels x points,
sampling locations from the reference points, then per level a ``grid_sample`` over a transposed
copy of the value, stack, weight and sum.

``HipMSDeformAttn`` keeps the projections, the softmax and the location arithmetic as the same
torch calls and replaces the core with ``MSDeformAttnFunction`` (csrc/msda.hip: one fused gather
kernel forward, one fused backward with atomics for the value gradient).  ``install(model)``
swaps the class of every HF module in place (parameters / state_dict keys unchanged).
"""
import torch
from torch import nn
from transformers.models.mask2former.modeling_mask2former import (
    Mask2FormerPixelDecoderEncoderMultiscaleDeformableAttention as _HFMSDA)

from . import _lib, ops
from ._lib import RGBD_BF16, RGBD_F32, check

_CODE = {torch.float32: RGBD_F32, torch.bfloat16: RGBD_BF16}


class MSDeformAttnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, value, shapes, loc, attw):
        ctx.shapes = [tuple(int(x) for x in hw) for hw in shapes]
        ctx.save_for_backward(value, loc, attw)
        ctx.loc_dtype, ctx.attw_dtype = loc.dtype, attw.dtype
        return ops.msda_forward(value, ctx.shapes, loc, attw)

    @staticmethod
    def backward(ctx, gout):
        value, loc, attw = ctx.saved_tensors
        gv, gl, ga = ops.msda_backward(value, ctx.shapes, loc, attw, gout)
        return gv.to(value.dtype), None, gl.to(ctx.loc_dtype), ga.to(ctx.attw_dtype)


class MSDALocationsFunction(torch.autograd.Function):
    """ref[:, :, None, :, None, :] + offsets / norm[None, None, None, :, None, :] (:990-994) in
    one kernel (rgbd_msda_locations): the division in the offsets' dtype, the sum in float32, as
    torch evaluates the expression; its backward forms the offsets' gradient the same way."""

    @staticmethod
    def forward(ctx, ref, offsets, norm):
        B, Q, NH, L, P, _ = offsets.shape
        off = offsets.contiguous()
        r = ref.detach().float().contiguous()
        loc = torch.empty(off.shape, dtype=torch.float32, device=off.device)
        check(_lib.lib().rgbd_msda_locations(_CODE[off.dtype], ops._p(r), ops._p(off), ops._p(norm), B, Q, NH, L, P,
                                             ops._p(loc), ops._stream(off.device)), "rgbd_msda_locations")
        ctx.save_for_backward(norm)
        ctx.dims, ctx.off_dtype = (B, Q, NH, L, P), off.dtype
        return loc

    @staticmethod
    def backward(ctx, gloc):
        (norm,) = ctx.saved_tensors
        B, Q, NH, L, P = ctx.dims
        g = gloc.float().contiguous()
        goff = torch.empty(g.shape, dtype=ctx.off_dtype, device=g.device)
        check(_lib.lib().rgbd_msda_locations_bwd(_CODE[ctx.off_dtype], ops._p(g), ops._p(norm), B, Q, NH, L, P,
                                                 ops._p(goff), ops._stream(g.device)), "rgbd_msda_locations_bwd")
        gref = g.sum(dim=(2, 4)) if ctx.needs_input_grad[0] else None
        return gref, goff, None


def location_norm(spatial_shapes_list, dtype, device):
    """The (w, h) normaliser of every level as float32 for rgbd_msda_locations.  The reference
    divides the offsets by an int64 tensor (modeling_mask2former.py:994-1001), which torch first
    casts to the offsets' dtype: for bf16 offsets a level size bf16 cannot hold (odd sizes above
    256) is rounded to bf16 the same way here."""
    rnd = (lambda v: float(torch.tensor(float(v)).to(dtype)))
    return ops.device_const([[rnd(w), rnd(h)] for h, w in spatial_shapes_list], torch.float32, device)


def multi_scale_deformable_attention(value, value_spatial_shapes, sampling_locations, attention_weights):
    """Drop-in for the reference function of the same name (same arguments, same output)."""
    return MSDeformAttnFunction.apply(value, value_spatial_shapes, sampling_locations, attention_weights)


class HipMSDeformAttn(_HFMSDA):
    def forward(self, hidden_states, attention_mask=None, encoder_hidden_states=None, encoder_attention_mask=None,
                position_embeddings=None, reference_points=None, spatial_shapes_list=None, level_start_index=None,
                output_attentions=False):
        if position_embeddings is not None:
            hidden_states = hidden_states + position_embeddings
        B, Q, _ = hidden_states.shape
        _, S, _ = encoder_hidden_states.shape
        if sum(h * w for h, w in spatial_shapes_list) != S:
            raise ValueError("Make sure to align the spatial shapes with the sequence length of the encoder hidden states")
        value = self.value_proj(encoder_hidden_states)
        if attention_mask is not None:
            value = value.masked_fill(attention_mask[..., None], float(0))
        value = value.view(B, S, self.n_heads, self.d_model // self.n_heads)
        offsets = self.sampling_offsets(hidden_states).view(B, Q, self.n_heads, self.n_levels, self.n_points, 2)
        weights = self.attention_weights(hidden_states).view(B, Q, self.n_heads, self.n_levels * self.n_points)
        weights = nn.functional.softmax(weights, -1).view(B, Q, self.n_heads, self.n_levels, self.n_points)
        if reference_points.shape[-1] == 2 and offsets.dtype in (torch.float32, torch.bfloat16):
            norm = location_norm(spatial_shapes_list, offsets.dtype, reference_points.device)
            loc = MSDALocationsFunction.apply(reference_points, offsets, norm)
        elif reference_points.shape[-1] == 2:
            norm = ops.device_const([[w, h] for h, w in spatial_shapes_list], torch.long, reference_points.device)
            loc = reference_points[:, :, None, :, None, :] + offsets / norm[None, None, None, :, None, :]
        elif reference_points.shape[-1] == 4:
            loc = (reference_points[:, :, None, :, None, :2]
                   + offsets / self.n_points * reference_points[:, :, None, :, None, 2:] * 0.5)
        else:
            raise ValueError(f"Last dim of reference_points must be 2 or 4, but got {reference_points.shape[-1]}")
        out = multi_scale_deformable_attention(value, spatial_shapes_list, loc, weights)
        return self.output_proj(out), weights


def install(model: nn.Module) -> int:
    n = 0
    for m in model.modules():
        if type(m) is _HFMSDA:
            m.__class__ = HipMSDeformAttn
            n += 1
    return n


def uninstall(model: nn.Module) -> int:
    n = 0
    for m in model.modules():
        if type(m) is HipMSDeformAttn:
            m.__class__ = _HFMSDA
            n += 1
    return n
