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

from . import ops


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
        if reference_points.shape[-1] == 2:
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
