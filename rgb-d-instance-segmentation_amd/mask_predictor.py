"""f1: the Mask2Former mask predictor on the HIP kernels.

Reference: ``Mask2FormerMaskPredictor`` (transformers 5.15 modeling_mask2former.py:2018-2056),
which produces the mask logits graded by BASELINE's 1e-3 criterion and, from them, the
binarised attention mask of the next masked-attention decoder layer (:1896, :1929).

``HipMaskPredictor`` is that class with ``forward`` replaced — same constructor, same
``mask_embedder`` parameters (state_dict keys unchanged), same outputs:
    mask_embeddings = mask_embedder(outputs.transpose(0, 1))      3-layer MLP, torch (tiny GEMMs)
    outputs_mask    = einsum(bqc,bchw->bqhw)                       K: rgbd_mask_logits (MFMA)
    attention_mask  = bilinear -> sigmoid -> < 0.5, x heads        K: rgbd_mask_attention
Backward of the einsum (grads for the mask embeddings and the pixel-decoder mask features) is
two batched HIP GEMMs (csrc/gemm.hip: d_emb = g pix^T split over the pixels, d_pix = emb^T g);
the attention mask is detached as in the reference.  ``install(model)`` swaps the class of the decoder's predictor in place (no
re-initialisation, no parameter change).
"""
import torch
from torch import nn
from transformers.models.mask2former.modeling_mask2former import Mask2FormerMaskPredictor

from . import dense, ops


class MaskLogitsFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, emb, pix):
        ctx.save_for_backward(emb, pix)
        return ops.mask_logits(emb, pix)

    @staticmethod
    def backward(ctx, g):
        emb, pix = ctx.saved_tensors
        B, Q, C = emb.shape
        emb = emb.contiguous()
        g2 = g.reshape(B, Q, -1).to(pix.dtype).contiguous()
        P = g2.shape[2]
        p2 = pix.reshape(B, C, P).contiguous()
        d_emb = d_pix = None
        if ctx.needs_input_grad[0]:   # d_emb[b] = g[b] pix[b]^T: K = pixels, split-K
            d_emb = dense.gemm(g2, p2, 0, 0, Q, C, P, batch=B, sa=Q * P, sb=C * P).reshape(emb.shape)
        if ctx.needs_input_grad[1]:   # d_pix[b] = emb[b]^T g[b]: K = queries
            d_pix = dense.gemm(emb, g2, 1, 1, C, P, Q, batch=B, sa=Q * C, sb=Q * P).reshape(pix.shape)
        return d_emb, d_pix


def mask_logits(emb, pix):
    if emb.dtype != pix.dtype:  # einsum under autocast / mixed inputs: compute in the wider type
        dt = torch.promote_types(emb.dtype, pix.dtype)
        emb, pix = emb.to(dt), pix.to(dt)
    return MaskLogitsFunction.apply(emb, pix)


class HipMaskPredictor(Mask2FormerMaskPredictor):
    def forward(self, outputs: torch.Tensor, pixel_embeddings: torch.Tensor, attention_mask_target_size=None):
        mask_embeddings = self.mask_embedder(outputs.transpose(0, 1))            # :2043
        outputs_mask = mask_logits(mask_embeddings, pixel_embeddings)             # :2046
        with torch.no_grad():                                                     # :2048-2054
            attention_mask = ops.mask_attention(outputs_mask.detach(), attention_mask_target_size, self.num_heads)
        return outputs_mask, attention_mask


def install(model: nn.Module) -> int:
    """Swap every Mask2FormerMaskPredictor inside ``model`` for the HIP one; returns the count."""
    n = 0
    for m in model.modules():
        if type(m) is Mask2FormerMaskPredictor:
            m.__class__ = HipMaskPredictor
            n += 1
    return n


def uninstall(model: nn.Module) -> int:
    """Inverse of ``install`` (tests run the reference HF predictor on the CPU as the checker)."""
    n = 0
    for m in model.modules():
        if type(m) is HipMaskPredictor:
            m.__class__ = Mask2FormerMaskPredictor
            n += 1
    return n
