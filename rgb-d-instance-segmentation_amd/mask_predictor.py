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
from transformers.models.mask2former.modeling_mask2former import (Mask2FormerMaskPredictor,
                                                                  Mask2FormerTransformerModule)

from . import _lib, dense, ops
from ._lib import RGBD_BF16, RGBD_F32, check


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


class LevelMemoryFunction(torch.autograd.Function):
    """(proj.flatten(2) + embed[None, :, None]).permute(2, 0, 1) — one feature level's decoder
    memory (modeling_mask2former.py:2102-2109) — written as a contiguous float32 [HW, B, C] by
    rgbd_level_memory_fwd; the backward transposes the gradient back into proj's dtype and sums
    it over pixels and images for the level embedding in the same pass."""

    @staticmethod
    def forward(ctx, proj, embed):
        B, C = proj.shape[:2]
        HW = proj.numel() // (B * C)
        p = proj.contiguous()
        e = embed.detach().float().contiguous()
        out = torch.empty((HW, B, C), dtype=torch.float32, device=proj.device)
        code = RGBD_BF16 if p.dtype == torch.bfloat16 else RGBD_F32
        check(_lib.lib().rgbd_level_memory_fwd(code, ops._p(p), ops._p(e), B, C, HW, ops._p(out),
                                               ops._stream(proj.device)), "rgbd_level_memory_fwd")
        ctx.shape, ctx.dtype, ctx.e_dtype = proj.shape, p.dtype, embed.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        HW, B, C = g.shape
        g = g.float().contiguous()
        dproj = torch.empty(ctx.shape, dtype=ctx.dtype, device=g.device)
        de = torch.empty((C,), dtype=torch.float32, device=g.device)
        L = _lib.lib()
        ws = ops._workspace(g.device, L.rgbd_level_memory_workspace_size(B, C, HW), "level_mem")
        code = RGBD_BF16 if ctx.dtype == torch.bfloat16 else RGBD_F32
        check(L.rgbd_level_memory_bwd(code, ops._p(g), B, C, HW, ops._p(dproj), ops._p(de), ops._p(ws),
                                      ops._stream(g.device)), "rgbd_level_memory_bwd")
        return dproj, de.to(ctx.e_dtype)


def level_memory(proj, embed):
    if proj.is_cuda and proj.dtype in (torch.float32, torch.bfloat16) and proj.dim() >= 3 and embed.dim() == 1:
        return LevelMemoryFunction.apply(proj, embed)
    return (proj.flatten(2) + embed[None, :, None]).permute(2, 0, 1)


class HipTransformerModule(Mask2FormerTransformerModule):
    """Mask2FormerTransformerModule with each level's memory from level_memory (the input
    projection + level embedding + permute of :2095-2109 in one kernel each way); the decoder
    call is the library's."""

    def forward(self, multi_scale_features, mask_features, output_hidden_states=False, output_attentions=False):
        feats, poss, sizes = [], [], []
        for i in range(self.num_feature_levels):
            f = multi_scale_features[i]
            sizes.append(f.shape[-2:])
            pos = self.position_embedder(f.shape, f.device, f.dtype, None).flatten(2)
            poss.append(pos.permute(2, 0, 1))
            feats.append(level_memory(self.input_projections[i](f), self.level_embed.weight[i]))
        batch_size = feats[0].shape[1]
        query_embeddings = self.queries_embedder.weight.unsqueeze(1).repeat(1, batch_size, 1)
        query_features = self.queries_features.weight.unsqueeze(1).repeat(1, batch_size, 1)
        return self.decoder(inputs_embeds=query_features, multi_stage_positional_embeddings=poss,
                            pixel_embeddings=mask_features, encoder_hidden_states=feats,
                            query_position_embeddings=query_embeddings, feature_size_list=sizes,
                            output_hidden_states=output_hidden_states, output_attentions=output_attentions,
                            return_dict=True)


def install(model: nn.Module) -> int:
    """Swap every Mask2FormerMaskPredictor inside ``model`` for the HIP one (and the transformer
    module around it for HipTransformerModule); returns the number of predictors swapped."""
    n = 0
    for m in model.modules():
        if type(m) is Mask2FormerMaskPredictor:
            m.__class__ = HipMaskPredictor
            n += 1
        if type(m) is Mask2FormerTransformerModule:
            m.__class__ = HipTransformerModule
    return n


def uninstall(model: nn.Module) -> int:
    """Inverse of ``install`` (tests run the reference HF predictor on the CPU as the checker)."""
    n = 0
    for m in model.modules():
        if type(m) is HipMaskPredictor:
            m.__class__ = Mask2FormerMaskPredictor
            n += 1
        if type(m) is HipTransformerModule:
            m.__class__ = Mask2FormerTransformerModule
    return n
