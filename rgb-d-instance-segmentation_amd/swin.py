"""f2: the Swin-T backbone's layers on the HIP kernels, forward only.

The reference calls the backbone at custom_model.py:330 and detaches its four feature maps
twice (:332-333), so v0.4.0 trains nothing inside it (Q1); the drop-in runs it under
torch.no_grad() and ``HipSwinLayer`` replaces ``SwinLayer.forward`` (transformers 5.15
modeling_swin.py:529-582) with

    h  = LayerNorm_before(x)                                   rgbd_layernorm_fwd
    qkv = h [Wq; Wk; Wv]^T + [bq; bk; bv]                      one rgbd_gemm (N = 3C)
    o  = window attention (pad, roll, 7x7 windows, relative-position bias, shift mask, softmax,
         P.V, un-window, roll back, crop)                      rgbd_swin_window_attn
    x  = x + o Wo^T + bo                                       rgbd_gemm, residual in the epilogue
    x  = x + GELU(LayerNorm_after(x) W1^T + b1) W2^T + b2      LayerNorm, rgbd_gemm (GELU in the
                                                               epilogue), rgbd_gemm (+ residual)

Under torch.autocast(bfloat16) the GEMMs and the attention take bf16 operands and the residual
stream stays float32 (autocast's LayerNorm returns float32, and float32 + bf16 promotes), as in
the HF layer.  DropPath in training draws its per-sample masks with the HF module itself, in
the HF order (attention branch only, as this SwinLayer applies it), and is applied outside
the GEMM epilogue.  Calls the kernels do not cover
(gradients required, a window shrunk below 7 for tiny inputs, float16, attention dropout in
training) run the HF forward.
"""
import torch
from torch import nn

from . import _lib
from ._lib import check
from .dense import _CODE, ACT_GELU, LayerNormFunction, cast_weight, compute_dtype, gemm
from .ops import _p, _stream

def _qkv_weights(attn, dt):
    """[Wq; Wk; Wv] in dt and [bq; bk; bv] float32, cached on the attention module under the
    same key as dense.cast_weight (address, version, optimizer-step epoch of all six tensors):
    the backbone is frozen in v0.4.0 (Q1), so this is built once."""
    ps = (attn.q_proj.weight, attn.k_proj.weight, attn.v_proj.weight)
    bs = (attn.q_proj.bias, attn.k_proj.bias, attn.v_proj.bias)
    key = tuple((t.data_ptr(), t._version, getattr(t, "_rgbd_epoch", 0)) for t in ps + bs if t is not None) + (dt,)
    hit = getattr(attn, "_rgbd_qkv", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    w = torch.cat([cast_weight(p, dt) for p in ps], 0).contiguous()
    b = None if bs[0] is None else torch.cat([x.detach().float() for x in bs], 0).contiguous()
    attn._rgbd_qkv = (key, (w, b))
    return w, b


def window_attention(qkv, bqkv, table, B, H, W, heads, shift, scale):
    """qkv [B*H*W, 3C] (q | k | v) -> out [B*H*W, C] of the same dtype."""
    C = qkv.shape[1] // 3
    out = torch.empty((qkv.shape[0], C), dtype=qkv.dtype, device=qkv.device)
    bq = bk = bv = None
    if bqkv is not None:
        bq, bk, bv = bqkv[:C], bqkv[C:2 * C], bqkv[2 * C:]
    t32 = table.detach().float().contiguous()
    check(_lib.lib().rgbd_swin_window_attn(_CODE[qkv.dtype], _p(qkv), _p(qkv[:, C:]), _p(qkv[:, 2 * C:]),
                                           qkv.stride(0), _p(bq), _p(bk), _p(bv), _p(t32), B, H, W, heads, 7,
                                           int(shift), float(scale), _p(out), C, _stream(qkv.device)),
          "rgbd_swin_window_attn")
    return out


def _covered(layer, x):
    attn = layer.attention
    return (x.is_cuda and compute_dtype(x) is not None and not torch.is_grad_enabled()
            and int(layer.window_size) == 7 and attn.head_dim == 32
            and layer.attention.relative_position_bias.window_size == (7, 7)
            and (not layer.training or (attn.attention_dropout == 0.0 and layer.dropout.p == 0.0)))


def _make_layer_class():
    from transformers.models.swin.modeling_swin import SwinLayer

    class HipSwinLayer(SwinLayer):
        def forward(self, hidden_states, input_dimensions, always_partition=False, **kwargs):
            if not always_partition:
                self.set_shift_and_window_size(input_dimensions)
            if not _covered(self, hidden_states) or kwargs.get("output_attentions"):
                return super().forward(hidden_states, input_dimensions, always_partition=True, **kwargs)
            H, W = input_dimensions
            B, N, C = hidden_states.shape
            attn = self.attention
            dt = compute_dtype(hidden_states)
            x = hidden_states.reshape(B * N, C)
            if x.dtype not in _CODE:
                x = x.float()
            x = x.contiguous()
            res_f32 = x.dtype == torch.float32
            # LayerNorm straight to the GEMM operand dtype (= autocast's float32 LayerNorm rounded
            # by the Linear's input cast)
            ln1, ln2 = self.layernorm_before, self.layernorm_after
            h = LayerNormFunction.apply(x, ln1.weight, ln1.bias, ln1.eps, dt)
            wqkv, bqkv = _qkv_weights(attn, dt)
            qkv = gemm(h, wqkv, 0, 0, B * N, 3 * C, C, bias=bqkv)
            o = window_attention(qkv, bqkv, attn.relative_position_bias.relative_position_bias_table, B, H, W,
                                 attn.num_attention_heads, int(self.shift_size), attn.scaling)
            wo = cast_weight(attn.o_proj.weight, dt)
            drop = self.training and not isinstance(self.drop_path, nn.Identity)
            if drop:  # DropPath's masks from the HF module, then the residual add
                a = gemm(o, wo, 0, 0, B * N, C, C, bias=attn.o_proj.bias)
                x = x + self.drop_path(a.view(B, N, C)).reshape(B * N, C)
            else:
                x = gemm(o, wo, 0, 0, B * N, C, C, bias=attn.o_proj.bias, R=x, c_f32=res_f32 and dt != torch.float32)
            h2 = LayerNormFunction.apply(x, ln2.weight, ln2.bias, ln2.eps, dt)
            mlp = self.mlp
            F_ = mlp.fc1.weight.shape[0]
            gelu = getattr(mlp.activation_fn, "__class__", None).__name__ in ("GELUActivation",)
            m = gemm(h2, cast_weight(mlp.fc1.weight, dt), 0, 0, B * N, F_, C,
                     bias=mlp.fc1.bias, act=ACT_GELU if gelu else 0)
            if not gelu:
                m = mlp.activation_fn(m)
            # the MLP branch has no DropPath in this SwinLayer (:578-580), only dropout (p = 0)
            x = gemm(m, cast_weight(mlp.fc2.weight, dt), 0, 0, B * N, C, F_, bias=mlp.fc2.bias, R=x,
                     c_f32=res_f32 and dt != torch.float32)
            return x.view(B, N, C).to(hidden_states.dtype), None

    return SwinLayer, HipSwinLayer


_CLS = []


def install(model: nn.Module) -> int:
    if not _CLS:
        _CLS.extend(_make_layer_class())
    base, cls = _CLS
    n = 0
    for m in model.modules():
        if type(m) is base:
            m.__class__ = cls
            n += 1
    return n


def uninstall(model: nn.Module) -> int:
    if not _CLS:
        return 0
    base, cls = _CLS
    n = 0
    for m in model.modules():
        if type(m) is cls:
            m.__class__ = base
            n += 1
    return n
