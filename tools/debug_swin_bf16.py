"""Diagnostic: the first non-finite intermediate of HipSwinLayer's bf16 path (test_gpu_swin
bf16_autocast arms measured NaN at stage 1 while the float32 arms match HF to 1e-6)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense, swin  # noqa: E402
from rgbd_amd.dense import LayerNormFunction, cast_weight, gemm  # noqa: E402


def fin(name, t):
    ok = bool(torch.isfinite(t.float()).all())
    print(f"{name:28s} {str(tuple(t.shape)):18s} {str(t.dtype):15s} finite={ok} max={float(t.float().abs().max()):.4g}")
    return ok


dev = torch.device("cuda")
torch.manual_seed(3)
C, heads, H, W, B = 96, 3, 60, 80, 2
from transformers.models.swin.modeling_swin import SwinLayer  # noqa: E402
from rgbd_amd.config import standard_config  # noqa: E402
cfg = standard_config(48).backbone_config
layer = SwinLayer(cfg, C, (H, W), heads, shift_size=3).to(dev).eval()
x = torch.randn((B * H * W, C), device=dev)
dt = torch.bfloat16
ln1 = layer.layernorm_before
h = LayerNormFunction.apply(x, ln1.weight, ln1.bias, ln1.eps, dt)
fin("ln_before (bf16 out)", h)
h32 = LayerNormFunction.apply(x, ln1.weight, ln1.bias, ln1.eps, torch.float32)
fin("ln_before (f32 out)", h32)
print("ln bf16 vs f32", float((h.float() - h32).abs().max()))
wqkv, bqkv = swin._qkv_weights(layer.attention, dt)
fin("wqkv", wqkv)
qkv = gemm(h, wqkv, 0, 0, B * H * W, 3 * C, C, bias=bqkv)
fin("qkv", qkv)
ref_qkv = h.float() @ wqkv.float().t() + bqkv
print("qkv vs ref", float((qkv.float() - ref_qkv).abs().max()))
for shift in (0, 3):
    o = swin.window_attention(qkv, bqkv, layer.attention.relative_position_bias.relative_position_bias_table, B, H,
                              W, heads, shift, layer.attention.scaling)
    fin(f"window attn bf16 shift {shift}", o)
    o32 = swin.window_attention(qkv.float(), bqkv, layer.attention.relative_position_bias.relative_position_bias_table,
                                B, H, W, heads, shift, layer.attention.scaling)
    fin(f"window attn f32 shift {shift}", o32)
    print("  bf16 vs f32", float((o.float() - o32).abs().max()))
wo = cast_weight(layer.attention.o_proj.weight, dt)
x2 = gemm(o, wo, 0, 0, B * H * W, C, C, bias=layer.attention.o_proj.bias, R=x, c_f32=True)
fin("o_proj + residual (c_f32)", x2)
ref = o.float() @ wo.float().t() + layer.attention.o_proj.bias + x
print("  vs ref", float((x2 - ref).abs().max()))
m = gemm(h, cast_weight(layer.mlp.fc1.weight, dt), 0, 0, B * H * W, 4 * C, C, bias=layer.mlp.fc1.bias,
         act=dense.ACT_GELU)
fin("fc1 + gelu", m)
