"""Diagnostic: where the bf16-autocast FFN weight gradient departs from torch's (test_gpu_dense
test_linear_and_ffn_modules[bf16_autocast] measured 9 % on fc1.weight while dX matched)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import dense  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


dev = torch.device("cuda")
torch.manual_seed(0)
fc1, fc2 = torch.nn.Linear(256, 2048).to(dev), torch.nn.Linear(2048, 256).to(dev)
x = torch.randn((800, 256), device=dev)
gy = torch.randn((800, 256), device=dev)
xb, w1, w2 = x.bfloat16(), fc1.weight.bfloat16(), fc2.weight.bfloat16()
h = torch.relu(xb.float() @ w1.float().t() + fc1.bias).bfloat16()
g2 = gy.bfloat16()
dh_ref = ((g2.float() @ w2.float()) * (h.float() > 0))
dw1_ref = dh_ref.bfloat16().float().t() @ xb.float()
dh = dense.gemm(g2, w2, 0, 1, 800, 2048, 256, act=dense.ACT_RELU_GRAD, R=h)
print("dh vs f32 ref", rel(dh, dh_ref))
dw1 = dense.gemm(dh, xb, 1, 1, 2048, 256, 800, c_f32=True)
print("dw1 (c_f32) vs ref", rel(dw1, dw1_ref))
dw1b = dense.gemm(dh, xb, 1, 1, 2048, 256, 800)
print("dw1 (bf16 out) vs ref", rel(dw1b, dw1_ref))
dw1f = dense.gemm(dh.float(), xb.float(), 1, 1, 2048, 256, 800)
print("dw1 (f32 operands) vs ref", rel(dw1f, dw1_ref))
dw1t = dense.gemm(dh.t().contiguous(), xb.t().contiguous(), 0, 0, 2048, 256, 800, c_f32=True)
print("dw1 as (0,0) layout vs ref", rel(dw1t, dw1_ref))
xa = x.clone().requires_grad_()
with torch.autocast("cuda", dtype=torch.bfloat16):
    y = fc2(torch.relu(fc1(xa)))
y.float().backward(gy)
print("torch autocast fc1.weight.grad vs ref", rel(fc1.weight.grad, dw1_ref))

# float64 truth (no bf16 rounding anywhere) and where each bf16 rounding moves dW1
xd, w1d, w2d, gd = x.double(), fc1.weight.double(), fc2.weight.double(), gy.double()
zd = xd @ w1d.t() + fc1.bias.double()
hd = torch.relu(zd)
dhd = (gd @ w2d) * (zd > 0)
dw1_true = dhd.t() @ xd
print("truth |dW1| max", float(dw1_true.abs().max()), " sum|terms| / |sum| ~", float((dhd.abs().t() @ xd.abs()).max() / dw1_true.abs().max()))
print("ours vs truth", rel(dw1, dw1_true))
print("bf16 emulation vs truth", rel(dw1_ref, dw1_true))
print("torch autocast vs truth", rel(fc1.weight.grad, dw1_true))
dh_x32 = (gd @ w2d) * (zd > 0)
print("dW1 from f32 dh and bf16 X vs truth", rel(dhd.t() @ xb.double(), dw1_true))
print("dW1 from bf16 dh and f32 X vs truth", rel(dh.double().t() @ xd, dw1_true))
print("dh (ours) vs truth", rel(dh, dhd))
print("h>0 mask flips", int(((h.float() > 0) != (zd > 0)).sum()), "of", zd.numel())
