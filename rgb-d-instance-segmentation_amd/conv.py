"""f2: the remaining convolutions of the drop-in model as MFMA GEMMs (csrc/gemm.hip + csrc/conv.hip).

Reference call sites (custom_model.py:330 ``self.encoder(rgb)``, :383 ``self.decoder(...)``;
transformers 5.15):
  * modeling_swin.py ``SwinPatchEmbeddings.projection``: Conv2d(3, 96, kernel 4, stride 4);
  * modeling_mask2former.py ``Mask2FormerPixelDecoder``: the input projections
    Conv2d(C, 256, 1) (+ GroupNorm), the FPN lateral Conv2d(96, 256, 1, bias=False)
    (+ GroupNorm), the FPN output Conv2d(256, 256, 3, padding=1, bias=False) (+ GroupNorm +
    ReLU) and ``mask_projection`` Conv2d(256, 256, 1).

In NCHW every one of them is the batched GEMM  Y[b][o][p] = sum_k W[o][k] col[b][k][p] + bias[o]
(bias on the GEMM's rows: RGBD_BIAS_M), col = x for 1x1, the im2col of x otherwise
(rgbd_im2col: 3x3 stride 1 pad 1, 4x4 stride 4).  Backward:
  dW = sum_b dY_b col_b^T   (one batched GEMM, float32 per image, summed over the batch)
  dX = W^T dY               (1x1; 4x4: then the patches back in place)
       conv3x3(dY, W')      (3x3: W'[c][o][ky][kx] = W[o][c][2-ky][2-kx], the transposed
                             convolution as a plain one: im2col of dY and one GEMM)
  db = sum over images and pixels of dY.
Precision as the module being replaced: float32 in -> exact-f32 MFMA; under
torch.autocast(bfloat16) bf16 operands with float32 sums and a bf16 output (autocast's conv2d).
Shapes outside these (other kernels / strides / groups / dilations / padding modes, CPU
tensors) take nn.Conv2d's own path.
"""
import torch
from torch import nn

from . import _lib
from ._lib import check
from .dense import _CODE, cast_weight, compute_dtype, gemm
from .ops import _p, _stream

ACT_NONE = 0
BIAS_M = 16  # RGBD_BIAS_M


def _im2col(x, k):
    B, C, H, W = x.shape
    Ho, Wo = (H, W) if k == 3 else (H // 4, W // 4)
    col = torch.empty((B, C * k * k, Ho * Wo), dtype=x.dtype, device=x.device)
    check(_lib.lib().rgbd_im2col(_CODE[x.dtype], _p(x), B, C, H, W, k, _p(col), _stream(x.device)), "rgbd_im2col")
    return col


def _col(x, k):
    B, C, H, W = x.shape
    return x.reshape(B, C, H * W) if k == 1 else _im2col(x, k)


def _conv_gemm(w2, col, bias):
    """Y[b] = w2 [O][K] @ col[b] [K][N] (+ bias[o]) -> [B][O][N]."""
    B, K, N = col.shape
    O = w2.shape[0]
    return gemm(w2, col, 0, 1, O, N, K, bias=bias, act=ACT_NONE | (BIAS_M if bias is not None else 0), batch=B,
                sa=0, sb=K * N)


class ConvFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, k, dt):
        xc = x.to(dt).contiguous()
        B, C, H, W = xc.shape
        O = w.shape[0]
        Ho, Wo = (H, W) if k != 4 else (H // 4, W // 4)
        wc = cast_weight(w, dt).reshape(O, -1).contiguous()
        y = _conv_gemm(wc, _col(xc, k), b)
        ctx.save_for_backward(xc, wc)
        ctx.k, ctx.x_dtype, ctx.w_dtype, ctx.w_shape, ctx.has_b = k, x.dtype, w.dtype, w.shape, b is not None
        return y.view(B, O, Ho, Wo)

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        k = ctx.k
        B, C, H, W = xc.shape
        O, K = wc.shape
        g = gy.to(xc.dtype).contiguous().reshape(B, O, -1)
        N = g.shape[2]
        dx = dw = db = None
        if ctx.needs_input_grad[1]:
            col = _col(xc, k)
            dwb = gemm(g, col, 0, 0, O, K, N, c_f32=True, batch=B, sa=O * N, sb=K * N)
            dw = dwb.view(B, O, K).sum(0).reshape(ctx.w_shape).to(ctx.w_dtype)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = g.float().sum((0, 2))
        if ctx.needs_input_grad[0]:
            if k == 1:   # dX_b [C][N] = W^T [C][O] dY_b [O][N]
                dx = gemm(wc, g, 1, 1, C, N, O, batch=B, sa=0, sb=O * N).view(B, C, H, W)
            elif k == 3:  # the transposed convolution as a convolution of dY
                wt = wc.view(O, C, 3, 3).flip(2, 3).transpose(0, 1).reshape(C, O * 9).contiguous()
                dx = _conv_gemm(wt, _im2col(g.view(B, O, H, W), 3), None).view(B, C, H, W)
            else:         # 4x4 stride 4: dcol = W^T dY, each patch back in place
                Hp, Wp = H // 4, W // 4
                dcol = gemm(wc, g, 1, 1, K, N, O, batch=B, sa=0, sb=O * N)
                dx = dcol.view(B, C, 4, 4, Hp, Wp).permute(0, 1, 4, 2, 5, 3).reshape(B, C, H, W)
            dx = dx.to(ctx.x_dtype)
        return dx, dw, db, None, None


def _kind(m: nn.Conv2d, x):
    """1 / 3 / 4 for the shapes the GEMM path covers, else None."""
    if (not x.is_cuda or x.dim() != 4 or x.numel() == 0 or m.groups != 1 or m.dilation != (1, 1)
            or m.padding_mode != "zeros" or compute_dtype(x) is None):
        return None
    if m.kernel_size == (1, 1) and m.stride == (1, 1) and m.padding in ((0, 0), "valid"):
        return 1
    if m.kernel_size == (3, 3) and m.stride == (1, 1) and m.padding in ((1, 1), "same"):
        return 3
    if m.kernel_size == (4, 4) and m.stride == (4, 4) and m.padding in ((0, 0), "valid") \
            and x.shape[2] % 4 == 0 and x.shape[3] % 4 == 0:
        return 4
    return None


class HipConv2d(nn.Conv2d):
    def forward(self, x):
        k = _kind(self, x)
        if k is None:
            return super().forward(x)
        return ConvFunction.apply(x, self.weight, self.bias, k, compute_dtype(x))
