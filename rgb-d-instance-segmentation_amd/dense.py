"""f1 / f2: the dense layers around the HIP attention cores — nn.Linear, the
fc1 -> ReLU -> fc2 feed-forward blocks and nn.LayerNorm — on the HIP GEMM / LayerNorm kernels
(csrc/gemm.hip, csrc/layernorm.hip), forward and backward.

Reference call sites (transformers 5.15, the modules the reference model instantiates through
``CustomMask2FormerForUniversalSegmentation``, custom_model.py:37-53):
  * masked-attention decoder layer ``Mask2FormerMaskedAttentionDecoderLayer.forward_post``
    (modeling_mask2former.py:1627-1683): cross-attention projections, self-attention
    (``Mask2FormerAttention`` :1487-1585, no mask: the HIP attention core with a NULL mask),
    fc1 -> relu -> fc2, three post-norm LayerNorms;
  * pixel decoder encoder layer ``Mask2FormerPixelDecoderEncoderLayer.forward`` (:1036-1102):
    deformable-attention projections, fc1 -> relu -> fc2, two LayerNorms;
  * Swin-T (modeling_swin.py): every nn.Linear / nn.LayerNorm of the backbone (forward only in
    v0.4.0: the reference detaches the colour features, custom_model.py:332-333).

Precision follows the module being replaced: float32 inputs run the exact-f32 MFMA GEMMs; under
torch.autocast(bfloat16) the GEMMs take bf16 operands (activations and weights cast per call)
with float32 sums and a bf16 output — what autocast's linear returns — and
LayerNorm returns float32, as autocast's layer_norm does.  Weight gradients are written in
float32 straight from the bf16 GEMM (autocast's path rounds them to bf16 first).

``install(model)`` swaps module classes in place (parameters and state_dict keys unchanged):
nn.Conv2d -> conv.HipConv2d (1x1, 3x3 and Swin's 4x4 patch embedding as GEMMs), nn.Linear -> HipLinear, nn.LayerNorm -> HipLayerNorm, the decoder and pixel-decoder encoder
layers -> classes whose forward fuses the ReLU into fc1's epilogue and its gradient into
fc2's dX epilogue.  Inputs the kernels do not cover (CPU tensors, float16, LayerNorm width
> 1536, dropout in training, GELU with gradients) take the module's own torch path.
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from ._lib import RGBD_BF16, RGBD_F32, check
from .ops import _p, _stream, _workspace

ACT_NONE, ACT_RELU, ACT_GELU, ACT_RELU_GRAD = 0, 1, 2, 3
_CODE = {torch.float32: RGBD_F32, torch.bfloat16: RGBD_BF16}


def compute_dtype(x: torch.Tensor):
    """The dtype a replaced module computes in for input x (None: not covered)."""
    if torch.is_autocast_enabled("cuda"):
        return torch.bfloat16 if torch.get_autocast_dtype("cuda") == torch.bfloat16 else None
    return x.dtype if x.dtype in _CODE else None


_STEP_HOOK = []


def _note_optimizer_step(opt, args, kwargs):
    """Global optimizer post-step hook: every parameter the step updated (the ones holding a
    gradient: AdamW skips the rest) advances its own step epoch."""
    for g in opt.param_groups:
        for p in g["params"]:
            if p.grad is not None:
                p._rgbd_epoch = getattr(p, "_rgbd_epoch", 0) + 1


def cast_weight(w: torch.Tensor, dt):
    """w (a parameter) in dtype dt, cached on the parameter.  The key is (storage address,
    version counter, optimizer-step epoch): torch's fused AdamW updates parameters in place
    WITHOUT bumping their version counters (measured, torch 2.10; a version-keyed cache went
    stale after the first step and the bf16 loss fell visibly slower, tools/diag_bf16_model.py),
    so every optimizer step advances the epoch of the parameters it updated (a global
    post-step hook).  Parameters no optimizer steps — the frozen Swin-T (the reference detaches
    its features, custom_model.py:332-333, Q1) — are cast once."""
    if w.dtype == dt:
        return w.detach()
    if not _STEP_HOOK:
        from torch.optim.optimizer import register_optimizer_step_post_hook
        _STEP_HOOK.append(register_optimizer_step_post_hook(_note_optimizer_step))
    key = (w.data_ptr(), w._version, getattr(w, "_rgbd_epoch", 0), dt)
    hit = getattr(w, "_rgbd_cast", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    c = w.detach().to(dt)
    w._rgbd_cast = (key, c)
    return c


def _splits(M, N, K):
    """split-K count: enough workgroups for the chip when the output tile grid is small."""
    tiles = math.ceil(M / 128) * math.ceil(N / 128)
    if tiles >= 256 or K < 1024:
        return 1
    return int(max(1, min(16, 256 // max(tiles, 1), K // 512)))


def gemm(A, B, a_t, b_t, M, N, K, bias=None, act=ACT_NONE, R=None, c_f32=False, batch=1, sa=0, sb=0, sr=0,
         out=None):
    """C [batch][M][N] = act(op(A) op(B) + bias) (+ R) on the HIP GEMM (see rgbd_gemm in
    include/rgbd_hip.h for a_t / b_t).  A, B (and R) 2-D with unit inner stride (or 3-D batched
    with the given batch strides); returns C contiguous."""
    dt = A.dtype
    c_dt = torch.float32 if (c_f32 or dt == torch.float32) else dt
    r_dt = dt if c_f32 == 2 else c_dt  # c_f32 = 2: bf16-rounded results stored as float32, R in dt
    if B.dtype != dt or dt not in _CODE or (R is not None and R.dtype != r_dt):
        raise TypeError(f"gemm: A / B must share float32 / bfloat16 and R must have C's dtype, got {A.dtype}, "
                        f"{B.dtype}, {None if R is None else R.dtype}")
    for t in (A, B, R):
        if t is not None and (not t.is_cuda or t.stride(-1) != 1):
            raise RuntimeError("gemm: CUDA tensors with unit inner stride expected")
    dev = A.device
    shape = (M, N) if batch == 1 else (batch, M, N)
    if out is None:
        out = torch.empty(shape, dtype=c_dt, device=dev)
    splits = _splits(M, N, K)
    L = _lib.lib()
    ws = None
    if splits > 1:
        ws = _workspace(dev, L.rgbd_gemm_workspace_size(M, N, batch, splits), "gemm")
    b32 = None if bias is None else bias.detach().float().contiguous()
    check(L.rgbd_gemm(_CODE[dt], int(a_t), int(b_t), M, N, K, _p(A), A.stride(-2), sa, _p(B), B.stride(-2), sb,
                      _p(b32), act, _p(R), 0 if R is None else R.stride(-2), sr, _p(out), N, M * N,
                      int(c_f32), batch, splits, _p(ws), _stream(dev)), "rgbd_gemm")
    return out


def colsum(y2):
    out = torch.empty((y2.shape[1],), dtype=torch.float32, device=y2.device)
    L = _lib.lib()
    ws = _workspace(y2.device, L.rgbd_colsum_workspace_size(y2.shape[0], y2.shape[1]), "colsum", zeroed=True)
    check(L.rgbd_colsum(_CODE[y2.dtype], _p(y2), y2.shape[0], y2.shape[1], y2.stride(0), _p(out), _p(ws),
                        _stream(y2.device)), "rgbd_colsum")
    return out


def _rows(x, dt):
    """x as contiguous [rows, C] in dt.  A cast is made once per tensor (and version): it is
    kept on x, so the projections that share an input (q / k of the self-attention, the sampling
    offsets / attention weights of the deformable attention) and a fused LayerNorm's bf16 twin
    (add_layer_norm) are not cast again."""
    if x.dtype != dt:
        hit = getattr(x, "_rgbd_rows", None)
        if hit is not None and hit[0] == (x._version, dt) and hit[1].shape[-1] == x.shape[-1]:
            return hit[1]
    x2 = x.reshape(-1, x.shape[-1])
    if x2.dtype != dt:
        x2 = x2.to(dt)
        x2 = x2.contiguous()
        x._rgbd_rows = ((x._version, dt), x2)
        return x2
    return x2.contiguous()


def _fwd(x2, wc, b, act, M, N, K):
    """y [M][N] = act(x W^T + b) for a Linear layer.  (Measured: the plain bf16 products on the
    vendor library through torch.mm / addmm made the whole-model step slower, 100.0 vs
    109.8 img/s, profiles/r04_v3/full_model_lib_ab.txt, so every product stays here.)"""
    return gemm(x2, wc, 0, 0, M, N, K, bias=b, act=act)


def _dx(g2, wc, M, K, N, act=ACT_NONE, R=None, out_dtype=None):
    """dX [M][K] = dY [M][N] W [N][K] (act ACT_RELU_GRAD: times R > 0).  bf16 with many rows: W
    transposed once (a [K][N] copy, 0.1-2 MB) so both operands are K-contiguous for the LDS-DMA
    kernel (csrc/gemm.hip k_gemm_lds); otherwise the transposed-operand layout (0, 1).
    out_dtype float32 for bf16 operands: the bf16-rounded results stored as float32 by the GEMM
    (the cast autograd would make for a float32 input, without its own pass)."""
    c_f32 = 2 if (out_dtype == torch.float32 and g2.dtype == torch.bfloat16) else 0
    if g2.dtype == torch.bfloat16 and M >= 1024 and K % 8 == 0 and N % 8 == 0:
        return gemm(g2, wc.t().contiguous(), 0, 0, M, K, N, act=act, R=R, c_f32=c_f32)
    return gemm(g2, wc, 0, 1, M, K, N, act=act, R=R, c_f32=c_f32)


class LinearFunction(torch.autograd.Function):
    """y = act(x W^T + b), act none / relu / gelu (gelu: forward only)."""

    @staticmethod
    def forward(ctx, x, w, b, act, dt):
        N, K = w.shape
        x2 = _rows(x, dt)
        wc = cast_weight(w, dt)
        y = _fwd(x2, wc, b, act, x2.shape[0], N, K)
        ctx.save_for_backward(x2, wc, y if act == ACT_RELU else None)
        ctx.act, ctx.x_dtype, ctx.w_dtype, ctx.has_b = act, x.dtype, w.dtype, b is not None
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        x2, wc, y = ctx.saved_tensors
        if ctx.act == ACT_GELU:
            raise RuntimeError("HipLinear: the fused GELU epilogue is forward-only")
        M, K = x2.shape
        N = wc.shape[0]
        g2 = _rows(gy, x2.dtype)
        if ctx.act == ACT_RELU:
            g2 = g2 * (y > 0)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _dx(g2, wc, M, K, N, out_dtype=ctx.x_dtype).to(ctx.x_dtype).view(*gy.shape[:-1], K)
        if ctx.needs_input_grad[1]:
            dw = gemm(g2, x2, 1, 1, N, K, M, c_f32=True).to(ctx.w_dtype)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = colsum(g2)
        return dx, dw, db, None, None


class FFNFunction(torch.autograd.Function):
    """fc2(relu(fc1(x))): the ReLU in fc1's epilogue, its gradient in fc2's dX epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, dt):
        F_, K = w1.shape
        N = w2.shape[0]
        x2 = _rows(x, dt)
        w1c, w2c = cast_weight(w1, dt), cast_weight(w2, dt)
        M = x2.shape[0]
        h = gemm(x2, w1c, 0, 0, M, F_, K, bias=b1, act=ACT_RELU)
        y = _fwd(h, w2c, b2, ACT_NONE, M, N, F_)
        ctx.save_for_backward(x2, h, w1c, w2c)
        ctx.x_dtype, ctx.w_dtypes = x.dtype, (w1.dtype, w2.dtype)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        x2, h, w1c, w2c = ctx.saved_tensors
        M, K = x2.shape
        F_, N = h.shape[1], w2c.shape[0]
        g2 = _rows(gy, x2.dtype)
        dh = _dx(g2, w2c, M, F_, N, act=ACT_RELU_GRAD, R=h)
        dw2 = gemm(g2, h, 1, 1, N, F_, M, c_f32=True).to(ctx.w_dtypes[1])
        db2 = colsum(g2)
        dx = _dx(dh, w1c, M, K, F_, out_dtype=ctx.x_dtype).to(ctx.x_dtype).view(*gy.shape[:-1], K)
        dw1 = gemm(dh, x2, 1, 1, F_, K, M, c_f32=True).to(ctx.w_dtypes[0])
        db1 = colsum(dh)
        return dx, dw1, db1, dw2, db2, None


class LayerNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, y_dtype):
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        if x2.dtype not in _CODE:
            x2 = x2.float()
        x2 = x2.contiguous()
        rows = x2.shape[0]
        y = torch.empty((rows, C), dtype=y_dtype, device=x.device)
        mean = torch.empty((rows,), dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        g32 = None if gamma is None else gamma.detach().float().contiguous()
        b32 = None if beta is None else beta.detach().float().contiguous()
        check(_lib.lib().rgbd_layernorm_fwd(_CODE[x2.dtype], _p(x2), _p(g32), _p(b32), rows, C, float(eps),
                                            _CODE[y_dtype], _p(y), _p(mean), _p(rstd), _stream(x.device)),
              "rgbd_layernorm_fwd")
        ctx.save_for_backward(x2, g32, mean, rstd)
        ctx.x_dtype, ctx.has_g, ctx.has_b = x.dtype, gamma is not None, beta is not None
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, g32, mean, rstd = ctx.saved_tensors
        rows, C = x2.shape
        g2 = gy.reshape(rows, C)
        if g2.dtype not in _CODE:
            g2 = g2.float()
        g2 = g2.contiguous()
        dx = torch.empty_like(x2)
        dg = torch.empty((C,), dtype=torch.float32, device=x2.device)
        db = torch.empty_like(dg)
        L = _lib.lib()
        ws = _workspace(x2.device, L.rgbd_layernorm_bwd_workspace_size(rows, C), "ln_bwd")
        check(L.rgbd_layernorm_bwd(_CODE[x2.dtype], _p(x2), _CODE[g2.dtype], _p(g2), _p(g32), _p(mean), _p(rstd),
                                   rows, C, _p(dx), _p(dg), _p(db), _p(ws), _stream(x2.device)), "rgbd_layernorm_bwd")
        return (dx.to(ctx.x_dtype).view(gy.shape), dg if ctx.has_g else None, db if ctx.has_b else None, None, None)


class AddLayerNormFunction(torch.autograd.Function):
    """y = LayerNorm(x + r) (then clamp(y, -clamp, clamp) when clamp > 0): the sum, the norm and
    the clamp in one kernel (rgbd_add_layernorm_fwd), the sum kept for the backward; its gradient
    goes to x and r in their own dtypes (what autograd's add backward hands each: the same values,
    the bf16 one written by the backward kernel itself).  With ``twin`` a second, non-
    differentiable output holds y in bf16 (the consuming GEMMs' operand)."""

    @staticmethod
    def forward(ctx, x, r, gamma, beta, eps, y_dtype, twin, clamp):
        ctx.set_materialize_grads(False)
        C = x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        r2 = r.reshape(-1, C).contiguous()
        x2 = x2 if x2.data_ptr() % 16 == 0 else x2.clone()  # the kernel's 16-byte row accesses
        r2 = r2 if r2.data_ptr() % 16 == 0 else r2.clone()
        rows = x2.shape[0]
        s_dtype = torch.promote_types(x2.dtype, r2.dtype)
        s = torch.empty((rows, C), dtype=s_dtype, device=x.device)
        y = torch.empty((rows, C), dtype=y_dtype, device=x.device)
        y2 = torch.empty((rows, C), dtype=torch.bfloat16, device=x.device) if twin else None
        mean = torch.empty((rows,), dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        g32 = None if gamma is None else gamma.detach().float().contiguous()
        b32 = None if beta is None else beta.detach().float().contiguous()
        check(_lib.lib().rgbd_add_layernorm_fwd(_CODE[x2.dtype], _p(x2), _CODE[r2.dtype], _p(r2), _p(g32), _p(b32),
                                                rows, C, float(eps), float(clamp), _CODE[y_dtype], _p(s), _p(y),
                                                _p(y2), _p(mean), _p(rstd), _stream(x.device)),
              "rgbd_add_layernorm_fwd")
        ctx.save_for_backward(s, g32, b32, mean, rstd)
        ctx.dtypes, ctx.has_g, ctx.has_b, ctx.clamp = (x.dtype, r.dtype), gamma is not None, beta is not None, clamp
        if y2 is None:
            y2 = torch.empty((0,), dtype=torch.bfloat16, device=x.device)
        ctx.mark_non_differentiable(y2)
        return y.view(x.shape), y2

    @staticmethod
    def backward(ctx, gy, _gy2):
        s, g32, b32, mean, rstd = ctx.saved_tensors
        rows, C = s.shape
        if gy is None:
            return None, None, None, None, None, None, None, None
        g2 = gy.reshape(rows, C)
        if g2.dtype not in _CODE:
            g2 = g2.float()
        g2 = g2.contiguous()
        if g2.data_ptr() % 16:
            g2 = g2.clone()
        ds = torch.empty_like(s)
        twin = s.dtype == torch.float32 and ctx.dtypes[1] == torch.bfloat16
        ds2 = torch.empty((rows, C), dtype=torch.bfloat16, device=s.device) if twin else None
        dg = torch.empty((C,), dtype=torch.float32, device=s.device)
        db = torch.empty_like(dg)
        L = _lib.lib()
        ws = _workspace(s.device, L.rgbd_layernorm_bwd_workspace_size(rows, C), "ln_bwd")
        check(L.rgbd_add_layernorm_bwd(_CODE[s.dtype], _p(s), _CODE[g2.dtype], _p(g2), _p(g32), _p(b32), _p(mean),
                                       _p(rstd), rows, C, float(ctx.clamp), _p(ds), _p(ds2), _p(dg), _p(db), _p(ws),
                                       _stream(s.device)), "rgbd_add_layernorm_bwd")
        ds = ds.view(gy.shape)
        dr = ds2.view(gy.shape) if twin else ds.to(ctx.dtypes[1])
        return (ds.to(ctx.dtypes[0]), dr, dg if ctx.has_g else None, db if ctx.has_b else None,
                None, None, None, None)


class GroupNormFunction(torch.autograd.Function):
    """nn.GroupNorm (+ the ReLU after it when ``relu``) on rgbd_groupnorm_fwd / _bwd, NCHW."""

    @staticmethod
    def forward(ctx, x, gamma, beta, groups, eps, relu, y_dtype):
        xc = x if x.dtype in _CODE else x.float()
        xc = xc.contiguous()
        B, C = xc.shape[0], xc.shape[1]
        HW = xc.numel() // max(B * C, 1)
        y = torch.empty(xc.shape, dtype=y_dtype, device=x.device)
        mr = torch.empty((B, groups, 2), dtype=torch.float32, device=x.device)
        g32 = None if gamma is None else gamma.detach().float().contiguous()
        b32 = None if beta is None else beta.detach().float().contiguous()
        L = _lib.lib()
        ws = _workspace(x.device, L.rgbd_groupnorm_workspace_size(B, C), "gn")
        check(L.rgbd_groupnorm_fwd(_CODE[xc.dtype], _p(xc), _p(g32), _p(b32), B, C, groups, HW, float(eps), int(relu),
                                   _CODE[y_dtype], _p(y), _p(mr), _p(ws), _stream(x.device)), "rgbd_groupnorm_fwd")
        ctx.save_for_backward(xc, g32, b32, mr)
        ctx.groups, ctx.relu, ctx.x_dtype = groups, relu, x.dtype
        ctx.has_g, ctx.has_b = gamma is not None, beta is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        xc, g32, b32, mr = ctx.saved_tensors
        B, C = xc.shape[0], xc.shape[1]
        HW = xc.numel() // max(B * C, 1)
        g2 = gy if gy.dtype in _CODE else gy.float()
        g2 = g2.contiguous()
        dx = torch.empty_like(xc)
        dg = torch.empty((C,), dtype=torch.float32, device=xc.device)
        db = torch.empty_like(dg)
        L = _lib.lib()
        ws = _workspace(xc.device, L.rgbd_groupnorm_workspace_size(B, C), "gn")
        check(L.rgbd_groupnorm_bwd(_CODE[xc.dtype], _p(xc), _CODE[g2.dtype], _p(g2), _p(g32), _p(b32), _p(mr), B, C,
                                   ctx.groups, HW, int(ctx.relu), _p(dx), _p(dg), _p(db), _p(ws), _stream(xc.device)),
              "rgbd_groupnorm_bwd")
        return (dx.to(ctx.x_dtype), dg if ctx.has_g else None, db if ctx.has_b else None, None, None, None, None)


class HipGroupNorm(nn.GroupNorm):
    """nn.GroupNorm on the HIP kernels; ``_fused_relu`` (set by ``install`` when a ReLU follows in
    the same nn.Sequential, Mask2FormerPixelDecoder's FPN output layer) applies that ReLU too."""
    _fused_relu = False

    def forward(self, x):
        if not x.is_cuda or x.numel() == 0 or x.dim() < 2 or x.dtype not in _CODE:
            y = super().forward(x)
            return torch.relu(y) if self._fused_relu else y
        y_dtype = torch.float32 if torch.is_autocast_enabled("cuda") else x.dtype
        return GroupNormFunction.apply(x, self.weight if self.affine else None, self.bias if self.affine else None,
                                       self.num_groups, self.eps, self._fused_relu, y_dtype)


class _FusedReLU(nn.ReLU):
    """The ReLU after a HipGroupNorm that already applied it (identity)."""

    def forward(self, x):
        return x


def linear(x, w, b=None, act=ACT_NONE):
    dt = compute_dtype(x)
    return LinearFunction.apply(x, w, b, act, dt)


def ffn(x, fc1, fc2):
    return FFNFunction.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, compute_dtype(x))


def layer_norm(x, ln):
    y_dtype = torch.float32 if torch.is_autocast_enabled("cuda") else x.dtype
    return LayerNormFunction.apply(x, ln.weight, ln.bias, ln.eps, y_dtype)


def add_layer_norm(x, r, ln, clamp=False):
    """ln(x + r) for the post-norm residual of a covered layer (with ``clamp`` then
    clamp(., -c, c), c = finfo(dtype).max - 1000, the encoder layer's training clamp): one fused
    kernel where the shapes allow it (HipLayerNorm's coverage, C % 4 == 0), else the add, the
    module and the clamp."""
    C = x.shape[-1]
    if (isinstance(ln, HipLayerNorm) and x.is_cuda and r.is_cuda and x.shape == r.shape and x.numel() > 0
            and len(ln.normalized_shape) == 1 and ln.normalized_shape[0] == C and C % 4 == 0 and C <= 1536
            and x.dtype in _CODE and r.dtype in _CODE):
        amp = torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
        y_dtype = torch.float32 if torch.is_autocast_enabled("cuda") else torch.promote_types(x.dtype, r.dtype)
        # under bf16 autocast the consumers are bf16 GEMMs: the kernel also writes y in bf16 and
        # _rows serves that instead of casting y again (the same RNE rounding of the same float)
        twin = amp and y_dtype == torch.float32
        c = torch.finfo(y_dtype).max - 1000 if clamp else 0.0
        y, y2 = AddLayerNormFunction.apply(x, r, ln.weight, ln.bias, ln.eps, y_dtype, twin, float(c))
        if twin:
            y._rgbd_rows = ((y._version, torch.bfloat16), y2)
        return y
    y = ln(x + r)
    if clamp:
        c = torch.finfo(y.dtype).max - 1000
        y = torch.clamp(y, min=-c, max=c)
    return y


def _cuda_ok(x):
    return x.is_cuda and compute_dtype(x) is not None and x.numel() > 0


class HipLinear(nn.Linear):
    def forward(self, x):
        if not _cuda_ok(x):
            return super().forward(x)
        return linear(x, self.weight, self.bias)


class HipLayerNorm(nn.LayerNorm):
    def forward(self, x):
        if (not x.is_cuda or x.numel() == 0 or len(self.normalized_shape) != 1 or self.normalized_shape[0] > 1536
                or x.dtype not in _CODE):
            return super().forward(x)
        return layer_norm(x, self)


# ----------------------------------------------------------------- decoder layer (f1)
def self_attention(attn, h, pos):
    """Mask2FormerAttention.forward (modeling_mask2former.py:1487-1585) for the decoder's
    self-attention, seq-first h [Q, B, E]: q / k from h + pos, v from h, softmax(q k^T / sqrt(d))
    v per head on the HIP attention core (no mask), out_proj."""
    from .masked_attention import masked_attention
    Q, B, E = h.shape
    H = attn.num_heads
    hq = h if pos is None else h + pos
    q = linear(hq, attn.q_proj.weight, attn.q_proj.bias).view(Q, B * H, E // H)
    k = linear(hq, attn.k_proj.weight, attn.k_proj.bias).view(Q, B * H, E // H)
    v = linear(h, attn.v_proj.weight, attn.v_proj.bias).view(Q, B * H, E // H)
    o = masked_attention(q, k, v, None, attn.scaling)
    return linear(o.view(Q, B, E), attn.out_proj.weight, attn.out_proj.bias)


def _decoder_layer_covered(layer, h):
    return (h.is_cuda and compute_dtype(h) is not None and not layer.pre_norm
            and (not layer.training or (layer.dropout == 0.0 and layer.self_attn.dropout == 0.0))
            and layer.config.activation_function == "relu" and layer.self_attn.head_dim == 32)


def _install_class(m, base, cls):
    if type(m) is base:
        m.__class__ = cls
        return 1
    return 0


def _make_decoder_layer_class():
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerMaskedAttentionDecoderLayer as _L

    class HipMaskedAttentionDecoderLayer(_L):
        def forward_post(self, hidden_states, level_index=None, attention_mask=None, position_embeddings=None,
                         query_position_embeddings=None, encoder_hidden_states=None, encoder_attention_mask=None,
                         output_attentions=False):
            if output_attentions or not _decoder_layer_covered(self, hidden_states):
                return super().forward_post(hidden_states, level_index, attention_mask, position_embeddings,
                                            query_position_embeddings, encoder_hidden_states,
                                            encoder_attention_mask, output_attentions)
            residual = hidden_states
            hidden_states, _ = self.cross_attn(
                query=self.with_pos_embed(hidden_states, query_position_embeddings),
                key=self.with_pos_embed(encoder_hidden_states[level_index], position_embeddings[level_index]),
                value=encoder_hidden_states[level_index], attn_mask=encoder_attention_mask, key_padding_mask=None)
            hidden_states = add_layer_norm(residual, hidden_states, self.cross_attn_layer_norm)
            residual = hidden_states
            hidden_states = self_attention(self.self_attn, hidden_states, query_position_embeddings)
            hidden_states = add_layer_norm(residual, hidden_states, self.self_attn_layer_norm)
            residual = hidden_states
            hidden_states = ffn(hidden_states, self.fc1, self.fc2)
            hidden_states = add_layer_norm(residual, hidden_states, self.final_layer_norm)
            return (hidden_states,)

    return _L, HipMaskedAttentionDecoderLayer


def _make_encoder_layer_class():
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerPixelDecoderEncoderLayer as _L

    class HipPixelDecoderEncoderLayer(_L):
        def forward(self, hidden_states, attention_mask, position_embeddings=None, reference_points=None,
                    spatial_shapes_list=None, level_start_index=None, output_attentions=False):
            if (not hidden_states.is_cuda or compute_dtype(hidden_states) is None
                    or (self.training and self.dropout > 0.0)):
                return super().forward(hidden_states, attention_mask, position_embeddings, reference_points,
                                       spatial_shapes_list, level_start_index, output_attentions)
            residual = hidden_states
            hidden_states, attn_weights = self.self_attn(
                hidden_states=hidden_states, attention_mask=attention_mask, encoder_hidden_states=hidden_states,
                encoder_attention_mask=attention_mask, position_embeddings=position_embeddings,
                reference_points=reference_points, spatial_shapes_list=spatial_shapes_list,
                level_start_index=level_start_index, output_attentions=output_attentions)
            hidden_states = add_layer_norm(residual, hidden_states, self.self_attn_layer_norm)
            residual = hidden_states
            hidden_states = ffn(hidden_states, self.fc1, self.fc2)
            # in training the reference clamps when any value is non-finite (:1094-1097, a host
            # sync per layer); clamping unconditionally is the same map (identity on finite
            # float32, +-inf -> +-(max - 1000) = +-max, NaN kept) without the sync, done by the
            # fused norm kernel (its backward masks the gradient where the clamp was not the identity)
            hidden_states = add_layer_norm(residual, hidden_states, self.final_layer_norm, clamp=self.training)
            outputs = (hidden_states,)
            if output_attentions:
                outputs += (attn_weights.transpose(1, 0),)
            return outputs

    return _L, HipPixelDecoderEncoderLayer


_CLASSES = {}


def _classes():
    if not _CLASSES:
        _CLASSES["decoder"] = _make_decoder_layer_class()
        _CLASSES["encoder"] = _make_encoder_layer_class()
    return _CLASSES


def install(model: nn.Module) -> int:
    """Swap nn.Linear / nn.LayerNorm and the decoder / pixel-decoder encoder layers inside
    ``model`` for the HIP classes; returns the number of modules swapped."""
    from .conv import HipConv2d
    cls = _classes()
    n = 0
    for m in model.modules():
        n += _install_class(m, nn.Conv2d, HipConv2d)
        n += _install_class(m, nn.Linear, HipLinear)
        n += _install_class(m, nn.LayerNorm, HipLayerNorm)
        n += _install_class(m, nn.GroupNorm, HipGroupNorm)
        n += _install_class(m, *cls["decoder"])
        n += _install_class(m, *cls["encoder"])
    for m in model.modules():  # GroupNorm -> ReLU pairs (the pixel decoder's FPN output layer)
        if isinstance(m, nn.Sequential):
            ch = list(m.children())
            for a, b in zip(ch, ch[1:]):
                if type(a) is HipGroupNorm and type(b) is nn.ReLU and not b.inplace:
                    a._fused_relu = True
                    b.__class__ = _FusedReLU
    return n


def uninstall(model: nn.Module) -> int:
    from .conv import HipConv2d
    cls = _classes()
    back = {HipConv2d: nn.Conv2d, HipLinear: nn.Linear, HipLayerNorm: nn.LayerNorm, HipGroupNorm: nn.GroupNorm, _FusedReLU: nn.ReLU,
            cls["decoder"][1]: cls["decoder"][0], cls["encoder"][1]: cls["encoder"][0]}
    n = 0
    for m in model.modules():
        b = back.get(type(m))
        if b is not None:
            if isinstance(m, HipGroupNorm):
                m.__dict__.pop("_fused_relu", None)
            m.__class__ = b
            n += b is not nn.ReLU
    return n
