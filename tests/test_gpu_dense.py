"""f1 / f2 dense layers on the HIP GEMM and LayerNorm kernels (csrc/gemm.hip, csrc/layernorm.hip;
rgbd_amd/dense.py) against plain PyTorch references.

* rgbd_gemm in every operand layout (forward / dX / dW of a linear layer), float32 and bf16,
  aligned and ragged shapes (N = 49: the class predictor's 48 labels + 1), batched, split-K,
  every epilogue — against a float64 matmul of the same operands.  Bars: float32 (exact f32
  products, f32 sums) 2e-5 relative to the max |C|; bf16 operands (exact products, f32 sums, one
  bf16 rounding of C) 1e-2 relative.
* LayerNorm forward / backward vs torch.nn.functional.layer_norm in float64.
* HipLinear / FFN / HipLayerNorm modules and the installed decoder and pixel-decoder encoder
  layers vs the Hugging Face modules they replace (same parameters; the HF arm in float32, the
  reference's arithmetic): outputs and every gradient, float32 2e-4 / 4e-4 (relative to the
  max), bf16 autocast 5e-2 outputs, 0.1 / 0.2 gradients (see _grad_tol).
"""
import copy
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import _rgbd_import  # noqa: E402,F401

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
F32_TOL, BF16_TOL = 2e-5, 1e-2


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _ref(A, B, a_t, b_t, bias=None, act=0, R=None):
    a = A.double().transpose(-1, -2) if a_t else A.double()
    b = B.double() if b_t else B.double().transpose(-1, -2)
    c = a @ b
    if act == 3:
        return c * (R.double() > 0)
    if bias is not None:
        c = c + bias.double()
    if act == 1:
        c = c.clamp_min(0)
    elif act == 2:
        c = torch.nn.functional.gelu(c)
    if R is not None:
        c = c + R.double()
    return c


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (800, 49, 256), (1000, 192, 96), (37, 130, 72), (3, 5, 7)])
def test_gemm_layouts(dt, a_t, b_t, M, N, K):
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    A = torch.randn((K, M) if a_t else (M, K), generator=g).to(DEV, dt)
    B = torch.randn((K, N) if b_t else (N, K), generator=g).to(DEV, dt)
    C = dense.gemm(A, B, a_t, b_t, M, N, K)
    tol = F32_TOL if dt == torch.float32 else BF16_TOL
    assert C.shape == (M, N)
    assert _rel(C, _ref(A, B, a_t, b_t)) < tol


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("act", [0, 1, 2, 3], ids=["none", "relu", "gelu", "relu_grad"])
def test_gemm_epilogues(dt, act):
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(act)
    M, N, K = 300, 200, 160
    A = torch.randn((M, K), generator=g).to(DEV, dt)
    B = torch.randn((N, K), generator=g).to(DEV, dt)
    bias = None if act == 3 else torch.randn((N,), generator=g).to(DEV)
    R = torch.randn((M, N), generator=g).to(DEV, dt)
    C = dense.gemm(A, B, 0, 0, M, N, K, bias=bias, act=act, R=R)
    ref = _ref(A, B, 0, 0, bias, act, R)
    tol = F32_TOL if dt == torch.float32 else BF16_TOL
    assert _rel(C, ref) < tol * (3 if act == 2 else 1)


@pytest.mark.parametrize("M,N,K", [(50400, 256, 1024), (50400, 1024, 256), (4000, 384, 96), (2000, 200, 96),
                                   (1500, 100, 72), (1029, 264, 200)])
@pytest.mark.parametrize("act", [0, 1, 2, 3], ids=["none", "relu", "gelu", "relu_grad"])
def test_gemm_lds_dma_path(M, N, K, act):
    """bf16, both operands K-contiguous, M >= 1024: the LDS-DMA kernel (k_gemm_lds; 128 x 256 tiles
    when N % 256 == 0, else 128 x 128), ragged M / N / K (K % 64 != 0: zero lines past K; N % 8
    != 0: scalar stores), every epilogue, against float64 on the same bf16 operands."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(M + N + K + act)
    A = torch.randn((M, K), generator=g).to(DEV, torch.bfloat16)
    B = torch.randn((N, K), generator=g).to(DEV, torch.bfloat16)
    bias = None if act == 3 else torch.randn((N,), generator=g).to(DEV)
    R = torch.randn((M, N), generator=g).to(DEV, torch.bfloat16) if act in (0, 3) else None
    C = dense.gemm(A, B, 0, 0, M, N, K, bias=bias, act=act, R=R)
    ref = _ref(A, B, 0, 0, bias, act, R)
    assert C.shape == (M, N) and C.dtype == torch.bfloat16
    assert _rel(C, ref) < BF16_TOL * (3 if act == 2 else 1)
    Cf = dense.gemm(A, B, 0, 0, M, N, K, bias=bias, act=act, R=None if R is None else R.float(), c_f32=True)
    assert Cf.dtype == torch.float32 and _rel(Cf, ref) < 2e-5 * (3 if act == 2 else 1) * K ** 0.5


@pytest.mark.parametrize("N,K,M", [(1024, 256, 50400), (256, 256, 50400), (264, 96, 3000), (96, 384, 1200),
                                   (136, 200, 1100)])
@pytest.mark.parametrize("c_f32", [True, False], ids=["f32_out", "bf16_out"])
def test_gemm_lds_dma_weight_gradient(N, K, M, c_f32):
    """dW [N][K] = dY^T [N][M] X [M][K] in bf16 (layout (1, 1), M >= 1024 tokens): the LDS-DMA
    kernel with transposed fragment reads and split-K over the tokens, ragged N / K / M, against
    float64 on the same bf16 operands."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(N + K + M)
    gy = torch.randn((M, N), generator=g).to(DEV, torch.bfloat16)
    x = torch.randn((M, K), generator=g).to(DEV, torch.bfloat16)
    dW = dense.gemm(gy, x, 1, 1, N, K, M, c_f32=c_f32)
    ref = gy.double().t() @ x.double()
    assert dW.shape == (N, K) and dW.dtype == (torch.float32 if c_f32 else torch.bfloat16)
    assert _rel(dW, ref) < (2e-5 if c_f32 else BF16_TOL)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_gemm_split_k_weight_gradient(dt):
    """dW = dY^T X with a long reduction (50 400 pixel-decoder tokens) and a small output: the
    split-K path (float32 partials summed in split order), float32 output; deterministic."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(5)
    M, N, K = 50400, 256, 256  # rows of dY / X
    dY = torch.randn((M, N), generator=g).to(DEV, dt)
    X = torch.randn((M, K), generator=g).to(DEV, dt)
    assert dense._splits(N, K, M) > 1
    dW = dense.gemm(dY, X, 1, 1, N, K, M, c_f32=True)
    assert dW.dtype == torch.float32
    ref = dY.double().t() @ X.double()
    assert _rel(dW, ref) < (1e-5 if dt == torch.float32 else 2e-3)
    assert torch.equal(dW, dense.gemm(dY, X, 1, 1, N, K, M, c_f32=True))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_gemm_split_k_epilogue_batched_and_reuse(dt):
    """Split-K in one launch: the last split of each output tile sums the partials in split order
    and applies the epilogue (bias + ReLU, residual), batched, with ragged M / N; successive calls
    of different shapes share the workspace (its tickets come back to zero)."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(9)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    for batch, M, N, K in [(1, 100, 72, 8192), (3, 64, 130, 4096), (1, 256, 256, 50400), (2, 40, 24, 3000)]:
        assert dense._splits(M, N, K) > 1, (M, N, K)
        A = torch.randn((batch, M, K), generator=g).to(DEV, dt)
        B = torch.randn((batch, N, K), generator=g).to(DEV, dt)
        bias = torch.randn((N,), generator=g).to(DEV)
        R = torch.randn((batch, M, N), generator=g).to(DEV, dt)
        C = dense.gemm(A, B, 0, 0, M, N, K, bias=bias, act=dense.ACT_RELU, R=R, batch=batch, sa=M * K, sb=N * K,
                       sr=M * N)
        ref = torch.relu(A.double() @ B.double().transpose(1, 2) + bias.double()) + R.double()
        assert _rel(C.view(batch, M, N), ref) < tol, (batch, M, N, K)
        C2 = dense.gemm(A, B, 0, 0, M, N, K, bias=bias, act=dense.ACT_RELU, R=R, batch=batch, sa=M * K, sb=N * K,
                        sr=M * N)
        assert torch.equal(C, C2)


def test_gemm_batched():
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(9)
    b, M, N, K = 4, 100, 256, 300
    A = torch.randn((b, M, K), generator=g).to(DEV)
    B = torch.randn((b, K, N), generator=g).to(DEV)
    C = dense.gemm(A, B, 0, 1, M, N, K, batch=b, sa=M * K, sb=K * N)
    assert C.shape == (b, M, N)
    assert _rel(C, A.double() @ B.double()) < F32_TOL


def test_colsum():
    """One launch per call; the workspace's tickets must come back to zero after every call, so
    repeated calls of different shapes on one workspace (and bf16) keep giving the column sums."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(5)
    for rows, N, dt in [(1234, 77, torch.float32), (50400, 256, torch.bfloat16), (7, 1000, torch.float32),
                        (1234, 77, torch.float32), (153600, 384, torch.bfloat16), (64, 3000, torch.float32)]:
        y = torch.randn((rows, N), generator=g).to(DEV, dt)
        first = dense.colsum(y)
        assert _rel(first, y.double().sum(0)) < 1e-5, (rows, N, dt)
        assert torch.equal(dense.colsum(y), first)  # deterministic, tickets rearmed


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("C,rows", [(96, 333), (96, 20000), (192, 4097), (256, 333), (384, 3333), (768, 333),
                                    (1536, 700), (1000, 333), (60, 777)])
def test_layernorm_fwd_bwd(dt, C, rows):
    """C % 4 == 0: the vectorised row-group kernels (many rows per wave, block partials of the
    parameter gradients); C = 1000 / 60: the one-wave-per-row kernels."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(C)
    ln = torch.nn.LayerNorm(C, eps=1e-5).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(torch.randn(C, generator=g))
        ln.bias.copy_(torch.randn(C, generator=g))
    x = (torch.randn((rows, C), generator=g) * 3 + 1).to(DEV, dt).requires_grad_()
    y = dense.layer_norm(x, ln)
    assert y.dtype == dt
    gy = torch.randn(y.shape, generator=g).to(DEV, dt)
    y.backward(gy)
    x64 = x.detach().double().requires_grad_()
    w64, b64 = ln.weight.detach().double().requires_grad_(), ln.bias.detach().double().requires_grad_()
    y64 = torch.nn.functional.layer_norm(x64, (C,), w64, b64, 1e-5)
    y64.backward(gy.double())
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert _rel(y, y64) < tol
    assert _rel(x.grad, x64.grad) < tol * 2
    assert _rel(ln.weight.grad, w64.grad) < 1e-5
    assert _rel(ln.bias.grad, b64.grad) < 1e-5


@pytest.mark.parametrize("a_t,b_t", [(0, 0), (0, 1)])
@pytest.mark.parametrize("M,N,K,act", [(4096, 256, 1024, 3), (800, 256, 256, 0), (37, 130, 72, 0), (50400, 256, 256, 0)])
def test_gemm_bf16_rounded_float32_store(a_t, b_t, M, N, K, act):
    """c_f32 = 2: a bf16 GEMM's results rounded to bf16 and stored as float32 (the dX a float32
    input receives under autocast) — the bits of the bf16 output widened, R read in bf16."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn((K, M) if a_t else (M, K), generator=g).to(DEV, torch.bfloat16)
    B = torch.randn((K, N) if b_t else (N, K), generator=g).to(DEV, torch.bfloat16)
    R = torch.randn((M, N), generator=g).to(DEV, torch.bfloat16) if act == 3 else None
    ref = dense.gemm(A, B, a_t, b_t, M, N, K, act=act, R=R)
    got = dense.gemm(A, B, a_t, b_t, M, N, K, act=act, R=R, c_f32=2)
    assert got.dtype == torch.float32 and torch.equal(got, ref.float())


@pytest.mark.parametrize("xdt,rdt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.bfloat16)], ids=["f32+f32", "f32+bf16", "bf16+bf16"])
@pytest.mark.parametrize("C,rows", [(256, 800), (256, 50400), (96, 333), (1536, 70)])
def test_add_layernorm_fused(xdt, rdt, C, rows):
    """LN(x + r) in one kernel (the decoder / encoder layers' post-norm residual): the sum in the
    promoted dtype exactly as torch's add (bitwise), the norm and every gradient against float64
    (x and r each get the sum's gradient in their own dtype)."""
    from rgbd_amd import dense
    g = torch.Generator(device="cpu").manual_seed(C + rows)
    ln = dense.HipLayerNorm(C, eps=1e-5).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(torch.randn(C, generator=g))
        ln.bias.copy_(torch.randn(C, generator=g))
    x = (torch.randn((rows, C), generator=g) * 3 + 1).to(DEV, xdt).requires_grad_()
    r = torch.randn((rows, C), generator=g).to(DEV, rdt).requires_grad_()
    y = dense.add_layer_norm(x, r, ln)
    sdt = torch.promote_types(xdt, rdt)
    assert y.dtype == sdt
    gy = torch.randn(y.shape, generator=g).to(DEV, sdt)
    y.backward(gy)
    assert x.grad.dtype == xdt and r.grad.dtype == rdt
    s = (x.detach() + r.detach())  # torch's add: the sum the norm must see
    s64 = s.double().requires_grad_()
    w64, b64 = ln.weight.detach().double().requires_grad_(), ln.bias.detach().double().requires_grad_()
    y64 = torch.nn.functional.layer_norm(s64, (C,), w64, b64, 1e-5)
    y64.backward(gy.double())
    tol = 1e-5 if sdt == torch.float32 else 1e-2
    assert _rel(y, y64) < tol
    assert _rel(x.grad, s64.grad) < tol * 2 + (1e-2 if xdt == torch.bfloat16 else 0)
    assert _rel(r.grad, s64.grad) < tol * 2 + (1e-2 if rdt == torch.bfloat16 else 0)
    assert _rel(ln.weight.grad, w64.grad) < 1e-5
    assert _rel(ln.bias.grad, b64.grad) < 1e-5
    # the unfused path (torch add + the HIP norm) gives the same bits
    ln2 = dense.HipLayerNorm(C, eps=1e-5).to(DEV)
    ln2.load_state_dict(ln.state_dict())
    assert torch.equal(dense.layer_norm(s, ln2), y.detach())


@pytest.mark.parametrize("rdt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_add_layernorm_clamp(rdt):
    """The encoder layer's training clamp folded into the fused norm: values that overflow to
    +-inf (one channel with gamma 1e38, large there in every third row) come out as +-max, and the
    backward zeroes the gradient exactly there (torch.clamp's backward) — the clamp pattern and
    values against torch's float32 add + layer_norm + clamp, the gradients against float64."""
    from rgbd_amd import dense
    C, rows = 256, 333
    g = torch.Generator(device="cpu").manual_seed(5)
    ln = dense.HipLayerNorm(C, eps=1e-5).to(DEV)
    with torch.no_grad():
        w = torch.randn(C, generator=g)
        w[7] = 1e38  # channel 7 overflows where its normalised value exceeds ~3.4
        ln.weight.copy_(w)
        ln.bias.copy_(torch.randn(C, generator=g))
    x0 = torch.randn((rows, C), generator=g)
    x0[::3, 7] = 10.0 * torch.sign(torch.randn(len(range(0, rows, 3)), generator=g))
    x = x0.to(DEV).requires_grad_()
    r = torch.randn((rows, C), generator=g).to(DEV, rdt).requires_grad_()
    y = dense.add_layer_norm(x, r, ln, clamp=True)
    c = torch.finfo(torch.float32).max - 1000
    assert torch.isfinite(y).all() and int((y.abs() == torch.finfo(torch.float32).max).sum()) >= rows // 3
    gy = torch.randn(y.shape, generator=g).to(DEV)
    y.backward(gy)
    # reference: torch's float32 forward decides where the clamp acts (the same overflow pattern as
    # the kernel, checked below); the gradient is the float64 LayerNorm backward of the masked dy
    s32 = x.detach() + r.detach()
    w, b = ln.weight.detach(), ln.bias.detach()
    y32 = torch.nn.functional.layer_norm(s32, (C,), w, b, 1e-5)
    big = torch.finfo(torch.float32).max
    yr = torch.clamp(y32, min=-c, max=c)
    assert torch.equal(y.detach().abs() == big, yr.abs() == big)
    fin = torch.isfinite(y32)
    assert _rel(y.detach()[fin], yr[fin]) < 1e-5
    s64 = s32.double().requires_grad_()
    w64, b64 = w.double().requires_grad_(), b.double().requires_grad_()
    torch.nn.functional.layer_norm(s64, (C,), w64, b64, 1e-5).backward(gy.double() * fin.double())
    # the clamped rows (every third): there the mask removes channel 7's 1e38-weighted gradient and
    # the input gradients are ordinary numbers (elsewhere they are ~1e35-1e38)
    assert torch.isfinite(x.grad[::3]).all() and float(x.grad[::3].abs().max()) < 1e6
    assert _rel(x.grad[::3], s64.grad[::3]) < 1e-4
    assert _rel(r.grad[::3].float(), s64.grad[::3]) < (1e-4 if rdt == torch.float32 else 1e-2)
    assert _rel(ln.bias.grad, b64.grad) < 1e-5


def _grads(m):
    return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("amp", [False, True], ids=["f32", "bf16_autocast"])
def test_linear_and_ffn_modules(amp):
    """fc2(relu(fc1(x))) on the fused FFN vs torch.  The weight gradients in bf16 are checked
    against float32 arithmetic on the same bf16-rounded operands: torch's own autocast weight
    gradient of fc1 here is 9.4 % (relative to its max) away from that (measured,
    tools/debug_ffn_bf16.py), ours 5.8e-4."""
    from rgbd_amd import dense
    torch.manual_seed(0)
    ref = torch.nn.Sequential(torch.nn.Linear(256, 2048), torch.nn.ReLU(), torch.nn.Linear(2048, 256)).to(DEV)
    hip = copy.deepcopy(ref)
    x = torch.randn((100, 8, 256), device=DEV)
    gy = torch.randn((100, 8, 256), device=DEV)
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        ya = ref(xa)
        yb = dense.ffn(xb, hip[0], hip[2])
    assert ya.dtype == yb.dtype
    ya.float().backward(gy)
    yb.float().backward(gy)
    tol = 3e-2 if amp else F32_TOL
    assert _rel(yb, ya) < tol
    assert _rel(xb.grad, xa.grad) < tol
    gb = _grads(hip)
    if amp:  # float32 arithmetic on the bf16 operands
        r = lambda t: t.detach().bfloat16().float()  # noqa: E731
        xr, w1, w2, g = r(x.reshape(800, 256)), r(ref[0].weight), r(ref[2].weight), r(gy.reshape(800, 256))
        z = xr @ w1.t() + ref[0].bias.detach()
        h = torch.relu(z).bfloat16().float()
        dh = ((g @ w2) * (h > 0)).bfloat16().float()
        ga = {"0.weight": dh.t() @ xr, "0.bias": dh.sum(0), "2.weight": g.t() @ h, "2.bias": g.sum(0)}
        tol_w = 5e-3
    else:
        ga, tol_w = _grads(ref), F32_TOL
    assert ga.keys() == gb.keys()
    for n in ga:
        err = _rel(gb[n], ga[n])
        print(f"{n}: {err:.3g}")
        assert err < tol_w, n
    # the plain module swap
    lin = torch.nn.Linear(256, 49).to(DEV)
    hl = copy.deepcopy(lin)
    hl.__class__ = dense.HipLinear
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        assert _rel(hl(x), lin(x)) < tol


def _grad_tol(name, amp):
    """Gradient bars against the HF float32 layer.  In bf16 the FFN's ReLU mask is taken from a
    bf16 pre-activation: about 0.07 % of the units sit within rounding of zero and flip (measured
    1 211 of 1.6 M at B = 8), which moves fc1's gradients by ~14 % of their max — torch's own
    autocast path lands at the same distance (tools/debug_ffn_bf16.py: 14.1 % vs ours 14.0 %)."""
    if not amp:
        return 4e-4
    if name.startswith("self_attn.sampling_offsets."):
        # the location gradient of bilinear sampling is a difference of neighbouring values, each
        # carrying bf16 rounding: measured 18 % of its max against float32
        return 0.3
    return 0.2 if name.startswith("fc1.") else 0.1


def _hf_config():
    from rgbd_amd.config import standard_config
    return standard_config(48)


@pytest.mark.parametrize("amp", [False, True], ids=["f32", "bf16_autocast"])
def test_decoder_layer_matches_hf(amp):
    """The installed masked-attention decoder layer (HIP cross-attention core, self-attention,
    FFN, LayerNorms) vs the HF layer with the same parameters on a C2-shaped call (B = 8, 100
    queries, level-2 memory of 4 800 keys), outputs and all gradients."""
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerMaskedAttentionDecoderLayer
    from rgbd_amd import dense, masked_attention
    torch.manual_seed(1)
    cfg = _hf_config()
    ref = Mask2FormerMaskedAttentionDecoderLayer(cfg).to(DEV).train()
    hip = copy.deepcopy(ref)
    assert dense.install(hip) == 1 + 3 + 4 + 2  # the layer, 3 LayerNorms, 4 self-attn + 2 FFN Linears
    assert masked_attention.install(hip) == 1
    Q, B, E, L = 100, 8, 256, 4800
    h = torch.randn((Q, B, E), device=DEV)
    qpos = torch.randn((Q, B, E), device=DEV)
    mem = [torch.randn((L, B, E), device=DEV)] * 3
    pos = [torch.randn((L, B, E), device=DEV)] * 3
    mask = torch.rand((B * 8, Q, L), device=DEV) < 0.3
    gy = torch.randn((Q, B, E), device=DEV)
    outs, grads = [], []
    for m, amp_ in ((ref, False), (hip, amp)):  # the HF arm in float32: the reference's arithmetic
        hh = h.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp_):
            y = m(hh, 2, None, pos, qpos, mem, encoder_attention_mask=mask)[0]
        y.float().backward(gy)
        outs.append((y.float(), hh.grad))
        grads.append(_grads(m))
    tol = 5e-2 if amp else 2e-4
    assert _rel(outs[1][0], outs[0][0]) < tol
    assert _rel(outs[1][1], outs[0][1]) < tol
    assert grads[0].keys() == grads[1].keys()
    scale = max(float(g.abs().max()) for g in grads[0].values())
    for n in grads[0]:
        if n == "self_attn.k_proj.bias":
            # a key bias shifts every score of a query by the same q.b: softmax-invariant, so its
            # gradient is zero in exact arithmetic and rounding noise in both arms
            assert float(grads[1][n].abs().max()) < 1e-4 * scale
            continue
        err = _rel(grads[1][n], grads[0][n])
        print(f"{n}: {err:.3g}")
        assert err < _grad_tol(n, amp), n


@pytest.mark.parametrize("amp", [False, True], ids=["f32", "bf16_autocast"])
def test_pixel_decoder_encoder_layer_matches_hf(amp):
    """One installed pixel-decoder encoder layer (HIP deformable attention, its four projections,
    FFN, two LayerNorms) vs the HF layer on the 320x240 level shapes (30x40, 15x20, 8x10), B = 2.
    The sampling-offset projection has zero weights and a fractional bias, so the sampling
    locations are exact in both arms: bilinear sampling is only piecewise smooth in the location,
    and a rounding-level location difference at a cell boundary would flip a cell and move the
    location gradients by O(1) — a property of the operator, not of either implementation."""
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerPixelDecoderEncoderLayer
    from rgbd_amd import deform_attn, dense
    torch.manual_seed(2)
    cfg = _hf_config()
    ref = Mask2FormerPixelDecoderEncoderLayer(cfg).to(DEV).train()
    with torch.no_grad():
        ref.self_attn.sampling_offsets.weight.zero_()
        ref.self_attn.sampling_offsets.bias.uniform_(-2.3, 2.3)
    hip = copy.deepcopy(ref)
    assert dense.install(hip) == 1 + 2 + 6 and deform_attn.install(hip) == 1
    shapes = [(30, 40), (15, 20), (8, 10)]
    S = sum(h * w for h, w in shapes)
    B = 2
    start = torch.tensor([0, 1200, 1500], device=DEV)
    x = torch.randn((B, S, 256), device=DEV)
    pos = torch.randn((B, S, 256), device=DEV)
    refp = torch.rand((B, S, 3, 2), device=DEV) * 0.9 + 0.05
    gy = torch.randn((B, S, 256), device=DEV)
    res = []
    for m, amp_ in ((ref, False), (hip, amp)):  # the HF arm in float32: the reference's arithmetic
        xx = x.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp_):
            y = m(xx, None, position_embeddings=pos, reference_points=refp, spatial_shapes_list=shapes,
                  level_start_index=start)[0]
        y.float().backward(gy)
        res.append((y.float(), xx.grad, _grads(m)))
    for k, arm in enumerate(("HF", "HIP")):
        assert torch.isfinite(res[k][0]).all() and torch.isfinite(res[k][1]).all(), f"{arm} arm not finite"
    tol = 5e-2 if amp else 2e-4
    assert _rel(res[1][0], res[0][0]) < tol
    assert _rel(res[1][1], res[0][1]) < tol
    for n in res[0][2]:
        err = _rel(res[1][2][n], res[0][2][n])
        print(f"{n}: {err:.3g}")
        assert err < _grad_tol(n, amp), n
