"""bf16 DSAM kernels (K5: code-merged forward, dX, dW) at the bench's full size, 640x480,
B=8, against a float32 PyTorch-GPU restatement of DSAModule.forward
(mask2former/utils/custom_model.py:682-699) on the same region codes:

    y = sum_{i<4} Conv3x3s2_i(x * m_i) + sum_{i<n_masks} b_i + Proj3x3s2(x),  m_i = bit i of code

The codes come from the HIP decomposition, which is pinned bit-exact elsewhere
(test_gpu_parity.py); here they only define the masks.  Tolerance: bf16 operands with f32
accumulation against f32 — max error <= 2e-2 of the reference's max magnitude, mean error
<= 4e-3 of its mean magnitude (the second bound catches a dropped or doubled tile that the
max-norm bound could hide)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import _rgbd_import  # noqa: F401
from rgbd_amd import init as winit, ops, synthetic

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ref_forward(x, code, n_masks, conv_w, conv_b, proj_w):
    y = F.conv2d(x, proj_w, stride=2, padding=1)
    for i in range(4):
        m = ((code >> i) & 1).float()[:, None]
        y = y + F.conv2d(x * m, conv_w[i], stride=2, padding=1)
    bias = torch.stack([conv_b[:int(n)].sum(0) if n > 0 else torch.zeros_like(conv_b[0]) for n in n_masks])
    return y + bias[:, :, None, None]


def _err(a, e):
    d = (a.float() - e).abs()
    return float(d.max() / e.abs().max()), float(d.mean() / e.abs().mean())


@pytest.mark.parametrize("k", [0, 1, 2])
def test_dsam_bf16_full_size(k):
    from rgbd_amd.modules import DSAModule
    cin, cout = [(96, 192), (192, 384), (384, 768)][k]
    B, H, W = 8, 480, 640
    h, w = [(120, 160), (60, 80), (30, 40)][k]
    m = DSAModule(cin, cout)
    winit.init_deterministic(m, prefix=f"full.dsam{k}.")
    m.compute_dtype = torch.bfloat16
    m = m.to(DEV)
    planes, _, _ = synthetic.make_batch(3, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    ratio = torch.linspace(0.05, 0.45, B, device=DEV)
    codes, info = ops.edsam_decompose(d3, ratio, [(h, w)])
    n_masks = ops.decode_info(info)["n_masks"]
    g = torch.Generator(device=DEV)
    g.manual_seed(100 + k)
    x = torch.randn((B, cin, h, w), generator=g, device=DEV).bfloat16()
    gout = (torch.randn((B, cout, (h + 1) // 2, (w + 1) // 2), generator=g, device=DEV) * 0.1).bfloat16()
    # HIP path, driven exactly as the fused hot path drives it
    from rgbd_amd.modules import _DSAMFn
    xg = x.clone().requires_grad_(True)
    y = _DSAMFn.apply(xg, codes[0], info, torch.bfloat16, m._pack_cache, *m._params())
    y.backward(gout)
    # float32 reference on the same (bf16-valued) inputs
    conv_w = torch.stack([m.conv_layers[i].weight.detach() for i in range(4)]).clone().requires_grad_(True)
    conv_b = torch.stack([m.conv_layers[i].bias.detach() for i in range(4)]).clone().requires_grad_(True)
    proj_w = m.rgb_projection.weight.detach().clone().requires_grad_(True)
    xr = x.float().requires_grad_(True)
    yr = _ref_forward(xr, codes[0].long(), n_masks, conv_w, conv_b, proj_w)
    yr.backward(gout.float())
    checks = {
        "y": (y.detach(), yr.detach()),
        "dx": (xg.grad, xr.grad),
        "dconv_w": (torch.stack([m.conv_layers[i].weight.grad for i in range(4)]), conv_w.grad),
        "dconv_b": (torch.stack([m.conv_layers[i].bias.grad for i in range(4)]), conv_b.grad),
        "dproj_w": (m.rgb_projection.weight.grad, proj_w.grad),
    }
    for name, (a, e) in checks.items():
        mx, mean = _err(a, e)
        assert mx <= 2e-2 and mean <= 4e-3, f"dsam{k} {name}: max {mx:.3g} mean {mean:.3g}"


def test_dsam_bf16_ragged_many_codes():
    """Odd sizes (ragged tiles, 64-px units crossing rows, border taps) and a code map using
    all 16 codes at random, B=3: the paths the full-size scenes rarely exercise."""
    from rgbd_amd.modules import _DSAMFn, DSAModule
    B, cin, cout, h, w = 3, 64, 96, 37, 53
    m = DSAModule(cin, cout)
    winit.init_deterministic(m, prefix="ragged.")
    m.compute_dtype = torch.bfloat16
    m = m.to(DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    code = torch.randint(0, 16, (B, h, w), generator=g, device=DEV).to(torch.uint8)
    info = torch.zeros((B, 2116), dtype=torch.uint8, device=DEV)
    rec = np.zeros(B, dtype=ops.DECOMP_INFO_DTYPE)
    rec["n_masks"] = [4, 2, 0]
    info.copy_(torch.from_numpy(rec.view(np.uint8).reshape(B, -1)))
    x = torch.randn((B, cin, h, w), generator=g, device=DEV).bfloat16()
    gout = torch.randn((B, cout, (h + 1) // 2, (w + 1) // 2), generator=g, device=DEV).bfloat16()
    xg = x.clone().requires_grad_(True)
    y = _DSAMFn.apply(xg, code, info, torch.bfloat16, m._pack_cache, *m._params())
    y.backward(gout)
    conv_w = torch.stack([m.conv_layers[i].weight.detach() for i in range(4)]).clone().requires_grad_(True)
    conv_b = torch.stack([m.conv_layers[i].bias.detach() for i in range(4)]).clone().requires_grad_(True)
    proj_w = m.rgb_projection.weight.detach().clone().requires_grad_(True)
    xr = x.float().requires_grad_(True)
    yr = _ref_forward(xr, code.long(), rec["n_masks"], conv_w, conv_b, proj_w)
    yr.backward(gout.float())
    for name, a, e in [("y", y.detach(), yr.detach()), ("dx", xg.grad, xr.grad),
                       ("dconv_w", torch.stack([m.conv_layers[i].weight.grad for i in range(4)]), conv_w.grad),
                       ("dproj_w", m.rgb_projection.weight.grad, proj_w.grad)]:
        mx, mean = _err(a, e)
        assert mx <= 2e-2 and mean <= 4e-3, f"{name}: max {mx:.3g} mean {mean:.3g}"


@pytest.mark.parametrize("k", [1, 2])
def test_dsam_bf16_dx_nhwc_only_and_nhwc_bias_sums(k):
    """The hot path's bf16 cascade writes dX in NHWC only, with the residual gradient given in
    NHWC (rgbd_dsam_bwd_data with dx_nchw = NULL, gin_nhwc), and takes the DSAM bias sums from the
    NHWC upstream gradient (rgbd_dsam_bwd_weight with gout_nchw = NULL).  Same arithmetic and
    rounding order as the NCHW path: dX bit-exact; bias sums differ only by float summation
    order (rel 1e-5)."""
    from rgbd_amd.modules import DSAModule
    cin, cout = [(96, 192), (192, 384), (384, 768)][k]
    B, H, W = 8, 480, 640
    h, w = [(120, 160), (60, 80), (30, 40)][k]
    m = DSAModule(cin, cout)
    winit.init_deterministic(m, prefix=f"nhwc.dsam{k}.")
    planes, _, _ = synthetic.make_batch(5, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    codes, info = ops.edsam_decompose(d3, torch.linspace(0.05, 0.45, B, device=DEV), [(h, w)])
    masks = ops.dsam_code_masks(codes)
    conv_w = torch.stack([m.conv_layers[i].weight.detach() for i in range(4)]).to(DEV)
    proj_w = m.rgb_projection.weight.detach().to(DEV)
    _, wb = ops.dsam_pack(conv_w, proj_w, torch.bfloat16, code_mask=masks[0:1])
    g = torch.Generator(device=DEV)
    g.manual_seed(300 + k)
    ho, wo = (h + 1) // 2, (w + 1) // 2
    gy = (torch.randn((B, ho, wo, cout), generator=g, device=DEV) * 0.1).bfloat16()
    gin = (torch.randn((B, cin, h, w), generator=g, device=DEV) * 0.1).bfloat16()
    dx_ref, dx_ref_nhwc = ops.dsam_bwd_data(gy, codes[0], wb, gin, want_nhwc=True)
    none, dx_nhwc = ops.dsam_bwd_data(gy, codes[0], wb, None, want_nhwc=True, want_nchw=False, cin=cin,
                                      gin_nhwc=ops.nchw_to_nhwc(gin))
    assert none is None
    assert torch.equal(dx_nhwc, dx_ref_nhwc)
    assert torch.equal(dx_nhwc, dx_ref.permute(0, 2, 3, 1))
    x = torch.randn((B, h, w, cin), generator=g, device=DEV).bfloat16()
    gy_nchw = gy.permute(0, 3, 1, 2).contiguous()
    a = ops.dsam_bwd_weight(gy_nchw, x, codes[0], info, gout_nhwc=gy)
    b = ops.dsam_bwd_weight(None, x, codes[0], info, gout_nhwc=gy)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    torch.testing.assert_close(b[2], a[2], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape", [(2, 96, 120, 160), (3, 40, 7, 8), (2, 768, 15, 20), (1, 12, 5, 5)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_nchw_to_nhwc_exact(shape, dtype):
    """rgbd_nchw_to_nhwc: the 16-byte bf16 path (h*w and C multiples of 8, ragged 64x64 tiles)
    and the element-wise fallback are exact copies."""
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    x = torch.randn(shape, generator=g, device=DEV).to(dtype)
    assert torch.equal(ops.nchw_to_nhwc(x), x.permute(0, 2, 3, 1).contiguous())


@pytest.mark.parametrize("shapes", [
    [(8, 768, 15, 20), (8, 384, 30, 40), (8, 192, 60, 80)],                    # the backward's G[3..1]
    [(8, 96, 120, 160), (8, 192, 60, 80), (8, 384, 30, 40), (8, 768, 15, 20)],  # the forward's colour maps
    [(3, 40, 7, 9), (1, 8, 1, 1), (2, 136, 33, 65)],                            # ragged tiles, HW % 8 != 0
])
def test_nchw_to_nhwc_multi_exact(shapes):
    """rgbd_nchw_to_nhwc_multi: every job an exact NHWC copy (16-byte loads where h*w % 8 == 0,
    element loads otherwise), one launch for all."""
    g = torch.Generator(device=DEV)
    g.manual_seed(17)
    xs = [torch.randn(s, generator=g, device=DEV).bfloat16() for s in shapes]
    for x, y in zip(xs, ops.nchw_to_nhwc_multi(xs)):
        assert torch.equal(y, x.permute(0, 2, 3, 1).contiguous())
    with pytest.raises(ops._lib.RgbdHipError):  # C % 8 != 0
        ops.nchw_to_nhwc_multi([torch.zeros((1, 12, 5, 5), device=DEV, dtype=torch.bfloat16)])


@pytest.mark.parametrize("k", [0, 1, 2])
def test_dsam_fwd_nhwc_equals_nchw_path(k):
    """rgbd_dsam_fwd_nhwc (NHWC residual in, NHWC out only: the hot path's bf16 cascade) gives
    bitwise the NHWC output of rgbd_dsam_fwd with the same residual in NCHW."""
    from rgbd_amd.modules import DSAModule
    cin, cout = [(96, 192), (192, 384), (384, 768)][k]
    B, H, W = 8, 480, 640
    h, w = [(120, 160), (60, 80), (30, 40)][k]
    m = DSAModule(cin, cout)
    winit.init_deterministic(m, prefix=f"nhwcfwd.dsam{k}.")
    planes, _, _ = synthetic.make_batch(4, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    codes, info = ops.edsam_decompose(d3, torch.linspace(0.05, 0.45, B, device=DEV), [(h, w)])
    masks = ops.dsam_code_masks(codes)
    conv_w = torch.stack([m.conv_layers[i].weight.detach() for i in range(4)]).to(DEV)
    proj_w = m.rgb_projection.weight.detach().to(DEV)
    bias4 = torch.stack([m.conv_layers[i].bias.detach() for i in range(4)]).to(DEV)
    wf, _ = ops.dsam_pack(conv_w, proj_w, torch.bfloat16, code_mask=masks[0:1], want_bwd=False)
    g = torch.Generator(device=DEV)
    g.manual_seed(500 + k)
    ho, wo = (h + 1) // 2, (w + 1) // 2
    x = torch.randn((B, h, w, cin), generator=g, device=DEV).bfloat16()
    res = torch.randn((B, cout, ho, wo), generator=g, device=DEV).bfloat16()
    _, ref_nhwc = ops.dsam_fwd(x, codes[0], info, wf, bias4, residual=res, want_nhwc=True)
    got = ops.dsam_fwd_nhwc(x, codes[0], info, wf, bias4, residual_nhwc=ops.nchw_to_nhwc(res))
    assert torch.equal(got, ref_nhwc)
    no_res = ops.dsam_fwd_nhwc(x, codes[0], info, wf, bias4)
    _, ref2 = ops.dsam_fwd(x, codes[0], info, wf, bias4, want_nhwc=True)
    assert torch.equal(no_res, ref2)


@pytest.mark.parametrize("shape", [(2, 96, 120, 160), (3, 192, 13, 17), (2, 384, 7, 9)])
def test_dggm_cp1_nhwc_equals_nchw(shape):
    """rgbd_dggm_fuse_fwd_multi_mixed with cp1 in NHWC gives bitwise the NCHW-cp1 result."""
    import golden_inputs as gi
    B, C, h, w = shape
    H, W = 4 * h, 4 * w
    pv = torch.from_numpy(gi.pixel_values(13, B, H, W)).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(9)
    color = torch.randn((B, C, h, w), generator=g, device=DEV).bfloat16()
    cp1 = torch.randn((B, C, h, w), generator=g, device=DEV).bfloat16()
    wt = torch.randn((C, 3, 1, 1), generator=g, device=DEV)
    bs = torch.randn((C,), generator=g, device=DEV)
    ref = ops.dggm_fuse_fwd_multi([cp1], [color], pv, [wt], [bs])[0]
    got = ops.dggm_fuse_fwd_multi([ops.nchw_to_nhwc(cp1)], [color], pv, [wt], [bs], cp1_nhwc=(0,))[0]
    assert torch.equal(got, ref)


def _pack_reference(conv_w, proj_w, codes_present):
    """numpy restatement of the bf16 code-merged packing (dsam_conv.hip, k_pack_codes):
    W_k = proj + sum_{i in k} conv_i in f32 (proj first, conv_0..3 ascending), rounded once to bf16,
    laid out as wfwd [k][tap][Cin/32][Cout][32 c] / wbwd [k][tap][Cout/32][Cin][32 o] with the
    16-byte chunk g of row n at slot g ^ (((n >> 3) & 1) << 1)."""
    conv = conv_w.cpu().numpy().astype(np.float32)
    proj = proj_w.cpu().numpy().astype(np.float32)
    _, Co, Ci = conv.shape[:3]
    nci, nco = Ci // 32, Co // 32
    wf = {}
    wb = {}
    n_o = np.arange(Co)
    n_c = np.arange(Ci)

    def slot(n, j):  # position of element j (0..31) of row n
        return ((((j >> 3) ^ (((n >> 3) & 1) << 1)) & 3) << 3) | (j & 7)
    for k in codes_present:
        t = proj.copy()
        for i in range(4):
            if (k >> i) & 1:
                t = (t + conv[i]).astype(np.float32)
        bf = torch.from_numpy(t).to(torch.bfloat16).view(torch.int16).numpy().reshape(Co, Ci, 9)
        f = np.zeros((9, nci, Co, 32), np.int16)
        b = np.zeros((9, nco, Ci, 32), np.int16)
        for tap in range(9):
            for cc in range(nci):
                blk = bf[:, cc * 32:(cc + 1) * 32, tap]  # [o][32 c]
                f[tap, cc][n_o[:, None], slot(n_o[:, None], np.arange(32)[None, :])] = blk
            for oc in range(nco):
                blk = bf[oc * 32:(oc + 1) * 32, :, tap].T  # [c][32 o]
                b[tap, oc][n_c[:, None], slot(n_c[:, None], np.arange(32)[None, :])] = blk
        wf[k], wb[k] = f, b
    return wf, wb


@pytest.mark.parametrize("cin,cout,mask", [(64, 96, 0b1000000000010011), (96, 192, 0xffff), (32, 32, 0b10)])
def test_pack_codes_layout_bit_exact(cin, cout, mask):
    """The bf16 code-merged filters (fwd and dX operands) equal, bit for bit, the numpy
    restatement of the packing for every code present; the one-tile tail pads are zero."""
    g = torch.Generator(device=DEV)
    g.manual_seed(cin + cout)
    conv_w = torch.randn((4, cout, cin, 3, 3), generator=g, device=DEV) * 0.05
    proj_w = torch.randn((cout, cin, 3, 3), generator=g, device=DEV) * 0.05
    cm = torch.tensor([mask], dtype=torch.int32, device=DEV)
    wf, wb = ops.dsam_pack(conv_w, proj_w, torch.bfloat16, code_mask=cm)
    present = [k for k in range(16) if (mask >> k) & 1]
    ref_f, ref_b = _pack_reference(conv_w, proj_w, present)
    slab = 9 * cin * cout
    wf16 = wf.view(torch.int16).cpu().numpy().reshape(-1)
    wb16 = wb.view(torch.int16).cpu().numpy().reshape(-1)
    for k in present:
        assert np.array_equal(wf16[k * slab:(k + 1) * slab], ref_f[k].reshape(-1)), f"wfwd code {k}"
        assert np.array_equal(wb16[k * slab:(k + 1) * slab], ref_b[k].reshape(-1)), f"wbwd code {k}"
    assert not wf16[16 * slab:16 * slab + 192 * 32].any() and not wb16[16 * slab:16 * slab + 192 * 32].any()
