"""HIP path vs oracle / golden vectors on a real MI355X (build contract ③).

Bars: bit-exact for integer / index / byte outputs (pixel_values DGGM planes, histograms,
modes, windows, region codes); float32 mode within FP32_TOL of the PyTorch-CPU fp32
oracle; bfloat16 mode within BF16_TOL (relative to the output scale).
"""
import numpy as np
import pytest
import torch

import golden_inputs as gi
from oracle import dggm as dggm_o, dggm_pre, edsam, hot_path as hot_o
from rgbd_amd import init as winit, synthetic

pytestmark = pytest.mark.gpu

FP32_TOL = dict(rtol=1e-4, atol=1e-4)
BF16_REL = 3e-2  # max-abs error / max-abs value, bf16 operands with f32 accumulation

DEV = "cuda"


def _ops():
    from rgbd_amd import ops
    return ops


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


# ------------------------------------------------------------------ K1
@pytest.mark.parametrize("H,W,B", [(64, 96, 3), (240, 320, 2), (90, 125, 2), (480, 640, 1)])
def test_assemble_pixel_values_bit_exact(H, W, B):
    ops = _ops()
    scenes = [synthetic.make_scene(5000 + 17 * H + b, H, W) for b in range(B)]
    depth = np.stack([s["depth_u8"] for s in scenes])
    rgb = np.stack([s["rgb_u8"] for s in scenes])
    pv = ops.assemble_pixel_values(torch.from_numpy(depth).to(DEV), torch.from_numpy(rgb).to(DEV)).cpu().numpy()
    for b in range(B):
        ref = np.concatenate([synthetic.rgbd_planes(scenes[b]), dggm_pre.dggm_planes(depth[b])])
        np.testing.assert_array_equal(bits(pv[b]), bits(ref))


def test_assemble_degenerate_depth():
    ops = _ops()
    d = np.zeros((2, 16, 24), np.uint8)          # all invalid -> no valid gradient
    d[1] = 77                                      # constant -> zero gradient everywhere
    pv = ops.assemble_pixel_values(torch.from_numpy(d).to(DEV)).cpu().numpy()
    for b in range(2):
        np.testing.assert_array_equal(bits(pv[b, 6:]), bits(dggm_pre.dggm_planes(d[b])))


# ------------------------------------------------------------------ K3
CASES = gi.decomposition_cases()


def _decompose(split, pv, ratio, sizes, code_masks=False):
    """The single-call decomposition, or its two phases (rgbd_edsam_modes, then
    rgbd_edsam_codes on the grey plane the first one kept) as the hot path runs them."""
    ops = _ops()
    if not split:
        return ops.edsam_decompose(pv, ratio, sizes, code_masks=code_masks)
    return ops.edsam_codes(ops.edsam_modes(pv), ratio, sizes, code_masks=code_masks)


@pytest.mark.parametrize("split", [False, True], ids=["one_call", "two_phases"])
@pytest.mark.parametrize("i", range(len(CASES)), ids=[c[0] for c in CASES])
def test_decomposition_matches_reference_fixture(golden, i, split):
    ops = _ops()
    g1 = golden("g1_decompose")
    name, d3, r = CASES[i]
    H, W = d3.shape[1:]
    sizes = gi.pool_sizes(H, W)
    codes, info = _decompose(split, torch.from_numpy(d3)[None].to(DEV),
                             torch.tensor([r], dtype=torch.float32, device=DEV), sizes)
    rec = ops.decode_info(info)[0]
    if str(g1["error"][i]):
        assert rec["status"] != 0
        with pytest.raises(ValueError):
            ops.raise_on_status(info)
        return
    assert rec["status"] == 0
    np.testing.assert_array_equal(rec["hist"], g1[f"{i}_hist"])
    n = int(g1[f"{i}_n_modes"])
    assert rec["n_modes"] == n
    assert rec["n_masks"] == (n + 1 if n else 4)
    np.testing.assert_array_equal(bits(rec["center"][:n]), bits(g1[f"{i}_centers"]))
    win = g1[f"{i}_windows"]
    np.testing.assert_array_equal(bits(rec["lo"][:n]), bits(win[:, 0].astype(np.float32)))
    np.testing.assert_array_equal(bits(rec["hi"][:n]), bits(win[:, 1].astype(np.float32)))
    for s in range(3):
        np.testing.assert_array_equal(codes[s][0].cpu().numpy(), g1[f"{i}_pooled{s}"])


@pytest.mark.parametrize("split", [False, True], ids=["one_call", "two_phases"])
def test_decomposition_batch_full_size(split):
    """Batch of 8 NYUv2-shaped (480x640) scenes, ratios in [0.01, 0.5]: every image matches
    the oracle bit-for-bit when decomposed together in one launch sequence (or in the hot
    path's two phases); the code-presence masks equal the codes' own."""
    ops = _ops()
    planes, _, _ = synthetic.make_batch(2, 8, 480, 640)
    ratios = np.linspace(0.01, 0.5, 8).astype(np.float32)
    sizes = gi.pool_sizes(480, 640)
    codes, info, masks = _decompose(split, torch.from_numpy(planes).to(DEV), torch.from_numpy(ratios).to(DEV), sizes,
                                    code_masks=True)
    for s in range(3):
        want = 0
        for v in np.unique(codes[s].cpu().numpy()):
            want |= 1 << int(v)
        assert int(masks[s]) == want
    rec = ops.decode_info(info)
    for b in range(8):
        dec = edsam.decompose(planes[b, 3:6], float(ratios[b]))
        np.testing.assert_array_equal(rec[b]["hist"], dec["hist"])
        assert rec[b]["n_modes"] == dec["n_modes"]
        for s, (oh, ow) in enumerate(sizes):
            np.testing.assert_array_equal(codes[s][b].cpu().numpy(), edsam.pooled_codes(dec["code"], oh, ow))


# ------------------------------------------------------------------ K5 DSAM
def _dsam_module(prefix, cin, cout, dtype=torch.float32):
    from rgbd_amd.modules import DSAModule
    m = DSAModule(cin, cout)
    winit.init_deterministic(m, prefix=prefix)
    m.compute_dtype = dtype
    return m.to(DEV)


@pytest.mark.parametrize("tag,cin,cout", [("a", 8, 16), ("b", 16, 32)])
def test_dsam_forward_golden(golden, tag, cin, cout):
    g2 = golden("g2_dsam")
    m = _dsam_module(f"g2.{tag}.", cin, cout)
    for ci, case_idx in enumerate(gi.G2_CASES):
        _, d3, r = CASES[case_idx]
        grey = torch.from_numpy(edsam.to_grayscale(d3)).to(DEV)
        with torch.no_grad():
            y = m(torch.from_numpy(g2[f"{tag}_{ci}_x"]).to(DEV), grey, r).cpu().numpy()
        np.testing.assert_allclose(y, g2[f"{tag}_{ci}_y"], **FP32_TOL)


def _oracle_dsam_params(m):
    return dict(conv_w=torch.stack([m.conv_layers[i].weight.detach().cpu() for i in range(4)]),
                conv_b=torch.stack([m.conv_layers[i].bias.detach().cpu() for i in range(4)]),
                proj_w=m.rgb_projection.weight.detach().cpu())


@pytest.mark.parametrize("k", [0, 1, 2])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dsam_real_channels_fwd_bwd(k, dtype):
    """Each v0.4.0 DSAM (96->192, 192->384, 384->768) at 240x320 input, B=2: forward and all
    gradients (dX, dW, db) against PyTorch-CPU fp32 autograd of the oracle."""
    cin, cout = [(96, 192), (192, 384), (384, 768)][k]
    H, W = 240, 320
    h, w = gi.swin_sizes(H, W)[k]
    m = _dsam_module(f"t.dsam{k}.", cin, cout, dtype)
    planes, _, _ = synthetic.make_batch(3, 2, H, W)
    ratios = [0.12, 0.31]
    x = torch.from_numpy(gi.feature(f"t.x{k}", (2, cin, h, w))).to(DEV).requires_grad_(True)
    gout = torch.from_numpy(gi.feature(f"t.g{k}", (2, cout, (h + 1) // 2, (w + 1) // 2)))
    from rgbd_amd import ops
    d3 = torch.from_numpy(planes[:, 3:6]).to(DEV)
    grey = (0.299 * d3[:, 0] + 0.587 * d3[:, 1]) + 0.114 * d3[:, 2]
    y = m(x, grey[:, None], torch.tensor(ratios, device=DEV))
    y.backward(gout.to(DEV))
    # oracle (per sample, reference semantics) with autograd
    p = {kk: v.clone().requires_grad_(True) for kk, v in _oracle_dsam_params(m).items()}
    xr = x.detach().cpu().clone().requires_grad_(True)
    ys = []
    for b in range(2):
        dec = edsam.decompose(planes[b, 3:6], ratios[b])
        ys.append(edsam.dsam_forward(xr[b:b + 1], dec["code"], dec["n_masks"], **p))
    yr = torch.cat(ys)
    yr.backward(gout)
    got = {"y": y.detach().float().cpu(), "dx": x.grad.float().cpu(),
           "dw": torch.stack([m.conv_layers[i].weight.grad.cpu() for i in range(4)]),
           "db": torch.stack([m.conv_layers[i].bias.grad.cpu() for i in range(4)]),
           "dp": m.rgb_projection.weight.grad.cpu()}
    ref = {"y": yr.detach(), "dx": xr.grad, "dw": p["conv_w"].grad, "db": p["conv_b"].grad, "dp": p["proj_w"].grad}
    for key in got:
        a, e = got[key].numpy(), ref[key].numpy()
        if dtype == torch.float32:
            scale = max(1.0, float(np.abs(e).max()))
            np.testing.assert_allclose(a, e, rtol=1e-4, atol=1e-4 * scale, err_msg=key)
        else:
            rel = np.abs(a - e).max() / max(np.abs(e).max(), 1e-6)
            assert rel < BF16_REL, f"{key}: bf16 rel err {rel}"


# ------------------------------------------------------------------ K2 DGGM
def test_dggm_forward_golden(golden):
    from rgbd_amd.modules import DepthGradientInjectionResidual
    g3 = golden("g3_dggm")
    m = DepthGradientInjectionResidual([4, 8, 16, 32], 3)
    winit.init_deterministic(m, prefix="g3.")
    m = m.to(DEV)
    with torch.no_grad():
        outs = m([torch.from_numpy(g3[f"color{i}"]).to(DEV) for i in range(4)],
                 torch.from_numpy(g3["grad"]).to(DEV), torch.from_numpy(g3["mask"]).to(DEV))
    for i in range(4):
        np.testing.assert_allclose(outs[i].cpu().numpy(), g3[f"out{i}"], rtol=1e-5, atol=1e-5)


def test_dggm_backward_vs_autograd(golden):
    from rgbd_amd.modules import DepthGradientInjectionResidual
    g3 = golden("g3_dggm")
    m = DepthGradientInjectionResidual([4, 8, 16, 32], 3)
    winit.init_deterministic(m, prefix="g3.")
    mr = DepthGradientInjectionResidual([4, 8, 16, 32], 3)
    mr.load_state_dict(m.state_dict())
    m = m.to(DEV)
    cols = [torch.from_numpy(g3[f"color{i}"]) for i in range(4)]
    gs = [torch.from_numpy(gi.feature(f"gg{i}", tuple(c.shape))) for i, c in enumerate(cols)]
    outs = m([c.to(DEV) for c in cols], torch.from_numpy(g3["grad"]).to(DEV), torch.from_numpy(g3["mask"]).to(DEV))
    torch.autograd.backward(outs, [g.to(DEV) for g in gs])
    ws = [l[0].weight.detach().clone().requires_grad_(True) for l in mr.depth_enhancement_layers]
    bs = [l[0].bias.detach().clone().requires_grad_(True) for l in mr.depth_enhancement_layers]
    ro = dggm_o.dggm_forward(cols, torch.from_numpy(g3["grad"]), torch.from_numpy(g3["mask"]), ws, bs)
    torch.autograd.backward(ro, gs)
    for i in range(4):
        np.testing.assert_allclose(m.depth_enhancement_layers[i][0].weight.grad.cpu().numpy(), ws[i].grad.numpy(),
                                   rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(m.depth_enhancement_layers[i][0].bias.grad.cpu().numpy(), bs[i].grad.numpy(),
                                   rtol=1e-4, atol=1e-4)


# ------------------------------------------------------------------ a1 hot path (fused)
def _hot_modules(dtype):
    from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual
    pre = "model.pixel_level_module."
    dsams = []
    for k, (ci, co) in enumerate([(96, 192), (192, 384), (384, 768)]):
        m = DSAModule(ci, co)
        winit.init_deterministic(m, prefix=f"{pre}dsam{k}.")
        dsams.append(m.to(DEV))
    dg = DepthGradientInjectionResidual([96, 192, 384, 768], 3)
    winit.init_deterministic(dg, prefix=f"{pre}depth_gradient_injection.")
    return dsams, dg.to(DEV)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_hot_path_fused_vs_oracle(dtype):
    """The fused HotPathFunction at 240x320, B=2 with injected ratios: the 4 backbone
    features and every hot-path parameter gradient against the oracle (custom_model.py:324-355)."""
    from rgbd_amd.hot_path import hot_path
    H, W, B = 240, 320, 2
    pv = torch.from_numpy(gi.pixel_values(7, B, H, W))
    ratios = torch.tensor([[0.2], [0.07]], dtype=torch.float32)
    sizes = gi.swin_sizes(H, W)
    colors = [torch.from_numpy(gi.feature(f"hp.c{k}", (B, c, *sizes[k])))
              for k, c in enumerate([96, 192, 384, 768])]
    gouts = [torch.from_numpy(gi.feature(f"hp.g{k}", tuple(c.shape))) for k, c in enumerate(colors)]
    dsams, dg = _hot_modules(dtype)
    outs = hot_path(pv.to(DEV), ratios.to(DEV), [c.to(DEV) for c in colors], dsams, dg, dtype=dtype,
                    check_status=True)
    torch.autograd.backward(outs, [g.to(DEV).to(dtype) for g in gouts])
    sd = {}
    for k, m in enumerate(dsams):
        for kk, v in m.state_dict().items():
            sd[f"dsam{k}.{kk}"] = v.detach().cpu().clone().requires_grad_(True)
    for kk, v in dg.state_dict().items():
        sd[f"depth_gradient_injection.{kk}"] = v.detach().cpu().clone().requires_grad_(True)
    # the oracle stacks conv weights itself; keep leaf tensors for grads
    ref, _, _ = hot_o.hot_path_forward(colors, pv, sd, ratios=ratios)
    torch.autograd.backward(ref, gouts)
    for k in range(4):
        a, e = outs[k].detach().float().cpu().numpy(), ref[k].detach().numpy()
        if dtype == torch.float32:
            np.testing.assert_allclose(a, e, rtol=1e-4, atol=1e-3, err_msg=f"feature {k}")
        else:
            assert np.abs(a - e).max() / np.abs(e).max() < BF16_REL, f"feature {k}"
    named = {}
    for k, m in enumerate(dsams):
        for n, p in m.named_parameters():
            named[f"dsam{k}.{n}"] = p
    for n, p in dg.named_parameters():
        named[f"depth_gradient_injection.{n}"] = p
    for n, p in named.items():
        a, e = p.grad.float().cpu().numpy(), sd[n].grad.numpy()
        scale = max(float(np.abs(e).max()), 1e-6)
        err = np.abs(a - e).max() / scale
        assert err < (2e-4 if dtype == torch.float32 else BF16_REL), f"{n}: rel err {err}"


def test_hot_path_joint_dw_bitwise():
    """bfloat16 backward: dsam1's and dsam0's dW GEMMs in one launch (hot_path.JOINT_DW) give
    bitwise the parameter gradients of the two-launch schedule."""
    from rgbd_amd import hot_path as hp
    H, W, B = 240, 320, 2
    pv = torch.from_numpy(gi.pixel_values(7, B, H, W)).to(DEV)
    ratios = torch.tensor([[0.2], [0.07]], dtype=torch.float32, device=DEV)
    sizes = gi.swin_sizes(H, W)
    colors = [torch.from_numpy(gi.feature(f"hp.c{k}", (B, c, *sizes[k]))).to(DEV)
              for k, c in enumerate([96, 192, 384, 768])]
    gouts = [torch.from_numpy(gi.feature(f"hp.g{k}", tuple(c.shape))).to(DEV, torch.bfloat16) for k, c in
             enumerate(colors)]
    dsams, dg = _hot_modules(torch.bfloat16)
    params = [p for m in dsams for p in m.parameters()] + list(dg.parameters())
    grads = []
    old = hp.JOINT_DW
    try:
        for joint in (True, False):
            hp.JOINT_DW = joint
            for p in params:
                p.grad = None
            outs = hp.hot_path(pv, ratios, colors, dsams, dg, dtype=torch.bfloat16)
            torch.autograd.backward(outs, gouts)
            grads.append([p.grad.clone() for p in params])
    finally:
        hp.JOINT_DW = old
    for a, b in zip(*grads):
        assert torch.equal(a, b)


# ------------------------------------------------------------------ C5: RealSense 1280x720
def test_c5_assemble_and_decompose_1280x720():
    """BASELINE config C5 (RealSense 1280x720): 10-channel assembly incl. the DGGM Sobel planes
    bit-exact, and the decomposition (histogram, modes, region codes at the three DSAM input
    resolutions 180x320 / 90x160 / 45x80) bit-exact against the oracle, two frames in one batch."""
    ops = _ops()
    H, W, B = 720, 1280, 2
    scenes = [synthetic.make_scene(synthetic.scene_seed(5, i), H, W) for i in range(B)]
    depth = torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(DEV)
    rgb = torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).contiguous().to(DEV)
    pv = ops.assemble_pixel_values(depth, rgb).cpu().numpy()
    for b, s in enumerate(scenes):
        exp = np.concatenate([synthetic.rgbd_planes(s), dggm_pre.dggm_planes(s["depth_u8"])])
        np.testing.assert_array_equal(bits(pv[b]), bits(exp))
    ratios = np.array([0.1, 0.33], dtype=np.float32)
    sizes = gi.pool_sizes(H, W)
    assert sizes[0] == (180, 320) and sizes[2] == (45, 80)
    codes, info = ops.edsam_decompose(torch.from_numpy(pv).to(DEV), torch.from_numpy(ratios).to(DEV), sizes)
    rec = ops.decode_info(info)
    for b in range(B):
        dec = edsam.decompose(pv[b, 3:6], float(ratios[b]))
        np.testing.assert_array_equal(rec[b]["hist"], dec["hist"])
        assert rec[b]["n_modes"] == dec["n_modes"]
        for s, (oh, ow) in enumerate(sizes):
            np.testing.assert_array_equal(codes[s][b].cpu().numpy(), edsam.pooled_codes(dec["code"], oh, ow))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_c5_hot_path_forward_1280x720(dtype):
    """C5 streaming inference shape (B=1, 1280x720; Swin maps 180x320 ... 23x40, so the last DSAM
    sees an odd 45x80 -> 23x40 reduction): fused forward vs the oracle."""
    from rgbd_amd.hot_path import hot_path
    H, W, B = 720, 1280, 1
    pv = torch.from_numpy(gi.pixel_values(9, B, H, W))
    ratios = torch.tensor([[0.15]], dtype=torch.float32)
    sizes = gi.swin_sizes(H, W)
    assert sizes[3] == (23, 40)
    colors = [torch.from_numpy(gi.feature(f"c5.c{k}", (B, c, *sizes[k])))
              for k, c in enumerate([96, 192, 384, 768])]
    dsams, dg = _hot_modules(dtype)
    with torch.no_grad():
        outs = hot_path(pv.to(DEV), ratios.to(DEV), [c.to(DEV) for c in colors], dsams, dg, dtype=dtype,
                        check_status=True)
    sd = {}
    for k, m in enumerate(dsams):
        sd.update({f"dsam{k}.{kk}": v.detach().cpu() for kk, v in m.state_dict().items()})
    sd.update({f"depth_gradient_injection.{kk}": v.detach().cpu() for kk, v in dg.state_dict().items()})
    with torch.no_grad():
        ref, _, _ = hot_o.hot_path_forward(colors, pv, sd, ratios=ratios)
    for k in range(4):
        a, e = outs[k].float().cpu().numpy(), ref[k].numpy()
        if dtype == torch.float32:
            np.testing.assert_allclose(a, e, rtol=1e-4, atol=1e-3, err_msg=f"feature {k}")
        else:
            assert np.abs(a - e).max() / np.abs(e).max() < BF16_REL, f"feature {k}"


def test_streaming_graph_replay_matches_eager():
    """stream.StreamingHotPath: the graph replay gives the eager path's features for a frame, and
    a new frame copied into the static buffers gives that frame's features (no stale state)."""
    from rgbd_amd.modules import EnhancedDepthImageRatioPredictor
    from rgbd_amd.stream import StreamingHotPath
    H, W = 96, 128
    rp = EnhancedDepthImageRatioPredictor(3)
    winit.init_deterministic(rp, prefix="model.pixel_level_module.ratio_predictor.")
    dsams, dg = _hot_modules(torch.bfloat16)
    sp = StreamingHotPath(rp.to(DEV), dsams, dg, H, W, B=1, dtype=torch.bfloat16)
    frames = [synthetic.make_scene(synthetic.scene_seed(6, i), H, W) for i in range(2)]
    g = torch.Generator(device=DEV).manual_seed(2)
    colors = [torch.randn(c.shape, generator=g, device=DEV).to(c.dtype) for c in sp.colors]
    for f in frames:
        d = torch.from_numpy(f["depth_u8"][None]).to(DEV)
        c = torch.from_numpy(f["rgb_u8"][None]).contiguous().to(DEV)
        feats, ratio = sp(d, c, colors)
        feats = [t.clone() for t in feats]
        ratio = ratio.clone()
        with torch.no_grad():
            ref_feats, ref_ratio = sp._run()
        assert torch.equal(ratio, ref_ratio)
        for a, e in zip(feats, ref_feats):
            assert torch.equal(a, e)


def test_graph_survives_a_larger_later_capture():
    """ADVICE r1 (workspaces and captured graphs): a graph keeps pointing at the workspaces it was
    captured with.  Capturing a second, larger path on the same capture stream grows those
    workspaces; the replaced buffers must stay alive (ops._ws_retired), so replaying the first
    graph afterwards still reproduces its own earlier output bit for bit."""
    from rgbd_amd.modules import EnhancedDepthImageRatioPredictor
    from rgbd_amd.stream import StreamingHotPath
    rp = EnhancedDepthImageRatioPredictor(3)
    winit.init_deterministic(rp, prefix="model.pixel_level_module.ratio_predictor.")
    rp = rp.to(DEV)
    dsams, dg = _hot_modules(torch.bfloat16)
    small = StreamingHotPath(rp, dsams, dg, 64, 96, B=1, dtype=torch.bfloat16)
    f = synthetic.make_scene(synthetic.scene_seed(8, 0), 64, 96)
    d = torch.from_numpy(f["depth_u8"][None]).to(DEV)
    c = torch.from_numpy(f["rgb_u8"][None]).contiguous().to(DEV)
    g = torch.Generator(device=DEV).manual_seed(4)
    colors = [torch.randn(t.shape, generator=g, device=DEV).to(t.dtype) for t in small.colors]
    first = [t.clone() for t in small(d, c, colors)[0]]
    big = StreamingHotPath(rp, dsams, dg, 192, 256, B=2, dtype=torch.bfloat16).capture()
    fb = synthetic.make_scene(synthetic.scene_seed(8, 1), 192, 256)
    big(torch.from_numpy(np.stack([fb["depth_u8"]] * 2)).to(DEV),
        torch.from_numpy(np.stack([fb["rgb_u8"]] * 2)).contiguous().to(DEV))
    torch.cuda.synchronize()
    again = small(d, c, colors)[0]
    for a, e in zip(again, first):
        assert torch.equal(a, e)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dggm_multi_scale_equals_per_scale(dtype):
    """rgbd_dggm_fuse_{fwd,bwd}_multi (all scales in one launch, as the fused hot path calls them)
    give bitwise the per-scale entry points' outputs and gradients, incl. PX = 8 / 4 / 1 scales."""
    ops = _ops()
    B, H, W = 2, 97, 130
    pv = torch.from_numpy(gi.pixel_values(12, B, H, W)).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(3)
    shapes = [(96, 25, 33), (192, 13, 17), (384, 7, 9), (768, 4, 4)]   # h*w % 8 / % 4 / odd
    colors = [torch.randn((B, c, h, w), generator=g, device=DEV).to(dtype) for c, h, w in shapes]
    cp1s = [torch.randn((B, c, h, w), generator=g, device=DEV).to(dtype) for c, h, w in shapes]
    wts = [torch.randn((c, 3, 1, 1), generator=g, device=DEV) for c, _, _ in shapes]
    bss = [torch.randn((c,), generator=g, device=DEV) for c, _, _ in shapes]
    for cps in (cp1s, None):
        multi = ops.dggm_fuse_fwd_multi(cps, colors, pv, wts, bss)
        for k in range(4):
            one = ops.dggm_fuse_fwd(None if cps is None else cps[k], colors[k], pv, wts[k], bss[k])
            assert torch.equal(multi[k], one), k
    douts = [torch.randn(c.shape, generator=g, device=DEV).to(dtype) for c in colors]
    multi = ops.dggm_fuse_bwd_multi(douts, pv, wts, bss)
    for k in range(4):
        dw, db = ops.dggm_fuse_bwd(douts[k], pv, wts[k], bss[k])
        assert torch.equal(multi[k][0], dw) and torch.equal(multi[k][1], db), k
