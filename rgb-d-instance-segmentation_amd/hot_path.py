"""The fused v0.4.0 hot path as one autograd Function over the HIP kernels.

Reference (mask2former/utils/custom_model.py:324-355), per step:
    cp1 = cp2 = detached clones of the 4 Swin maps                          (:332-333, Q1)
    r   = ratio_predictor(depth) -> .item() per sample (no grad)            (:336, :339-351, Q2)
    for k in 0..2: cp1[k+1] += stack_b dsam_k(cp1[k][b], grey(depth[b]), r[b])   (:339-352, Q4)
    cp2 = DGGM(cp2, grad, mask)                                             (:354)
    out = [cp1_k + cp2_k]                                                   (:355, Q3)
Here:
    decomposition once per image for the three DSAM input resolutions (K3),
    dsam_k over the whole batch in one masked implicit-GEMM launch whose epilogue adds the
      residual colour map (cp1[k+1] = colour[k+1] + dsam_k) and writes the NHWC copy the next
      DSAM reads (K5),
    DGGM gate + final sum in one elementwise pass over all four scales (K2, one launch).
Backward produces exactly the gradients the reference graph has: DSAM / DGGM parameters,
nothing for the colour maps (detached) or the ratio (left the graph via .item()).
"""
import ctypes

import torch

from . import ops

DSAM_PARAMS_PER_MODULE = 9  # conv_layers.{0..3}.{weight,bias}, rgb_projection.weight
_SIDE_STREAMS = {}
_HIP = None


def _hip_stream(dev):
    """A stream of its own (hipStreamCreateWithFlags, non-blocking) wrapped for torch.  torch's
    Stream() hands out one of a fixed pool of 32 streams round-robin, so after enough stream
    creations in a process a "new" capture stream can be the very stream used as a side branch,
    which corrupts a captured graph; these streams are never in that pool."""
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    with torch.cuda.device(dev):
        h = ctypes.c_void_p()
        rc = _HIP.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1))  # hipStreamNonBlocking
        if rc != 0:
            raise RuntimeError(f"hipStreamCreateWithFlags failed ({rc})")
    return torch.cuda.ExternalStream(h.value, device=dev)


def side_stream(dev):
    """The per-device side stream the bf16 path runs its off-critical-path launches on (a
    process-lifetime stream of its own, never one of torch's pooled streams)."""
    s = _SIDE_STREAMS.get(dev.index)
    if s is None:
        s = _SIDE_STREAMS[dev.index] = _hip_stream(dev)
    return s


# bf16 backward: the dW GEMMs of dsam1 and dsam0 in one launch (rgbd_dsam_bwd_weight_planned_multi);
# False runs them as two launches, dW1 on the side stream (bitwise the same gradients)
JOINT_DW = True


class _Side:
    """Fork/join of launches onto the side stream (works eagerly and under graph capture: the side
    stream joins the capture through the fork's event).  One side stream, and never two forks
    back to back from the same point of the main stream: captured graphs with either (a second
    side stream forked beside the first, or the same one forked twice) made hipGraphLaunch
    segfault on ROCm 7.2 once the process had captured and replayed other graphs (measured; see
    DESIGN.md §5.1).  Inputs are recorded on the side stream
    so the allocator does not hand their memory to the main stream while side work reads it;
    outputs are recorded on the main stream at the join."""

    def __init__(self, dev, enabled):
        self.on = enabled
        if enabled:
            self.main = torch.cuda.current_stream(dev)
            self.side = side_stream(dev)
        self.outs = []
        self.forked = False  # launches on the side stream since the last join

    def run(self, fn, *inputs):
        if not self.on:
            return fn()
        self.side.wait_stream(self.main)
        self.forked = True
        for t in inputs:
            t.record_stream(self.side)
        with torch.cuda.stream(self.side):
            out = fn()
        self.outs.append(out)
        return out

    def join(self):
        # a join without a fork since the last one is a no-op: under graph capture, waiting on a
        # side stream that is not part of the capture would tie the graph to outside work
        if not self.on or not self.forked:
            return
        self.forked = False
        self.main.wait_stream(self.side)

        def rec(o):
            if isinstance(o, torch.Tensor):
                o.record_stream(self.main)
            elif isinstance(o, (list, tuple)):
                for x in o:
                    rec(x)
        rec(self.outs)
        self.outs = []


def stack4(ts, view_only=False):
    """torch.stack(ts) for same-shape tensors — as a free view when they already sit back to back
    in one storage (DSAModule keeps its conv weights / biases that way); ``view_only``: None
    instead of copying."""
    t0 = ts[0]
    n, es = t0.numel(), t0.element_size()
    adjacent = all(t.is_contiguous() and t.dtype == t0.dtype and t.device == t0.device and t.shape == t0.shape
                   and t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr()
                   and t.data_ptr() == t0.data_ptr() + i * n * es for i, t in enumerate(ts))
    if adjacent and t0.storage_offset() + len(ts) * n <= t0.untyped_storage().nbytes() // es:
        return t0.as_strided((len(ts),) + tuple(t0.shape), (n,) + tuple(t0.stride()), t0.storage_offset())
    return None if view_only else torch.stack(ts)


class _PackCache:
    """Packed implicit-GEMM weights, built on every call from the current parameters: float32 in
    the segment form, bfloat16 in the code-merged form for the region codes present in this
    batch (``code_mask``), into fresh tensors so a pending backward keeps the filters its forward
    used; ``want_bwd`` adds the dX operand.  (No reuse keyed on parameter versions: the fused
    AdamW step updates parameters in place without bumping their version counters, so such a
    key would go stale after the first optimizer step.)"""

    def get(self, conv_ws, proj_w, dtype, code_mask=None, want_bwd=True):
        if dtype == torch.bfloat16:
            return ops.dsam_pack(stack4([w.detach() for w in conv_ws]), proj_w.detach(), dtype,
                                 code_mask=code_mask, want_bwd=want_bwd)
        return ops.dsam_pack(stack4([w.detach() for w in conv_ws]), proj_w.detach(), dtype)


class Prepared:
    """What the hot path needs before the ratio exists (``prepare``): phase A of the depth
    decomposition (grey plane, histogram, modes: ops.edsam_modes) and, in bf16, the NHWC copies
    of the colour maps — launched on the side stream so they run beside the ratio predictor."""

    def __init__(self, side, pixel_values, modes, colors, nhwc, dtype, sources, packs=None):
        self.side, self.pixel_values, self.modes = side, pixel_values, modes
        self.colors, self.nhwc, self.dtype = colors, nhwc, dtype
        self.packs = packs or {}  # DSAM index -> bf16 packed filters for all 16 codes
        self.sources = sources  # (data_ptr, shape) of the pixel_values and colour maps it was built from

    def check(self, pixel_values, colors):
        """Refuse a Prepared built from other tensors than the ones hot_path() is given: it would
        silently compute features of another batch (the autograd inputs would not be the
        tensors whose copies the kernels read)."""
        got = _sources(pixel_values, colors)
        if got != self.sources:
            raise ValueError("hot_path: `prepared` was built from other pixel_values / colour maps than the ones "
                             "passed (prepare() and hot_path() must get the same tensors)")

    def join(self):
        self.side.join()


def _sources(pixel_values, colors):
    return tuple((t.data_ptr(), tuple(t.shape)) for t in (pixel_values, *colors))


# DSAMs whose bf16 filters prepare() packs for all 16 region codes beside the ratio predictor
# (small: 5 MB / 42 MB; off the critical path), instead of for the codes present after the
# decomposition; dsam2's (16 x 21 MB) stays packed for the present codes only, beside dsam0
PREPACK = (0, 1)


def _pack_all(m, k, dtype):
    conv_ws = [m.conv_layers[i].weight for i in range(4)]
    want_bwd = k > 0 and torch.is_grad_enabled() and m.rgb_projection.weight.requires_grad
    return m._pack_cache.get(conv_ws, m.rgb_projection.weight, dtype, code_mask=None, want_bwd=want_bwd)


def prepare(pixel_values, colors, dtype=torch.float32, overlap=True, dsam_modules=None):
    """Launch the ratio-independent part of the hot path (call it before the ratio predictor,
    pass the result to ``hot_path(..., prepared=)``).  bf16 on the GPU: on the side stream
    (``overlap`` False: on the current stream).  With ``dsam_modules`` (bf16) the filters of the
    PREPACK DSAMs are packed here too, from the parameters as they are now (after the previous
    optimizer step)."""
    pv = pixel_values.detach().float().contiguous()
    cols = [c.detach().to(dtype).contiguous() for c in colors]
    bf16 = dtype == torch.bfloat16
    side = _Side(pv.device, bf16 and pv.is_cuda and overlap)
    held = {}

    def work():
        held["modes"] = m = ops.edsam_modes(pv)
        nhwc = ops.nchw_to_nhwc_multi(cols) if bf16 else None
        packs = {}
        if bf16 and dsam_modules is not None:
            for k in PREPACK:
                packs[k] = _pack_all(dsam_modules[k], k, dtype)
        held["packs"] = packs
        return [m.info, m.ws, m.masks, nhwc, [t for pk in packs.values() for t in pk if t is not None]]
    _, _, _, nhwc, _ = side.run(work, pv, *cols)
    return Prepared(side, pv, held["modes"], cols, nhwc, dtype, _sources(pixel_values, colors), held["packs"])


class HotPathFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pixel_values, ratio, cfg, c0, c1, c2, c3, *params):
        dtype = cfg["dtype"]
        prepared = cfg.get("prepared")
        if prepared is None:
            prepared = prepare(pixel_values, (c0, c1, c2, c3), dtype)
        if prepared.dtype != dtype:
            raise ValueError("hot_path: prepared for another compute dtype")
        colors = prepared.colors
        dsam_p = [params[9 * k:9 * k + 9] for k in range(3)]
        dggm_p = params[27:35]
        sizes = [tuple(c.shape[2:]) for c in colors[:3]]
        bf16 = dtype == torch.bfloat16
        # bf16 on the GPU: the decomposition's modes and the colour-map layout changes ran beside
        # the ratio predictor (prepare); the dsam1 / dsam2 packing runs beside dsam0 and the dW
        # plans beside dsam1 / dsam2 (side stream; joined before their consumers)
        side = _Side(pixel_values.device, bf16 and pixel_values.is_cuda and cfg.get("overlap", True))
        prepared.join()
        nhwc = prepared.nhwc
        if bf16:  # the code-presence masks the bf16 filter packing needs come out of the decomposition
            codes, info, masks = ops.edsam_codes(prepared.modes, ratio.detach(), sizes, code_masks=True)
        else:
            codes, info = ops.edsam_codes(prepared.modes, ratio.detach(), sizes)
            masks = None
        if cfg.get("check_status"):
            ops.raise_on_status(info)
        if cfg.get("status_sink") is not None:
            cfg["status_sink"].append(ops.DeferredStatus(info))
        training = any(ctx.needs_input_grad[7:])
        chans = [(colors[k].shape[1], colors[k + 1].shape[1]) for k in range(3)]
        conv_plans = dw_plans = None
        if bf16:
            # every leg's code-dependent set-up planned once, right after the decomposition: the
            # forward and dX legs by two launches here, the dW legs on the side stream below
            legs = [(ops.LEG_FWD, codes[k], *chans[k]) for k in range(3)]
            if training:
                legs += [(ops.LEG_DX, codes[k], *chans[k]) for k in (1, 2)]
            conv_plans = ops.dsam_plan(legs)

        def pack(k):
            pre = prepared.packs.get(k)
            if pre is not None and (pre[1] is not None or not (training and k > 0)):
                return pre  # packed for all codes beside the ratio predictor
            return cfg["pack_cache"][k].get(dsam_p[k][0:8:2], dsam_p[k][8], dtype,
                                            code_mask=None if masks is None else masks[k:k + 1],
                                            want_bwd=training and k > 0)  # dsam0's input takes no gradient
        cp1 = [colors[0]]
        if bf16:
            packs = [pack(0)]
            packs += side.run(lambda: [pack(1), pack(2)], masks)
            x_nhwc = [nhwc[0]]
            res_nhwc = nhwc[1:]
            # bf16 cascade entirely in NHWC: each DSAM adds its residual colour map in NHWC and writes
            # cp1[k+1] once, in the layout the next DSAM reads and the DGGM pass accepts
            dggm_early = None
            for k in range(3):
                if k == 1:
                    side.join()  # the dsam1 / dsam2 packs
                    if training:  # dW plans beside the rest of the forward
                        dw_plans = side.run(lambda: ops.dsam_plan([(ops.LEG_DW, codes[j], *chans[j]) for j in range(3)]),
                                            *codes)
                if k == 2:  # DGGM gate + sum of scales 0-2 beside dsam2 (their cp1 are final now)
                    dggm_early = side.run(lambda: ops.dggm_fuse_fwd_multi(cp1[0:3], colors[0:3], pixel_values,
                                                                          dggm_p[0:6:2], dggm_p[1:6:2],
                                                                          cp1_nhwc=(1, 2)),
                                          *cp1[0:3], *colors[0:3], pixel_values)
                bias4 = stack4([b.detach() for b in dsam_p[k][1:8:2]])
                out_nhwc = ops.dsam_fwd_nhwc(x_nhwc[k], codes[k], info, packs[k][0], bias4, residual_nhwc=res_nhwc[k],
                                             plan=conv_plans[k])
                cp1.append(out_nhwc)
                if k < 2:
                    x_nhwc.append(out_nhwc)
            cp1_nhwc = (1, 2, 3)
        else:
            packs = [pack(k) for k in range(3)]
            x_nhwc = [ops.nchw_to_nhwc(colors[0])]
            for k in range(3):
                bias4 = stack4([b.detach() for b in dsam_p[k][1:8:2]])
                out, out_nhwc = ops.dsam_fwd(x_nhwc[k], codes[k], info, packs[k][0], bias4, residual=colors[k + 1],
                                             want_nhwc=(k < 2))
                cp1.append(out)
                if k < 2:
                    x_nhwc.append(out_nhwc)
            cp1_nhwc = ()
        if bf16:  # scale 3 after dsam2; scales 0-2 ran beside it
            outs = dggm_early + ops.dggm_fuse_fwd_multi(cp1[3:], colors[3:], pixel_values, dggm_p[6::2], dggm_p[7::2],
                                                        cp1_nhwc=(0,))
        else:  # DGGM gate + final sum of all four scales in one launch
            outs = ops.dggm_fuse_fwd_multi(cp1, colors, pixel_values, dggm_p[0::2], dggm_p[1::2], cp1_nhwc=cp1_nhwc)
        side.join()  # the dW plans, DGGM scales 0-2
        ctx.cfg = cfg
        ctx.dx_plans = {1: conv_plans[3], 2: conv_plans[4]} if conv_plans and training else {}
        ctx.dw_plans = dw_plans
        ctx.codes = codes
        ctx.info = info
        ctx.x_nhwc = x_nhwc
        ctx.packs = packs
        ctx.save_for_backward(pixel_values, *dggm_p)
        ctx.dtype = dtype
        ctx.in_dtypes = [c.dtype for c in (c0, c1, c2, c3)]
        return tuple(outs)

    @staticmethod
    def backward(ctx, g0, g1, g2, g3):
        pixel_values, *dggm_p = ctx.saved_tensors
        dtype = ctx.dtype
        G = []
        for k, g in enumerate((g0, g1, g2, g3)):
            if g is None:
                shape = ctx.x_nhwc[0].shape if k == 0 else None
                raise RuntimeError("hot-path backward needs gradients for all four backbone features"
                                   if shape is None else "missing gradient for scale 0")
            G.append(g.to(dtype).contiguous())
        bf16 = dtype == torch.bfloat16
        # bf16 on the GPU: the main stream runs dX2 -> dX1 -> dW1 + dW0 (one launch); the DGGM backward
        # and the dW of dsam2 run beside it on the side stream (their persistent kernels take CUs as the
        # other stream's work drains; every kernel assigns its work dynamically)
        side = _Side(G[0].device, bf16 and G[0].is_cuda and ctx.cfg.get("overlap", True) and ctx.cfg.get("overlap_bwd", True))

        def dggm_bwd():
            out = []
            for k, (dw, db) in enumerate(ops.dggm_fuse_bwd_multi(G, pixel_values, dggm_p[0::2], dggm_p[1::2])):
                out += [dw.reshape(dggm_p[2 * k].shape).to(dggm_p[2 * k].dtype), db.to(dggm_p[2 * k + 1].dtype)]
            return out
        grads_dggm = side.run(dggm_bwd, *G, pixel_values)
        # DSAM cascade backward: d cp1[k+1] = G[k+1] + dX_{k+1}.  bfloat16 keeps the cascade in
        # NHWC (dX written NHWC only, its residual G[k] converted once; bias sums from NHWC).
        hook = ctx.cfg.get("grad_hook")
        dcp = G[3]
        # bf16: the three upstream gradients the cascade reads in NHWC, converted by one launch
        g_nhwc = dict(zip((3, 2, 1), ops.nchw_to_nhwc_multi([G[3], G[2], G[1]]))) if bf16 else {}
        dcp_nhwc = g_nhwc[3] if bf16 else ops.nchw_to_nhwc(dcp)
        grads_dsam = [None, None, None]
        def dsam_dw(k, dcp, dcp_nhwc):
            dconv, dproj, dbias = ops.dsam_bwd_weight(None if bf16 else dcp, ctx.x_nhwc[k], ctx.codes[k], ctx.info,
                                                      gout_nhwc=dcp_nhwc,
                                                      plan=ctx.dw_plans[k] if ctx.dw_plans else None)
            if k == 0:  # dW0 needs nothing from the side stream; the hook and the caller do
                side.join()
            return dsam_dw_grads(k, dconv, dproj, dbias)

        def dsam_dw_grads(k, dconv, dproj, dbias):
            gk = []
            for i in range(4):
                gk += [dconv[i], dbias[i]]
            gk.append(dproj)
            if hook is not None:  # DDP: this module's all-reduce runs under the rest of the cascade
                hook(2 - k, gk if k > 0 else gk + grads_dggm)
            return gk

        def dsam_dx(k, dcp, dcp_nhwc):
            if bf16:
                return ops.dsam_bwd_data(dcp_nhwc, ctx.codes[k], ctx.packs[k][1], None, want_nhwc=True,
                                         want_nchw=False, gin_nhwc=g_nhwc[k], plan=ctx.dx_plans.get(k))
            return ops.dsam_bwd_data(dcp_nhwc, ctx.codes[k], ctx.packs[k][1], G[k], want_nhwc=(k > 1))
        # dW2 beside the cascade; dX2, dX1, then dW1 and dW0 on the main stream (the side stream
        # already carries the DGGM backward, dW2 and, with in-backward optimizer steps, the
        # dsam2 update)
        grads_dsam = [None, None, None]
        grads_dsam[2] = side.run(lambda: dsam_dw(2, dcp, dcp_nhwc), dcp_nhwc, ctx.x_nhwc[2], ctx.codes[2], ctx.info)
        dcp1, dcp1_nhwc = dsam_dx(2, dcp, dcp_nhwc)
        dcp0, dcp0_nhwc = dsam_dx(1, dcp1, dcp1_nhwc)
        if bf16 and JOINT_DW and ctx.dw_plans:
            # dW1 and dW0 are ready together: their GEMMs share one launch (two whole-chip launches
            # queue behind each other and each drains on a partly idle chip)
            (dw1, dw0) = ops.dsam_bwd_weight_multi([(dcp1_nhwc, ctx.x_nhwc[1], ctx.codes[1], ctx.dw_plans[1]),
                                                    (dcp0_nhwc, ctx.x_nhwc[0], ctx.codes[0], ctx.dw_plans[0])],
                                                   ctx.info)
            side.join()  # the last launches of the backward, the join after them
            grads_dsam[1] = dsam_dw_grads(1, *dw1)
            grads_dsam[0] = dsam_dw_grads(0, *dw0)
        else:
            grads_dsam[1] = side.run(lambda: dsam_dw(1, dcp1, dcp1_nhwc), dcp1_nhwc, ctx.x_nhwc[1], ctx.codes[1],
                                     ctx.info)
            grads_dsam[0] = dsam_dw(0, dcp0, dcp0_nhwc)  # the last launches of the backward, the join after them
        pgrads = grads_dsam[0] + grads_dsam[1] + grads_dsam[2] + grads_dggm
        return (None, None, None, None, None, None, None, *pgrads)


def hot_path(pixel_values, ratio, colors, dsam_modules, dggm_module, dtype=torch.float32, check_status=False,
             grad_hook=None, status_sink=None, prepared=None, overlap=True, overlap_bwd=True):
    """Run the fused hot path.  ``dsam_modules``: the three DSAModule instances;
    ``dggm_module``: the DepthGradientInjectionResidual instance.  ``check_status`` raises the
    reference's ValueError for a degenerate depth histogram right away (synchronising);
    ``status_sink`` (a list) instead receives an ``ops.DeferredStatus`` to check later.
    ``grad_hook(i, grads)``, if
    given, is called during backward as each parameter group's gradients are enqueued, in the
    order of ``distributed.hot_path_grad_groups`` (dsam2, dsam1, dsam0 + DGGM) — the data-parallel
    reducer uses it to overlap the gradient all-reduce with the rest of the backward.
    ``prepared``: ``prepare(pixel_values, colors, dtype)``, launched before the ratio predictor
    (the same pixel_values / colours), so the ratio-free work overlaps it; None = inline.
    ``overlap_bwd`` False keeps only the backward's launches on the current stream (a captured
    data-parallel step overlaps its gradient all-reduces there instead: graph_guard's two branches).
    ``overlap`` False keeps every launch on the current stream (no side stream of the hot path's
    own: a caller that runs other work beside it on a stream of its own, e.g. the next batch's
    ratio predictor, stays within two concurrent branches when captured)."""
    params = []
    for m in dsam_modules:
        for i in range(4):
            params += [m.conv_layers[i].weight, m.conv_layers[i].bias]
        params.append(m.rgb_projection.weight)
    for i in range(4):
        conv = dggm_module.depth_enhancement_layers[i][0]
        params += [conv.weight, conv.bias]
    cfg = {"dtype": dtype, "check_status": check_status, "grad_hook": grad_hook, "status_sink": status_sink,
           "pack_cache": [m._pack_cache for m in dsam_modules], "overlap": overlap, "overlap_bwd": overlap_bwd,
           "prepared": prepared}
    if prepared is not None:
        prepared.check(pixel_values, colors)
    pv = prepared.pixel_values if prepared is not None else pixel_values.detach().float().contiguous()
    return list(HotPathFunction.apply(pv, ratio, cfg, *colors, *params))
