"""Torch-facing wrappers of the librgbd_hip.so entry points (one per C-ABI function).

Every wrapper validates shapes/devices on the host, allocates outputs with torch (device
memory is plumbing), passes raw pointers + the current HIP stream to the C ABI and raises
``RgbdHipError`` on a non-zero return.  Nothing here synchronises with the device except
``decode_info`` (explicitly a host read-back for tests/diagnostics).
"""
import collections
import contextlib
import threading
import ctypes
import math

import numpy as np
import torch

from . import _lib
from ._lib import RGBD_BF16, RGBD_F32, DECOMP_INFO_DTYPE, check

_ws_cache = {}
# Workspaces replaced by a larger one stay alive for the life of the process: a HIP graph
# captured earlier (stream.StreamingHotPath) keeps the raw pointer of the buffer it was
# captured with, so that buffer must never return to the caching allocator.
_ws_retired = []


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return RGBD_F32
    if t.dtype == torch.bfloat16:
        return RGBD_BF16
    raise TypeError(f"rgbd_amd kernels take float32 or bfloat16 tensors, got {t.dtype}")


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("rgbd_amd ops run on the GPU only (no CPU fallback); got a CPU tensor")
        if t is not None and not t.is_contiguous():
            raise RuntimeError("rgbd_amd ops expect contiguous tensors")


_ws_zeroed = set()  # keys of the workspaces whose contents calls rely on (counters left at zero)


def _workspace(dev, nbytes: int, tag: str, zeroed: bool = False):
    """Scratch buffer for one entry point, one per (device, tag, stream): launches on two
    streams never share one, and launches on one stream are ordered.  Never freed (see
    ``_ws_retired``).  ``zeroed``: a new buffer starts as zeros (entry points whose workspace
    holds counters that each call leaves at zero, e.g. rgbd_colsum's tickets)."""
    key = (dev, tag, torch.cuda.current_stream(dev).cuda_stream)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        if buf is not None:
            _ws_retired.append(buf)
        alloc = torch.zeros if zeroed else torch.empty
        buf = alloc(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
        _ws_cache[key] = buf
    if zeroed:
        _ws_zeroed.add(key)
    return buf


# ------------------------------------------------------------------ small host constants
# Shapes, offsets and counts the model builds from Python numbers every step (the pixel decoder's
# level shapes, the matcher's per-image offsets, the loss's instance count) would each be a
# blocking host->device copy — torch synchronises the stream behind a pageable copy, draining the
# GPU queue — and cannot be captured into a graph.  They are the same numbers step after step,
# so each distinct value is copied once and the device tensor reused (read-only by contract).
# Values that change with the batch (the matcher's per-image target counts) would make the table
# grow without bound over a training run, so it is least-recently-used with a cap; a constant a
# captured graph reads is pinned (the graph holds its address, not a reference).
_consts = collections.OrderedDict()
_pinned = set()
_CONST_CAP = 512


def capturing() -> bool:
    """True while the current stream is being captured into a graph (False without a GPU)."""
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _freeze(v):
    if isinstance(v, (list, tuple)):
        return tuple(_freeze(x) for x in v)
    if isinstance(v, (bool, int, float)):
        return v
    raise TypeError("device_const: numbers or nested lists / tuples of numbers only")


def device_const(values, dtype, device, _nonblocking=False):
    """A device tensor holding ``values`` (numbers, nested lists / tuples), copied once per
    distinct (values, dtype, device) and shared: callers must not modify it."""
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (_freeze(values), dtype, device)
    t = _consts.get(key)
    cap = device.type == "cuda" and capturing()
    if t is None:
        if cap:
            raise RuntimeError("device_const: a new constant during graph capture (run the step eagerly first)")
        if _nonblocking and device.type == "cuda":
            # the caching host allocator keeps the pinned block until the copy has run
            t = torch.tensor(values, dtype=dtype).pin_memory().to(device, non_blocking=True)
        else:
            t = torch.tensor(values, dtype=dtype).to(device)
        _consts[key] = t
        if len(_consts) > _CONST_CAP:
            for old in [k for k in _consts if k not in _pinned][:len(_consts) - _CONST_CAP]:
                del _consts[old]
    else:
        _consts.move_to_end(key)
    if cap:
        _pinned.add(key)
    return t


def device_vec(values, dtype, device):
    """A device tensor of ``values`` (a number or a flat list) that change from call to call
    (per-batch counts and offsets): device_const's shared tensor when these values were seen
    before (no copy at all), else a copy from pinned memory that neither blocks the host nor
    drains the stream, kept in device_const's cache — so a graph capture after an eager warm-up
    step of the same batch finds it (a capture cannot copy from host memory: replays would read
    stale bytes)."""
    return device_const(values, dtype, device, _nonblocking=True)


_hc_local = threading.local()
_hc_lock = threading.Lock()
_hc_state = {"orig": None, "users": 0}


def _hc_as_tensor(data, dtype=None, device=None):
    orig = _hc_state["orig"]
    if (getattr(_hc_local, "depth", 0) > 0 and device is not None and torch.device(device).type == "cuda"
            and not isinstance(data, torch.Tensor)):
        try:
            frozen = _freeze(data)
        except TypeError:
            return orig(data, dtype=dtype, device=device)
        return device_const(frozen, orig(data, dtype=dtype).dtype, device)
    return orig(data, dtype=dtype, device=device)


@contextlib.contextmanager
def host_constants():
    """Inside the block, ``torch.as_tensor(numbers, device=cuda)`` called FROM THIS THREAD returns
    the shared ``device_const`` (library code outside this package calls it on every forward, e.g.
    the HF pixel decoder's level shapes, modeling_mask2former.py:1347); other threads (data
    loaders, pin-memory workers) and anything else go to torch's own function unchanged."""
    with _hc_lock:
        if _hc_state["users"] == 0:
            _hc_state["orig"] = torch.as_tensor
            torch.as_tensor = _hc_as_tensor
        _hc_state["users"] += 1
    _hc_local.depth = getattr(_hc_local, "depth", 0) + 1
    try:
        yield
    finally:
        _hc_local.depth -= 1
        with _hc_lock:
            _hc_state["users"] -= 1
            if _hc_state["users"] == 0:
                torch.as_tensor = _hc_state["orig"]
                _hc_state["orig"] = None


# ------------------------------------------------------------------ K1 DGGM-pre / assembly
def assemble_pixel_values(depth_u8: torch.Tensor, rgb_u8: torch.Tensor = None, out: torch.Tensor = None):
    """depth_u8 [B,H,W] uint8 (+ rgb_u8 [B,H,W,3]) -> pixel_values float32 [B,10,H,W]
    (map_10channel_case2 layout, dataloader.py:386-425; DGGM-pre data_process.py:1247-1305)."""
    depth_u8 = depth_u8.contiguous()
    rgb_u8 = None if rgb_u8 is None else rgb_u8.contiguous()
    _need_cuda(depth_u8, rgb_u8)
    if depth_u8.dtype != torch.uint8 or depth_u8.dim() != 3:
        raise ValueError("depth_u8 must be uint8 [B,H,W]")
    B, H, W = depth_u8.shape
    if rgb_u8 is not None and (rgb_u8.dtype != torch.uint8 or tuple(rgb_u8.shape) != (B, H, W, 3)):
        raise ValueError("rgb_u8 must be uint8 [B,H,W,3]")
    if out is None:  # every plane is written when RGB is given; planes 0:3 stay zero otherwise
        alloc = torch.empty if rgb_u8 is not None else torch.zeros
        out = alloc((B, 10, H, W), dtype=torch.float32, device=depth_u8.device)
    L = _lib.lib()
    ws = _workspace(depth_u8.device, L.rgbd_assemble_workspace_size(B), "assemble")
    check(L.rgbd_assemble_pixel_values(_p(rgb_u8), _p(depth_u8), B, H, W, _p(out), _p(ws),
                                       _stream(depth_u8.device)), "rgbd_assemble_pixel_values")
    return out


# ------------------------------------------------------------------ K3 decomposition
def _depth_planes(pixel_values):
    _need_cuda(pixel_values)
    if pixel_values.dtype != torch.float32:
        raise TypeError("the decomposition consumes float32 depth (SURVEY §7 (i))")
    B, C, H, W = pixel_values.shape
    nch = 1 if C == 1 else 3
    depth3 = pixel_values if C in (1, 3) else pixel_values[:, 3:6]
    return depth3, nch, B, H, W


def _ratio_vec(ratio, B):
    _need_cuda(ratio)
    r = ratio.reshape(-1).to(torch.float32).contiguous()
    if r.numel() != B:
        raise ValueError("one ratio per image expected")
    return r


def _scale_args(sizes, B, dev):
    n = len(sizes)
    codes = [torch.empty((B, h, w), dtype=torch.uint8, device=dev) for (h, w) in sizes]
    oh = (ctypes.c_int * max(n, 1))(*[s[0] for s in sizes])
    ow = (ctypes.c_int * max(n, 1))(*[s[1] for s in sizes])
    cp = (ctypes.c_void_p * max(n, 1))(*[c.data_ptr() for c in codes])
    return n, codes, oh, ow, cp


def edsam_decompose(pixel_values: torch.Tensor, ratio: torch.Tensor, sizes, code_masks=False):
    """Depth decomposition of every image, once for all DSAMs.

    pixel_values: float32 [B,C>=6,H,W] (depth planes = channels 3:6, custom_model.py:326), a
    [B,3,H,W] depth tensor, or a [B,1,H,W] already-grey map; ratio: float32 [B] or [B,1] on device; sizes: list of (h, w).
    Returns (codes list of uint8 [B,h,w], info uint8 [B, 2116] device tensor); with
    ``code_masks`` also the int32 device tensor [len(sizes)] of dsam_code_masks(codes), made by
    the decomposition itself (rgbd_edsam_decompose_masks).  Both phases on the current stream;
    ``edsam_modes`` + ``edsam_codes`` split them (the hot path runs the first beside the ratio
    predictor)."""
    depth3, nch, B, H, W = _depth_planes(pixel_values)
    r = _ratio_vec(ratio, B)
    dev = pixel_values.device
    n, codes, oh, ow, cp = _scale_args(sizes, B, dev)
    info = torch.empty((B, DECOMP_INFO_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    L = _lib.lib()
    ws = _workspace(dev, L.rgbd_edsam_decompose_workspace_size(B), "decompose")
    if code_masks:
        masks = torch.empty((max(n, 1),), dtype=torch.int32, device=dev)
        check(L.rgbd_edsam_decompose_masks(ctypes.c_void_p(depth3.data_ptr()), depth3.stride(0), nch, B, H, W, _p(r),
                                           n, oh, ow, cp, _p(info), _p(masks), _p(ws), _stream(dev)),
              "rgbd_edsam_decompose_masks")
        return codes, info, masks[:n]
    check(L.rgbd_edsam_decompose(ctypes.c_void_p(depth3.data_ptr()), depth3.stride(0), nch, B, H, W, _p(r), n,
                                 oh, ow, cp, _p(info), _p(ws), _stream(dev)), "rgbd_edsam_decompose")
    return codes, info


class EdsamModes:
    """Phase A of the decomposition (rgbd_edsam_modes): the grey plane, histogram and modes of
    every image — everything that does not depend on the ratio.  ``info`` holds the per-image
    records (status, histogram, centres); ``ws`` the grey plane phase B reads."""

    def __init__(self, info, ws, masks, B, H, W):
        self.info, self.ws, self.masks, self.B, self.H, self.W = info, ws, masks, B, H, W


def edsam_modes(pixel_values: torch.Tensor, n_masks: int = 3) -> EdsamModes:
    """Launch phase A on the current stream (the hot path puts it on its side stream, beside
    the ratio predictor); ``n_masks``: code-presence masks (zeroed here) for up to that many
    scales of the codes call.  The workspace is per (device, stream): one EdsamModes per
    stream may be pending at a time."""
    depth3, nch, B, H, W = _depth_planes(pixel_values)
    dev = pixel_values.device
    info = torch.empty((B, DECOMP_INFO_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    masks = torch.empty((max(n_masks, 1),), dtype=torch.int32, device=dev)
    L = _lib.lib()
    ws = _workspace(dev, L.rgbd_edsam_modes_workspace_size(B, H, W), "edsam_modes")
    check(L.rgbd_edsam_modes(ctypes.c_void_p(depth3.data_ptr()), depth3.stride(0), nch, B, H, W, _p(info), _p(masks),
                             n_masks, _p(ws), _stream(dev)), "rgbd_edsam_modes")
    return EdsamModes(info, ws, masks, B, H, W)


def edsam_codes(modes: EdsamModes, ratio: torch.Tensor, sizes, code_masks=False):
    """Phase B (rgbd_edsam_codes) on the current stream, after ``modes`` (stream-ordered by
    the caller): the windows at ``ratio`` and the region codes at ``sizes`` from the grey
    plane.  Returns what edsam_decompose returns."""
    B, H, W = modes.B, modes.H, modes.W
    r = _ratio_vec(ratio, B)
    dev = modes.info.device
    n, codes, oh, ow, cp = _scale_args(sizes, B, dev)
    masks = None
    if code_masks:
        if modes.masks.numel() < n:
            raise ValueError(f"edsam_codes: the modes call zeroed {modes.masks.numel()} code masks, {n} needed")
        masks = modes.masks
    check(_lib.lib().rgbd_edsam_codes(_p(modes.ws), B, H, W, _p(r), n, oh, ow, cp, _p(modes.info), _p(masks),
                                      _stream(dev)), "rgbd_edsam_codes")
    return (codes, modes.info, masks[:n]) if code_masks else (codes, modes.info)


def decode_info(info: torch.Tensor) -> np.ndarray:
    """Host copy of the per-image decomposition records (synchronises)."""
    return info.cpu().numpy().view(DECOMP_INFO_DTYPE).reshape(-1)


def _raise_statuses(statuses):
    for b, s in enumerate(statuses):
        if s == 1:
            raise ValueError(f"image {b}: supplied range of depth is not finite (np.histogram)")
        if s == 2:
            raise ValueError(f"image {b}: Too many bins for data range. Cannot create 512 finite-sized bins.")


def raise_on_status(info: torch.Tensor):
    """Mirror the reference's ValueError for degenerate histograms (numpy raises inside
    DSAModule._calculate_depth_histogram, custom_model.py:715-717).  Synchronises."""
    _raise_statuses(decode_info(info)["status"])


class DeferredStatus:
    """The per-image decomposition status, copied to pinned host memory behind the
    decomposition on its stream.  ``check()`` waits only for that copy (the kernels enqueued
    after it keep running) and raises the reference's ValueError; the drop-in module calls it
    at the end of its forward, after the pixel decoder has been enqueued."""

    def __init__(self, info: torch.Tensor):
        st = info.view(torch.int32)[:, 0]  # rgbd_decomp_info.status, the record's first word
        self.captured = capturing()
        if self.captured:
            # inside a graph: a device copy (a pinned-host copy breaks the capture); the replay
            # rewrites it, check() reads it back after the replay
            self.dev = st.clone()
            return
        self.host = torch.empty(st.shape, dtype=torch.int32, pin_memory=True)
        self.host.copy_(st, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record(torch.cuda.current_stream(info.device))

    def check(self):
        """Eager: wait for the copy and raise.  Captured: call after the replay has finished;
        reads that replay's statuses (synchronises)."""
        if self.captured:
            _raise_statuses(self.dev.tolist())
            return
        self.event.synchronize()
        _raise_statuses(self.host.tolist())


# ------------------------------------------------------------------ K2 DGGM fusion
def _grad_mask(pv):
    if pv.dtype != torch.float32 or pv.shape[1] not in (4, 10):
        raise ValueError("DGGM planes must be float32 [B,10,H,W] pixel_values or [B,4,H,W] (grad x3, mask)")
    return (pv[:, 6:9], pv[:, 9:10]) if pv.shape[1] == 10 else (pv[:, 0:3], pv[:, 3:4])


def dggm_fuse_fwd(cp1, color, pixel_values, weight, bias):
    """out = cp1 + (color + ReLU(W . (bilinear(grad) * nearest(mask)) + b)), one scale
    (cp1=None: out = color + ReLU(...), the bare DepthGradientInjectionResidual output).
    ``pixel_values``: float32 [B, >=4, H, W] holding grad planes at channels -4:-1 and the
    mask at channel -1 when it has 4 channels, or the full 10-channel tensor."""
    _need_cuda(cp1, color, pixel_values, weight, bias)
    B, C, h, w = color.shape
    _, _, H, W = pixel_values.shape
    if cp1 is not None and (cp1.shape != color.shape or cp1.dtype != color.dtype):
        raise ValueError("cp1/color mismatch")
    if weight.shape[0] != C or bias.shape[0] != C:
        raise AssertionError(f"Expected {C} channels in the DGGM projection")
    out = torch.empty_like(color)
    wt = weight.reshape(C, 3).float().contiguous()
    bs = bias.float().contiguous()
    grad, mask = _grad_mask(pixel_values)
    check(_lib.lib().rgbd_dggm_fuse_fwd(_dtype_code(color), _p(cp1), _p(color), ctypes.c_void_p(grad.data_ptr()),
                                        ctypes.c_void_p(mask.data_ptr()), pixel_values.stride(0), B, H, W, C,
                                        h, w, _p(wt), _p(bs), _p(out), _stream(color.device)),
          "rgbd_dggm_fuse_fwd")
    return out


def dggm_fuse_bwd(dout, pixel_values, weight, bias):
    _need_cuda(dout, pixel_values, weight, bias)
    B, C, h, w = dout.shape
    _, _, H, W = pixel_values.shape
    wt = weight.reshape(C, 3).float().contiguous()
    bs = bias.float().contiguous()
    dw = torch.empty((C, 3), dtype=torch.float32, device=dout.device)
    db = torch.empty((C,), dtype=torch.float32, device=dout.device)
    L = _lib.lib()
    ws = _workspace(dout.device, L.rgbd_dggm_fuse_bwd_workspace_size(B, C, h, w), "dggm_bwd")
    grad, mask = _grad_mask(pixel_values)
    check(L.rgbd_dggm_fuse_bwd(_dtype_code(dout), _p(dout), ctypes.c_void_p(grad.data_ptr()),
                               ctypes.c_void_p(mask.data_ptr()), pixel_values.stride(0), B, H, W, C, h, w,
                               _p(wt), _p(bs), _p(dw), _p(db), _p(ws), _stream(dout.device)),
          "rgbd_dggm_fuse_bwd")
    return dw, db


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])


def _ints(xs):
    return (ctypes.c_int * len(xs))(*[int(x) for x in xs])


def dggm_fuse_fwd_multi(cp1s, colors, pixel_values, weights, biases, cp1_nhwc=()):
    """dggm_fuse_fwd for every scale in one launch (rgbd_dggm_fuse_fwd_multi[_mixed]); cp1s may be
    None; scales listed in ``cp1_nhwc`` take their cp1 as NHWC [B,h,w,C] (the DSAM cascade's
    output layout) instead of NCHW."""
    _need_cuda(*colors, pixel_values)
    n = len(colors)
    B, _, H, W = pixel_values.shape
    cp1_mask = 0
    if cp1s is not None:
        _need_cuda(*cp1s)
        for k, (a, c) in enumerate(zip(cp1s, colors)):
            exp = (c.shape[0], c.shape[2], c.shape[3], c.shape[1]) if k in cp1_nhwc else tuple(c.shape)
            if tuple(a.shape) != exp or a.dtype != c.dtype:
                raise ValueError("cp1/color mismatch")
            cp1_mask |= (1 << k) if k in cp1_nhwc else 0
    for c, w, b in zip(colors, weights, biases):
        if c.dtype != colors[0].dtype or c.shape[0] != B:
            raise ValueError("colour maps must share dtype and batch")
        if w.shape[0] != c.shape[1] or b.shape[0] != c.shape[1]:
            raise AssertionError(f"Expected {c.shape[1]} channels in the DGGM projection")
    outs = [torch.empty_like(c) for c in colors]
    wts = [w.reshape(w.shape[0], 3).float().contiguous() for w in weights]
    bss = [b.float().contiguous() for b in biases]
    grad, gmask = _grad_mask(pixel_values)
    check(_lib.lib().rgbd_dggm_fuse_fwd_multi_mixed(
        _dtype_code(colors[0]), n, None if cp1s is None else _ptrs(cp1s), cp1_mask, _ptrs(colors), _ptrs(outs),
        _ptrs(wts), _ptrs(bss), _ints([c.shape[1] for c in colors]), _ints([c.shape[2] for c in colors]),
        _ints([c.shape[3] for c in colors]), ctypes.c_void_p(grad.data_ptr()), ctypes.c_void_p(gmask.data_ptr()),
        pixel_values.stride(0), B, H, W, _stream(pixel_values.device)), "rgbd_dggm_fuse_fwd_multi_mixed")
    return outs


def dggm_fuse_bwd_multi(douts, pixel_values, weights, biases):
    """dggm_fuse_bwd for every scale: one partial launch + one final launch.  -> [(dw, db)]."""
    _need_cuda(*douts, pixel_values)
    n = len(douts)
    B, _, H, W = pixel_values.shape
    Cs, hs, ws_ = [d.shape[1] for d in douts], [d.shape[2] for d in douts], [d.shape[3] for d in douts]
    wts = [w.reshape(w.shape[0], 3).float().contiguous() for w in weights]
    bss = [b.float().contiguous() for b in biases]
    dws = [torch.empty((c, 3), dtype=torch.float32, device=pixel_values.device) for c in Cs]
    dbs = [torch.empty((c,), dtype=torch.float32, device=pixel_values.device) for c in Cs]
    L = _lib.lib()
    ci, hi, wi = _ints(Cs), _ints(hs), _ints(ws_)
    ws = _workspace(pixel_values.device, L.rgbd_dggm_fuse_bwd_multi_workspace_size(n, ci, hi, wi, B), "dggm_bwd_multi")
    grad, mask = _grad_mask(pixel_values)
    check(L.rgbd_dggm_fuse_bwd_multi(_dtype_code(douts[0]), n, _ptrs(douts), _ptrs(wts), _ptrs(bss), _ptrs(dws),
                                     _ptrs(dbs), ci, hi, wi, ctypes.c_void_p(grad.data_ptr()),
                                     ctypes.c_void_p(mask.data_ptr()), pixel_values.stride(0), B, H, W, _p(ws),
                                     _stream(pixel_values.device)), "rgbd_dggm_fuse_bwd_multi")
    return list(zip(dws, dbs))


# ------------------------------------------------------------------ layout / packing
def nchw_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    _need_cuda(x)
    B, C, H, W = x.shape
    y = torch.empty((B, H, W, C), dtype=x.dtype, device=x.device)
    check(_lib.lib().rgbd_nchw_to_nhwc(_dtype_code(x), _p(x), _p(y), B, C, H, W, _stream(x.device)),
          "rgbd_nchw_to_nhwc")
    return y


class _NhwcJob(ctypes.Structure):  # rgbd_nhwc_job
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("B", ctypes.c_int), ("C", ctypes.c_int),
                ("H", ctypes.c_int), ("W", ctypes.c_int)]


def nchw_to_nhwc_multi(xs):
    """Up to four bfloat16 NCHW tensors -> their NHWC copies in one launch
    (rgbd_nchw_to_nhwc_multi); bitwise nchw_to_nhwc of each."""
    if not 1 <= len(xs) <= 4:
        raise ValueError("nchw_to_nhwc_multi: one to four tensors")
    _need_cuda(*xs)
    arr = (_NhwcJob * len(xs))()
    ys = []
    for i, x in enumerate(xs):
        if x.dtype != torch.bfloat16 or x.dim() != 4:
            raise ValueError("nchw_to_nhwc_multi: bfloat16 [B,C,H,W] tensors")
        B, C, H, W = x.shape
        y = torch.empty((B, H, W, C), dtype=x.dtype, device=x.device)
        arr[i] = _NhwcJob(x.data_ptr(), y.data_ptr(), B, C, H, W)
        ys.append(y)
    check(_lib.lib().rgbd_nchw_to_nhwc_multi(len(xs), arr, _stream(xs[0].device)), "rgbd_nchw_to_nhwc_multi")
    return ys


def dsam_code_masks(codes):
    """codes: list of uint8 region-code maps -> uint32 device tensor [len(codes)], bit k set when
    code k occurs in map i (the codes the bf16 packed filters are needed for)."""
    _need_cuda(*codes)
    n = len(codes)
    masks = torch.empty((n,), dtype=torch.int32, device=codes[0].device)
    ptrs = (ctypes.c_void_p * n)(*[c.data_ptr() for c in codes])
    sizes = (ctypes.c_longlong * n)(*[c.numel() for c in codes])
    check(_lib.lib().rgbd_dsam_code_masks(n, ptrs, sizes, _p(masks), _stream(codes[0].device)),
          "rgbd_dsam_code_masks")
    return masks


def dsam_pack(conv_w: torch.Tensor, proj_w: torch.Tensor, dtype: torch.dtype, code_mask: torch.Tensor = None,
              want_bwd: bool = True):
    """conv_w float32 [4,Co,Ci,3,3], proj_w [Co,Ci,3,3] -> (wfwd, wbwd):
    float32 segment form wfwd [Co,45*Ci], wbwd [Ci,45*Co]; bfloat16 code-merged tiles, flat
    (include/rgbd_hip.h: [16][9][Ci/32][Co][32] and [16][9][Co/32][Ci][32] + a tail pad), written
    for the codes of ``code_mask`` (a one-element device tensor from dsam_code_masks; None = all
    16).  ``want_bwd=False`` skips wbwd (None is returned for it)."""
    cw = conv_w.detach().float().contiguous()
    pw = proj_w.detach().float().contiguous()
    _need_cuda(cw, pw, code_mask)
    Co, Ci = pw.shape[:2]
    if dtype == torch.bfloat16:
        if Ci % 32 or Co % 32:
            raise ValueError(f"bfloat16 DSAM needs channel counts that are multiples of 32, got {Ci}->{Co}")
        n = _lib.lib().rgbd_dsam_packed_elems(RGBD_BF16, Ci, Co)
        fshape = bshape = (n,)
    else:
        fshape, bshape = (Co, 45 * Ci), (Ci, 45 * Co)
        n = _lib.lib().rgbd_dsam_packed_elems(RGBD_F32, Ci, Co)
        assert n == math.prod(fshape) == math.prod(bshape), (n, fshape, bshape)
    wfwd = torch.empty(fshape, dtype=dtype, device=cw.device)
    wbwd = torch.empty(bshape, dtype=dtype, device=cw.device) if want_bwd else None
    check(_lib.lib().rgbd_dsam_pack_weights(_dtype_code(wfwd), _p(cw), _p(pw), Ci, Co, _p(code_mask), _p(wfwd),
                                            _p(wbwd), _stream(cw.device)), "rgbd_dsam_pack_weights")
    return wfwd, wbwd


# ------------------------------------------------------------------ K5 DSAM convs
LEG_FWD, LEG_DX, LEG_DW = 0, 1, 2  # include/rgbd_hip.h RGBD_LEG_*


class _Leg(ctypes.Structure):  # rgbd_dsam_leg
    _fields_ = [("kind", ctypes.c_int), ("code", ctypes.c_void_p), ("B", ctypes.c_int), ("Cin", ctypes.c_int),
                ("h", ctypes.c_int), ("w", ctypes.c_int), ("Cout", ctypes.c_int), ("plan", ctypes.c_void_p)]


def dsam_plan(legs):
    """Plan bfloat16 DSAM legs ahead (rgbd_dsam_plan): ``legs`` is a list of (kind, code [B,h,w]
    uint8, Cin, Cout) with kind one of LEG_FWD / LEG_DX / LEG_DW; returns one plan buffer per
    leg, to be passed as ``plan=`` to dsam_fwd_nhwc / dsam_bwd_data / dsam_bwd_weight.  All
    forward / dX legs are planned by two launches together on the current stream."""
    codes = [c for _, c, _, _ in legs]
    _need_cuda(*codes)
    L = _lib.lib()
    arr = (_Leg * len(legs))()
    plans = []
    for i, (kind, code, ci, co) in enumerate(legs):
        B, h, w = code.shape
        nb = L.rgbd_dsam_plan_size(kind, B, ci, h, w, co)
        if nb == 0:
            raise ValueError(f"dsam_plan: bad leg {kind} {tuple(code.shape)} {ci}->{co}")
        p = torch.empty((nb,), dtype=torch.uint8, device=code.device)
        plans.append(p)
        arr[i] = _Leg(kind, code.data_ptr(), B, ci, h, w, co, p.data_ptr())
    check(L.rgbd_dsam_plan(len(legs), arr, _stream(codes[0].device)), "rgbd_dsam_plan")
    return plans


def dsam_fwd(x_nhwc, code, info, wfwd, bias4, residual=None, want_nhwc=False):
    """x_nhwc [B,h,w,Ci] -> (out_nchw [B,Co,ho,wo], out_nhwc or None)."""
    _need_cuda(x_nhwc, code, info, wfwd, bias4, residual)
    B, h, w, Ci = x_nhwc.shape
    Co = bias4.shape[-1]
    ho, wo = (h + 1) // 2, (w + 1) // 2
    if tuple(code.shape) != (B, h, w):
        raise ValueError(f"region code {tuple(code.shape)} does not match features {(B, h, w)}")
    if residual is not None and tuple(residual.shape) != (B, Co, ho, wo):
        raise ValueError(f"residual {tuple(residual.shape)} != {(B, Co, ho, wo)}")
    out = torch.empty((B, Co, ho, wo), dtype=x_nhwc.dtype, device=x_nhwc.device)
    out_nhwc = torch.empty((B, ho, wo, Co), dtype=x_nhwc.dtype, device=x_nhwc.device) if want_nhwc else None
    b4 = bias4.detach().float().contiguous()
    L = _lib.lib()
    dt = _dtype_code(x_nhwc)
    ws = _workspace(x_nhwc.device, L.rgbd_dsam_conv_workspace_size(dt, B, Ci, h, w, Co), "dsam_conv")
    check(L.rgbd_dsam_fwd(dt, _p(x_nhwc), _p(code), _p(info), B, Ci, h, w, Co, _p(wfwd), _p(b4), _p(residual),
                          _p(out), _p(out_nhwc), _p(ws), _stream(x_nhwc.device)), "rgbd_dsam_fwd")
    return out, out_nhwc


def dsam_fwd_nhwc(x_nhwc, code, info, wfwd, bias4, residual_nhwc=None, plan=None):
    """bfloat16 forward with NHWC residual and NHWC output only -> out_nhwc [B,ho,wo,Co]
    (rgbd_dsam_fwd_nhwc; the hot path's cascade).  ``plan``: this leg's buffer from dsam_plan."""
    _need_cuda(x_nhwc, code, info, wfwd, bias4, residual_nhwc, plan)
    if x_nhwc.dtype != torch.bfloat16:
        raise TypeError("dsam_fwd_nhwc is the bfloat16 path")
    B, h, w, Ci = x_nhwc.shape
    Co = bias4.shape[-1]
    ho, wo = (h + 1) // 2, (w + 1) // 2
    if tuple(code.shape) != (B, h, w):
        raise ValueError(f"region code {tuple(code.shape)} does not match features {(B, h, w)}")
    if residual_nhwc is not None and tuple(residual_nhwc.shape) != (B, ho, wo, Co):
        raise ValueError(f"residual {tuple(residual_nhwc.shape)} != {(B, ho, wo, Co)}")
    out = torch.empty((B, ho, wo, Co), dtype=x_nhwc.dtype, device=x_nhwc.device)
    b4 = bias4.detach().float().contiguous()
    L = _lib.lib()
    if plan is not None:
        ws = _workspace(x_nhwc.device, L.rgbd_dsam_run_workspace_size(LEG_FWD, B, Ci, h, w, Co), "dsam_conv")
        check(L.rgbd_dsam_fwd_nhwc_planned(RGBD_BF16, _p(x_nhwc), _p(code), _p(info), B, Ci, h, w, Co, _p(wfwd),
                                           _p(b4), _p(residual_nhwc), _p(out), _p(plan), _p(ws),
                                           _stream(x_nhwc.device)), "rgbd_dsam_fwd_nhwc_planned")
        return out
    ws = _workspace(x_nhwc.device, L.rgbd_dsam_conv_workspace_size(RGBD_BF16, B, Ci, h, w, Co), "dsam_conv")
    check(L.rgbd_dsam_fwd_nhwc(RGBD_BF16, _p(x_nhwc), _p(code), _p(info), B, Ci, h, w, Co, _p(wfwd), _p(b4),
                               _p(residual_nhwc), _p(out), _p(ws), _stream(x_nhwc.device)), "rgbd_dsam_fwd_nhwc")
    return out


def dsam_bwd_data(gout_nhwc, code, wbwd, gin_nchw, want_nhwc=False, cin=None, gin_nhwc=None, want_nchw=True,
                  plan=None):
    """dX of one DSAM (+ gin).  The input channel count comes from ``cin``, ``gin_nchw`` /
    ``gin_nhwc`` or the 2-D float32 wbwd (the flat bfloat16 tiles do not carry it).
    ``want_nchw=False`` (bfloat16 only) writes the NHWC result alone, with the residual given as
    ``gin_nhwc``: the hot path's cascade, which never needs dX in NCHW."""
    _need_cuda(gout_nhwc, code, wbwd, gin_nchw, gin_nhwc, plan)
    B, ho, wo, Co = gout_nhwc.shape
    if cin is not None:
        Ci = int(cin)
    elif gin_nchw is not None:
        Ci = gin_nchw.shape[1]
    elif gin_nhwc is not None:
        Ci = gin_nhwc.shape[-1]
    elif wbwd.dim() == 2:
        Ci = wbwd.shape[-2]
    else:
        raise ValueError("dsam_bwd_data needs cin (or gin) with the flat bfloat16 filter tiles")
    _, h, w = code.shape
    if gin_nchw is not None and tuple(gin_nchw.shape) != (B, Ci, h, w):
        raise ValueError("gin shape mismatch")
    if gin_nhwc is not None and (want_nchw or tuple(gin_nhwc.shape) != (B, h, w, Ci)):
        raise ValueError("gin_nhwc goes with want_nchw=False and shape [B, h, w, Cin]")
    if not want_nchw and not want_nhwc:
        raise ValueError("dsam_bwd_data: nothing to write")
    dx = torch.empty((B, Ci, h, w), dtype=gout_nhwc.dtype, device=gout_nhwc.device) if want_nchw else None
    dx_nhwc = torch.empty((B, h, w, Ci), dtype=gout_nhwc.dtype, device=gout_nhwc.device) if want_nhwc else None
    L = _lib.lib()
    dt = _dtype_code(gout_nhwc)
    if plan is not None:
        ws = _workspace(gout_nhwc.device, L.rgbd_dsam_run_workspace_size(LEG_DX, B, Ci, h, w, Co), "dsam_conv")
        check(L.rgbd_dsam_bwd_data_planned(dt, _p(gout_nhwc), _p(code), B, Ci, h, w, Co, _p(wbwd), _p(gin_nchw),
                                           _p(gin_nhwc), _p(dx), _p(dx_nhwc), _p(plan), _p(ws),
                                           _stream(gout_nhwc.device)), "rgbd_dsam_bwd_data_planned")
        return dx, dx_nhwc
    ws = _workspace(gout_nhwc.device, L.rgbd_dsam_conv_workspace_size(dt, B, Ci, h, w, Co), "dsam_conv")
    check(L.rgbd_dsam_bwd_data(dt, _p(gout_nhwc), _p(code), B, Ci, h, w, Co, _p(wbwd), _p(gin_nchw), _p(gin_nhwc),
                               _p(dx), _p(dx_nhwc), _p(ws), _stream(gout_nhwc.device)), "rgbd_dsam_bwd_data")
    return dx, dx_nhwc


def dsam_bwd_weight(gout_nchw, x_nhwc, code, info, gout_nhwc=None, plan=None):
    """dW/db of one DSAM.  The bfloat16 path contracts the NHWC copy of the upstream gradient
    (``gout_nhwc``; made here when not given); bias gradients use the NCHW one when given, else
    (bfloat16) the NHWC one.  ``plan``: this leg's buffer from dsam_plan (bfloat16)."""
    _need_cuda(gout_nchw, x_nhwc, code, info, gout_nhwc, plan)
    if gout_nchw is None:
        if gout_nhwc is None or gout_nhwc.dtype != torch.bfloat16:
            raise ValueError("dsam_bwd_weight: gout_nchw is required unless a bfloat16 gout_nhwc is given")
        B, ho, wo, Co = gout_nhwc.shape
        ref = gout_nhwc
    else:
        B, Co, ho, wo = gout_nchw.shape
        ref = gout_nchw
    _, h, w, Ci = x_nhwc.shape
    dev = ref.device
    dt = _dtype_code(ref)
    if dt == RGBD_BF16 and gout_nhwc is None:
        gout_nhwc = nchw_to_nhwc(gout_nchw)
    if gout_nhwc is not None and tuple(gout_nhwc.shape) != (B, ho, wo, Co):
        raise ValueError(f"gout_nhwc {tuple(gout_nhwc.shape)} != {(B, ho, wo, Co)}")
    dconv = torch.empty((4, Co, Ci, 3, 3), dtype=torch.float32, device=dev)
    dproj = torch.empty((Co, Ci, 3, 3), dtype=torch.float32, device=dev)
    dbias = torch.empty((4, Co), dtype=torch.float32, device=dev)
    L = _lib.lib()
    if plan is not None:
        if dt != RGBD_BF16:
            raise ValueError("dsam_bwd_weight: a plan goes with the bfloat16 path")
        ws = _workspace(dev, L.rgbd_dsam_run_workspace_size(LEG_DW, B, Ci, h, w, Co), "dsam_wgrad")
        check(L.rgbd_dsam_bwd_weight_planned(dt, _p(gout_nchw), _p(gout_nhwc), _p(x_nhwc), _p(code), _p(info), B, Ci,
                                             h, w, Co, _p(dconv), _p(dproj), _p(dbias), _p(plan), _p(ws),
                                             _stream(dev)), "rgbd_dsam_bwd_weight_planned")
        return dconv, dproj, dbias
    ws = _workspace(dev, L.rgbd_dsam_bwd_weight_workspace_size(dt, B, Ci, h, w, Co), "dsam_wgrad")
    check(L.rgbd_dsam_bwd_weight(dt, _p(gout_nchw), _p(gout_nhwc), _p(x_nhwc), _p(code), _p(info), B, Ci, h, w,
                                 Co, _p(dconv), _p(dproj), _p(dbias), _p(ws), _stream(dev)), "rgbd_dsam_bwd_weight")
    return dconv, dproj, dbias


class _DwRun(ctypes.Structure):  # rgbd_dsam_dw_run
    _fields_ = [("gout_nhwc", ctypes.c_void_p), ("x_nhwc", ctypes.c_void_p), ("code", ctypes.c_void_p),
                ("B", ctypes.c_int), ("Cin", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
                ("Cout", ctypes.c_int), ("dconv_w", ctypes.c_void_p), ("dproj_w", ctypes.c_void_p),
                ("dbias", ctypes.c_void_p), ("plan", ctypes.c_void_p), ("ws", ctypes.c_void_p)]


def dsam_bwd_weight_multi(runs, info):
    """dW/db of bfloat16 DSAM legs that are ready together, their GEMMs in one persistent launch
    (rgbd_dsam_bwd_weight_planned_multi).  ``runs``: up to two (gout_nhwc [B,ho,wo,Co], x_nhwc
    [B,h,w,Ci], code [B,h,w], plan) tuples, each plan from dsam_plan(LEG_DW); returns per run
    (dconv, dproj, dbias), bitwise those of dsam_bwd_weight(None, ..., gout_nhwc=, plan=)."""
    if not 1 <= len(runs) <= 2:
        raise ValueError("dsam_bwd_weight_multi: one or two runs")
    L = _lib.lib()
    arr = (_DwRun * len(runs))()
    outs = []
    for j, (gout_nhwc, x_nhwc, code, plan) in enumerate(runs):
        _need_cuda(gout_nhwc, x_nhwc, code, plan, info)
        if gout_nhwc.dtype != torch.bfloat16 or x_nhwc.dtype != torch.bfloat16:
            raise ValueError("dsam_bwd_weight_multi: bfloat16 legs only")
        B, ho, wo, Co = gout_nhwc.shape
        _, h, w, Ci = x_nhwc.shape
        if (ho, wo) != ((h + 1) // 2, (w + 1) // 2) or tuple(code.shape) != (B, h, w):
            raise ValueError(f"dsam_bwd_weight_multi: run {j} shapes {tuple(gout_nhwc.shape)} {tuple(x_nhwc.shape)}")
        dev = gout_nhwc.device
        dconv = torch.empty((4, Co, Ci, 3, 3), dtype=torch.float32, device=dev)
        dproj = torch.empty((Co, Ci, 3, 3), dtype=torch.float32, device=dev)
        dbias = torch.empty((4, Co), dtype=torch.float32, device=dev)
        ws = _workspace(dev, L.rgbd_dsam_run_workspace_size(LEG_DW, B, Ci, h, w, Co), f"dsam_wgrad_run{j}")
        arr[j] = _DwRun(gout_nhwc.data_ptr(), x_nhwc.data_ptr(), code.data_ptr(), B, Ci, h, w, Co, dconv.data_ptr(),
                        dproj.data_ptr(), dbias.data_ptr(), plan.data_ptr(), ws.data_ptr())
        outs.append((dconv, dproj, dbias))
    check(L.rgbd_dsam_bwd_weight_planned_multi(len(runs), arr, _p(info), _stream(runs[0][0].device)),
          "rgbd_dsam_bwd_weight_planned_multi")
    return outs


# ------------------------------------------------------------------ f1 mask predictor
def mask_logits(emb: torch.Tensor, pix: torch.Tensor) -> torch.Tensor:
    """einsum("bqc,bchw->bqhw", emb, pix) (modeling_mask2former.py:2046) on the MFMA kernel.
    emb [B,Q,C], pix [B,C,H,W], same dtype (float32 or bfloat16) -> [B,Q,H,W] of that dtype."""
    emb = emb.contiguous()
    pix = pix.contiguous()
    _need_cuda(emb, pix)
    if emb.dim() != 3 or pix.dim() != 4 or emb.shape[0] != pix.shape[0] or emb.shape[2] != pix.shape[1]:
        raise ValueError(f"mask_logits: emb {tuple(emb.shape)} and pix {tuple(pix.shape)} do not contract")
    if emb.dtype != pix.dtype:
        raise TypeError(f"mask_logits: emb {emb.dtype} != pix {pix.dtype}")
    B, Q, C = emb.shape
    H, W = pix.shape[2:]
    out = torch.empty((B, Q, H, W), dtype=pix.dtype, device=pix.device)
    check(_lib.lib().rgbd_mask_logits(_dtype_code(pix), _p(emb), _p(pix), B, Q, C, H, W, _p(out),
                                      _stream(pix.device)), "rgbd_mask_logits")
    return out


def mask_attention(logits: torch.Tensor, size, heads: int) -> torch.Tensor:
    """The binarised attention mask of modeling_mask2former.py:2048-2054: bilinear resample of
    ``logits`` [B,Q,H,W] to ``size`` (align_corners=False), sigmoid, < 0.5, repeated over
    ``heads`` -> bool [B*heads, Q, th*tw]."""
    logits = logits.contiguous()
    _need_cuda(logits)
    B, Q, H, W = logits.shape
    th, tw = (int(size), int(size)) if isinstance(size, int) else (int(size[0]), int(size[1]))
    attn = torch.empty((B * heads, Q, th * tw), dtype=torch.bool, device=logits.device)
    check(_lib.lib().rgbd_mask_attention(_dtype_code(logits), _p(logits), B, Q, H, W, th, tw, int(heads),
                                         _p(attn), _stream(logits.device)), "rgbd_mask_attention")
    return attn


# ------------------------------------------------------------------ f3 matcher assignment
class LsaResult(list):
    """The per-matrix [(row_ind, col_ind)] list, plus ``rows_all`` / ``cols_all`` (every matrix's
    indices concatenated, views of the kernel's output: no copy) and ``counts`` (host ints)."""
    rows_all = cols_all = None
    counts = ()


def linear_sum_assignment_batch(costs, validate=False, return_status=False):
    """scipy.optimize.linear_sum_assignment for a list of 2-D float32 CUDA cost matrices in one
    launch (rgbd_lsa_batch).  Returns [(row_ind, col_ind)] as int64 CUDA tensors, scipy's order
    (with ``return_status`` also the int32 device tensor of per-matrix statuses: 0 ok,
    1 infeasible, 2 invalid entries — scipy's two ValueErrors).  Nothing synchronises unless
    ``validate`` (then a status read-back raises scipy's ValueErrors)."""
    if not costs:
        return ([], None) if return_status else []
    dev = costs[0].device
    flat, meta, coff, ooff, mr, mc = [], [], 0, 0, 0, 0
    for c in costs:
        if c.dim() != 2:
            raise ValueError("cost matrix must be 2-D")
        c = c.detach().float().contiguous()
        _need_cuda(c)
        r, k = c.shape
        meta += [coff, r, k, ooff]
        flat.append(c.reshape(-1))
        coff += r * k
        ooff += min(r, k)
        mr, mc = max(mr, r), max(mc, k)
    if max(mr, mc) > 2048:
        raise ValueError("rgbd_lsa_batch: matrices up to 2048 on a side")
    cost = torch.cat(flat) if coff > 0 else torch.zeros(1, dtype=torch.float32, device=dev)
    meta_t = device_const(meta, torch.int64, dev)
    # zero-initialised: a matrix the kernel rejects (status != 0) leaves valid indices behind,
    # never uninitialised ones
    rows = torch.zeros(max(ooff, 1), dtype=torch.int64, device=dev)
    cols = torch.zeros(max(ooff, 1), dtype=torch.int64, device=dev)
    status = torch.zeros(len(costs), dtype=torch.int32, device=dev)
    check(_lib.lib().rgbd_lsa_batch(len(costs), _p(cost), _p(meta_t), mr, mc, _p(rows), _p(cols), _p(status),
                                    _stream(dev)), "rgbd_lsa_batch")
    if validate:
        st = status.cpu().tolist()
        for s in st:
            if s == 1:
                raise ValueError("cost matrix is infeasible")
            if s == 2:
                raise ValueError("matrix contains invalid numeric entries")
    out, o, counts = LsaResult(), 0, []
    for i in range(len(costs)):
        n = int(min(meta[4 * i + 1], meta[4 * i + 2]))
        out.append((rows[o:o + n], cols[o:o + n]))
        counts.append(n)
        o += n
    out.rows_all, out.cols_all, out.counts = rows[:o], cols[:o], tuple(counts)
    return (out, status) if return_status else out


# ------------------------------------------------------------------ f2 deformable attention
def _msda_args(value, shapes, loc, attw):
    _need_cuda(value, loc, attw)
    B, S, NH, D = value.shape
    _, Q, nh2, L, P, two = loc.shape
    if nh2 != NH or two != 2 or tuple(attw.shape) != (B, Q, NH, L, P) or len(shapes) != L:
        raise ValueError(f"msda: value {tuple(value.shape)}, loc {tuple(loc.shape)}, attw {tuple(attw.shape)}, "
                         f"{len(shapes)} levels do not match")
    if sum(int(h) * int(w) for h, w in shapes) != S:
        raise ValueError("msda: spatial shapes do not add up to the value length")
    arr = (ctypes.c_int * (2 * L))(*[int(x) for hw in shapes for x in hw])
    return B, S, NH, D, Q, L, P, arr


def msda_forward(value, shapes, loc, attw):
    """multi_scale_deformable_attention(value, shapes, loc, attw) (modeling_mask2former.py:798) on
    the HIP kernel.  value [B,S,NH,D] f32/bf16; loc [B,Q,NH,L,P,2] and attw [B,Q,NH,L,P] float32."""
    value = value.contiguous()
    loc = loc.float().contiguous()
    attw = attw.float().contiguous()
    B, S, NH, D, Q, L, P, arr = _msda_args(value, shapes, loc, attw)
    out = torch.empty((B, Q, NH * D), dtype=value.dtype, device=value.device)
    check(_lib.lib().rgbd_msda_fwd(_dtype_code(value), _p(value), B, L, arr, NH, D, Q, P, _p(loc), _p(attw),
                                   _p(out), _stream(value.device)), "rgbd_msda_fwd")
    return out


def msda_backward(value, shapes, loc, attw, gout):
    """-> (grad_value float32 [B,S,NH,D], grad_loc, grad_attw)."""
    value = value.contiguous()
    loc = loc.float().contiguous()
    attw = attw.float().contiguous()
    gout = gout.to(value.dtype).contiguous()
    B, S, NH, D, Q, L, P, arr = _msda_args(value, shapes, loc, attw)
    gv = torch.empty((B, S, NH, D), dtype=torch.float32, device=value.device)
    gl = torch.empty_like(loc)
    ga = torch.empty_like(attw)
    check(_lib.lib().rgbd_msda_bwd(_dtype_code(value), _p(value), B, L, arr, NH, D, Q, P, _p(loc), _p(attw),
                                   _p(gout), _p(gv), _p(gl), _p(ga), _stream(value.device)), "rgbd_msda_bwd")
    return gv, gl, ga
