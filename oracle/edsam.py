"""Oracle for the E-DSAM depth decomposition and DSAM masked conv.

Every function restates one reference method of ``DSAModule``
(mask2former/utils/custom_model.py:622-798) with the float32 rounding sequence that
numpy 2.2 (NEP 50 promotion) and scipy 1.15 produce.
"""
import numpy as np
import torch
import torch.nn.functional as F

NBINS = 512
NUM_REGIONS = 3
F32 = np.float32


# ---------------------------------------------------------------- a2: to_grayscale
def to_grayscale(depth3: np.ndarray) -> np.ndarray:
    """[3,H,W] f32 -> [H,W] f32; custom_model.py:466-480 (torch f32: scalar cast to f32,
    one rounding per op, left-to-right)."""
    d = depth3.astype(F32, copy=False)
    return (F32(0.299) * d[0] + F32(0.587) * d[1]) + F32(0.114) * d[2]


# ---------------------------------------------------------------- a5: histogram
class HistogramError(ValueError):
    pass


def histogram_range(d: np.ndarray):
    """(first_edge, last_edge) f32: np.nanmin/np.nanmax (custom_model.py:714-715), then
    numpy's _get_outer_edges expansion by +-0.5 for a constant image."""
    v = d[~np.isnan(d)]
    if v.size == 0:
        raise HistogramError("supplied range of [nan, nan] is not finite")
    first, last = F32(v.min()), F32(v.max())
    if not (np.isfinite(first) and np.isfinite(last)):
        raise HistogramError(f"supplied range of [{first}, {last}] is not finite")
    if first == last:
        first = F32(first - F32(0.5))
        last = F32(last + F32(0.5))
    return first, last


def histogram_edges(first, last) -> np.ndarray:
    """np.linspace(first, last, 513, dtype=f32) as numpy 2.2 computes it: i*step + first in
    f32 with step = (last-first)/512, last edge forced to ``last``."""
    delta = F32(last - first)
    step = F32(delta / F32(NBINS))
    if step == 0:
        raise HistogramError("Too many bins for data range.")
    e = np.arange(NBINS + 1, dtype=F32) * step + first
    e[-1] = last
    if np.any(e[:-1] >= e[1:]):
        raise HistogramError("Too many bins for data range.")
    return e.astype(F32)


def histogram(d: np.ndarray):
    """np.histogram(d.flatten(), 512, (nanmin, nanmax)) -> (hist int64[512], edges f32[513]).
    custom_model.py:701-718; numpy _histograms_impl uniform-bin fast path."""
    d = d.astype(F32, copy=False).ravel()
    first, last = histogram_range(d)
    edges = histogram_edges(first, last)
    v = d[(d >= first) & (d <= last)]
    denom = F32(last - first)
    f = ((v - first) / denom) * F32(NBINS)
    idx = f.astype(np.int64)
    idx[idx == NBINS] -= 1
    idx[v < edges[idx]] -= 1
    inc = (v >= edges[idx + 1]) & (idx != NBINS - 1)
    idx[inc] += 1
    return np.bincount(idx, minlength=NBINS).astype(np.int64), edges


# ---------------------------------------------------------------- a6: peaks
def local_maxima(x: np.ndarray):
    """scipy.signal._peak_finding_utils._local_maxima_1d: plateau midpoints (floor),
    endpoints never peaks."""
    n = x.shape[0]
    peaks = []
    i, i_max = 1, n - 1
    while i < i_max:
        if x[i - 1] < x[i]:
            j = i + 1
            while j < i_max and x[j] == x[i]:
                j += 1
            if x[j] < x[i]:
                peaks.append((i + j - 1) // 2)
                i = j
        i += 1
    return np.array(peaks, dtype=np.int64)


def prominences(x: np.ndarray, peaks: np.ndarray) -> np.ndarray:
    """scipy _peak_prominences with wlen=-1 (whole signal)."""
    out = np.zeros(len(peaks), dtype=np.float64)
    n = x.shape[0]
    for k, p in enumerate(peaks):
        i = p; lmin = x[p]
        while i >= 0 and x[i] <= x[p]:
            lmin = min(lmin, x[i]); i -= 1
        i = p; rmin = x[p]
        while i <= n - 1 and x[i] <= x[p]:
            rmin = min(rmin, x[i]); i += 1
        out[k] = x[p] - max(lmin, rmin)
    return out


def find_peaks_prominence(hist: np.ndarray, rel: float = 0.01) -> np.ndarray:
    """find_peaks(hist, prominence=rel*max(hist)) (custom_model.py:738): indices, ascending."""
    x = hist.astype(np.float64)
    pk = local_maxima(x)
    if pk.size == 0:
        return pk
    pmin = rel * np.max(hist)          # np.int64 * python float -> float64
    keep = pmin <= prominences(x, pk)
    return pk[keep]


def select_modes(hist: np.ndarray, edges: np.ndarray, num_modes: int = NUM_REGIONS):
    """custom_model.py:720-752 -> (centers f32 list, peak bin indices list), top ``num_modes``
    by (count, center) descending."""
    pk = find_peaks_prominence(hist)
    if pk.size == 0:
        return [], []
    heights = hist[pk]
    centers = edges[:-1][pk] + np.diff(edges)[pk] / F32(2.0)
    data = sorted(zip(heights.tolist(), centers.tolist(), pk.tolist()), reverse=True)
    top = data[:num_modes]
    return [F32(c) for _, c, _ in top], [int(p) for _, _, p in top]


# ---------------------------------------------------------------- a7: windows
def define_windows(centers, ratio: float):
    """custom_model.py:754-772: half = c*r/2 (f32), lo = max(0, c-half), hi = c+half."""
    r = F32(ratio)
    wins = []
    for c in centers:
        half = F32(F32(c * r) / F32(2.0))
        lo = F32(c - half)
        lo = lo if lo > 0 else F32(0.0)
        wins.append((lo, F32(c + half)))
    return wins


# ---------------------------------------------------------------- a8: masks + pool
def region_masks(d: np.ndarray, windows):
    """custom_model.py:774-798 (+ the zero-mode branch :676-678): list of bool [H,W]."""
    if not windows:
        return [np.zeros(d.shape, dtype=bool)] * (NUM_REGIONS + 1)
    masks, comb = [], np.zeros(d.shape, dtype=bool)
    for lo, hi in windows:
        m = (d >= lo) & (d <= hi)
        masks.append(m)
        comb |= m
    masks.append(~comb)
    return masks


def adaptive_max_pool_bool(m: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """adaptive_max_pool2d of a {0,1} mask (custom_model.py:687): bins
    [floor(i*H/oh), ceil((i+1)*H/oh))."""
    H, W = m.shape
    out = np.zeros((oh, ow), dtype=bool)
    for i in range(oh):
        y0, y1 = (i * H) // oh, ((i + 1) * H + oh - 1) // oh
        row = m[y0:y1].any(axis=0)
        for j in range(ow):
            x0, x1 = (j * W) // ow, ((j + 1) * W + ow - 1) // ow
            out[i, j] = row[x0:x1].any()
    return out


def region_code(masks) -> np.ndarray:
    """Pack a list of <=4 bool masks into one u8 plane: bit i <-> conv_layers[i]."""
    code = np.zeros(masks[0].shape, dtype=np.uint8)
    for i, m in enumerate(masks):
        code |= (m.astype(np.uint8) << i)
    return code


def pooled_codes(code: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """OR-pool of the packed region code == per-mask adaptive max pool, packed."""
    H, W = code.shape
    if H % oh == 0 and W % ow == 0:  # exact bins: same result, vectorised
        blocks = code.reshape(oh, H // oh, ow, W // ow)
        return np.bitwise_or.reduce(np.bitwise_or.reduce(blocks, axis=3), axis=1).astype(np.uint8)
    out = np.zeros((oh, ow), dtype=np.uint8)
    for bit in range(4):
        out |= adaptive_max_pool_bool(((code >> bit) & 1).astype(bool), oh, ow).astype(np.uint8) << bit
    return out


def decompose(depth3: np.ndarray, ratio: float):
    """Whole decomposition for one image (the part of DSAModule.forward before the convs,
    custom_model.py:661-679).  Returns dict with grey, hist, edges, centers, peak bins,
    windows, n_masks (=len(region_masks)), n_modes, code (u8 [H,W])."""
    g = to_grayscale(depth3)
    hist, edges = histogram(g)
    centers, bins = select_modes(hist, edges)
    wins = define_windows(centers, ratio) if centers else []
    masks = region_masks(g, wins)
    return dict(grey=g, hist=hist, edges=edges, centers=centers, peak_bins=bins,
                windows=wins, n_modes=len(centers), n_masks=len(masks), code=region_code(masks))


# ---------------------------------------------------------------- a4: DSAM conv
def dsam_forward(x: torch.Tensor, code_full: np.ndarray, n_masks: int, conv_w, conv_b, proj_w):
    """DSAModule.forward after decomposition (custom_model.py:682-699), one sample.
    x [1,Cin,h,w] f32; code_full u8 [H,W]; conv_w [4,Cout,Cin,3,3]; conv_b [4,Cout];
    proj_w [Cout,Cin,3,3].  Same op sequence as the reference (fp32, PyTorch CPU)."""
    h, w = x.shape[2:]
    enhanced = 0
    for i in range(n_masks):
        m = torch.from_numpy(((code_full >> i) & 1).astype(np.float32))[None, None]
        rm = F.adaptive_max_pool2d(m, (h, w))
        enhanced = enhanced + F.conv2d(x * rm, conv_w[i], conv_b[i], stride=2, padding=1)
    return enhanced + F.conv2d(x, proj_w, None, stride=2, padding=1)
