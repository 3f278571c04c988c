"""Oracle (test infrastructure only): the two resizes of the reference's data map
(mask2former/utils/dataloader.py:405-414, ``map_10channel_case2``) for frames that do not arrive
at model resolution.

* The image processor's resize: ``Mask2FormerImageProcessor`` (the PIL backend transformers
  instantiates without torchvision) resizes the colour image and the depth-as-RGB image with
  ``PIL.Image.resize((w, h), BILINEAR)`` on uint8 data and the instance map with NEAREST
  (transformers image_transforms.resize -> Pillow).  Restated here from Pillow's published
  ``libImaging/Resample.c`` (precompute_coeffs, normalize_coeffs_8bpc, ImagingResampleHorizontal_8bpc
  / Vertical_8bpc, ImagingResampleInner: horizontal pass first into a uint8 image of the rows
  the vertical pass needs) and ``Geometry.c`` (the NEAREST resize: an affine transform walked
  incrementally in double).  Pinned against Pillow itself (importable here: tests/test_oracle_resize.py).
* ``cv2.resize(depth, (h, w), interpolation=cv2.INTER_LINEAR)`` (:414; note the reference passes
  (h, w) as dsize = (width, height), which transposes non-square frames, Q18).  OpenCV is not
  installed: restated from OpenCV 4's fixed-point linear resize of 8-bit data (source coordinate
  (d + 0.5) * in / out - 0.5 clamped at the borders, 11-bit coefficients, integer horizontal
  sums, (sum * cy + 2^21) >> 22 vertically) — parity unpinned.
"""
import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _bilinear_filter(x):
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def precompute_coeffs(in_size, out_size, in0=0.0, in1=None):
    """Resample.c precompute_coeffs + normalize_coeffs_8bpc for BILINEAR (support 1.0):
    returns ksize, bounds [out][2] (xmin, count) and int32 coefficients [out][ksize]."""
    in1 = float(in_size) if in1 is None else in1
    scale = float(np.float32(in1) - np.float32(in0)) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.float64)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        for x in range(xmax):
            w = _bilinear_filter((x + xmin - center + 0.5) * ss)
            kk[xx, x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                kk[xx, x] /= ww
        bounds[xx] = (xmin, xmax)
    one = 1 << PRECISION_BITS
    ik = np.where(kk < 0, (-0.5 + kk * one).astype(np.int64), (0.5 + kk * one).astype(np.int64)).astype(np.int32)
    # the C cast truncates toward zero, as astype does
    return ksize, bounds, ik


def _clip8(ss):
    return np.clip(ss >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(img, axis, bounds, ik, offset=0):
    """One 8bpc pass along axis (1: horizontal, 0: vertical) of an [H][W](, C) uint8 image."""
    src = np.moveaxis(img.astype(np.int64), axis, 0)
    out_n = bounds.shape[0]
    out = np.empty((out_n,) + src.shape[1:], np.uint8)
    for o in range(out_n):
        xmin, cnt = int(bounds[o, 0]) + offset, int(bounds[o, 1])
        ss = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for x in range(cnt):
            ss += src[xmin + x] * int(ik[o, x])
        out[o] = _clip8(ss)
    return np.moveaxis(out, 0, axis)


def pil_bilinear(img, out_h, out_w):
    """PIL.Image.fromarray(img).resize((out_w, out_h), BILINEAR) for a uint8 [H][W] or [H][W][C]."""
    H, W = img.shape[:2]
    need_h = out_w != W
    need_v = out_h != H
    _, bh, kh = precompute_coeffs(W, out_w)
    _, bv, kv = precompute_coeffs(H, out_h)
    cur = img
    if need_h:
        first = int(bv[0, 0])
        last = int(bv[-1, 0] + bv[-1, 1])
        cur = _pass(img[first:last], 1, bh, kh)
        bv = bv.copy()
        bv[:, 0] -= first
    if need_v:
        cur = _pass(cur, 0, bv, kv)
    return np.ascontiguousarray(cur)


def pil_nearest_index(in_size, out_size):
    """Source index per output index of Pillow's NEAREST resize: an affine transform whose
    nearest fast path walks the source coordinate incrementally in double (Geometry.c:
    xx = a2 + 0.5 a0, then xx += a0 per output pixel, index = (int)xx; rows the same with a5, a4),
    a0 = in / out.  The increments matter: at exact integers the accumulated value can sit one
    ulp below (checked against Pillow over 300 random size pairs, tests/test_oracle_resize.py)."""
    a0 = float(in_size) / out_size
    xx = 0.5 * a0
    out = np.empty(out_size, np.int64)
    for x in range(out_size):
        out[x] = min(max(int(xx), 0), in_size - 1)
        xx += a0
    return out


def pil_nearest(img, out_h, out_w):
    iy = pil_nearest_index(img.shape[0], out_h)
    ix = pil_nearest_index(img.shape[1], out_w)
    return np.ascontiguousarray(img[iy][:, ix])


CV_COEF_BITS = 11


def cv2_linear_coeffs(in_size, out_size):
    """Per output index: source index s0 (s1 = min(s0 + 1, in - 1)) and the 11-bit coefficient
    of s1 (s0's is 2048 minus it)."""
    scale = in_size / out_size
    s0 = np.empty(out_size, np.int64)
    c1 = np.empty(out_size, np.int64)
    for d in range(out_size):
        f = (d + 0.5) * scale - 0.5
        s = int(math.floor(f))
        f -= s
        if s < 0:
            s, f = 0, 0.0
        if s >= in_size - 1:
            s, f = in_size - 1, 0.0
        s0[d] = s
        c1[d] = int(round(f * (1 << CV_COEF_BITS)))
    return s0, c1


def cv2_linear(img, dsize):
    """cv2.resize(img, dsize=(width, height), interpolation=INTER_LINEAR) for uint8 [H][W]."""
    out_w, out_h = dsize
    H, W = img.shape
    if (out_h, out_w) == (H, W):
        return img.copy()
    one = 1 << CV_COEF_BITS
    sx, cx = cv2_linear_coeffs(W, out_w)
    sy, cy = cv2_linear_coeffs(H, out_h)
    src = img.astype(np.int64)
    sx1 = np.minimum(sx + 1, W - 1)
    hrow = src[:, sx] * (one - cx) + src[:, sx1] * cx            # [H][out_w], scaled by 2^11
    sy1 = np.minimum(sy + 1, H - 1)
    v = hrow[sy] * (one - cy)[:, None] + hrow[sy1] * cy[:, None]  # scaled by 2^22
    return ((v + (1 << (2 * CV_COEF_BITS - 1))) >> (2 * CV_COEF_BITS)).clip(0, 255).astype(np.uint8)
