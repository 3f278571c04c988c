"""Oracle (test infrastructure only): COCO run-length encoding as pycocotools computes it.

pycocotools is not installed here; the reference calls
``pycocotools.mask.encode(np.asfortranarray(binary_mask))`` and decodes the byte string to UTF-8
(mask2former/predictor.py:430-435, 590-595).  This restates the published C routines of
pycocotools 2.0 ``common/maskApi.c`` step for step, as plain Python loops:

  rleEncode   column-major scan; counts alternate zeros / ones starting with zeros (a mask whose
              first pixel is set starts with a 0 count)
  rleToString LEB128-like: count i (minus count i-2 for i > 2) in 5-bit groups, low first, bit
              0x20 = more groups follow, bit 0x10 of the last group = sign, each char + 48
  rleFrString the inverse, rleDecode the mask back

Parity is pinned by these restatements (and their round trip), not by the library itself.
"""
import numpy as np


def rle_encode(mask: np.ndarray):
    """maskApi.c rleEncode for one [h, w] {0,1} mask -> (h, w, counts list)."""
    h, w = mask.shape
    flat = [int(v) for v in np.asarray(mask, dtype=np.uint8).T.reshape(-1)]  # column-major (Fortran)
    counts, p, c = [], 0, 0
    for v in flat:
        if v != p:
            counts.append(c)
            c = 0
            p = v
        c += 1
    counts.append(c)
    return h, w, counts


def rle_to_string(counts) -> str:
    """maskApi.c rleToString."""
    out = []
    for i, cnt in enumerate(counts):
        x = int(cnt)
        if i > 2:
            x -= int(counts[i - 2])
        more = True
        while more:
            c = x & 0x1F
            x >>= 5  # arithmetic shift, as C's on a signed long
            more = (x != -1) if (c & 0x10) else (x != 0)
            if more:
                c |= 0x20
            out.append(chr(c + 48))
    return "".join(out)


def rle_from_string(s: str):
    """maskApi.c rleFrString -> counts."""
    counts, p = [], 0
    while p < len(s):
        x, k, more = 0, 0, True
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(counts) > 2:
            x += counts[-2]
        counts.append(x)
    return counts


def rle_decode(h: int, w: int, counts) -> np.ndarray:
    """maskApi.c rleDecode -> [h, w] uint8."""
    flat, v = [], 0
    for c in counts:
        flat += [v] * int(c)
        v = 1 - v
    return np.asarray(flat, dtype=np.uint8).reshape(w, h).T


def encode(mask: np.ndarray) -> dict:
    """pycocotools.mask.encode of a Fortran-ordered [h, w] mask, counts decoded to str (the
    reference's use)."""
    h, w, counts = rle_encode(mask)
    return {"size": [h, w], "counts": rle_to_string(counts)}


def bbox_from_mask(mask: np.ndarray):
    """predictor.py:463-488 _calculate_bbox_from_mask: [x, y, w, h] of the set pixels (None if empty)."""
    ys, xs = np.where(mask > 0)
    if len(ys) == 0:
        return None
    return [float(xs.min()), float(ys.min()), float(xs.max() - xs.min() + 1), float(ys.max() - ys.min() + 1)]
