"""Oracle for DGGM-pre — PARITY UNPINNED (OpenCV absent).

Restates ``calculate_gradient_features`` (reference mask2former/utils/data_process.py:1247-1305)
as called from ``map_10channel_case2`` (mask2former/utils/dataloader.py:414-421) on a u8
depth image.  OpenCV's ``Sobel(src, CV_32F, dx, dy, ksize=3)`` uses the kernel
[-1 0 1] x [1 2 1]^T with BORDER_REFLECT_101; on integer-valued input every partial sum is
an exact integer in float32, so the result does not depend on OpenCV's summation order.
"""
import numpy as np


def sobel3_reflect101(d: np.ndarray):
    """(gx, gy) float32 for a float32 [H,W] image (data_process.py:1268-1269)."""
    p = np.pad(d, 1, mode="reflect")  # numpy 'reflect' == OpenCV BORDER_REFLECT_101
    f2 = np.float32(2.0)
    gx = (p[0:-2, 2:] - p[0:-2, :-2]) + f2 * (p[1:-1, 2:] - p[1:-1, :-2]) + (p[2:, 2:] - p[2:, :-2])
    gy = (p[2:, 0:-2] - p[:-2, 0:-2]) + f2 * (p[2:, 1:-1] - p[:-2, 1:-1]) + (p[2:, 2:] - p[:-2, 2:])
    return gx.astype(np.float32), gy.astype(np.float32)


def calculate_gradient_features(depth: np.ndarray, invalid_depth_value: float = 0.0):
    """Returns (normalized_magnitude, grad_x, grad_y, valid_gradient_mask), all float32 [H,W].

    Follows data_process.py:1262-1305 line by line:
      valid = (d != invalid) & ~isnan(d)                          :1265
      mag = sqrt(gx^2 + gy^2); gx, gy, mag zeroed where invalid    :1272-1278
      mask = (mag > 0)                                             :1282
      norm = (mag - min(mag[mask])) / (max(mag) - min(mag[mask]))  :1286-1291
             (zero-magnitude pixels become negative: Q14)
    """
    d = depth.astype(np.float32)
    valid = (d != np.float32(invalid_depth_value)) & ~np.isnan(d)
    gx, gy = sobel3_reflect101(d)
    mag = np.sqrt(gx * gx + gy * gy).astype(np.float32)
    gx[~valid] = 0
    gy[~valid] = 0
    mag[~valid] = 0
    mask = (mag > 0).astype(np.float32)
    vm = mag[mask > 0]
    if vm.size > 0:
        mn = np.float32(vm.min())
        mx = np.float32(mag.max())
        if mx > mn:
            norm = ((mag - mn) / (mx - mn)).astype(np.float32)
        else:
            norm = np.zeros_like(mag, dtype=np.float32)
    else:
        norm = np.zeros_like(mag, dtype=np.float32)
    return norm, gx, gy, mask


def dggm_planes(depth_u8: np.ndarray) -> np.ndarray:
    """Channels 6:10 of pixel_values for one image: [norm, norm, norm, mask] (dataloader.py:415-421)."""
    norm, _, _, mask = calculate_gradient_features(depth_u8)
    return np.stack([norm, norm, norm, mask], axis=0)
