"""DGGM-pre oracle (a10).  calculate_gradient_features calls OpenCV (absent here), so the
reference cannot be run for this row: PARITY UNPINNED against the reference itself.  The
restatement is cross-checked against an independent implementation of OpenCV's documented
semantics (scipy.ndimage.correlate with mode='mirror' == BORDER_REFLECT_101), exact on u8
input, and against the reference's own quirks (Q14)."""
import numpy as np
import pytest
from scipy import ndimage

from oracle import dggm_pre
from rgbd_amd import synthetic

KX = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], dtype=np.float64)


@pytest.mark.parametrize("seed,H,W", [(1, 48, 64), (2, 240, 320), (3, 7, 5), (4, 2, 9)])
def test_sobel_matches_scipy_mirror(seed, H, W):
    d = synthetic.make_scene(seed, max(H, 8), max(W, 8))["depth_u8"][:H, :W]
    gx, gy = dggm_pre.sobel3_reflect101(d.astype(np.float32))
    rx = ndimage.correlate(d.astype(np.float64), KX, mode="mirror")
    ry = ndimage.correlate(d.astype(np.float64), KX.T, mode="mirror")
    np.testing.assert_array_equal(gx, rx.astype(np.float32))
    np.testing.assert_array_equal(gy, ry.astype(np.float32))


def test_quirks_q14():
    d = synthetic.make_scene(9, 64, 96)["depth_u8"]
    norm, gx, gy, mask = dggm_pre.calculate_gradient_features(d)
    assert mask.dtype == np.float32 and set(np.unique(mask)) <= {0.0, 1.0}
    assert (mask[d == 0] == 0).all()                      # invalid depth -> no gradient
    mn = np.float32(np.sqrt(gx * gx + gy * gy)[mask > 0].min())
    assert (norm[mask == 0] <= 0).all() and (norm[mask == 0] < 0).any() == (mn > 0)  # zeros go negative
    assert np.isclose(norm.max(), 1.0)


def test_degenerate_inputs():
    z = np.zeros((10, 12), np.uint8)
    norm, _, _, mask = dggm_pre.calculate_gradient_features(z)
    assert not norm.any() and not mask.any()
    c = np.full((10, 12), 77, np.uint8)
    norm, _, _, mask = dggm_pre.calculate_gradient_features(c)
    assert not norm.any() and not mask.any()
