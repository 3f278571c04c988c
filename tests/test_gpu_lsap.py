"""f3: batched GPU linear sum assignment (csrc/lsap.hip) vs scipy.optimize.linear_sum_assignment
on the same float32 matrices — identical (row_ind, col_ind), ties included — and the
HipHungarianMatcher vs the HF matcher (transformers 5.15 modeling_mask2former.py:412-483)."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment as scipy_lsa

from rgbd_amd import matcher, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mats(seed):
    rng = np.random.default_rng(seed)
    out = []
    for shape in [(100, 7), (7, 100), (100, 1), (1, 1), (100, 37), (100, 100), (100, 150), (12, 5), (3, 64),
                  (65, 130), (100, 0)]:
        out.append(rng.standard_normal(shape).astype(np.float32))
        out.append(rng.integers(0, 3, shape).astype(np.float32))   # tie-heavy
    out.append(np.zeros((100, 20), np.float32))
    out.append(np.full((10, 10), 1e10, np.float32))
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lsa_batch_matches_scipy(seed):
    mats = _mats(seed)
    got = ops.linear_sum_assignment_batch([torch.from_numpy(m).to(DEV) for m in mats], validate=True)
    for m, (a, b) in zip(mats, got):
        ea, eb = scipy_lsa(m.astype(np.float64))
        np.testing.assert_array_equal(a.cpu().numpy(), ea, err_msg=str(m.shape))
        np.testing.assert_array_equal(b.cpu().numpy(), eb, err_msg=str(m.shape))


def test_lsa_many_small_tie_heavy():
    rng = np.random.default_rng(5)
    mats = [rng.integers(-1, 2, (int(rng.integers(1, 30)), int(rng.integers(1, 30)))).astype(np.float32)
            for _ in range(300)]
    got = ops.linear_sum_assignment_batch([torch.from_numpy(m).to(DEV) for m in mats], validate=True)
    for m, (a, b) in zip(mats, got):
        ea, eb = scipy_lsa(m)
        assert np.array_equal(a.cpu().numpy(), ea) and np.array_equal(b.cpu().numpy(), eb), m


def test_lsa_invalid_entries_raise():
    m = torch.zeros((4, 5), device=DEV)
    m[1, 2] = float("nan")
    with pytest.raises(ValueError):
        ops.linear_sum_assignment_batch([m], validate=True)
    m = torch.zeros((4, 5), device=DEV)
    m[0, 0] = float("-inf")
    with pytest.raises(ValueError):
        ops.linear_sum_assignment_batch([m], validate=True)
    m = torch.full((3, 3), float("inf"), device=DEV)
    with pytest.raises(ValueError):
        ops.linear_sum_assignment_batch([m], validate=True)


def test_hip_matcher_matches_hf():
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerHungarianMatcher
    ref = Mask2FormerHungarianMatcher(cost_class=2.0, cost_mask=5.0, cost_dice=5.0, num_points=12544)
    hip = Mask2FormerHungarianMatcher(cost_class=2.0, cost_mask=5.0, cost_dice=5.0, num_points=12544)
    assert matcher.install(hip) == 1
    g = torch.Generator(device=DEV).manual_seed(0)
    B, Q, L, H, W = 3, 100, 49, 60, 80
    masks = torch.randn((B, Q, H, W), generator=g, device=DEV)
    classes = torch.randn((B, Q, L), generator=g, device=DEV)
    mask_labels, class_labels = [], []
    for n in (5, 0, 23):
        mask_labels.append((torch.rand((n, H * 4, W * 4), generator=g, device=DEV) > 0.7).float())
        class_labels.append(torch.randint(0, L - 1, (n,), generator=g, device=DEV))
    torch.manual_seed(11)
    r = ref(masks, classes, mask_labels, class_labels)
    torch.manual_seed(11)
    h = hip(masks, classes, mask_labels, class_labels)
    for (ra, rb), (ha, hb) in zip(r, h):
        assert ha.is_cuda and ha.dtype == torch.int64
        assert torch.equal(ra, ha.cpu()) and torch.equal(rb, hb.cpu())
