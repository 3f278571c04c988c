"""The LSA restatement (oracle/lsap.py) against scipy itself: identical assignments — including
which optimum is returned on ties — on random float and tie-heavy integer cost matrices of the
shapes the Mask2Former matcher produces (100 queries x N targets, both orientations)."""
import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment as scipy_lsa

from oracle import lsap


def _cases():
    rng = np.random.default_rng(0)
    out = []
    for shape in [(1, 1), (3, 3), (5, 2), (2, 5), (100, 7), (7, 100), (12, 12), (100, 20)]:
        out.append(rng.standard_normal(shape))
        out.append(rng.integers(0, 3, shape).astype(np.float64))   # many ties
        out.append(np.zeros(shape))                                 # all tied
    out.append(np.full((4, 6), 1e10))
    out.append(rng.integers(-2, 2, (30, 9)).astype(np.float32).astype(np.float64))
    return out


@pytest.mark.parametrize("i", range(len(_cases())))
def test_oracle_lsap_matches_scipy(i):
    c = _cases()[i]
    a0, b0 = scipy_lsa(c)
    a1, b1 = lsap.linear_sum_assignment(c)
    np.testing.assert_array_equal(a0, a1)
    np.testing.assert_array_equal(b0, b1)


def test_oracle_lsap_empty():
    a, b = lsap.linear_sum_assignment(np.zeros((100, 0)))
    assert a.size == 0 and b.size == 0
