"""The warp kernels divide by launch constants (Wf, Hf for the grid normalisation
of geometry.py:155-156, V for the mean of fusion.py:20) as
``(float)((double)a * (1.0 / (double)b))`` instead of an f32 division
(csrc/bev_geometry.h: div_rcp).  The claim is that this equals the IEEE f32
quotient for every float a.  Because a/b scales exactly with a's exponent, all
2^23 significands at one exponent plus the subnormal-result range cover every
case for a divisor; checked here for the divisors the path uses and more.
"""
import numpy as np
import pytest

DIVISORS = list(range(1, 17)) + [23, 31, 63, 97, 135, 240, 301, 1080, 1920, 16383]


def _check(a: np.ndarray, b: int):
    a = a.astype(np.float32)
    want = a / np.float32(b)
    got = (a.astype(np.float64) * (1.0 / float(b))).astype(np.float32)
    bad = want.view(np.uint32) != got.view(np.uint32)
    both_nan = np.isnan(want) & np.isnan(got)
    return int((bad & ~both_nan).sum())


@pytest.mark.parametrize("b", DIVISORS)
def test_div_rcp_all_significands(b):
    sig = np.arange(1 << 23, dtype=np.uint32)
    for exp in (127, 1):  # [1,2) and the smallest normal binade
        a = ((np.uint32(exp) << np.uint32(23)) | sig).view(np.float32)
        assert _check(a, b) == 0


@pytest.mark.parametrize("b", [1, 3, 7, 240, 1920])
def test_div_rcp_subnormal_and_specials(b):
    sub = np.arange(1 << 23, dtype=np.uint32).view(np.float32)  # every subnormal and +0
    assert _check(sub, b) == 0
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, np.finfo(np.float32).max,
                         -np.finfo(np.float32).max, np.finfo(np.float32).tiny], np.float32)
    assert _check(specials, b) == 0
