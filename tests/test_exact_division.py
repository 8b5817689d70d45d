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


def test_cell_ixy_reciprocal_randomized(tmp_path):
    """cell_ixy's u0 / ws through one refined double reciprocal (bev_geometry.h) equals the IEEE f32 quotient:
    tools/verify_div_rcp_ws.c on 3e6 random (u0, ws) pairs, subnormal / overflowing quotients included (the full
    3e8-sample run is recorded in the header comment)."""
    import os
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "verify_div_rcp_ws.c")
    exe = str(tmp_path / "vrw")
    subprocess.run(["gcc", "-O2", "-o", exe, src, "-lm"], check=True)
    out = subprocess.run([exe, "3000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "0 mismatches" in out.stdout
