"""C ABI of libbev_mi355x.so (include/bev_mi355x.h): loads, exports every declared
entry point, validates arguments on the host.  No GPU compute is launched here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, REPO

HEADER = os.path.join(REPO, "include", "bev_mi355x.h")
LIB = os.path.join(PKG, "libbev_mi355x.so")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bev_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    import bev_native
    if not os.path.exists(LIB):
        bev_native.build()
    return bev_native.lib()


def test_every_declared_symbol_is_exported(lib):
    syms = declared_symbols()
    assert len(syms) >= 15, syms
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    for s in syms:
        assert hasattr(lib, s)


def test_ctypes_signatures_cover_header(lib):
    import bev_native
    assert sorted(bev_native.SIGNATURES) == declared_symbols()


def test_abi_version(lib):
    import bev_native
    assert lib.bev_abi_version() == bev_native.ABI_VERSION


def test_linspace_host_entry_bit_exact(lib):
    """bev_linspace_f32 (host) == torch.linspace CPU as the reference calls it (geometry.py:26-27)."""
    import bev_native
    d = np.load(os.path.join(GOLDEN, "linspace_cases.npz"))
    pos = 0
    for lo, hi, n in zip(d["lo"], d["hi"], d["n"]):
        ref = d["out"][pos:pos + n]
        pos += n
        got = bev_native.linspace(float(lo), float(hi), int(n)).numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (lo, hi, n)


def test_argument_validation_without_gpu(lib):
    """Bad shapes are rejected on the host with BEV_ERR_ARGS (-1) before any launch."""
    null = None
    assert lib.bev_ipm_warp_f32(null, 0, 0, 0, 0, null, null, null, -1, 1, 1, 1, 1.0, 1.0, 1, 1, null, null) == -1
    assert lib.bev_ipm_warp_f32(null, 0, 0, 0, 0, null, null, null, 1, 1, 0, 1, 1.0, 1.0, 1, 1, null, null) == -1
    assert lib.bev_ipm_warp_fuse_f32(null, 0, 0, 0, 0, null, null, null, 1, 0, 1, 1, 1, 1.0, 1.0, 1, 1, 1, null,
                                     null) == -1
    assert lib.bev_ipm_warp_fuse_f32(null, 0, 0, 0, 0, null, null, null, 1, 1, 1, 1, 1, 1.0, 1.0, 1, 1, 7, null,
                                     null) == -1  # bad mode
    assert lib.bev_view_fuse_f32(null, 1, 0, 10, 0, null, null) == -1
    assert lib.bev_ipm_warp_fuse_bwd_f32(null, null, null, null, 1, 1, 1, 1, 1, 1.0, 1.0, 1, 1, 2, null, null) == -1
    # conv: output size inconsistent with the geometry, null pointers
    assert lib.bev_conv2d_f32(null, 0, 1, 8, 8, 16, null, null, null, 16, 3, 3, 1, 1, 0, null, 8, 8, null) == -1
    assert lib.bev_conv_packed_size(64, 64, 3, 3) > 0
    assert lib.bev_conv_packed_size(0, 64, 3, 3) == 0
    assert lib.bev_maxpool2d_nhwc_f32(null, 1, 8, 8, 4, 3, 2, 1, null, 4, 4, null) == -1
    # empty work is a successful no-op
    assert lib.bev_homography_f32(null, null, 0, null, null) == 0


def test_tune_knobs_host_only(lib):
    """bev_tune: every knob returns its previous value, rejects out-of-range values and unknown knobs;
    no GPU involved (knobs are read at launch)."""
    import bev_native as nat
    assert lib.bev_tune(99, 0) == -1
    for knob, good, bad in ((nat.TUNE_CONV_TILE, 3, 5), (nat.TUNE_WARP_POOL_KB, 16, 151), (nat.TUNE_WARP_KERNEL, 1, 5),
                            (nat.TUNE_WARP_BWD_POOL, 96, 1 << 20),
                            (nat.TUNE_CONV_XCD, 0, 2), (nat.TUNE_CONV_NBUF, 1, 3), (nat.TUNE_CONV_DMA, 2, 3),
                            (nat.TUNE_WGRAD_MFMA, 0, 3), (nat.TUNE_CONV_X6_TILE, 2, 3),
                            (nat.TUNE_CONV_X6_KERNEL, 1, 3), (nat.TUNE_CONV_H16_KERNEL, 1, 4),
                            (nat.TUNE_CONV_PW_SMALL, 0, 5),
                            (nat.TUNE_DW_RUN, 1, 4), (nat.TUNE_CONV_X6_NT, 1, 2),
                            (nat.TUNE_STEM3_STAGE, 1, 3), (nat.TUNE_WARP_PERSIST, 2, 3),
                            (nat.TUNE_WARP_SPAN, 50, 101), (nat.TUNE_WARP_TILE_BAND, 4, 65)):
        old = lib.bev_tune(knob, good)
        assert old >= 0
        assert lib.bev_tune(knob, bad) == -1
        assert lib.bev_tune(knob, old) == good
    with nat.tuned(WARP_KERNEL=1, WARP_POOL_KB=8):
        assert lib.bev_tune(nat.TUNE_WARP_KERNEL, 1) == 1
    assert lib.bev_tune(nat.TUNE_WARP_KERNEL, 0) == 0  # the default kernel stays selected
    # the round-6 warp knobs' defaults: span staging off, automatic tile bands, the per-tile kernel
    assert lib.bev_tune(nat.TUNE_WARP_SPAN, 0) == 0
    assert lib.bev_tune(nat.TUNE_WARP_TILE_BAND, 0) == 0
    assert lib.bev_tune(nat.TUNE_WARP_PERSIST, 0) == 0


def test_no_environment_knobs_in_library():
    """The shipped library reads no environment variables (performance knobs are bev_tune only)."""
    import glob
    for src in glob.glob(os.path.join(PKG, "csrc", "*.hip")) + glob.glob(os.path.join(PKG, "csrc", "*.h")):
        assert "getenv" not in open(src).read(), src
