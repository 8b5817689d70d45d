"""Pin the CPU oracle (oracle/bev_oracle.c) to the reference's own outputs.

The fixtures were produced by importing the reference modules
(tests/golden/make_golden.py): geometry.py:142-162 (grid_sample branch),
geometry.py:33-64 (_compute_homography), fusion.py:11-46, cnn_encoder.py:31-37.
Bit-exact everywhere except the conv (tolerance; MKL-DNN order not restated).
"""
import glob
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def feats_for(d):
    B, V, C, Hf, Wf = (int(d[k]) for k in ("B", "V", "C", "Hf", "Wf"))
    return np.random.default_rng(int(d["seed"])).standard_normal(size=(B, V, C, Hf, Wf), dtype=np.float32)


WARP_FILES = sorted(glob.glob(os.path.join(GOLDEN, "warp_*.npz")))


def test_linspace_bit_exact(oracle):
    d = np.load(os.path.join(GOLDEN, "linspace_cases.npz"))
    pos = 0
    for lo, hi, n in zip(d["lo"], d["hi"], d["n"]):
        ref = d["out"][pos:pos + n]
        pos += n
        assert np.array_equal(bits(oracle.linspace(float(lo), float(hi), int(n))), bits(ref)), (lo, hi, n)


def test_homography_branches_bit_exact(oracle):
    d = np.load(os.path.join(GOLDEN, "homography_cases.npz"))
    names = sorted({f.rsplit("_", 1)[0] for f in d.files})
    assert len(names) == 7
    for k in names:
        K33, G33 = oracle.homography_operands(d[k + "_K"], d[k + "_Rt"])
        assert np.array_equal(bits(oracle.homography(K33, G33)[0]), bits(d[k + "_H"])), k


@pytest.mark.parametrize("path", WARP_FILES, ids=[os.path.basename(p)[:-4] for p in WARP_FILES])
def test_warp_bit_exact(oracle, path):
    d = np.load(path)
    bounds = tuple(float(x) for x in d["bounds"])
    img = (int(d["img_h"]), int(d["img_w"]))
    xs, ys = oracle.bev_axes(int(d["bev_h"]), int(d["bev_w"]), bounds)
    assert np.array_equal(bits(xs), bits(d["xs"])) and np.array_equal(bits(ys), bits(d["ys"]))
    out = oracle.geometry_forward(feats_for(d), d["K"], d["Rt"], img, int(d["bev_h"]), int(d["bev_w"]), bounds)
    assert tuple(out.shape) == tuple(d["out_shape"])
    assert sha(out) == str(d["out_sha"])
    if "out" in d.files:
        assert np.array_equal(bits(out), bits(d["out"]))
    else:
        assert np.array_equal(bits(out.reshape(-1)[d["out_idx"]]), bits(d["out_val"]))


def test_grid_bit_exact(oracle):
    d = np.load(os.path.join(GOLDEN, "warp_w1_7cam_1080p.npz"))
    B, V, Hf, Wf = (int(d[k]) for k in ("B", "V", "Hf", "Wf"))
    ops = [oracle.homography_operands(d["K"][b, v], d["Rt"][b, v]) for b in range(B) for v in range(V)]
    H = oracle.homography(np.stack([o[0] for o in ops]), np.stack([o[1] for o in ops]))
    assert np.array_equal(bits(H), bits(d["H"].reshape(-1, 3, 3)))
    g = oracle.grid(H, d["xs"], d["ys"], Hf, Wf, (int(d["img_h"]), int(d["img_w"])))
    assert sha(g) == str(d["grid_sha"])
    assert np.array_equal(bits(g.reshape(-1, 2)[d["grid_idx"]]), bits(d["grid_val"]))


def test_degenerate_case_exercises_w_safe(oracle):
    """W6 must really contain |w| < 1e-6 cells and w < 0 cells (geometry.py:147, quirk Q5)."""
    d = np.load(os.path.join(GOLDEN, "warp_w6_degenerate.npz"))
    H = d["H"].reshape(-1, 3, 3).astype(np.float64)
    xs, ys = d["xs"].astype(np.float64), d["ys"].astype(np.float64)
    w = H[:, 2, 0][:, None, None] * xs[None, None, :] + H[:, 2, 1][:, None, None] * ys[None, :, None] + H[:, 2, 2][:, None, None]
    assert (np.abs(w) < 1e-6).any() and (w < 0).any()


@pytest.mark.parametrize("V", [2, 3, 7, 16])
def test_fusion_bit_exact(oracle, V):
    d = np.load(os.path.join(GOLDEN, "fusion_cases.npz"))
    x = d[f"V{V}_in"]
    for m in ("sum", "mean", "max"):
        assert np.array_equal(bits(oracle.fuse(x, m)), bits(d[f"V{V}_{m}"])), m
    assert np.array_equal(bits(oracle.fuse(x, "mean")), bits(d[f"V{V}_attention"]))  # fusion.py:36
    assert np.array_equal(x.reshape(x.shape[0], -1, *x.shape[3:]), d[f"V{V}_concat"])  # fusion.py:46


def test_fusion_full_size_mean(oracle):
    d = np.load(os.path.join(GOLDEN, "fusion_cases.npz"))
    x = np.random.default_rng(77).standard_normal(size=(1, 7, 2, 480, 1440), dtype=np.float32)
    m = oracle.fuse(x, "mean")
    assert sha(m) == str(d["big_mean_sha"])


def test_encoder_fallback_conv(oracle):
    """cnn_encoder.py:31-37 restated as two direct convs (+ReLU); tolerance only."""
    d = np.load(os.path.join(GOLDEN, "encoder_fallback.npz"))
    w0, b0 = d["w_backbone_0_weight"], d["w_backbone_0_bias"]
    w2, b2 = d["w_backbone_2_weight"], d["w_backbone_2_bias"]
    for x, y in ((d["x5"].reshape(-1, *d["x5"].shape[2:]), d["y5"].reshape(-1, *d["y5"].shape[2:])), (d["x4"], d["y4"][0])):
        h = oracle.conv2d(x, w0, b0, 2, 1, True)
        z = oracle.conv2d(h, w2, b2, 2, 1, True)
        np.testing.assert_allclose(z, y, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("path", [p for p in WARP_FILES if "16cam" not in p], ids=lambda p: os.path.basename(p)[:-4])
def test_fused_stream_equals_stacked_fuse(oracle, path):
    """Oracle.fused_stream (view-at-a-time, used for the full-size GPU references) == fuse(geometry_forward)."""
    d = np.load(path)
    feats = feats_for(d)
    img = (int(d["img_h"]), int(d["img_w"]))
    bh, bw = int(d["bev_h"]), int(d["bev_w"])
    bounds = tuple(float(x) for x in d["bounds"])
    per_view = oracle.geometry_forward(feats, d["K"], d["Rt"], img, bh, bw, bounds)
    got = oracle.fused_stream(feats, d["K"], d["Rt"], img, bh, bw, bounds)
    for mode in ("sum", "mean", "max"):
        assert np.array_equal(bits(got[mode]), bits(oracle.fuse(per_view, mode))), mode
