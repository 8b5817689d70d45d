"""The reference's kornia branch (geometry.py:124-141) -- parity UNPINNED.

kornia is not installed here (nor pinned by the reference), so there is no kornia oracle and no
reference fixture for this branch.  `oracle/kornia_ref.py` restates kornia's published
warp_perspective algorithm in float64; these tests check the drop-in's kornia mode
(`models.fusion.geometry.KORNIA_AVAILABLE = True`, warp_impl='kornia') against that restatement:

* CPU: the sampling coordinates the HIP kernel will compute from the folded homography H'
  (ix = (H'_0 . p) / (H'_2 . p) over the normalized axes) agree with kornia's
  (grid from T, then grid_sample's align_corners=False un-normalization) to fp32 rounding;
* GPU: the warped maps (per view and fused mean) agree with the float64 restatement, including a
  view whose M is singular (the grid_sample fallback).  Tolerance: bilinear sampling is continuous
  in the coordinates except where a tap crosses the image border, so 99.9 % of the elements within
  1e-4 x max|feat| and all but 0.1 % within 1e-3 x max|feat|.
Default behaviour (KORNIA_AVAILABLE = False, as in the reference without kornia) is covered by the
bit-exact grid_sample tests (test_warp_gpu.py).
"""
import numpy as np
import pytest
import torch

import bev_rig
import kornia_ref
from models.fusion import geometry as G

BOUNDS = (-24.0, 24.0, -7.2, 7.2)


def _setup(V=4, B=1, img=(270, 480), feat=(34, 60), bev=(40, 120)):
    K, Rt = bev_rig.rig(V, img[0], img[1], B)
    return torch.from_numpy(K), torch.from_numpy(Rt), img, feat, bev


def test_folded_homography_matches_kornia_grid():
    K, Rt, img, (Hf, Wf), (Hb, Wb) = _setup()
    geom = G.GeometryTransformer(Hb, Wb, BOUNDS, warp_impl="kornia")
    Hp, xs, ys, hw = geom.kornia_homographies(K, Rt, 1, K.shape[1], Hf, Wf, img, torch.device("cpu"))
    assert hw == (Hf, Wf) and xs.shape == (Wb,) and ys.shape == (Hb,)
    yy, xx = torch.meshgrid(ys.double(), xs.double(), indexing="ij")
    p = torch.stack([xx, yy, torch.ones_like(xx)], dim=-1)
    S = torch.diag(torch.tensor([img[1] / Wf, img[0] / Hf, 1.0], dtype=torch.float64))
    rx, ry = 48.0 / Wb, 14.4 / Hb
    A = torch.tensor([[1 / rx, 0, 24.0 / rx], [0, 1 / ry, 7.2 / ry], [0, 0, 1.0]], dtype=torch.float64)
    for v in range(K.shape[1]):
        q = p @ Hp[v].view(3, 3).double().T
        ix, iy = q[..., 0] / q[..., 2], q[..., 1] / q[..., 2]
        M = A @ torch.linalg.inv(kornia_ref._homography(K[0, v], Rt[0, v])) @ S
        T = torch.linalg.inv(kornia_ref._ntp(Hb, Wb) @ M @ torch.linalg.inv(kornia_ref._ntp(Hf, Wf)))
        r = p @ T.T
        gx, gy = r[..., 0] / (r[..., 2] + 1e-8), r[..., 1] / (r[..., 2] + 1e-8)
        kx, ky = ((gx + 1) * Wf - 1) / 2, ((gy + 1) * Hf - 1) / 2
        ok = (kx.abs() < 4 * Wf) & (ky.abs() < 4 * Hf)  # cells that can sample the map
        assert ok.any()
        assert ((ix - kx).abs()[ok] <= 1e-3 + 1e-5 * kx.abs()[ok]).all()
        assert ((iy - ky).abs()[ok] <= 1e-3 + 1e-5 * ky.abs()[ok]).all()


def _close(got, ref, what):
    scale = ref.abs().max().item()
    d = (got.double() - ref).abs() / scale
    assert (d > 1e-3).double().mean().item() <= 1e-3, (what, d.max().item())
    assert (d > 1e-4).double().mean().item() <= 1e-3, (what, (d > 1e-4).double().mean().item())


@pytest.mark.gpu
@pytest.mark.parametrize("C", [8, 64])
def test_kornia_mode_vs_restatement(C, monkeypatch):
    monkeypatch.setattr(G, "KORNIA_AVAILABLE", True)
    K, Rt, img, (Hf, Wf), (Hb, Wb) = _setup(V=4, B=2)
    K = K.clone()
    K[1, 2] = 0.0  # frame 1, view 2: singular homography -> pinv -> singular M -> grid_sample fallback
    feats = torch.from_numpy(np.random.default_rng(3).standard_normal((2, 4, C, Hf, Wf), dtype=np.float32))
    ref = kornia_ref.kornia_branch(feats, K, Rt, img, Hb, Wb, BOUNDS)
    geom = G.GeometryTransformer(Hb, Wb, BOUNDS, warp_impl="kornia")
    dev = torch.device("cuda:0")
    fd = feats.to(dev)
    if C % 64 == 0:
        fd = fd.permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)  # channels-last: the LDS-DMA kernel
    with torch.no_grad():
        per_view = geom(fd, K.to(dev), Rt.to(dev), img).cpu()
        fused = geom.forward_fused(fd, K.to(dev), Rt.to(dev), img, "mean").cpu()
    _close(per_view, ref, "per-view")
    _close(fused, ref.mean(dim=1), "fused mean")
    # default: the reference without kornia (grid_sample semantics) differs from the kornia branch
    monkeypatch.setattr(G, "KORNIA_AVAILABLE", False)
    with torch.no_grad():
        gs = geom(fd, K.to(dev), Rt.to(dev), img).cpu()
    assert not torch.allclose(gs, per_view)
