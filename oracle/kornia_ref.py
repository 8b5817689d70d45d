"""CPU restatement of the reference's kornia branch (geometry.py:124-141) -- TEST INFRASTRUCTURE ONLY.

Imported by tests/ only, never by the product package.  Parity status: **UNPINNED**.  The branch calls
`kornia.geometry.transform.warp_perspective` (kornia: unpinned, not listed in the reference's
requirements, absent from this image), so there is neither a kornia oracle nor a reference fixture.
This restates kornia's published algorithm (kornia 0.6/0.7 `warp_perspective`, `normalize_homography`,
`normal_transform_pixel`, `create_meshgrid`, `transform_points`, `convert_points_from_homogeneous`)
in float64 torch on the CPU, around the reference's own call site:

    H_i2w = _compute_img_to_world_homography(K, Rt)          (inv; pinv if |det| < 1e-8 / NaN / inf)
    S_feat2img = diag(W_img / Wf, H_img / Hf, 1)
    A_w2bev = [[1/res_x, 0, -min_x/res_x], [0, 1/res_y, -min_y/res_y], [0, 0, 1]]
    M = A_w2bev @ H_i2w @ S_feat2img                         (feature pixel -> BEV pixel)
    if M is not singular: warp_perspective(feat, M, dsize=(bev_h, bev_w), bilinear, zeros,
                                           align_corners=False)
    else: the grid_sample branch (geometry.py:143-162)

warp_perspective(src [C,H,W], M, (h, w)):
    D = N(h, w) @ M @ inv(N(H, W)),  N(h, w) = [[2/(w-1), 0, -1], [0, 2/(h-1), -1], [0, 0, 1]]
    T = inv(D)
    grid over xn = (linspace(0, w-1, w)/(w-1) - 0.5) * 2 (likewise yn):  q = T (xn, yn, 1)
    (gx, gy) = q.xy * (1 / (q.z + 1e-8) if |q.z| > 1e-8 else 1)
    F.grid_sample(src, (gx, gy), bilinear, zeros, align_corners=False)
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _ntp(h: int, w: int) -> torch.Tensor:
    T = torch.eye(3, dtype=torch.float64)
    T[0, 0] = 2.0 / (1e-14 if w == 1 else w - 1.0)
    T[1, 1] = 2.0 / (1e-14 if h == 1 else h - 1.0)
    T[0, 2] = T[1, 2] = -1.0
    return T


def warp_perspective(src: torch.Tensor, M: torch.Tensor, dsize) -> torch.Tensor:
    """kornia warp_perspective(src[None], M[None], dsize, 'bilinear', 'zeros', align_corners=False)[0]."""
    C, H, W = src.shape
    h, w = dsize
    D = _ntp(h, w) @ M.double() @ torch.linalg.inv(_ntp(H, W))
    T = torch.linalg.inv(D)
    xn = (torch.linspace(0, w - 1, w, dtype=torch.float64) / max(w - 1, 1) - 0.5) * 2
    yn = (torch.linspace(0, h - 1, h, dtype=torch.float64) / max(h - 1, 1) - 0.5) * 2
    yy, xx = torch.meshgrid(yn, xn, indexing="ij")
    p = torch.stack([xx, yy, torch.ones_like(xx)], dim=-1)  # [h, w, 3]
    q = p @ T.T
    z = q[..., 2:3]
    scale = torch.where(z.abs() > 1e-8, 1.0 / (z + 1e-8), torch.ones_like(z))
    grid = (q[..., :2] * scale)[None]
    return F.grid_sample(src.double()[None], grid, mode="bilinear", padding_mode="zeros", align_corners=False)[0]


def _homography(K: torch.Tensor, Rt: torch.Tensor) -> torch.Tensor:
    G = torch.stack([Rt[:3, 0], Rt[:3, 1], Rt[:3, 3]], dim=1)
    return K[:3, :3].double() @ G.double()


def grid_sample_branch(feat: torch.Tensor, K, Rt, img_size, bev_h, bev_w, bounds) -> torch.Tensor:
    """geometry.py:143-162 in float64 (the fallback of a singular M)."""
    C, Hf, Wf = feat.shape
    H_img, W_img = img_size
    min_x, max_x, min_y, max_y = bounds
    rx, ry = (max_x - min_x) / bev_w, (max_y - min_y) / bev_h
    xs = torch.linspace(min_x + 0.5 * rx, max_x - 0.5 * rx, bev_w, dtype=torch.float64)
    ys = torch.linspace(min_y + 0.5 * ry, max_y - 0.5 * ry, bev_h, dtype=torch.float64)
    yy, xx = torch.meshgrid(ys, xs, indexing="ij")
    uvw = torch.stack([xx, yy, torch.ones_like(xx)], dim=-1) @ _homography(K, Rt).T
    w = uvw[..., 2]
    w = torch.where(w.abs() < 1e-6, torch.ones_like(w), w)
    fx = uvw[..., 0] / w * (Wf / float(W_img))
    fy = uvw[..., 1] / w * (Hf / float(H_img))
    grid = torch.stack([(fx + 0.5) / Wf * 2 - 1, (fy + 0.5) / Hf * 2 - 1], dim=-1)[None]
    return F.grid_sample(feat.double()[None], grid, mode="bilinear", padding_mode="zeros", align_corners=False)[0]


def kornia_branch(feats: torch.Tensor, K: torch.Tensor, Rt: torch.Tensor, img_size, bev_h: int, bev_w: int,
                  bounds) -> torch.Tensor:
    """feats [B, V, C, Hf, Wf], K [B, V, 3, 3], Rt [B, V, 4, 4] -> [B, V, C, bev_h, bev_w] float64."""
    B, V, C, Hf, Wf = feats.shape
    H_img, W_img = img_size
    min_x, max_x, min_y, max_y = bounds
    rx, ry = (max_x - min_x) / bev_w, (max_y - min_y) / bev_h
    S = torch.diag(torch.tensor([W_img / float(Wf), H_img / float(Hf), 1.0], dtype=torch.float64))
    A = torch.tensor([[1.0 / rx, 0.0, -min_x / rx], [0.0, 1.0 / ry, -min_y / ry], [0.0, 0.0, 1.0]],
                     dtype=torch.float64)
    out = torch.zeros(B, V, C, bev_h, bev_w, dtype=torch.float64)
    for b in range(B):
        for v in range(V):
            Hw = _homography(K[b, v], Rt[b, v])
            det = torch.linalg.det(Hw)
            if torch.isnan(det) or torch.isinf(det) or det.abs() < 1e-8:
                Hi = torch.linalg.pinv(Hw)
            else:
                Hi = torch.linalg.inv(Hw)
            M = A @ Hi @ S
            dM = torch.linalg.det(M)
            if torch.isnan(dM) or torch.isinf(dM) or dM.abs() < 1e-8:
                out[b, v] = grid_sample_branch(feats[b, v], K[b, v], Rt[b, v], img_size, bev_h, bev_w, bounds)
            else:
                out[b, v] = warp_perspective(feats[b, v], M, (bev_h, bev_w))
    return out
