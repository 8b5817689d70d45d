"""GeometryTransformer -- IPM homography warp of per-camera features onto the BEV ground grid.

Drop-in for the reference's `project/models/fusion/geometry.py` (class
GeometryTransformer, geometry.py:12-163): same constructor, same attributes
(`bev_h`, `bev_w`, `bounds`, `res_x`, `res_y`, `warp_impl`, non-persistent
`ground_grid` buffer), same `forward(feats, intrinsics, extrinsics,
img_size)` contract and the same static `_compute_homography` /
`_compute_img_to_world_homography` helpers (used externally at
model_wrapper.py:330,336).

What changes is HOW: the reference loops over (b, v) in Python and launches
~20 torch kernels plus one `F.grid_sample` per view (geometry.py:120-162).
Here every view of every frame is warped by ONE HIP kernel on gfx950
(`bev_ipm_warp_f32`), whose grid arithmetic restates the reference CPU's
rounding exactly, so the output is bit-identical to the reference's on the
same inputs.  `forward_fused` additionally folds the N-view reduction of
SimpleFusion into the warp (`bev_ipm_warp_fuse_f32`) and never materialises
the [B, V, C, Hb, Wb] intermediate -- the layout the benchmark uses.

There is no CPU path: forward() raises on CPU tensors (the HIP library is
the product; the CPU restatement lives in oracle/ for testing only).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

import bev_native as _nat

__all__ = ["GeometryTransformer", "ViewProjection", "gather_calibration", "KORNIA_AVAILABLE"]

# The reference's `_HAS_KORNIA` (geometry.py:5-9).  kornia is absent from this image, so by default
# warp_impl='kornia' runs the grid_sample semantics exactly like the reference does here (quirk Q7).
# Set True to get the branch the reference takes where kornia IS installed (geometry.py:124-141):
# kornia.geometry.transform.warp_perspective semantics, restated (kornia's published algorithm:
# normalize_homography -> inverse -> normalized meshgrid -> transform_points -> grid_sample,
# align_corners=False) and run on the same fused HIP warp kernel.  Parity UNPINNED (no kornia here).
KORNIA_AVAILABLE = False


def _normal_transform_pixel(h: int, w: int, dtype, device) -> torch.Tensor:
    """kornia normal_transform_pixel: pixel [0, w-1] x [0, h-1] -> [-1, 1]^2 (eps 1e-14 for size 1)."""
    T = torch.eye(3, dtype=dtype, device=device)
    T[0, 0] = 2.0 / (1e-14 if w == 1 else w - 1.0)
    T[1, 1] = 2.0 / (1e-14 if h == 1 else h - 1.0)
    T[0, 2] = T[1, 2] = -1.0
    return T


def _kornia_axis(n: int) -> torch.Tensor:
    """kornia create_meshgrid(normalized_coordinates=True) axis: (linspace(0, n-1, n) / (n-1) - 0.5) * 2."""
    a = torch.linspace(0, n - 1, n, dtype=torch.float32)
    return (a / (n - 1) - 0.5) * 2 if n > 1 else a


def _homography_operands(K: torch.Tensor, Rt: torch.Tensor):
    """(K33, G33) per geometry.py:35-62 shape rules, for ONE view (any device)."""
    if not isinstance(K, torch.Tensor) or K.dim() != 2 or K.shape[0] < 3 or K.shape[1] < 3:
        device = K.device if hasattr(K, "device") else torch.device("cpu")
        K = torch.eye(3, device=device)
        K[0, 0] = K[1, 1] = 1000.0
    else:
        K = K[:3, :3]
    if isinstance(Rt, torch.Tensor) and Rt.dim() == 2 and tuple(Rt.shape) in ((4, 4), (3, 4)):
        R = Rt[:3, :3] if Rt.shape[0] == 4 else Rt[:, :3]
        t = Rt[:3, 3:4] if Rt.shape[0] == 4 else Rt[:, 3:4]
    elif isinstance(Rt, torch.Tensor) and Rt.dim() == 2 and tuple(Rt.shape) == (3, 3):
        R = Rt
        t = torch.zeros(3, 1, device=Rt.device)
    else:
        device = Rt.device if hasattr(Rt, "device") else torch.device("cpu")
        R = torch.eye(3, device=device)
        t = torch.zeros(3, 1, device=device)
    G = torch.cat([R[:, 0:1], R[:, 1:2], t.to(R.dtype)], dim=1)
    return K, G


def _select(calib, b: int, v: int, B: int, V: int, eye: int, device):
    """get_K / get_Rt of geometry.py:96-118."""
    if isinstance(calib, torch.Tensor):
        if calib.dim() == 4:
            return calib[b, v]
        if calib.dim() == 3:
            return calib[v] if calib.shape[0] == V else calib[b]
        if calib.dim() == 2:
            return calib[:eye, :eye]
        return torch.eye(eye, device=device)
    return calib[b][v]


def gather_calibration(intrinsics, extrinsics, B: int, V: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Resolve the reference's calibration conventions into K33, G33 [B*V, 3, 3] fp32 on `device`.

    Fast path: 4-D tensors [B, V, >=3, >=3] and [B, V, 4|3, 4] (one batched
    slice, no per-view Python).  Anything else (lists of lists, 2-D/3-D
    tensors, odd shapes) follows the per-(b, v) rules of geometry.py:96-118
    and 33-64 verbatim.
    """
    if (isinstance(intrinsics, torch.Tensor) and intrinsics.dim() == 4 and tuple(intrinsics.shape[:2]) == (B, V)
            and intrinsics.shape[2] >= 3 and intrinsics.shape[3] >= 3 and isinstance(extrinsics, torch.Tensor)
            and extrinsics.dim() == 4 and tuple(extrinsics.shape[:2]) == (B, V)
            and tuple(extrinsics.shape[2:]) in ((4, 4), (3, 4))):
        K33 = intrinsics[:, :, :3, :3]
        R = extrinsics[:, :, :3, :3]
        t = extrinsics[:, :, :3, 3:4]
        G33 = torch.cat([R[..., 0:1], R[..., 1:2], t], dim=-1)
        K33 = K33.reshape(B * V, 3, 3)
        G33 = G33.reshape(B * V, 3, 3)
    else:
        Ks, Gs = [], []
        for b in range(B):
            for v in range(V):
                k, g = _homography_operands(_select(intrinsics, b, v, B, V, 3, device),
                                            _select(extrinsics, b, v, B, V, 4, device))
                Ks.append(k.to(device=device, dtype=torch.float32))
                Gs.append(g.to(device=device, dtype=torch.float32))
        K33 = torch.stack(Ks) if Ks else torch.empty(0, 3, 3, device=device)
        G33 = torch.stack(Gs) if Gs else torch.empty(0, 3, 3, device=device)
    return (K33.to(device=device, dtype=torch.float32).contiguous(),
            G33.to(device=device, dtype=torch.float32).contiguous())


class _WarpFn(torch.autograd.Function):
    """Per-view warp with a gradient to feats (the grid is constant)."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, feats4, H, xs, ys, img_hw):
        ctx.save_for_backward(H, xs, ys)
        ctx.meta = (feats4.shape[2], feats4.shape[3], img_hw)
        return _nat.warp(feats4, H, xs, ys, img_hw)

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, gout):
        H, xs, ys = ctx.saved_tensors
        Hf, Wf, img_hw = ctx.meta
        return _nat.warp_bwd(gout, H, xs, ys, Hf, Wf, img_hw), None, None, None, None


class _WarpFuseFn(torch.autograd.Function):
    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, feats5, H, xs, ys, img_hw, mode):
        if mode == "max":  # the backward re-samples the views to find each element's maximal one
            ctx.save_for_backward(H, xs, ys, feats5)
        else:
            ctx.save_for_backward(H, xs, ys)
        ctx.meta = (feats5.shape[1], feats5.shape[3], feats5.shape[4], img_hw, mode)
        return _nat.warp_fuse(feats5, H, xs, ys, img_hw, mode)

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, gout):
        V, Hf, Wf, img_hw, mode = ctx.meta
        if mode in ("sum", "mean"):
            H, xs, ys = ctx.saved_tensors
            return _nat.warp_fuse_bwd(gout, H, xs, ys, V, Hf, Wf, img_hw, mode), None, None, None, None, None
        # max (fusion.py:22 after geometry.py:161): the per-view samples again (bit-identical to the forward's),
        # the gradient to the view torch's max(dim) picks, then the per-view warp backward
        H, xs, ys, feats5 = ctx.saved_tensors
        B, C = feats5.shape[0], feats5.shape[2]
        f4 = feats5.reshape(B * V, C, Hf, Wf)
        per_view = _nat.warp(f4, H, xs, ys, img_hw).view(B, V, C, gout.shape[2], gout.shape[3])
        gv = _nat.view_max_bwd(per_view, gout)
        del per_view
        gf = _nat.warp_bwd(gv.view(B * V, C, gout.shape[2], gout.shape[3]), H, xs, ys, Hf, Wf, img_hw)
        return gf.view(B, V, C, Hf, Wf), None, None, None, None, None


class GeometryTransformer(nn.Module):
    def __init__(self, bev_h: int, bev_w: int, bev_bounds: tuple, warp_impl: str = "grid_sample"):
        super().__init__()
        self.bev_h = bev_h
        self.bev_w = bev_w
        self.bounds = bev_bounds  # (x_min, x_max, y_min, y_max)
        self.res_x = (bev_bounds[1] - bev_bounds[0]) / bev_w
        self.res_y = (bev_bounds[3] - bev_bounds[2]) / bev_h
        # 'kornia': grid_sample semantics like the reference without kornia (geometry.py:124, quirk Q7),
        # or kornia's warp_perspective semantics when KORNIA_AVAILABLE is set (see kornia_homographies).
        self.warp_impl = warp_impl if warp_impl in ("grid_sample", "kornia") else "grid_sample"
        xs, ys = self._axes()
        self.register_buffer("ground_grid", self._create_ground_grid(xs, ys), persistent=False)
        self._axes_cpu = (xs, ys)
        self._axes_dev = {}
        self._grid_cache = {}

    # ---- geometry.py:24-31 ------------------------------------------------------
    def _axes(self):
        min_x, max_x, min_y, max_y = self.bounds
        xs = _nat.linspace(min_x + 0.5 * self.res_x, max_x - 0.5 * self.res_x, self.bev_w)
        ys = _nat.linspace(min_y + 0.5 * self.res_y, max_y - 0.5 * self.res_y, self.bev_h)
        return xs, ys

    @staticmethod
    def _create_ground_grid(xs, ys):
        yy, xx = torch.meshgrid(ys, xs, indexing="ij")
        return torch.stack([xx, yy, torch.ones_like(xx)], dim=-1)  # [H, W, 3]

    def _device_axes(self, device):
        key = str(device)
        if key not in self._axes_dev:
            self._axes_dev[key] = tuple(a.to(device) for a in self._axes_cpu)
        return self._axes_dev[key]

    # ---- geometry.py:33-78 (static helpers kept for external callers) ----------
    @staticmethod
    def _compute_homography(K: torch.Tensor, Rt: torch.Tensor) -> torch.Tensor:
        K33, G = _homography_operands(K, Rt)
        if K33.is_cuda:
            return _nat.homography(K33[None].float(), G[None].float().to(K33.device)).view(3, 3)
        return K33 @ G

    @staticmethod
    def _compute_img_to_world_homography(K: torch.Tensor, Rt: torch.Tensor) -> torch.Tensor:
        H_w2i = GeometryTransformer._compute_homography(K, Rt)
        try:
            det = torch.det(H_w2i)
        except Exception:
            det = torch.tensor(float("nan"), device=H_w2i.device)
        if torch.isnan(det) or torch.isinf(det) or det.abs().item() < 1e-8:
            return torch.linalg.pinv(H_w2i)
        try:
            return torch.linalg.inv(H_w2i)
        except Exception:
            return torch.linalg.pinv(H_w2i)

    # ---- forward ----------------------------------------------------------------
    def homographies(self, intrinsics, extrinsics, B: int, V: int, device) -> torch.Tensor:
        """[B*V, 9] world->image homographies on `device` (bit-identical to geometry.py:143)."""
        K33, G33 = gather_calibration(intrinsics, extrinsics, B, V, device)
        return _nat.homography(K33, G33)

    def kornia_homographies(self, intrinsics, extrinsics, B: int, V: int, Hf: int, Wf: int, img_size, device):
        """kornia-branch sampling maps (geometry.py:124-141) in the kernel's parametrization.

        Per view: M = A_w2bev @ inv(K [r1 r2 t]) @ S_feat2img (feature pixel -> BEV pixel; the reference
        falls back to pinv when |det| < 1e-8); kornia's warp_perspective samples src at
        T (xn, yn, 1) with T = inv(N_bev @ M @ inv(N_feat)) over the normalized BEV meshgrid, then
        grid_sample(align_corners=False) un-normalizes ix = ((gx + 1) Wf - 1) / 2.  Folding that
        un-normalization into T gives one homography H' with ix = (H'_0 . p) / (H'_2 . p), p = (xn, yn, 1):
        the warp kernel runs it with the normalized axes and a unit feature scale.  Views whose M is
        singular (NaN / inf / |det| < 1e-8) take the reference's grid_sample fallback, expressed in the
        same parametrization (world x = a xn + b).  Computed in float64 on the device, no host sync.
        Returns (H' [B*V, 9] fp32, xs [Wb], ys [Hb]) and the kernel's img_hw = (Hf, Wf).
        """
        K33, G33 = gather_calibration(intrinsics, extrinsics, B, V, device)
        f64 = torch.float64
        Hw = K33.to(f64) @ G33.to(f64)  # world plane -> image pixels
        det = torch.linalg.det(Hw)
        bad = torch.isnan(det) | torch.isinf(det) | (det.abs() < 1e-8)
        Hw_safe = torch.where(bad[:, None, None], torch.eye(3, dtype=f64, device=device), Hw)
        Hi = torch.where(bad[:, None, None], torch.linalg.pinv(Hw), torch.linalg.inv(Hw_safe))
        H_img, W_img = img_size
        S = torch.diag(torch.tensor([W_img / float(Wf), H_img / float(Hf), 1.0], dtype=f64, device=device))
        min_x, _, min_y, _ = self.bounds
        A = torch.tensor([[1.0 / self.res_x, 0.0, -min_x / self.res_x], [0.0, 1.0 / self.res_y, -min_y / self.res_y],
                          [0.0, 0.0, 1.0]], dtype=f64, device=device)
        M = A @ Hi @ S
        detM = torch.linalg.det(M)
        singular = torch.isnan(detM) | torch.isinf(detM) | (detM.abs() < 1e-8)
        Nd = _normal_transform_pixel(self.bev_h, self.bev_w, f64, device)
        Ns = _normal_transform_pixel(Hf, Wf, f64, device)
        D = Nd @ torch.where(singular[:, None, None], torch.eye(3, dtype=f64, device=device), M) @ torch.linalg.inv(Ns)
        T = torch.linalg.inv(D)  # src_norm <- dst_norm
        U = torch.tensor([[Wf / 2.0, 0.0, (Wf - 1) / 2.0], [0.0, Hf / 2.0, (Hf - 1) / 2.0], [0.0, 0.0, 1.0]],
                         dtype=f64, device=device)
        Hk = U @ T
        # grid_sample fallback in the normalized parametrization: world = a * n + b per axis
        ax = self.res_x * (self.bev_w - 1) / 2.0
        ay = self.res_y * (self.bev_h - 1) / 2.0
        Nw = torch.tensor([[ax, 0.0, min_x + 0.5 * self.res_x + ax], [0.0, ay, min_y + 0.5 * self.res_y + ay],
                           [0.0, 0.0, 1.0]], dtype=f64, device=device)
        Sg = torch.diag(torch.tensor([Wf / float(W_img), Hf / float(H_img), 1.0], dtype=f64, device=device))
        Hg = Sg @ Hw @ Nw
        Hp = torch.where(singular[:, None, None], Hg, Hk).to(torch.float32).reshape(-1, 9).contiguous()
        xs = _kornia_axis(self.bev_w).to(device)
        ys = _kornia_axis(self.bev_h).to(device)
        return Hp, xs, ys, (Hf, Wf)

    def _sampling(self, feats, intrinsics, extrinsics, img_size):
        B, V, _, Hf, Wf = feats.shape
        device = feats.device
        if self.warp_impl == "kornia" and KORNIA_AVAILABLE:
            return self.kornia_homographies(intrinsics, extrinsics, B, V, Hf, Wf, img_size, device)
        H = self.homographies(intrinsics, extrinsics, B, V, device)
        xs, ys = self._device_axes(device)
        return H, xs, ys, tuple(img_size)

    def forward(self, feats: torch.Tensor, intrinsics, extrinsics,
                img_size: Tuple[int, int] = (1080, 1920)) -> torch.Tensor:
        """feats [B,V,C,Hf,Wf] -> per-view BEV maps [B,V,C,H_bev,W_bev] (geometry.py:80-163)."""
        B, V, C, Hf, Wf = feats.shape
        H, xs, ys, hw = self._sampling(feats, intrinsics, extrinsics, img_size)
        f4 = feats.reshape(B * V, C, Hf, Wf) if feats.is_contiguous() else feats.flatten(0, 1)
        out = _WarpFn.apply(f4, H, xs, ys, hw)
        return out.view(B, V, C, self.bev_h, self.bev_w)

    def forward_fused(self, feats: torch.Tensor, intrinsics, extrinsics, img_size: Tuple[int, int] = (1080, 1920),
                      mode: str = "mean", rows_per_chunk: Optional[int] = None,
                      memory_format: torch.memory_format = torch.contiguous_format,
                      num_chunks: Optional[int] = None) -> torch.Tensor:
        """SimpleFusion(mode)(self.forward(...)) in one kernel: [B,V,C,Hf,Wf] -> [B,C,H_bev,W_bev] (NCHW storage,
        as the reference's torch.mean over the stacked views gives).  memory_format=torch.channels_last (inference,
        channels-last features with C % 64 == 0): the same values in [B,H_bev,W_bev,C] storage
        (bev_ipm_warp_fuse_nhwc_f32), for a consumer that reads channels-last -- at the bench geometry the launch is
        ~4 % slower than the NCHW one (profiles/r05as_warp_nhwc_ab.txt), so it is not the default.
        rows_per_chunk (< H_bev, inference only): the same values in rank-chunk-major row order,
        [ceil(H_bev / rows_per_chunk), B, C, rows_per_chunk, W_bev] (padding rows zero) -- the layout the camera-shard
        reduce-scatter over BEV rows consumes without a permute (bev_dist.camera_sharded_forward); `num_chunks` (the
        world size, >= that count) pads the layout with all-zero chunks to exactly that many."""
        H, xs, ys, hw = self._sampling(feats, intrinsics, extrinsics, img_size)
        grad = torch.is_grad_enabled() and feats.requires_grad
        if rows_per_chunk is not None and (rows_per_chunk < self.bev_h or num_chunks):
            if grad:
                raise RuntimeError("forward_fused(rows_per_chunk=...) is an inference layout (no autograd)")
            return _nat.warp_fuse(feats, H, xs, ys, hw, mode, rows_per_chunk=rows_per_chunk, num_chunks=num_chunks)
        C = feats.shape[2]
        if (not grad and memory_format == torch.channels_last and feats.is_cuda and C % 64 == 0
                and feats.stride(2) == 1 and feats.shape[1] <= 64):
            return _nat.warp_fuse(feats, H, xs, ys, hw, mode, channels_last=True)
        return _WarpFuseFn.apply(feats, H, xs, ys, hw, mode)


# north_star vocabulary alias
ViewProjection = GeometryTransformer
