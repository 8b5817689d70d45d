"""ctypes front-end of the CPU oracle (bev_oracle.c) + the torch-CPU composition.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  Parity status:
pinned against tests/golden (generated from the reference by
tests/golden/make_golden.py).

Two things live here:

* `Oracle` -- thin numpy wrappers over the bit-exact C restatement of
  SURVEY.md Appendix A (grid, bilinear taps, per-view warp, view fusion,
  homography, linspace) and a direct conv2d.
* `reference_composition_cpu` -- the reference's own torch-CPU composition
  (geometry.py:120-163 per-(b,v) loop + fusion.py:21 mean), restated with the
  same torch ops.  It is what bench.py times as the CPU baseline ("port").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_bev.so")

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB


def _p(a, t=_f32p):
    return a.ctypes.data_as(t)


def _c(a, dt=np.float32):
    return np.ascontiguousarray(a, dtype=dt)


class Oracle:
    """Bit-exact CPU restatement.  variant 0 = AVX-512 MKL dot3."""

    def __init__(self, variant: int = 0):
        if not os.path.exists(LIB):
            build()
        self.lib = ctypes.CDLL(LIB)
        self.variant = variant
        L = self.lib
        L.oracle_linspace_f32.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int, _f32p]
        L.oracle_homography_f32.argtypes = [_f32p, _f32p, ctypes.c_int, _f32p, ctypes.c_int]
        geo = [_f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
               ctypes.c_int, ctypes.c_int]
        L.oracle_grid_f32.argtypes = geo + [_f32p, ctypes.c_int]
        L.oracle_taps_f32.argtypes = geo + [_i32p, _f32p, _u8p, ctypes.c_int]
        L.oracle_warp_f32.argtypes = [_f32p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                      _f32p, ctypes.c_int]
        L.oracle_fuse_f32.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, _f32p]
        L.oracle_conv2d_f32.argtypes = [_f32p, _f32p, _f32p] + [ctypes.c_int] * 10 + [_f32p]

    # ---- geometry.py:18-31 -------------------------------------------------
    def linspace(self, lo: float, hi: float, n: int) -> np.ndarray:
        out = np.empty(max(n, 0), np.float32)
        self.lib.oracle_linspace_f32(lo, hi, n, _p(out))
        return out

    def bev_axes(self, bev_h: int, bev_w: int, bounds):
        """xs[Wb], ys[Hb] cell centres (geometry.py:18-19,26-27; res in Python double)."""
        x0, x1, y0, y1 = bounds
        rx = (x1 - x0) / bev_w
        ry = (y1 - y0) / bev_h
        return self.linspace(x0 + 0.5 * rx, x1 - 0.5 * rx, bev_w), self.linspace(y0 + 0.5 * ry, y1 - 0.5 * ry, bev_h)

    # ---- geometry.py:33-64 -------------------------------------------------
    @staticmethod
    def homography_operands(K: np.ndarray, Rt: np.ndarray):
        """Restates the shape-tolerance branches of _compute_homography: returns (K33, G33)."""
        K = np.asarray(K, np.float32)
        Rt = np.asarray(Rt, np.float32)
        if K.ndim != 2 or K.shape[0] < 3 or K.shape[1] < 3:
            K = np.eye(3, dtype=np.float32)
            K[0, 0] = K[1, 1] = 1000.0
        else:
            K = K[:3, :3]
        R = np.eye(3, dtype=np.float32)
        t = np.zeros(3, np.float32)
        if Rt.ndim == 2:
            if Rt.shape == (4, 4):
                R, t = Rt[:3, :3], Rt[:3, 3]
            elif Rt.shape == (3, 4):
                R, t = Rt[:, :3], Rt[:, 3]
            elif Rt.shape == (3, 3):
                R = Rt
        G = np.stack([R[:, 0], R[:, 1], t], axis=1)
        return _c(K), _c(G)

    def homography(self, K33: np.ndarray, G33: np.ndarray) -> np.ndarray:
        K33 = _c(K33).reshape(-1, 9)
        G33 = _c(G33).reshape(-1, 9)
        H = np.empty_like(K33)
        self.lib.oracle_homography_f32(_p(K33), _p(G33), K33.shape[0], _p(H), self.variant)
        return H.reshape(-1, 3, 3)

    # ---- geometry.py:143-161 -----------------------------------------------
    def grid(self, H, xs, ys, Hf, Wf, img_hw):
        H = _c(H).reshape(-1, 9)
        n = H.shape[0]
        sx, sy = np.float32(Wf / float(img_hw[1])), np.float32(Hf / float(img_hw[0]))
        g = np.empty((n, len(ys), len(xs), 2), np.float32)
        self.lib.oracle_grid_f32(_p(H), _p(_c(xs)), _p(_c(ys)), n, Hf, Wf, sx, sy, len(ys), len(xs), _p(g),
                                 self.variant)
        return g

    def taps(self, H, xs, ys, Hf, Wf, img_hw):
        H = _c(H).reshape(-1, 9)
        n = H.shape[0]
        sx, sy = np.float32(Wf / float(img_hw[1])), np.float32(Hf / float(img_hw[0]))
        Hb, Wb = len(ys), len(xs)
        x0y0 = np.empty((n, Hb, Wb, 2), np.int32)
        wts = np.empty((n, Hb, Wb, 4), np.float32)
        valid = np.empty((n, Hb, Wb), np.uint8)
        self.lib.oracle_taps_f32(_p(H), _p(_c(xs)), _p(_c(ys)), n, Hf, Wf, sx, sy, Hb, Wb, _p(x0y0, _i32p),
                                 _p(wts), _p(valid, _u8p), self.variant)
        return x0y0, wts, valid

    def warp(self, feats, H, xs, ys, img_hw):
        """feats [N,C,Hf,Wf] -> [N,C,Hb,Wb] (the per-(b,v) body of geometry.py:120-162)."""
        feats = _c(feats)
        n, C, Hf, Wf = feats.shape
        H = _c(H).reshape(n, 9)
        sx, sy = np.float32(Wf / float(img_hw[1])), np.float32(Hf / float(img_hw[0]))
        out = np.empty((n, C, len(ys), len(xs)), np.float32)
        self.lib.oracle_warp_f32(_p(feats), _p(H), _p(_c(xs)), _p(_c(ys)), n, C, Hf, Wf, sx, sy, len(ys), len(xs),
                                 _p(out), self.variant)
        return out

    def geometry_forward(self, feats, K, Rt, img_hw, bev_h, bev_w, bounds):
        """GeometryTransformer.forward (grid_sample branch) on [B,V,C,Hf,Wf] with K [B,V,3,3], Rt [B,V,4,4]."""
        B, V = feats.shape[:2]
        ops = [self.homography_operands(K[b, v], Rt[b, v]) for b in range(B) for v in range(V)]
        H = self.homography(np.stack([o[0] for o in ops]), np.stack([o[1] for o in ops]))
        xs, ys = self.bev_axes(bev_h, bev_w, bounds)
        out = self.warp(feats.reshape((B * V,) + feats.shape[2:]), H, xs, ys, img_hw)
        return out.reshape((B, V) + out.shape[1:])

    # ---- fusion.py:17-22 ---------------------------------------------------
    def fuse(self, x, mode: str):
        x = _c(x)
        B, V = x.shape[:2]
        M = int(np.prod(x.shape[2:]))
        out = np.empty((B,) + x.shape[2:], np.float32)
        self.lib.oracle_fuse_f32(_p(x), B, V, M, {"sum": 0, "mean": 1, "max": 2}[mode], _p(out))
        return out

    def fused_stream(self, feats, K, Rt, img_hw, bev_h, bev_w, bounds, modes=("sum", "mean", "max")):
        """SimpleFusion(mode)(GeometryTransformer.forward(...)) for each mode, one view at a time.

        Same arithmetic as `fuse(geometry_forward(...))` (oracle_fuse_f32: sum from +0 in view
        order, mean = sum / f32(V), max = first view then `t > acc`), but never materialises the
        [B, V, C, Hb, Wb] stack -- full-size 16-camera rigs fit in host memory.  No NaNs expected."""
        B, V = feats.shape[:2]
        xs, ys = self.bev_axes(bev_h, bev_w, bounds)
        res = {}
        for b in range(B):
            acc_s, acc_m = None, None
            for v in range(V):
                Kv, Gv = self.homography_operands(K[b, v], Rt[b, v])
                H = self.homography(Kv[None], Gv[None])
                x = self.warp(feats[b, v][None], H, xs, ys, img_hw)[0]
                acc_s = x + np.float32(0.0) if acc_s is None else acc_s + x
                acc_m = x if acc_m is None else np.where(x > acc_m, x, acc_m)
            for m in modes:
                r = {"sum": acc_s, "mean": acc_s / np.float32(V), "max": acc_m}[m]
                res.setdefault(m, []).append(r.astype(np.float32, copy=False))
        return {m: np.stack(r) for m, r in res.items()}

    # ---- cnn_encoder.py:31-37 (direct conv) --------------------------------
    def conv2d(self, x, w, b, stride, pad, relu):
        x, w = _c(x), _c(w)
        N, Ci, H, W = x.shape
        Co, _, KH, KW = w.shape
        Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
        y = np.empty((N, Co, Ho, Wo), np.float32)
        bp = _p(_c(b)) if b is not None else None
        self.lib.oracle_conv2d_f32(_p(x), _p(w), bp, N, Ci, H, W, Co, KH, KW, stride, pad, int(relu), _p(y))
        return y


def reference_grid_cpu(K, Rt, img_hw, Hf, Wf, bev_h, bev_w, bounds):
    """The grid_sample grid the reference builds for each (b, v): geometry.py:26-27 (linspace ground grid),
    :143-158 (H = K [r1 r2 t], uvw = H g, w_safe, u / w, rescale, normalise), torch CPU fp32 ops as the
    reference runs them.  K [B,V,3,3], Rt [B,V,4,4] -> grid [B,V,Hb,Wb,2] fp32."""
    import torch

    B, V = K.shape[:2]
    H_img, W_img = img_hw
    x0, x1, y0, y1 = bounds
    rx, ry = (x1 - x0) / bev_w, (y1 - y0) / bev_h
    xs = torch.linspace(x0 + 0.5 * rx, x1 - 0.5 * rx, bev_w)
    ys = torch.linspace(y0 + 0.5 * ry, y1 - 0.5 * ry, bev_h)
    yy, xx = torch.meshgrid(ys, xs, indexing="ij")
    ground = torch.stack([xx, yy, torch.ones_like(xx)], dim=-1)
    g_flat = ground.reshape(-1, 3).T
    grid = torch.empty(B, V, bev_h, bev_w, 2)
    for b in range(B):
        for v in range(V):
            Kb, Rtb = K[b, v][:3, :3], Rt[b, v]
            G = torch.cat([Rtb[:3, 0:1], Rtb[:3, 1:2], Rtb[:3, 3:4]], dim=1)
            Hm = Kb @ G
            uvw = Hm @ g_flat
            w = uvw[2:3, :]
            w_safe = torch.where(w.abs() < 1e-6, torch.ones_like(w), w)
            u = uvw[0:1, :] / w_safe
            v_ = uvw[1:2, :] / w_safe
            pts = torch.stack([u.squeeze(0), v_.squeeze(0)], dim=1).reshape(bev_h, bev_w, 2)
            fp = pts.clone()
            fp[..., 0] = fp[..., 0] * (Wf / float(W_img))
            fp[..., 1] = fp[..., 1] * (Hf / float(H_img))
            nrm = fp.clone()
            nrm[..., 0] = (nrm[..., 0] + 0.5) / Wf * 2.0 - 1.0
            nrm[..., 1] = (nrm[..., 1] + 0.5) / Hf * 2.0 - 1.0
            grid[b, v] = nrm
    return grid


def reference_composition_cpu(feats, K, Rt, img_hw, bev_h, bev_w, bounds):
    """The reference's torch-CPU warp + mean composition, op for op.

    Restates geometry.py:90-163 (grid_sample branch, per-(b,v) Python loop,
    zero-initialised bev_out) followed by SimpleFusion('mean') (fusion.py:21).
    Used as the CPU baseline that bench.py times; inputs are torch CPU tensors.
    """
    import torch
    import torch.nn.functional as F

    B, V, C, Hf, Wf = feats.shape
    grid = reference_grid_cpu(K, Rt, img_hw, Hf, Wf, bev_h, bev_w, bounds)
    bev = torch.zeros(B, V, C, bev_h, bev_w)
    for b in range(B):
        for v in range(V):
            s = F.grid_sample(feats[b, v][None], grid[b, v][None], mode="bilinear", padding_mode="zeros",
                              align_corners=False)
            bev[b, v] = s[0]
    return bev.mean(dim=1)
