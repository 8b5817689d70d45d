"""Deterministic Wildtrack-shaped synthetic camera rig.

The reference has no synthetic-input generator; its calibration comes from the
Wildtrack XML files (`project/data/wildtrack_loader.py:154-247`).  For
measurement and parity we use a fixed, RNG-free rig that reproduces the
properties the hot path cares about: V cameras on an ellipse around the BEV
area, partial view overlap, and some BEV cells behind a camera (w < 0, quirk
Q5 of SURVEY.md Appendix C).

Everything is computed in float64 and cast to float32 at the end, exactly as
Appendix B states, so the same rig is produced on every host.
"""
from __future__ import annotations

import math

import numpy as np


def camera(v: int, V: int, img_h: int, img_w: int):
    """Return (K[3,3], Rt[4,4]) float32 for camera v of a V-camera rig.

    Rt maps world (z up, ground plane z=0) to camera coordinates; K is the
    pinhole intrinsic at image resolution img_h x img_w.
    """
    th = 2.0 * math.pi * v / V
    c = np.array([26.4 * math.cos(th), 12.0 * math.sin(th), 4.0 + 0.25 * (v % 8)])
    p = np.array([0.5 * (v % 7) - 1.5, 0.3 * (v % 7) - 0.9, 0.0])
    z = (p - c) / np.linalg.norm(p - c)
    x = np.cross(z, np.array([0.0, 0.0, 1.0]))
    x = x / np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z], axis=0)
    t = -R @ c
    Rt = np.eye(4)
    Rt[:3, :3] = R
    Rt[:3, 3] = t
    f = (1700.0 + 25.0 * (v % 7)) * img_w / 1920.0
    K = np.array([[f, 0.0, img_w / 2.0], [0.0, f, img_h / 2.0], [0.0, 0.0, 1.0]])
    return K.astype(np.float32), Rt.astype(np.float32)


def rig(V: int, img_h: int, img_w: int, B: int = 1):
    """Return (K[B,V,3,3], Rt[B,V,4,4]) float32 numpy arrays (same rig per frame)."""
    Ks, Rts = [], []
    for v in range(V):
        K, Rt = camera(v, V, img_h, img_w)
        Ks.append(K)
        Rts.append(Rt)
    K = np.stack(Ks)[None].repeat(B, axis=0)
    Rt = np.stack(Rts)[None].repeat(B, axis=0)
    return np.ascontiguousarray(K), np.ascontiguousarray(Rt)
