"""Footprint statistics of the fused warp's tiles (k_warp_boxes, the corner boxes every (frame, 16 x 16 tile, view)
gets) for the bench geometries: how many (tile, view) pairs are empty, take the corner box, or need the exact
per-cell reduction (w sign change / near the 1e-6 clamp); the box sizes in pixels against the LDS pool; and per tile
the sum of its live views' images (does everything fit the pool at once).  Boxes are computed with the pool knob at
its maximum, so "too large" is decided here per pool size.

    python tools/warp_box_stats.py            # K2: 7 cams 1080p batch 2 -> 135 x 240 maps; K5: 16 cams 4K -> 270 x 480
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
import bev_rig  # noqa: E402
from models.fusion.geometry import GeometryTransformer  # noqa: E402
from bench import BOUNDS  # noqa: E402


def stats(name, B, V, H, W, Hf, Wf, pools_kib=(24, 36, 49, 72, 100)):
    dev = torch.device("cuda")
    geom = GeometryTransformer(480, 1440, BOUNDS)
    K, Rt = bev_rig.rig(V, H, W, B)
    feats = torch.empty(B, V, Hf, Wf, 64, device=dev).permute(0, 1, 4, 2, 3)
    Hm, xs, ys, hw = geom._sampling(feats, torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev), (H, W))
    old = nat.tune(nat.TUNE_WARP_POOL_KB, 150)
    try:
        ws = nat.warp_fuse_boxes(Hm, xs, ys, B, V, Hf, Wf, hw, "mean")
    finally:
        nat.tune(nat.TUNE_WARP_POOL_KB, old)
    torch.cuda.synchronize()
    nt = 90 * 30
    bx = ws.view(torch.int32).cpu().numpy().view(np.uint32)[4: 4 + B * nt * V * 2].reshape(B, nt, V, 2)  # after the 16-B header
    a, c = bx[..., 0].astype(np.int64), bx[..., 1].astype(np.int64)
    bad = (a >> 31) & 1
    x0, y0 = a & 0xFFFF, (a >> 16) & 0x7FFF
    x1, y1 = (c & 0xFFFF) - 1, (c >> 16) - 1
    empty = (x1 < 0) & (bad == 0)
    npix = np.where(x1 >= 0, (x1 - x0 + 1) * (y1 - y0 + 1), 0)
    live = ~empty
    tv = B * nt * V
    print(f"== {name}: {B} frame(s) x {nt} tiles x {V} views = {tv} (tile, view) pairs")
    print(f"   empty {empty.sum()} ({empty.mean():.3f}), corner box {(live & (bad == 0)).sum()}, exact per-cell "
          f"(corner bound n/a) {bad.sum()} ({bad.mean():.4f}); live views per tile {live.sum(-1).mean():.2f}")
    ok = live & (bad == 0)
    q = np.percentile(npix[ok], [10, 50, 90, 99, 100])
    print(f"   corner-box pixels: mean {npix[ok].mean():.1f}, p10/50/90/99/max {q.astype(int).tolist()}, "
          f"bytes/pixel 272 -> mean {npix[ok].mean() * 272 / 1024:.1f} KiB")
    tot = np.where(ok, npix, 0).sum(-1) * 272  # per (frame, tile)
    anybad = (live & (bad == 1)).any(-1)
    for kb in pools_kib:
        pool = kb * 1024
        maxpix = pool // 272 - 4
        fit1 = ok & (npix <= maxpix)
        two = ok & (npix * 2 * 272 <= pool)
        print(f"   pool {kb:3d} KiB: views fitting {fit1.sum() / max(1, ok.sum()):.3f}, views fitting twice (double "
              f"buffer) {two.sum() / max(1, ok.sum()):.3f}, tiles whose live views all fit at once "
              f"{((tot <= pool) & ~anybad).mean():.3f}")


def main():
    stats("K2 (7 cams, 1080p, batch 2, 135 x 240 maps)", 2, 7, 1080, 1920, 135, 240)
    stats("K5 (16 cams, 4K, 1 frame, 270 x 480 maps)", 1, 16, 2160, 3840, 270, 480)


if __name__ == "__main__":
    main()
