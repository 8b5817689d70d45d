"""Per-wave phase timing of the default fused warp (k_warp_fuse_v2; BEV_WARP_DEBUG=64, results garbage).

Usage (GPU): BEV_WARP_DEBUG=64 [BEV_WARP_OCC=2] python tools/warp_phases_v2.py
Cycles (s_memtime) per wave: prologue (corner boxes), first DMA + barrier, and summed over views:
synchronous staging, look-ahead DMA issue, taps + LDS sampling, end-of-view vmcnt wait + barrier; store.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd")]
import bev_rig  # noqa: E402
from models.fusion.geometry import GeometryTransformer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    V, C = 7, 64
    g = GeometryTransformer(480, 1440, (-24.0, 24.0, -7.2, 7.2))
    K, Rt = bev_rig.rig(V, 1080, 1920, 1)
    f = torch.randn(1, V, 135, 240, C, device=dev).permute(0, 1, 4, 2, 3)
    Kd, Rtd = torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev)
    for _ in range(3):
        out = g.forward_fused(f, Kd, Rtd, (1080, 1920), "mean")
    torch.cuda.synchronize()
    nt = (480 // 8) * (1440 // 32)
    rec = out.view(-1)[: nt * 4 * 12].view(torch.int32).cpu().numpy().reshape(nt * 4, 12).astype(np.int64)
    names = ["prologue", "dma0+bar", "sync stage", "dma issue", "taps+sample", "wait+bar", "store", "life"]
    for q, n in enumerate(names):
        x = rec[:, q]
        print(f"{n:12s} mean {x.mean():9.0f}  p50 {np.median(x):9.0f}  p90 {np.percentile(x, 90):9.0f}  "
              f"max {x.max():9.0f}")
    t0 = rec[:, 8] - rec[:, 8].min()
    t1 = rec[:, 9] - rec[:, 8].min()
    print(f"launch span {t1.max()} cycles; waves in flight (mean) {(t1 - t0).sum() / max(t1.max(), 1):.1f}")
    # start-time histogram: how many tiles start in each tenth of the launch
    h, _ = np.histogram(t0[::4], bins=10, range=(0, t1.max()))
    print("tile starts per tenth:", h.tolist())


if __name__ == "__main__":
    main()
