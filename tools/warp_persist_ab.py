"""Interleaved A/B of the fused warp's persistent kernel (BEV_TUNE_WARP_PERSIST 1, k_warp_fuse_p) against the
one-workgroup-per-tile kernel (0, k_warp_fuse_v2): bench geometry (7 cams, C = 64 NHWC features 135 x 240 ->
480 x 1440, B = 2, mean) or the K5 rig (--k5: 16 cams 4K, 270 x 480 maps, sum); footprint boxes computed once,
HIP events around the fused launches alone; us per launch, HBM fraction of the algorithmic bytes, and a bit check.

    python tools/warp_persist_ab.py [--k5] [--iters 20] [--rounds 4] [--pools 0:40] [--spans 0:80:100] [--bands 1:2:4]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
from bev_rig import rig  # noqa: E402
from models.fusion.geometry import GeometryTransformer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k5", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--pools", default="", help="WARP_POOL_KB values, comma- or colon-separated: A/B the per-tile kernel's pool")
    ap.add_argument("--spans", default="", help="WARP_SPAN values (colon-separated): A/B the span-staging threshold")
    ap.add_argument("--bands", default="", help="WARP_TILE_BAND values (colon-separated): A/B the tile order")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = GeometryTransformer(480, 1440, (-24.0, 24.0, -7.2, 7.2))
    if a.k5:
        V, H, W, Hf, Wf, B, mode = 16, 2160, 3840, 270, 480, 1, "sum"
    else:
        V, H, W, Hf, Wf, B, mode = 7, 1080, 1920, 135, 240, 2, "mean"
    K, Rt = rig(V, H, W, B)
    torch.manual_seed(0)
    f = torch.randn(B, V, Hf, Wf, 64, device=dev).permute(0, 1, 4, 2, 3)  # NHWC storage
    Kt, Rtt = torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev)
    Hm, xs, ys, hw = g._sampling(f, Kt, Rtt, (H, W))
    boxes = nat.warp_fuse_boxes(Hm, xs, ys, B, V, Hf, Wf, hw, mode)
    import bench
    alg, _, _ = bench.warp_alg_bytes(g, Hm, tuple(f.shape), (H, W), B)
    variants = [("persist", 1), ("persist", 2), ("persist", 0)]
    if a.pools:
        variants = [("pool", int(x)) for x in a.pools.replace(":", ",").split(",")]
    if a.spans:
        variants = [("span", int(x)) for x in a.spans.replace(":", ",").split(",")]
    if a.bands:
        variants = [("band", int(x)) for x in a.bands.replace(":", ",").split(",")]
    res = {v: [] for v in variants}
    ref = None
    for _ in range(a.rounds):
        for var in variants:
            knobs = {{"persist": "WARP_PERSIST", "pool": "WARP_POOL_KB", "span": "WARP_SPAN", "band": "WARP_TILE_BAND"}[var[0]]: var[1]}
            with nat.tuned(**knobs):
                bx = boxes if var[0] == "persist" else nat.warp_fuse_boxes(Hm, xs, ys, B, V, Hf, Wf, hw, mode)
                out = nat.warp_fuse(f, Hm, xs, ys, hw, mode, boxes=bx)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                elif not torch.equal(out, ref):
                    print(f"MISMATCH {var}", flush=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    nat.warp_fuse(f, Hm, xs, ys, hw, mode, boxes=bx, out=out)
                e1.record()
                torch.cuda.synchronize()
                res[var].append(e0.elapsed_time(e1) / a.iters * 1e3)
    for var, v in res.items():
        us = statistics.median(v)
        name = (["per-tile", "persistent 8 queues", "persistent 1 queue"][var[1]] if var[0] == "persist"
                else f"pool {var[1]} KiB" if var[0] == "pool" else f"span {var[1]} %" if var[0] == "span"
                else f"tile band {var[1]}")
        print(f"{name:20s} {us:8.2f} us  frac {alg / (us * 1e-6) / 8e12:.4f}  "
              f"(all: {', '.join(f'{x:.1f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
