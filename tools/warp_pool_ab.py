"""A/B of the fused warp's LDS pool (BEV_TUNE_WARP_POOL_KB) on the bench workload (7-cam 1080p ResNet-50
features, C = 64 channels-last, 480 x 1440 BEV, mean), HIP-event time per launch, interleaved rounds.

    python tools/warp_pool_ab.py --pools 0 36 32 --batch 2
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
import bev_rig  # noqa: E402
from models.encoders.cnn_encoder import CNNEncoder  # noqa: E402
from models.fusion.geometry import GeometryTransformer  # noqa: E402
from bench import BOUNDS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pools", type=int, nargs="*", default=[0])
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, V, H, W = a.batch, 7, 1080, 1920
    torch.manual_seed(1234)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(dev)
    geom = GeometryTransformer(480, 1440, BOUNDS)
    K, Rt = bev_rig.rig(V, H, W, B)
    Kd, Rtd = torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev)
    imgs = torch.randn(B, V, 3, H, W, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    with torch.no_grad():
        feats = enc(imgs)
        ref = geom.forward_fused(feats, Kd, Rtd, (H, W), "mean").clone()
    for rnd in range(a.rounds):
        for p in a.pools:
            old = nat.tune(nat.TUNE_WARP_POOL_KB, p)
            with torch.no_grad():
                out = geom.forward_fused(feats, Kd, Rtd, (H, W), "mean")
                same = torch.equal(out.view(torch.int32), ref.view(torch.int32))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                nat.spans_start()
                for _ in range(a.iters):
                    geom.forward_fused(feats, Kd, Rtd, (H, W), "mean")
                sp = nat.spans_stop()
            nat.tune(nat.TUNE_WARP_POOL_KB, old)
            us = sum(sp["warp_fuse"]) / len(sp["warp_fuse"]) * 1e3
            print(f"round {rnd} pool {p:3d} KiB: {us:7.1f} us per launch, bit-exact vs default: {same}", flush=True)


if __name__ == "__main__":
    main()
