"""Micro-benchmark of the depthwise conv (bev_dwconv2d_f32, SiLU, with SE partial sums) on EfficientNet-B3
layer shapes at 7 x 1080p (features_only to stride 8): time per call and HBM bytes / time.

    python tools/dwconv_micro.py [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))

import torch  # noqa: E402

import bev_native as nat  # noqa: E402

N = 7
# name: (C, K, stride, H_in, W_in)  -- B3: stem 40 @ 540x960; stage 1 dw 40; stage 2 e6 144 (s2), 192; stage 3 k5
LAYERS = {
    "s1.dw40": (40, 3, 1, 540, 960),
    "s2.dw144s2": (144, 3, 2, 540, 960),
    "s2.dw192": (192, 3, 1, 270, 480),
    "s3.dw192k5s2": (192, 5, 2, 270, 480),
    "s3.dw288k5": (288, 5, 1, 135, 240),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("layers", nargs="*", default=list(LAYERS))
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name in a.layers:
        C, K, s, H, W = LAYERS[name]
        p = K // 2
        x = torch.randn(N, H, W, C, device=dev, generator=g)
        wt = torch.randn(K * K, C, device=dev, generator=g) * 0.2
        b = torch.randn(C, device=dev, generator=g) * 0.1
        for _ in range(2):
            y, ps = nat.dwconv2d_nhwc(x, wt, b, K, s, p, nat.ACT_SILU, want_psum=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            y, ps = nat.dwconv2d_nhwc(x, wt, b, K, s, p, nat.ACT_SILU, want_psum=True)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        byts = 4 * (x.numel() + y.numel())
        print(f"{name:13s} {ms * 1e3:8.1f} us  {byts / ms / 1e6:7.1f} GB/s(io)  in {x.numel() * 4 / 1e6:.0f} MB "
              f"out {y.numel() * 4 / 1e6:.0f} MB", flush=True)


if __name__ == "__main__":
    main()
