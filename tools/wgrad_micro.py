"""Micro-benchmark of the conv weight gradient (bev_conv_wgrad_f32) on ResNet-50 layer shapes at 7 x 1080p.

    python tools/wgrad_micro.py [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))

import torch  # noqa: E402

import bev_native as nat  # noqa: E402

N = 7
# name: (Ci, Co, k, stride, H_in, W_in)
LAYERS = {
    "l1.c2": (64, 64, 3, 1, 270, 480),
    "l1.c1": (256, 64, 1, 1, 270, 480),
    "l1.c3": (64, 256, 1, 1, 270, 480),
    "l2.c2": (128, 128, 3, 1, 135, 240),
    "l2.c1": (512, 128, 1, 1, 135, 240),
    "l2.c3": (128, 512, 1, 1, 135, 240),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("layers", nargs="*", default=list(LAYERS))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--kernels", type=int, nargs="*", default=[2, 1], help="BEV_TUNE_WGRAD_MFMA values to A/B")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name in a.layers:
        Ci, Co, k, s, H, W = LAYERS[name]
        p = k // 2
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Ci, device=dev, generator=g)
        dz = torch.randn(N, Ho, Wo, Co, device=dev, generator=g)
        ref = None
        for kern in a.kernels:
            with nat.tuned(WGRAD_MFMA=kern):
                for _ in range(2):
                    dw = nat.conv_wgrad(x, dz, k, k, s, p)
                ref = dw if ref is None else ref
                err = float((dw - ref).abs().max() / ref.abs().max())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    nat.conv_wgrad(x, dz, k, k, s, p)
                e1.record()
                torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            flops = 2.0 * N * Ho * Wo * Co * Ci * k * k
            print(f"{name:6s} kernel {kern}: {ms * 1e3:8.1f} us  {flops / ms / 1e9:6.1f} TF  (rel diff vs first {err:.1e})",
                  flush=True)


if __name__ == "__main__":
    main()
