"""Micro-benchmark of single backbone conv layers (ResNet-50 at 7 x 1080x1920) on the HIP kernel.

    python tools/conv_micro.py l1.0.c3 l2.1.c2 stem --iters 20

Prints one line per layer: time per call (HIP events) and TFLOP/s.  Used with
rocprofv3 --pmc to attribute counters to one layer shape at a time.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))

import torch  # noqa: E402

import bev_native as nat  # noqa: E402

N = 7
ARITH = "f32"  # --arith: panel of the plain / dual layers (bf16x6 = the split-bf16 kernels)
SPLIT_IN = False  # --split-in: bf16x6 layers read pre-split operand planes
# name: (Ci, Co, k, stride, H_in, W_in, residual, nchw_in)
LAYERS = {
    "stem": (3, 64, 7, 2, 1080, 1920, False, True),
    "l1.0.ds": (64, 256, 1, 1, 270, 480, False, False),
    "l1.0.c1": (64, 64, 1, 1, 270, 480, False, False),
    "l1.1.c1": (256, 64, 1, 1, 270, 480, False, False),
    "l1.0.c2": (64, 64, 3, 1, 270, 480, False, False),
    "l1.0.c3": (64, 256, 1, 1, 270, 480, True, False),
    "l2.0.ds": (256, 512, 1, 2, 270, 480, False, False),
    "l2.0.c1": (256, 128, 1, 1, 270, 480, False, False),
    "l2.0.c2": (128, 128, 3, 2, 270, 480, False, False),
    "l2.1.c1": (512, 128, 1, 1, 135, 240, False, False),
    "l2.1.c2": (128, 128, 3, 1, 135, 240, False, False),
    "l2.1.c3": (128, 512, 1, 1, 135, 240, True, False),
    "proj": (512, 64, 1, 1, 135, 240, False, False),
    "g512": (512, 512, 1, 1, 135, 240, False, False),  # plain GEMM shape (M 226800 x N 512 x K 512): loop ceiling
    # EfficientNet-B3 pointwise layers at 1080p (stride-2 stem: 540 x 960)
    "b3.p40": (40, 24, 1, 1, 540, 960, False, False),
    "b3.p24": (24, 24, 1, 1, 540, 960, True, False),
    "b3.e24": (24, 144, 1, 1, 540, 960, False, False),
    "b3.p144": (144, 32, 1, 1, 270, 480, False, False),
    "b3.e32": (32, 192, 1, 1, 270, 480, False, False),
    "b3.p192": (192, 32, 1, 1, 270, 480, True, False),
    "b3.e48": (48, 288, 1, 1, 135, 240, False, False),
    "b3.p288": (288, 48, 1, 1, 135, 240, True, False),
}
# fused bottleneck tails (bev_conv2d_dual_f32): name: (Ci conv3 in, Ci2 block in, Co, s2, H2, W2)
DUAL = {
    "l1.0.tail": (64, 64, 256, 1, 270, 480),
    "l2.0.tail": (128, 256, 512, 2, 270, 480),
}


def run_dual(name, iters):
    Ci, Ci2, Co, s2, H2, W2 = DUAL[name]
    Ho, Wo = (H2 - 1) // s2 + 1, (W2 - 1) // s2 + 1
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(N, Ho, Wo, Ci, device=dev, generator=g)
    x = torch.randn(N, H2, W2, Ci2, device=dev, generator=g)
    w = torch.randn(Co, Ci + Ci2, 1, 1, device=dev, generator=g) * (2.0 / (Ci + Ci2)) ** 0.5
    b = torch.randn(Co, device=dev, generator=g)
    packed = nat.pack_conv_weight_x6(w) if ARITH == "bf16x6" else nat.pack_conv_weight(w)
    out = torch.empty(N, Ho, Wo, Co, device=dev)
    for _ in range(3):
        nat.conv2d_dual_nhwc(h, x, s2, packed, b, Co, True, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        nat.conv2d_dual_nhwc(h, x, s2, packed, b, Co, True, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2 * N * Ho * Wo * Co * (Ci + Ci2)
    byts = 4 * (N * H * W * Ci + N * Ho * Wo * Ci2 + out.numel())
    print(f"{name:8s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:6.1f} TF  {byts / ms / 1e6:7.1f} GB/s(io)", flush=True)


# chained bottleneck bodies (bev_conv2d_chain_f32): name: (Ci, Co, Co2, H, W) -- 3x3 Ci->Co, 1x1 Co->Co2 + x
CHAIN = {
    "l1.1.chain": (64, 64, 256, 270, 480),
    "l2.1.chain": (128, 128, 512, 135, 240),
}
# chained block-0 bodies (bev_conv2d_chain_dual_f32): name: (Ci, Co, Co2, H, W, stride, Ci2) -- 3x3 Ci->Co
# (stride), then [h2 | x[::stride]] 1x1 -> Co2; x [N][H][W][Ci2] is the block input
CHAIN_DUAL = {
    "l1.0.chain": (64, 64, 256, 270, 480, 1, 64),
    "l2.0.chain": (128, 128, 512, 270, 480, 2, 256),
}


def run_chain_dual(name, iters):
    Ci, Co, Co2, H, W, s, Ci2 = CHAIN_DUAL[name]
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(N, H, W, Ci, device=dev, generator=g)
    x = torch.randn(N, H, W, Ci2, device=dev, generator=g)
    pk = nat.pack_conv_weight_x6 if ARITH == "bf16x6" else nat.pack_conv_weight
    p1 = pk(torch.randn(Co, Ci, 3, 3, device=dev, generator=g) * (2.0 / (Ci * 9)) ** 0.5)
    p2 = pk(torch.randn(Co2, Co + Ci2, 1, 1, device=dev, generator=g) * (2.0 / (Co + Ci2)) ** 0.5)
    if SPLIT_IN and ARITH == "bf16x6":
        h = nat.split3(h)  # conv1's split output (k_conv_x6s CHAIN)
    b1, b2 = torch.randn(Co, device=dev, generator=g), torch.randn(Co2, device=dev, generator=g)
    out = torch.empty(N, Ho, Wo, Co2, device=dev)
    for _ in range(3):
        nat.conv2d_chain_dual_nhwc(h, p1, b1, Co, 3, 3, s, 1, 1, x, s, p2, b2, Co2, 1, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        nat.conv2d_chain_dual_nhwc(h, p1, b1, Co, 3, 3, s, 1, 1, x, s, p2, b2, Co2, 1, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2 * N * Ho * Wo * (Co * Ci * 9 + Co2 * (Co + Ci2))
    byts = 4 * (N * H * W * Ci + N * Ho * Wo * Ci2 + out.numel())
    print(f"{name:8s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:6.1f} TF  {byts / ms / 1e6:7.1f} GB/s(io)", flush=True)


def run_chain(name, iters):
    Ci, Co, Co2, H, W = CHAIN[name]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(N, H, W, Ci, device=dev, generator=g)
    x = torch.randn(N, H, W, Co2, device=dev, generator=g)
    pk = nat.pack_conv_weight_x6 if ARITH == "bf16x6" else nat.pack_conv_weight
    p1 = pk(torch.randn(Co, Ci, 3, 3, device=dev, generator=g) * (2.0 / (Ci * 9)) ** 0.5)
    p2 = pk(torch.randn(Co2, Co, 1, 1, device=dev, generator=g) * (2.0 / Co) ** 0.5)
    if SPLIT_IN and ARITH == "bf16x6":
        h = nat.split3(h)  # conv1's split output (k_conv_x6s CHAIN)
    b1, b2 = torch.randn(Co, device=dev, generator=g), torch.randn(Co2, device=dev, generator=g)
    out = torch.empty(N, H, W, Co2, device=dev)
    for _ in range(3):
        nat.conv2d_chain_nhwc(h, p1, b1, Co, 3, 3, 1, 1, 1, p2, b2, Co2, 1, residual=x, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        nat.conv2d_chain_nhwc(h, p1, b1, Co, 3, 3, 1, 1, 1, p2, b2, Co2, 1, residual=x, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2 * N * H * W * Co * (Ci * 9 + Co2)
    byts = 4 * (N * H * W * Ci + x.numel() + out.numel())
    print(f"{name:8s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:6.1f} TF  {byts / ms / 1e6:7.1f} GB/s(io)", flush=True)


def run(name, iters):
    Ci, Co, k, s, H, W, res, nchw = LAYERS[name]
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((N, Ci, H, W) if nchw else (N, H, W, Ci), device=dev, generator=g)
    w = torch.randn(Co, Ci, k, k, device=dev, generator=g) * (2.0 / (Ci * k * k)) ** 0.5
    b = torch.randn(Co, device=dev, generator=g)
    r = torch.randn(N, Ho, Wo, Co, device=dev, generator=g) if res else None
    packed = nat.pack_conv_weight_x6(w) if (ARITH == "bf16x6" and not nchw) else nat.pack_conv_weight(w)
    if SPLIT_IN and ARITH == "bf16x6" and not nchw and Ci % 32 == 0:
        x = nat.split3(x)  # pre-split operand planes (k_conv_x6s)
    out = torch.empty(N, Ho, Wo, Co, device=dev)
    for _ in range(3):
        nat.conv2d_nhwc(x, packed, b, Co, k, k, s, p, True, residual=r, in_nchw=nchw, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        nat.conv2d_nhwc(x, packed, b, Co, k, k, s, p, True, residual=r, in_nchw=nchw, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2 * N * Ho * Wo * Co * Ci * k * k
    byts = 4 * (N * H * W * Ci + out.numel() + (r.numel() if res else 0))
    print(f"{name:8s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:6.1f} TF  {byts / ms / 1e6:7.1f} GB/s(io)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("layers", nargs="*", default=[k for k in LAYERS if k != "g512"] + list(DUAL) + list(CHAIN) + list(CHAIN_DUAL))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--knob", default="CONV_TILE", help="bev_tune knob to A/B (TUNE_<name>)")
    ap.add_argument("--values", type=int, nargs="*", default=[0], help="knob values, interleaved per round")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--arith", choices=("f32", "bf16x6"), default="f32")
    ap.add_argument("--split-in", action="store_true")
    a = ap.parse_args()
    global ARITH, SPLIT_IN
    ARITH = a.arith
    SPLIT_IN = a.split_in
    knob = getattr(nat, "TUNE_" + a.knob)
    for rnd in range(a.rounds):  # interleaved rounds, same process
        for v in a.values:
            old = nat.tune(knob, v)
            print(f"-- round {rnd} {a.knob}={v}")
            for name in a.layers:
                (run_dual if name in DUAL else run_chain if name in CHAIN else run_chain_dual if name in CHAIN_DUAL
                 else run)(name, a.iters)
            nat.tune(knob, old)


if __name__ == "__main__":
    main()
