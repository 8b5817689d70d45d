"""A/B of the ResNet-50 trunk execution plans on the bench workload (7 cams x 1080p x 2 frames, eval, no_grad).

    python tools/trunk_ab.py --iters 10 --rounds 2

Variants are interleaved in one process (same clocks, same caches): the conv arithmetic (f32 = exact-f32 MFMA kernels
and chains, bf16x6 = split-bf16 kernels), the stages that keep the exact-f32 chained bottleneck kernels under
bf16x6, and pre-split conv1 -> conv2 operands.  Prints ms per step (HIP events around CNNEncoder.forward).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
from models.encoders.cnn_encoder import CNNEncoder  # noqa: E402

# name: (arith, stages on the exact-f32 chains, stages on the split-arithmetic chains, pre-split conv1 -> conv2)
VARIANTS = {
    "f32": ("f32", set(), set(), False),
    "x6": ("bf16x6", set(), set(), False),
    "x6+f32chain1": ("bf16x6", {1}, set(), False),
    "x6+x6chain1": ("bf16x6", set(), {1}, False),
    "x6+x6chain12": ("bf16x6", set(), {1, 2}, False),
    "x6+split": ("bf16x6", set(), set(), True),
}
# stream-group variants of the default plan: "sg<G>"; split-kernel choice: "k<knob>" (BEV_TUNE_CONV_X6_KERNEL)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", default=list(VARIANTS))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--frames", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(dev)
    imgs = torch.randn(a.frames, 7, 3, 1080, 1920, device=dev)
    rn = enc.backbone
    with torch.no_grad():
        for rnd in range(a.rounds):
            for name in a.variants:
                knob = int(name[1:]) if name.startswith("k") else 0
                nat.tune(nat.TUNE_CONV_X6_KERNEL, knob)
                if name.startswith("k"):
                    arith, stages, stages6, split = VARIANTS["x6+x6chain1"]
                    rn.stream_groups = 2
                elif name.startswith("sg"):
                    arith, stages, stages6, split = VARIANTS["x6+x6chain1"]
                    rn.stream_groups = int(name[2:])
                else:
                    arith, stages, stages6, split = VARIANTS[name]
                    rn.stream_groups = 2
                rn.f32_chain_stages, rn.x6_chain_stages, rn.split_edges = stages, stages6, split
                with nat.conv_arith_mode(arith):
                    for _ in range(3):
                        enc(imgs)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        enc(imgs)
                    e1.record()
                    torch.cuda.synchronize()
                print(f"round {rnd} {name:16s} {e0.elapsed_time(e1) / a.iters:8.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
