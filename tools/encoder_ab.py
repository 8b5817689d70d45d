"""Interleaved A/B of ResNet-50 encoder plan switches on the bench workload (7 cams x 1080p x 2 frames, eval).

    python tools/encoder_ab.py base nosplitchain splitedges --iters 10 --rounds 3

Each variant sets module / trunk attributes, then times CNNEncoder.forward with HIP events on the caller's stream;
variants alternate inside one process (same clocks, same caches: cdna_hip_programming.md §5.4 rule 24).  Prints one
line per (round, variant) and the median per variant, and checks that every variant's output equals the first's.
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
from models.encoders import resnet  # noqa: E402
from models.encoders.cnn_encoder import CNNEncoder  # noqa: E402


def apply(name, rn):
    if hasattr(rn, "x6_expand"):  # EfficientNet (--backbone efficientnet_b3): base / x6expand / nostem3
        if name not in ("base", "x6expand", "nostem3", "nopwstream", "noirfuse"):
            raise SystemExit(f"unknown EfficientNet variant {name}")
        rn.ir_fuse = name != "noirfuse"
        rn.x6_expand = name == "x6expand"
        rn.stem3 = name != "nostem3"
        rn.pw_stream = name != "nopwstream"
        return
    resnet.SPLIT_CHAIN = True
    resnet.FUSE_NEXT_CONV1 = False
    rn.split_edges = False
    if name == "nosplitchain":
        resnet.SPLIT_CHAIN = False
    elif name == "fuse":
        resnet.FUSE_NEXT_CONV1 = True
    elif name == "splitedges":
        rn.split_edges = True
    elif name != "base":
        raise SystemExit(f"unknown variant {name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", default=["base", "nosplitchain"])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--backbone", default="resnet50")
    ap.add_argument("--stream-groups", type=int, default=2, help="1: launches attributable per layer (profiling)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    enc = CNNEncoder(out_channels=64, backbone=a.backbone, pretrained=False).eval().to(dev)
    imgs = torch.randn(a.frames, 7, 3, 1080, 1920, device=dev)
    rn = enc.backbone
    if hasattr(rn, "stream_groups"):
        rn.stream_groups = a.stream_groups
    res = {n: [] for n in a.variants}
    first = None
    with torch.no_grad():
        for rnd in range(a.rounds):
            for name in a.variants:
                apply(name, rn)
                out = enc(imgs)  # warm-up (and the repack after a plan change)
                torch.cuda.synchronize()
                if first is None:
                    first = out.clone()
                elif not torch.equal(out, first):
                    print(f"MISMATCH: {name} differs from {a.variants[0]}", flush=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    enc(imgs)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                res[name].append(ms)
                print(f"round {rnd} {name:14s} {ms:8.3f} ms/step", flush=True)
    for n, v in res.items():
        print(f"median {n:14s} {statistics.median(v):8.3f} ms  min {min(v):8.3f}", flush=True)


if __name__ == "__main__":
    main()
