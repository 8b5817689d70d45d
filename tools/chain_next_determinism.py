"""Repeatability of bev_conv2d_chain_next_x6_f32 (and the plain pre-split chain) at the bench's layer1 size
(14 images x 270 x 480): every repeat's y / h3 must equal the first bit for bit.  Reports where a difference sits
(row within the 128-row tile, channel) to locate a race.

    python tools/chain_next_determinism.py [--repeats 4] [--n 14]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))

import torch  # noqa: E402

import bev_native as nat  # noqa: E402


def where(a, b, Co):
    d = (a != b).reshape(-1, Co)
    rows = d.any(1).nonzero().flatten()
    chans = d.any(0).nonzero().flatten()
    tile_rows = torch.unique(rows % 128)
    return (f"{int(d.sum())} values, {rows.numel()} pixels (first {rows[:4].tolist()}, tiles "
            f"{torch.unique(rows // 128)[:6].tolist()}), rows-in-tile {tile_rows[:12].tolist()}"
            f"{'...' if tile_rows.numel() > 12 else ''} ({tile_rows.numel()}), channels {chans[:12].tolist()}"
            f"{'...' if chans.numel() > 12 else ''} ({chans.numel()})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=4)
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--h", type=int, default=270)
    ap.add_argument("--w", type=int, default=480)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    N, H, W, Ci, Co, Co2 = a.n, a.h, a.w, 64, 64, 256
    x = torch.randn(N, H, W, Ci, generator=g).to(dev)
    xs = nat.split3(x)
    res = torch.randn(N, H, W, Co2, generator=g).to(dev)
    xb = torch.randn(N, H, W, 64, generator=g).to(dev)
    w2 = (torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5).to(dev)
    p2 = nat.pack_conv_weight_x6(w2)
    b2 = (torch.randn(Co, generator=g) * 0.1).to(dev)
    b3 = (torch.randn(Co2, generator=g) * 0.1).to(dev)
    cases = []
    for dual in (False, True):
        w3 = (torch.randn(Co2, Co + (64 if dual else 0), 1, 1, generator=g) / Co ** 0.5).to(dev)
        p3 = nat.pack_conv_weight_x6(w3)
        for Co3, split in ((0, True), (64, True), (128, False), (128, True)):
            if dual and Co3 > 0:  # refused by the library since r06o (its kernel was not repeatable)
                continue
            wn = (torch.randn(max(Co3, 64), Co2, 1, 1, generator=g) / Co2 ** 0.5).to(dev)
            pn, bn = nat.pack_conv_weight_x6(wn), (torch.randn(max(Co3, 64), generator=g) * 0.1).to(dev)

            def run(dual=dual, Co3=Co3, split=split, p3=p3, pn=pn, bn=bn):
                if Co3 == 0:
                    if dual:
                        return nat.conv2d_chain_dual_nhwc(xs, p2, b2, Co, 3, 3, 1, 1, 1, xb, 1, p3, b3, Co2, 1), None
                    return nat.conv2d_chain_nhwc(xs, p2, b2, Co, 3, 3, 1, 1, 1, p3, b3, Co2, 1, residual=res), None
                kw = dict(x2=xb) if dual else dict(residual=res)
                y, h3 = nat.conv2d_chain_next_nhwc(xs, p2, b2, Co, 3, 3, 1, 1, 1, p3, b3, Co2, 1, pn, bn, Co3, 1,
                                                   split3_out=split, **kw)
                return y, (h3.planes if split else h3)
            cases.append((f"{'dual' if dual else 'chain'} Co3={Co3} {'split' if split else 'fp32'}", run, Co3))
    with torch.no_grad():
        for name, run, Co3 in cases:
            y0, h0 = run()
            y0 = y0.clone()
            h0 = h0.clone() if h0 is not None else None
            bad = 0
            for r in range(1, a.repeats):
                y, h = run()
                torch.cuda.synchronize()
                ok = torch.equal(y, y0) and (h is None or torch.equal(h, h0))
                if not ok:
                    bad += 1
                    if not torch.equal(y, y0):
                        print(f"  {name} repeat {r}: y {where(y, y0, Co2)}", flush=True)
                    if h is not None and not torch.equal(h, h0):
                        print(f"  {name} repeat {r}: h3 {where(h, h0, Co3)}", flush=True)
            print(f"{name:22s}: {bad} of {a.repeats - 1} repeats differ", flush=True)


if __name__ == "__main__":
    main()
