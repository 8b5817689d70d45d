"""Minimal reproducer behind tools/loss_graph_check.py: which torch op of the round-5 (torch-op) focal loss goes wrong
when replayed from a captured HIP graph?  Each case is captured once with torch.cuda.graph (after a warm-up on a
side stream, as make_graphed_callables does) and replayed N times with fresh inputs copied into the static input;
every replay is compared bit for bit with the eager op on the same input.

    python tools/graph_reduce_check.py [--n 691200] [--replays 12]
"""
import argparse

import torch


def focal(logits, gt):
    p = torch.sigmoid(logits).clamp(1e-4, 1 - 1e-4)
    peak = gt == 1.0
    pos = torch.where(peak, p.log() * (1 - p).pow(2.0), torch.zeros_like(p))
    neg = torch.where(gt < 1.0, (1 - p).log() * p.pow(2.0) * (1 - gt).pow(4.0), torch.zeros_like(p))
    return -(pos.sum() + neg.sum()) / peak.sum().float().clamp(min=1.0)


CASES = {
    "sum": lambda x, g: x.sum(),
    "sum2": lambda x, g: x.sum() + (x * 2).sum(),
    "bool_sum": lambda x, g: (g == 1.0).sum().float(),
    "where_sum": lambda x, g: torch.where(g < 1.0, x, torch.zeros_like(x)).sum(),
    "focal": focal,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=691200)
    ap.add_argument("--replays", type=int, default=12)
    ap.add_argument("cases", nargs="*", default=list(CASES))
    a = ap.parse_args()
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(0)
    for name in a.cases:
        fn = CASES[name]
        sx = torch.randn(a.n, device=dev, generator=gen)
        sg = torch.rand(a.n, device=dev, generator=gen)
        sg[:: 997] = 1.0
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn(sx, sg)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = fn(sx, sg)
        bad = []
        for r in range(a.replays):
            x = torch.randn(a.n, device=dev, generator=gen)
            gt = torch.rand(a.n, device=dev, generator=gen)
            gt[r % 7:: 991] = 1.0
            sx.copy_(x)
            sg.copy_(gt)
            g.replay()
            got = out.clone()
            ref = fn(x, gt)
            torch.cuda.synchronize()
            if not torch.equal(got, ref):
                bad.append((r + 1, float(got), float(ref)))
        print(f"{name:10s} n={a.n}: {len(bad)} of {a.replays} replays differ" +
              (f" (first: replay {bad[0][0]} graphed {bad[0][1]:.6g} eager {bad[0][2]:.6g})" if bad else ""),
              flush=True)
        del g


if __name__ == "__main__":
    main()
