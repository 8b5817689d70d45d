"""Diagnostic for the graphed-loss failure of round 5 (profiles/r05ar_loss_graph_check.txt: BEVNet.loss replayed as a
captured graph pair returned a focal loss of -375 from the fifth replay on).  The graphed loss was removed from the
model (commit af958c9); this tool rebuilds it OUTSIDE the model with torch.cuda.make_graphed_callables over the
model's own target construction + loss terms, runs the AMP BEVNet training step of tools/train_step_bench.py, and
compares every replay with the eager loss on the same predictions.

    python tools/loss_graph_check.py [--variant full|terms|targets] [--steps 10] [--sync] [--no-amp] [--no-opt]

  full     targets + loss terms captured together (what 69d574d shipped)
  terms    targets eager, the loss terms captured
  --sync   torch.cuda.synchronize() after every step (timing hazards)
  --no-opt no optimizer step (parameters frozen: the same predictions every step)
  --torch-loss  the focal / L1 losses and the gaussian radius as torch ops, as in round 5's graphed loss
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "vision-based-spatio-temporal-analysis_amd"))
import bev_native  # noqa: E402,F401
import bev_rig  # noqa: E402
import models.model_wrapper as mw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="full", choices=("full", "terms"))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--sync", action="store_true")
    ap.add_argument("--no-amp", action="store_true")
    ap.add_argument("--no-opt", action="store_true")
    ap.add_argument("--bev", type=int, nargs=2, default=(480, 1440))
    ap.add_argument("--torch-loss", action="store_true", help="the loss terms / radius as torch ops (round 5's graph)")
    a = ap.parse_args()
    if a.torch_loss:
        mw.NATIVE_LOSS = False
    dev = torch.device("cuda:0")
    V, H, W = 7, 1080, 1920
    K, Rt = bev_rig.rig(V, H, W, 1)
    Kd, Rtd = torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev)
    torch.manual_seed(a.seed)
    images = torch.randn(1, V, 3, H, W, device=dev)
    cfg = {"MODEL": {"BACKBONE": "resnet50", "PRETRAINED": False, "FEAT_DIM": 64, "OUT_INDEX": 2,
                     "BEV_SIZE": [32, a.bev[0], a.bev[1]], "BEV_BOUNDS": [-24.0, 24.0, -7.2, 7.2], "BEV_PROJ_CH": 128},
           "LOSS": {}, "EVAL": {"CONF_THRESH": 0.99}}
    model = mw.BEVNet(cfg).to(dev)
    batch = {"images": images, "calib": {"intrinsic": Kd, "extrinsic": Rtd}}
    targets = [{"boxes_world": torch.tensor([[1.0, 0.5, 0.6, 0.6], [-3.0, 2.0, 0.6, 0.6]])}]
    with torch.no_grad():
        model.eval()(batch)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    scaler = torch.amp.GradScaler("cuda", enabled=not a.no_amp)
    B = len(targets)
    graphed = None

    def loss_full(logits, offset, size_raw, boxes, frame, bound):
        t = model._targets_from_boxes(boxes, frame, bound, B)
        return model._loss_terms(logits, offset, size_raw, t["heatmap"], t["indices"], t["mask"], t["offset"],
                                 t["size_log"])

    for it in range(a.steps):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16, enabled=not a.no_amp):
            preds = model(batch)
        pr = (preds["heatmap_logits"], preds["offset"], preds["size_raw"])
        boxes, frame, bound = model._target_boxes(targets, dev)
        if a.variant == "full":
            args = pr + (boxes, frame)
            fn = lambda *x: loss_full(*x, bound=bound)  # noqa: E731
        else:
            tg = model._targets_from_boxes(boxes, frame, bound, B)
            args = pr + (tg["heatmap"], tg["indices"], tg["mask"], tg["offset"], tg["size_log"])
            fn = model._loss_terms
        if graphed is None:
            samples = tuple(x.detach().clone().requires_grad_(x.requires_grad) for x in args)
            with torch.autocast("cuda", enabled=False):
                graphed = torch.cuda.make_graphed_callables(fn, samples, allow_unused_input=True)
        outs = graphed(*args)
        ls = torch.stack(outs)
        scaler.scale(ls[3]).backward()
        if not a.no_opt:
            scaler.step(opt)
            scaler.update()
        if a.sync:
            torch.cuda.synchronize()
        with torch.no_grad():
            ref = torch.stack(fn(*[x.detach() for x in args]))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        g, r = ls.detach().cpu().tolist(), ref.cpu().tolist()
        bad = [i for i in range(4) if g[i] != r[i]]
        print(f"step {it} {dt * 1e3:7.1f} ms scale {scaler.get_scale():.0f} graphed {[f'{x:.6g}' for x in g]} "
              f"eager {[f'{x:.6g}' for x in r]}" + (f"  MISMATCH {bad}" if bad else ""), flush=True)


if __name__ == "__main__":
    main()
