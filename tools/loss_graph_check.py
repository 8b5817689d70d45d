"""Diagnostic: the AMP BEVNet training step of tools/train_step_bench.py with the graphed loss, each step's losses
compared with the eager loss terms on the same predictions (and the same targets), printed per step.
Needs the graphed loss (models.model_wrapper.LOSS_GRAPHS) of commit 69d574d, removed after this check found wrong
replays (profiles/r05ar_loss_graph_check.txt); kept as the reproducer for that investigation."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vision-based-spatio-temporal-analysis_amd"))
import bev_native  # noqa: E402,F401
import bev_rig  # noqa: E402
import models.model_wrapper as mw  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    V, H, W = 7, 1080, 1920
    K, Rt = bev_rig.rig(V, H, W, 1)
    Kd, Rtd = torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev)
    torch.manual_seed(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
    images = torch.randn(1, V, 3, H, W, device=dev)
    cfg = {"MODEL": {"BACKBONE": "resnet50", "PRETRAINED": False, "FEAT_DIM": 64, "OUT_INDEX": 2,
                     "BEV_SIZE": [32, 480, 1440], "BEV_BOUNDS": [-24.0, 24.0, -7.2, 7.2], "BEV_PROJ_CH": 128},
           "LOSS": {}, "EVAL": {"CONF_THRESH": 0.99}}
    model = mw.BEVNet(cfg).to(dev)
    batch = {"images": images, "calib": {"intrinsic": Kd, "extrinsic": Rtd}}
    targets = [{"boxes_world": torch.tensor([[1.0, 0.5, 0.6, 0.6], [-3.0, 2.0, 0.6, 0.6]])}]
    with torch.no_grad():
        model.eval()(batch)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    scaler = torch.amp.GradScaler("cuda")
    for it in range(8):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            preds = model(batch)
            ls = model.loss(preds, targets, {})
        scaler.scale(ls["total_loss"]).backward()
        scaler.step(opt)
        scaler.update()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        with torch.no_grad():
            mw.LOSS_GRAPHS = False
            ref = model.loss({k: v.detach() for k, v in preds.items() if isinstance(v, torch.Tensor)}, targets, {})
            mw.LOSS_GRAPHS = True
        vals = {k: (float(ls[k]), float(ref[k])) for k in ls}
        bad = [k for k, (a, b) in vals.items() if a != b]
        print(f"step {it} {dt * 1e3:7.1f} ms scale {scaler.get_scale():.0f} graphs {len(model.__dict__.get('_loss_graphs', {}))} "
              + " ".join(f"{k}={a:.6g}/{b:.6g}" for k, (a, b) in vals.items()) + (f"  MISMATCH {bad}" if bad else ""),
              flush=True)


if __name__ == "__main__":
    main()
