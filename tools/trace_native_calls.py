"""List the library entry points one AMP BEVNet training step calls (tools/train_step_bench.py --bevnet --amp shape),
with their integer arguments -- to attribute a kernel of a rocprofv3 trace (e.g. an exact-f32 k_conv inside the AMP
step) to the layer that launches it.

    python tools/trace_native_calls.py [--filter conv] [--steps 1]
"""
import argparse
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
import bev_rig  # noqa: E402
import models.model_wrapper as mw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="conv")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--stack", action="store_true", help="print the Python caller of every call")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    V, H, W = 7, 1080, 1920
    K, Rt = bev_rig.rig(V, H, W, 1)
    torch.manual_seed(0)
    cfg = {"MODEL": {"BACKBONE": "resnet50", "PRETRAINED": False, "FEAT_DIM": 64, "OUT_INDEX": 2,
                     "BEV_SIZE": [32, 480, 1440], "BEV_BOUNDS": [-24.0, 24.0, -7.2, 7.2], "BEV_PROJ_CH": 128},
           "LOSS": {}, "EVAL": {"CONF_THRESH": 0.99}}
    model = mw.BEVNet(cfg).to(dev)
    batch = {"images": torch.randn(1, V, 3, H, W, device=dev),
             "calib": {"intrinsic": torch.from_numpy(K).to(dev), "extrinsic": torch.from_numpy(Rt).to(dev)}}
    targets = [{"boxes_world": torch.tensor([[1.0, 0.5, 0.6, 0.6], [-3.0, 2.0, 0.6, 0.6]])}]
    with torch.no_grad():
        model.eval()(batch)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    scaler = torch.amp.GradScaler("cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            preds = model(batch)
            ls = model.loss(preds, targets, {})
        scaler.scale(ls["total_loss"]).backward()
        scaler.step(opt)
        scaler.update()

    step()  # warm-up (packs, lazy modules)
    L = nat.lib()
    calls = collections.Counter()
    orig = {}
    for name in nat.SIGNATURES:
        if a.filter not in name:
            continue
        fn = getattr(L, name)
        orig[name] = fn

        def wrap(*args, _n=name, _f=fn):
            ints = tuple(x for x in args if isinstance(x, int) and abs(x) < 2 ** 31)  # not the pointers
            where = ""
            if a.stack:
                fr = [f for f in traceback.extract_stack()[:-1] if "bev_native" not in f.filename]
                where = " <- " + " / ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:])
            calls[(_n, ints, where)] += 1
            return _f(*args)
        setattr(L, name, wrap)
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    for (n, ints, where), c in sorted(calls.items()):
        print(f"{c:3d} x {n}{ints}{where}")


if __name__ == "__main__":
    main()
