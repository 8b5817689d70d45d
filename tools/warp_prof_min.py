"""Minimal fused-warp workload for counter passes: the bench geometry (7 cams, 1080p / 8 features, 480 x 1440 BEV,
B = 2, C = 64, channels-last maps), N forward calls (default kernel) and N fused-mean backward calls.  (GPU box)
    python tools/warp_prof_min.py [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
import torch  # noqa: E402

import bev_native as nat  # noqa: E402
import bev_rig  # noqa: E402
from models.fusion.geometry import GeometryTransformer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B, V, C, H, W = 2, 7, 64, 1080, 1920
Hf, Wf = H // 8, W // 8
dev = torch.device("cuda:0")
geom = GeometryTransformer(480, 1440, (-24.0, 24.0, -7.2, 7.2))
K, Rt = bev_rig.rig(V, H, W, B)
Hm = geom.homographies(torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev), B, V, dev)
xs, ys = geom._device_axes(dev)
feats = torch.randn(B, V, Hf, Wf, C, device=dev).permute(0, 1, 4, 2, 3)
gout = torch.randn(B, C, ys.numel(), xs.numel(), device=dev)
for _ in range(n):
    nat.warp_fuse(feats, Hm, xs, ys, (H, W), "mean")
for _ in range(n):
    nat.warp_fuse_bwd(gout, Hm, xs, ys, V, Hf, Wf, (H, W), "mean")
torch.cuda.synchronize()
print("done", flush=True)
