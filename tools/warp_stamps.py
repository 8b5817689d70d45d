"""Per-workgroup phase times of the fused warp (k_warp_fuse_v2) from s_memtime stamps (timing builds with
-DWARP_STAMP=1, tools/warp_ablate.sh with EXTRA=-DWARP_STAMP=1 SUF=s): prologue (corner boxes), first DMA,
view loop, store, per workgroup in shader cycles, on the bench workload (tools/warp_ablate.py's launch).

    python tools/warp_stamps.py 0s 30s
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
import bev_rig  # noqa: E402
from models.fusion.geometry import GeometryTransformer  # noqa: E402
from bench import BOUNDS  # noqa: E402


def main():
    names = sys.argv[1:] or ["0s"]
    dev = torch.device("cuda")
    B, V, C, H, W, Hf, Wf = 2, 7, 64, 1080, 1920, 135, 240
    feats = torch.randn(B, V, Hf, Wf, C, device=dev).permute(0, 1, 4, 2, 3)
    geom = GeometryTransformer(480, 1440, BOUNDS)
    K, Rt = bev_rig.rig(V, H, W, B)
    Hm, xs, ys, hw = geom._sampling(feats, torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev), (H, W))
    sx, sy = nat._scales(Hf, Wf, hw)
    out = torch.empty(B, C, 480, 1440, device=dev)
    s = feats.stride()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ws = torch.empty(nat.lib().bev_ipm_warp_fuse_workspace_bytes(B, V, 480, 1440), device=dev, dtype=torch.uint8)
    args = (nat._ptr(feats), s[1], s[2], s[3], s[4], nat._ptr(Hm), nat._ptr(xs), nat._ptr(ys), B, V, C, Hf, Wf, sx, sy,
            480, 1440, 1, nat._ptr(out), nat._ptr(ws), ws.numel(), st)
    nwg = ((1440 + 15) // 16) * ((480 + 15) // 16) * B
    for name in names:
        L = ctypes.CDLL(os.path.join(REPO, "tools", "_ablate", f"libwarp_ablate_{name}.so"))
        if name.startswith("w"):  # the wave-independent kernel (a separate copy of the library)
            tune = getattr(L, "_ZN3bev9warp_tuneEii")  # bev::warp_tune (bev_warp.hip alone has no bev_tune)
            tune.restype = ctypes.c_int
            tune.argtypes = [ctypes.c_int, ctypes.c_int]
            assert tune(nat.TUNE_WARP_KERNEL, 2) >= 0
        L.bev_ipm_warp_fuse_ws_f32.restype = ctypes.c_int
        L.bev_ipm_warp_fuse_ws_f32.argtypes = nat.SIGNATURES["bev_ipm_warp_fuse_ws_f32"][1]
        for _ in range(5):
            assert L.bev_ipm_warp_fuse_ws_f32(*args) == 0
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (16384 * 6))()
        assert L.bev_warp_stamp_read(buf, 16384 * 6) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(16384, 6)[:nwg, :5].astype(np.int64)
        d = np.diff(a, axis=1)
        life = a[:, 4] - a[:, 0]
        span = a[:, 4].max() - a[:, 0].min()
        print(f"{name}: {nwg} workgroups, span {span} cyc; per workgroup mean cycles: prologue {d[:, 0].mean():.0f}, "
              f"first DMA {d[:, 1].mean():.0f}, view loop {d[:, 2].mean():.0f}, store {d[:, 3].mean():.0f}, "
              f"lifetime {life.mean():.0f} (p10 {np.percentile(life, 10):.0f}, p90 {np.percentile(life, 90):.0f})",
              flush=True)
        # per XCD (linear workgroup id mod 8; one s_memtime clock per XCD): its span, slot utilisation at
        # 3 workgroups x 32 CUs, and when the last quarter / last workgroup started relative to the span
        for x in range(8):
            sel = np.arange(nwg) % 8 == x
            t0, t1 = a[sel, 0].min(), a[sel, 4].max()
            sp = t1 - t0
            starts = np.sort(a[sel, 0] - t0)
            ends = np.sort(a[sel, 4] - t0)
            print(f"  xcd {x}: span {sp} cyc, busy slots {life[sel].sum() / sp:.1f} of 96, "
                  f"start of last wg {starts[-1] / sp:.2f}, end of first wg {ends[0] / sp:.2f}, "
                  f"75% done at {ends[int(0.75 * len(ends))] / sp:.2f}", flush=True)


if __name__ == "__main__":
    main()
