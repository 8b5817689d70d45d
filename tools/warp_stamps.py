"""Per-wave phase cycles of the fused-warp pipeline kernel (k_warp_fuse_pc), from the profiling
build libbev_mi355x_stamps.so (`make -C vision-based-spatio-temporal-analysis_amd stamps`).

Runs the benchmark workload's fused warp (7 cams, C=64 channels-last, 480x1440, Appendix-B rig) once
after warm-up and prints, for the loader waves and the sampler waves, the mean / p50 / p90 over
workgroups of each phase (s_memtime cycles).  Usage: python tools/warp_stamps.py [--wgs 2|3] [--pool KB]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd")
sys.path.insert(0, PKG)

import bev_native as nat  # noqa: E402

LOADER = ["total", "corner boxes", "reserve (ring wait)", "DMA issue", "publish waits", "exact boxes", "images",
          "items"]
SAMPLER = ["total", "poll (desc wait)", "taps", "LDS sampling", "stores", "descs", "-", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wgs", type=int, default=2)
    ap.add_argument("--pool", type=int, default=0)
    ap.add_argument("--views", type=int, default=7)
    ap.add_argument("--img", type=int, nargs=2, default=(1080, 1920))
    ap.add_argument("--lib", default="libbev_mi355x_stamps.so", help="stamps build (…_nostore: store ablation)")
    args = ap.parse_args()
    nat.LIB_PATH = os.path.join(PKG, args.lib)
    L = nat.lib()
    L.bev_pc_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    import bev_rig
    from models.fusion.geometry import GeometryTransformer
    dev = torch.device("cuda:0")
    V = args.views
    H, W = args.img
    Hf, Wf = H // 8, W // 8
    g = GeometryTransformer(480, 1440, (-24.0, 24.0, -7.2, 7.2))
    K, Rt = bev_rig.rig(V, H, W, 1)
    Kd, Rtd = torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev)
    f = torch.randn(1, V, Hf, Wf, 64, device=dev).permute(0, 1, 4, 2, 3)
    nat.tune(nat.TUNE_WARP_KERNEL, nat.WARP_KERNEL_PIPELINE)
    nat.tune(nat.TUNE_WARP_WGS, args.wgs)
    nat.tune(nat.TUNE_WARP_POOL_KB, args.pool)
    for _ in range(5):
        g.forward_fused(f, Kd, Rtd, (H, W), "mean")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.forward_fused(f, Kd, Rtd, (H, W), "mean")
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 5 * 8, np.int64)
    rc = L.bev_pc_stamps(buf.ctypes.data, buf.nbytes)
    assert rc == 0, rc
    st = buf.reshape(4096, 5, 8)
    nwg = 256 * args.wgs
    st = st[:nwg]
    print(f"kernel+homography span {e0.elapsed_time(e1) * 1e3:.1f} us, {nwg} workgroups")
    for name, rows, labels in (("loader", st[:, 4, :], LOADER), ("samplers", st[:, :4, :].reshape(-1, 8), SAMPLER)):
        print(f"== {name}")
        for q, lab in enumerate(labels):
            if lab == "-":
                continue
            col = rows[:, q].astype(np.float64)
            print(f"  {lab:22s} mean {col.mean():10.0f}  p50 {np.percentile(col, 50):10.0f}  "
                  f"p90 {np.percentile(col, 90):10.0f}  max {col.max():10.0f}")


if __name__ == "__main__":
    main()
