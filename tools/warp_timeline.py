"""Timeline of the fused warp (k_warp_fuse_v2) from s_memtime stamps (timing builds with -DWARP_STAMP=1, e.g.
EXTRA=-DWARP_STAMP=1 SUF=s bash tools/warp_ablate.sh 0): per workgroup its phases, per live view (the first six) the
time from taps to the end of the LDS sampling (compute) and from there to the end-of-view barrier (wait for the
next view's LDS-DMA and the other waves), and per CU (HW_ID / XCC_ID) how many workgroups were resident over the
launch and the idle gaps between one workgroup's end and the next one's start.  Bench workload (7 cams, C = 64,
135 x 240 -> 480 x 1440, mean, batch 2).

    python tools/warp_timeline.py s
"""
import collections
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

N = 24


def main():
    names = sys.argv[1:] or ["s"]
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
    nwg = 2700 * B
    for name in names:
        L = ctypes.CDLL(os.path.join(REPO, "tools", "_ablate", f"libwarp_ablate_{name}.so"))
        L.bev_ipm_warp_fuse_ws_f32.restype = ctypes.c_int
        L.bev_ipm_warp_fuse_ws_f32.argtypes = nat.SIGNATURES["bev_ipm_warp_fuse_ws_f32"][1]
        for _ in range(8):
            assert L.bev_ipm_warp_fuse_ws_f32(*args) == 0
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (16384 * N))()
        assert L.bev_warp_stamp_read(buf, 16384 * N) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(16384, N)[:nwg].astype(np.int64)
        t0 = a[:, 0].min()
        st_, en = a[:, 0] - t0, a[:, 4] - t0
        d = np.diff(a[:, :5], axis=1)
        print(f"{name}: span {en.max()} cyc, workgroup life mean {np.mean(en - st_):.0f} "
              f"(prologue {d[:, 0].mean():.0f}, first DMA {d[:, 1].mean():.0f}, views {d[:, 2].mean():.0f}, "
              f"store {d[:, 3].mean():.0f})")
        for v in range(6):
            tv = a[:, 6 + 3 * v: 9 + 3 * v]
            ok = (tv[:, 0] > 0) & (tv[:, 1] >= tv[:, 0]) & (tv[:, 2] >= tv[:, 1])
            if ok.sum() == 0:
                continue
            comp = (tv[ok, 1] - tv[ok, 0]).mean()
            wait = (tv[ok, 2] - tv[ok, 1]).mean()
            print(f"  live view {v}: {ok.sum():5d} workgroups, taps->sampled {comp:6.0f} cyc, sampled->barrier "
                  f"{wait:6.0f} cyc")
        hw = a[:, 5]
        hwid, xcc = hw & 0xffffffff, (hw >> 32) & 0xf
        cu = (xcc << 8) | ((hwid >> 8) & 0xff)  # xcc, se, sh, cu
        per = collections.defaultdict(list)
        for k in range(nwg):
            per[int(cu[k])].append((int(st_[k]), int(en[k])))
        conc, gaps, counts = [], [], []
        for key, lst in per.items():
            lst.sort()
            counts.append(len(lst))
            ev = sorted([(x, 1) for x, _ in lst] + [(y, -1) for _, y in lst])
            cur, last, area = 0, ev[0][0], 0
            for t, dlt in ev:
                area += cur * (t - last)
                cur += dlt
                last = t
            conc.append(area / max(1, ev[-1][0] - ev[0][0]))
            ends = sorted(y for _, y in lst)
            starts = sorted(x for x, _ in lst)
            for x in starts[3:]:  # a start after the first three: the slot freed by the latest end before it
                prev = [y for y in ends if y <= x]
                if prev:
                    gaps.append(x - prev[-1])
        print(f"  CUs seen {len(per)}, workgroups per CU {np.mean(counts):.1f} (min {min(counts)}, max {max(counts)}), "
              f"mean resident workgroups {np.mean(conc):.2f}, start-after-free gap mean {np.mean(gaps):.0f} cyc, "
              f"CU busy-span mean {np.mean([max(y for _, y in l) - min(x for x, _ in l) for l in per.values()]):.0f}")


if __name__ == "__main__":
    main()
