"""Time the fused warp with parts of its work removed (tools/warp_ablate.sh variants; WARP_ABLATE bits in
bev_warp.hip: 1 no mean division, 2 no staging, 4 no LDS sampling, 8 no tap arithmetic, 16 no stores) on the
bench workload (7 cams, C = 64 channels-last, 135 x 240 features -> 480 x 1440, mean, batch 2).  Results of
the variants are wrong by construction; only their launch times are read.

    python tools/warp_ablate.py 0 1 2 4 8 16
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bev_native as nat  # noqa: E402
import bev_rig  # noqa: E402
from models.fusion.geometry import GeometryTransformer  # noqa: E402
from bench import BOUNDS  # noqa: E402


def main():
    bits = sys.argv[1:] or ["0"]
    dev = torch.device("cuda")
    B, V, C, H, W, Hf, Wf = 2, 7, 64, 1080, 1920, 135, 240
    if os.environ.get("GEOM") == "k5":  # BASELINE configs[4]: 16 cameras at 4K, one frame, SUM (the per-rank partial)
        B, V, H, W, Hf, Wf = 1, 16, 2160, 3840, 270, 480
    feats = torch.randn(B, V, Hf, Wf, C, device=dev).permute(0, 1, 4, 2, 3)
    geom = GeometryTransformer(480, 1440, BOUNDS)
    K, Rt = bev_rig.rig(V, H, W, B)
    Hm, xs, ys, hw = geom._sampling(feats, torch.from_numpy(K).to(dev), torch.from_numpy(Rt).to(dev), (H, W))
    sx, sy = nat._scales(Hf, Wf, hw)
    out = torch.empty(B, C, 480, 1440, device=dev)
    s = feats.stride()
    # a trailing "n" times the same library without the workspace (the in-kernel corner-box prologue)
    libs = {b: ctypes.CDLL(os.path.join(REPO, "tools", "_ablate", f"libwarp_ablate_{(b.rstrip('n') or b).split('_p')[0]}.so"))
            for b in bits}  # "p0" / "w0": copies of libwarp_ablate_0.so built as p0 / w0 (their own knob state)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ws = torch.empty(nat.lib().bev_ipm_warp_fuse_workspace_bytes(B, V, 480, 1440), device=dev, dtype=torch.uint8)
    args = (nat._ptr(feats), s[1], s[2], s[3], s[4], nat._ptr(Hm), nat._ptr(xs), nat._ptr(ys), B, V, C, Hf, Wf, sx, sy,
            480, 1440, 0 if os.environ.get("GEOM") == "k5" else 1, nat._ptr(out), nat._ptr(ws), ws.numel(), st)
    for L in libs.values():
        L.bev_ipm_warp_fuse_ws_f32.restype = ctypes.c_int
        L.bev_ipm_warp_fuse_ws_f32.argtypes = nat.SIGNATURES["bev_ipm_warp_fuse_ws_f32"][1]
    args_n = args[:-3] + (None, 0, st)
    # a leading "w" times the wave-independent kernel (bev_tune(BEV_TUNE_WARP_KERNEL, 2)); libwarp_ablate_w<b>.so
    # must be a separate copy of the library (its own knob state)
    for b, L in libs.items():
        if b.startswith("w") or b.startswith("p"):  # "p": the persistent kernel (BEV_TUNE_WARP_KERNEL 3)
            tune = getattr(L, "_ZN3bev9warp_tuneEii")  # bev::warp_tune (bev_warp.hip alone has no bev_tune)
            tune.restype = ctypes.c_int
            tune.argtypes = [ctypes.c_int, ctypes.c_int]
            assert tune(nat.TUNE_WARP_KERNEL, 2 if b.startswith("w") else 3) >= 0
    pool_kb = os.environ.get("POOL_KB")  # a variant name containing "_p<KB>" sets that LDS pool (BEV_TUNE_WARP_POOL_KB)
    for b, L in libs.items():
        if "_p" in b:
            tune = getattr(L, "_ZN3bev9warp_tuneEii")
            tune.restype = ctypes.c_int
            tune.argtypes = [ctypes.c_int, ctypes.c_int]
            assert tune(nat.TUNE_WARP_POOL_KB, int(b.split("_p")[1].split("_")[0])) >= 0
    del pool_kb
    for rnd in range(int(os.environ.get("ROUNDS", "5"))):
        for b, L in libs.items():
            a = args_n if b.endswith("n") else args
            for _ in range(3):
                assert L.bev_ipm_warp_fuse_ws_f32(*a) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            n = 30
            for _ in range(n):
                L.bev_ipm_warp_fuse_ws_f32(*a)
            e1.record()
            torch.cuda.synchronize()
            print(f"round {rnd} variant {b:>6}: {e0.elapsed_time(e1) / n * 1e3:8.1f} us per launch", flush=True)
    check_exact(libs, args, out)


def check_exact(libs, args, out):
    """Variants without ablation bits ("0" + build suffixes) must produce the baseline's output bit for bit."""
    ref = None
    for b, L in libs.items():
        if b.lstrip("wp").rstrip("nsw") not in ("0", ""):
            continue
        out.zero_()
        assert L.bev_ipm_warp_fuse_ws_f32(*args) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        else:
            print(f"variant {b}: bit-identical to the first exact variant: {torch.equal(out, ref)}", flush=True)


if __name__ == "__main__":
    main()
