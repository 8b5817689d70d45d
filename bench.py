"""Benchmark: multi-cam frames/sec (7-cam -> 480x1440 BEV) on MI355X.

Workload = BASELINE.json configs[1] (default): Wildtrack-shaped 7 cameras x 3 x
1080 x 1920 fp32 images -> ResNet-50 (timm features_only, out_index=2, stride
8) -> 1x1 proj to C=64 -> IPM warp onto the 480x1440 ground grid -> mean
fusion over views.  One step = one batch of B frames through that whole hot
path (CNNEncoder.forward + GeometryTransformer.forward_fused); B = 2 by default,
the reference's own Wildtrack inference batch (inference.py:27 builds its
DataLoader with cfg['DATA']['BATCH_SIZE'], configs/wildtrack.yaml:2 = 2); inputs resident
in HBM, random-init weights of that architecture, synthetic images, the fixed
Appendix-B camera rig.

Other BASELINE configs (each its own JSON line, never the default):
  --backbone efficientnet_b3   configs[3]: EfficientNet-B3 + AttentionFusion, which in the
                               reference is the mean placeholder (fusion.py:25-36, quirk Q8)
  --camera-shard               configs[4]: 16 cameras at 4K (2160 x 3840 -> 270 x 480
                               features), cameras sharded over the ranks (2 per GPU at 8
                               GPUs): each rank runs the trunk + the fused warp (SUM) on its
                               cameras, then ONE reduce-scatter over BEV rows (RCCL/xGMI)
                               and the division by 16 (bev_dist.camera_sharded_forward).
                               Total work per frame is fixed: strong scaling.

Multi-GPU, one process per GPU: `python bench.py --gpus N` starts N rank processes
itself (torch.distributed.run on 127.0.0.1, before this process touches the GPU);
under an external torchrun, WORLD_SIZE must equal --gpus.  Frame-sharded configs
run B frames per rank with no data-path collective (weak scaling); only the timing
barrier and a MAX-reduction of the elapsed time cross ranks.  `n_gpus` is the world
size of the initialised process group.

Prints ONE JSON line on rank 0 (contract in the task statement), with a
`roofline` object for the dominant kernel family (backbone convs; by default in
the split-bf16 fp32 arithmetic, --conv-arith f32 for the exact-f32 MFMA kernels), `roofline_warp` for the IPM warp kernel (HBM-bound), and, at N = 1, a
`cpu_baseline` (the reference's torch-CPU composition, timed on this host on
a bounded sample).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

BOUNDS = (-24.0, 24.0, -7.2, 7.2)
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_F32_MFMA_TF = 157.3  # MI355X fp32 matrix spec (= vector peak)
PEAK_BF16_MFMA_TF = 2500.0  # MI355X bf16 matrix, dense (MI355X_MICROARCH.md)
# the split arithmetic spends 6 bf16 partial products per fp32 product: its fp32-equivalent dense peak
PEAK_X6_TF = PEAK_BF16_MFMA_TF / 6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (rank processes) of this node; default 1")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=2, help="frames per GPU per step (frame-sharded configs); default 2 = "
                    "the reference's Wildtrack inference batch (inference.py:27 DataLoader(batch_size=cfg['DATA']"
                    "['BATCH_SIZE']), configs/wildtrack.yaml:2 BATCH_SIZE: 2)")
    ap.add_argument("--views", type=int, default=None, help="cameras (default 7; 16 with --camera-shard)")
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--backbone", default="resnet50")
    ap.add_argument("--img", type=int, nargs=2, default=None, help="image H W (default 1080 1920; 2160 3840 "
                                                                   "with --camera-shard)")
    ap.add_argument("--bev", type=int, nargs=2, default=(480, 1440))
    ap.add_argument("--camera-shard", action="store_true", help="BASELINE configs[4]: cameras sharded over ranks")
    ap.add_argument("--stream-groups", type=int, default=None, help="ResNet inference: image groups on separate "
                    "streams (default: the model's)")
    ap.add_argument("--stream-offset", type=int, default=None, help="ResNet inference: stagger of the stream groups")
    ap.add_argument("--cpu-iters", type=int, default=3, help="frames timed for the CPU baseline (median; 0 = skip)")
    ap.add_argument("--warp-only", action="store_true", help="time only the fused warp (for profiling)")
    ap.add_argument("--warp-nhwc", action="store_true", help="A/B: the fused warp writes its output channels-last "
                    "(bev_ipm_warp_fuse_nhwc_f32) instead of the default NCHW storage")
    ap.add_argument("--conv-arith", choices=("bf16x6", "f32"), default="bf16x6",
                    help="trunk conv arithmetic: bf16x6 = fp32 through exact 3-way bf16 splits (default), f32 = the "
                         "exact-f32 MFMA kernels")
    ap.add_argument("--stem-f32", action="store_true", help="ResNet: the exact-f32 stem kernel instead of the "
                    "split-arithmetic one (A/B only; resnet.STEM_X6)")
    ap.add_argument("--no-stem-pool", action="store_true", help="ResNet: the stem output written and max-pooled "
                    "by its own launch instead of the fused stem + max-pool (A/B)")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=V",
                    help="set a performance knob (include/bev_mi355x.h BEV_TUNE_<NAME>) before the run; repeatable")
    ap.add_argument("--warp-kernel", choices=("dma", "register", "rows"), default="dma",
                    help="fused warp kernel (bev_tune BEV_TUNE_WARP_KERNEL; A/B only, same results): dma = "
                         "k_warp_fuse_v2 (default), register = k_warp_fuse, rows = k_warp_fuse_v3")
    ap.add_argument("--warp-touch", choices=("none", "tlb", "full", "sleep"), default="none",
                    help="experiment: read the encoder's features before the warp (tlb: one float per 4 KiB page, "
                         "full: every byte) or idle the GPU ~60 us (sleep), inside the timed geometry stage; "
                         "profiles/r04u_warp_touch_ab.txt")
    ap.add_argument("--dry-run", action="store_true",
                    help="orchestration check on the CPU (gloo): the rank spawning, barriers, timing and MAX "
                         "reduction of this script with a placeholder step (rank r sleeps (r + 1) x 5 ms); no hot "
                         "path runs and the line is marked so.  Used by tests/test_dist_gloo.py")
    args = ap.parse_args()
    if args.views is None:
        args.views = 16 if args.camera_shard else 7
    if args.img is None:
        args.img = (2160, 3840) if args.camera_shard else (1080, 1920)
    return args


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """Run this same command as n rank processes (one per GPU) and return their exit code.  Called before
    this process makes any GPU call, so nothing is inherited from a HIP context."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def backbone_flops(enc, H, W):
    """2 * MACs of every conv executed per image (stem..out_index + proj)."""
    import torch.nn as nn
    net = enc.backbone
    total = 0

    def conv(c: nn.Conv2d, h, w):
        ho = (h + 2 * c.padding[0] - c.kernel_size[0]) // c.stride[0] + 1
        wo = (w + 2 * c.padding[1] - c.kernel_size[1]) // c.stride[1] + 1
        return (2 * ho * wo * c.out_channels * (c.in_channels // c.groups) * c.kernel_size[0] * c.kernel_size[1],
                ho, wo)

    if enc._use_timm and hasattr(net, "conv_stem"):  # EfficientNet: stem, (pw,) dw, SE FCs, pw(l)
        from models.encoders.efficientnet import FEATURE_STAGE, DepthwiseSeparableConv
        f, h, w = conv(net.conv_stem, H, W)
        total += f
        for si in range(FEATURE_STAGE[enc.out_index] + 1):
            for blk in net.blocks[si]:
                if not isinstance(blk, DepthwiseSeparableConv):
                    total += conv(blk.conv_pw, h, w)[0]
                f, h, w = conv(blk.conv_dw, h, w)
                total += f
                total += 2 * (blk.se.conv_reduce.in_channels * blk.se.conv_reduce.out_channels) * 2
                last = blk.conv_pw if isinstance(blk, DepthwiseSeparableConv) else blk.conv_pwl
                total += conv(last, h, w)[0]
        return total + 2 * h * w * enc.proj.in_channels * enc.proj.out_channels
    if not enc._use_timm:
        f0, h, w = conv(net[0], H, W)
        f1, h, w = conv(net[2], h, w)
        return f0 + f1
    f, h, w = conv(net.conv1, H, W)
    total += f
    h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
    for li, layer in enumerate((net.layer1, net.layer2, net.layer3, net.layer4), start=1):
        if li > enc.out_index:
            break
        for blk in layer:
            hi, wi = h, w
            for c, _, _ in blk.convs():
                f, h, w = conv(c, h, w)
                total += f
            if blk.downsample is not None:
                total += conv(blk.downsample[0], hi, wi)[0]
    total += 2 * h * w * enc.proj.in_channels * enc.proj.out_channels
    return total


def stem_flops(enc, H, W):
    """2 * MACs of the ResNet stem conv per image."""
    c = enc.backbone.conv1
    ho = (H + 2 * c.padding[0] - c.kernel_size[0]) // c.stride[0] + 1
    wo = (W + 2 * c.padding[1] - c.kernel_size[1]) // c.stride[1] + 1
    return 2 * ho * wo * c.out_channels * c.in_channels * c.kernel_size[0] * c.kernel_size[1]


def backbone_bytes(enc, H, W):
    """Algorithmic HBM bytes of one image through the EfficientNet trunk + proj as the launches run it: every
    launch reads its input once and writes its output once (+ the residual it adds), fp32 NHWC; the SE
    excitation is applied in the projection conv's operand load (no extra pass); a fused inverted residual
    (bev_ir_expand_dw_f32) reads its input and writes the depthwise output only.  Weights are negligible."""
    from models.encoders.efficientnet import FEATURE_STAGE, DepthwiseSeparableConv
    net = enc.backbone

    def out_hw(c, h, w):
        return (h + 2 * c.padding[0] - c.kernel_size[0]) // c.stride[0] + 1, \
            (w + 2 * c.padding[1] - c.kernel_size[1]) // c.stride[1] + 1

    h, w = out_hw(net.conv_stem, H, W)
    total = 4 * (3 * H * W + h * w * net.conv_stem.out_channels)
    for si in range(FEATURE_STAGE[enc.out_index] + 1):
        for blk in net.blocks[si]:
            cin = blk.conv_dw.in_channels if isinstance(blk, DepthwiseSeparableConv) else blk.conv_pw.in_channels
            x_bytes = 4 * h * w * cin
            cdw = blk.conv_dw.in_channels
            h2, w2 = out_hw(blk.conv_dw, h, w)
            if net.ir_fused_block(blk, cin):  # expansion + depthwise in one pass: the expanded tensor never moves
                total += x_bytes + 4 * h2 * w2 * cdw
            else:
                if not isinstance(blk, DepthwiseSeparableConv):
                    total += x_bytes + 4 * h * w * blk.conv_pw.out_channels  # expand 1x1
                total += 4 * (h * w * cdw + h2 * w2 * cdw)  # depthwise
            last = blk.conv_pw if isinstance(blk, DepthwiseSeparableConv) else blk.conv_pwl
            total += 4 * (h2 * w2 * cdw + h2 * w2 * last.out_channels)  # projection (+ excitation)
            if blk.has_skip:
                total += 4 * h2 * w2 * last.out_channels  # residual read
            h, w = h2, w2
    return total + 4 * h * w * (enc.proj.in_channels + enc.proj.out_channels)


def warp_alg_bytes(geom, H, feats_shape, img, B):
    """out bytes + distinct touched source bytes, counted from the real taps."""
    import bev_native as nat
    _, _, C, Hf, Wf = feats_shape
    xs, ys = geom._device_axes(H.device)
    x0y0, _, valid = nat.taps(H, xs, ys, Hf, Wf, img)
    touched = 0
    for n in range(H.shape[0]):
        m = torch.zeros(Hf + 1, Wf + 1, dtype=torch.bool, device=H.device)
        v = valid[n].to(torch.int32)
        x0 = x0y0[n, ..., 0].long()
        y0 = x0y0[n, ..., 1].long()
        for bit, dx, dy in ((1, 0, 0), (2, 1, 0), (4, 0, 1), (8, 1, 1)):
            sel = (v & bit) > 0
            m[(y0 + dy)[sel], (x0 + dx)[sel]] = True
        touched += int(m.sum().item())
    out_bytes = 4 * C * geom.bev_h * geom.bev_w * B
    return out_bytes + 4 * C * touched, out_bytes, touched


def cpu_baseline(enc, args, K, Rt):
    """The reference's CPU path (timm-style ResNet on torch CPU + geometry.py grid_sample loop + mean),
    timed on this host on a bounded sample of the workload (median over `cpu_iters` frames).  For the
    16-camera 4K config the trunk runs on 2 of the 16 cameras per frame and its time is scaled by 8."""
    import backbone_ref
    from oracle import reference_composition_cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    enc_cpu = enc.to("cpu")
    H, W = args.img
    V = args.views
    v_enc = 2 if args.camera_shard else V
    gen = torch.Generator().manual_seed(1)
    times = []
    for _ in range(args.cpu_iters):
        imgs = torch.randn(1, v_enc, 3, H, W, generator=gen)
        t0 = time.perf_counter()
        feats = backbone_ref.encoder_forward(enc_cpu, imgs)
        t_enc = (time.perf_counter() - t0) * V / v_enc
        if v_enc != V:
            feats = feats.repeat(1, (V + v_enc - 1) // v_enc, 1, 1, 1)[:, :V].contiguous()
        t1 = time.perf_counter()
        reference_composition_cpu(feats, torch.from_numpy(K[:1]), torch.from_numpy(Rt[:1]), (H, W), args.bev[0],
                                  args.bev[1], BOUNDS)
        times.append(t_enc + time.perf_counter() - t1)
    t = float(np.median(times))
    enc_note = (f"trunk timed on {v_enc} of the {V} cameras and scaled x{V // v_enc}, " if v_enc != V else "")
    # the reference's warp + mean (geometry.py grid_sample loop + fusion.py mean) on ONE host thread
    torch.set_num_threads(1)
    t1 = time.perf_counter()
    reference_composition_cpu(feats[:, :V].contiguous(), torch.from_numpy(K[:1]), torch.from_numpy(Rt[:1]), (H, W),
                              args.bev[0], args.bev[1], BOUNDS)
    warp_1t = time.perf_counter() - t1
    torch.set_num_threads(threads)
    return {"value": round(1.0 / t, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{args.cpu_iters} frame(s) of the same workload ({V}x3x{H}x{W} -> {args.backbone} "
                      f"layer2 + proj C={args.channels} -> grid_sample warp -> mean), {enc_note}median {t:.2f} "
                      "s/frame, torch CPU fp32 (oracle/backbone_ref.py + oracle.reference_composition_cpu)",
            "per_frame_s": [round(x, 3) for x in times],
            "warp_mean_1thread": {"value": round(1.0 / warp_1t, 4), "unit": "frames/s", "cores": 1,
                                  "sample": f"1 frame: the {V}-view grid_sample warp + mean alone (geometry.py:120-162, "
                                            f"fusion.py:21) on one host thread, {warp_1t:.2f} s"}}


def cpu_k1(args, K, Rt):
    """BASELINE configs[0] (K1): the reference's v1.0 CPU-only path with a ResNet-18 trunk (README.md:48-55):
    7 cameras x 1080p -> ResNet-18 features_only[2] + 1x1 proj -> geometry.py grid_sample warp -> mean, on this
    host's cores (torch CPU fp32, random init), one frame.  Reported beside the GPU line, never as `value`."""
    import torch.nn as nn

    import backbone_ref
    from models.encoders.cnn_encoder import CNNEncoder
    from oracle import reference_composition_cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    torch.manual_seed(18)
    enc = CNNEncoder(out_channels=args.channels, backbone="resnet18", pretrained=False).eval()
    enc.proj = nn.Conv2d(enc.backbone.feature_info[2], args.channels, 1)  # the lazy proj, built on the CPU
    H, W = args.img
    imgs = torch.randn(1, args.views, 3, H, W, generator=torch.Generator().manual_seed(3))
    t0 = time.perf_counter()
    feats = backbone_ref.encoder_forward(enc, imgs)
    t1 = time.perf_counter()
    reference_composition_cpu(feats, torch.from_numpy(K[:1]), torch.from_numpy(Rt[:1]), (H, W), args.bev[0],
                              args.bev[1], BOUNDS)
    t2 = time.perf_counter()
    return {"config": "BASELINE configs[0]: 7-cam ResNet-18 + IPM + mean, CPU-only forward (v1.0 path)",
            "value": round(1.0 / (t2 - t0), 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"1 frame ({args.views}x3x{H}x{W} -> resnet18 layer2 + proj C={args.channels} -> grid_sample "
                      f"warp -> mean, {args.bev[0]}x{args.bev[1]}): trunk {t1 - t0:.2f} s + warp/mean {t2 - t1:.2f} s, "
                      "torch CPU fp32 (oracle/backbone_ref.py + oracle.reference_composition_cpu)"}


def pmc_traffic(args, world: int = 1) -> dict:
    """HBM bytes from the committed rocprofv3 PMC passes of this same command (tools/pmc_traffic.py):
    conv = bytes per step over all backbone conv launches, warp = bytes per fused-warp launch.
    Only reported for the default workload those passes ran; {} otherwise.  These are the profile
    file's numbers (named in `traffic_source`), not counters read by this run."""
    default = (args.views, args.channels, tuple(args.img), tuple(args.bev), args.batch, args.backbone,
               args.camera_shard, args.warp_kernel) == \
        (7, 64, (1080, 1920), (480, 1440), 2, "resnet50", False, "dma")
    # the camera-shard line (BASELINE configs[4]) at world 1: its own passes (tools/gpu_r05_warp_pmc.sh cam_fetch /
    # cam_write -> tools/pmc_traffic.py -> profiles/r*_pmc_traffic_k5.json)
    k5 = (args.views, args.channels, tuple(args.img), tuple(args.bev), args.backbone, args.camera_shard,
          args.warp_kernel, world) == (16, 64, (2160, 3840), (480, 1440), "resnet50", True, "dma", 1)
    # the EfficientNet-B3 line (BASELINE configs[3]): its own passes (tools/pmc_traffic.py ... k4 ->
    # profiles/r*_pmc_traffic_k4.json); "conv" = every encoder launch of a step
    k4 = (args.views, args.channels, tuple(args.img), tuple(args.bev), args.batch, args.backbone, args.camera_shard,
          args.warp_kernel) == (7, 64, (1080, 1920), (480, 1440), 2, "efficientnet_b3", False, "dma")
    pat = "r*_pmc_traffic_k5.json" if k5 else "r*_pmc_traffic_k4.json" if k4 else "r*_pmc_traffic.json"
    files = sorted(glob.glob(os.path.join(REPO, "profiles", pat)))
    if not (default or k5 or k4) or not files:
        return {}
    d = json.load(open(files[-1]))
    if d.get("conv_arith", "f32") != args.conv_arith:  # profiled under the other conv arithmetic
        d.pop("conv", None)
    res = {k: d[k]["traffic_bytes"] for k in ("conv", "warp") if k in d}
    res["source"] = f"profiles/{os.path.basename(files[-1])}: {d.get('note', '')}"
    return res


def workload(args, world):
    V, C = args.views, args.channels
    H, W = args.img
    if args.camera_shard:
        return ("BASELINE configs[4]", f"{V}-cam {H}x{W} -> {args.backbone}(stride-8 features)+proj C={C} -> IPM warp "
                f"(SUM of each rank's {V // world if V % world == 0 else '~' + str(V // world)} cameras) -> reduce-scatter "
                f"over BEV rows -> /{V} -> {args.bev[0]}x{args.bev[1]} BEV")
    if args.backbone.startswith("efficientnet"):
        return ("BASELINE configs[3]", f"{V}-cam {H}x{W} -> {args.backbone}(stride-8 features)+proj C={C} -> IPM warp -> "
                f"AttentionFusion (the reference's mean placeholder, fusion.py:25-36) -> {args.bev[0]}x{args.bev[1]} BEV")
    return ("BASELINE configs[1]", f"{V}-cam {H}x{W} -> {args.backbone}(stride-8 features)+proj C={C} -> IPM warp -> "
            f"mean -> {args.bev[0]}x{args.bev[1]} BEV")


def timed_steps(step, steps: int, sync, world: int):
    """The contract's timed region: barrier + sync, exactly `steps` steps, barrier + sync, then the MAX of the
    elapsed time over the ranks (all_reduce MAX on the default group).  Returns (elapsed_s, own_elapsed_s)."""
    def barrier():
        if world > 1:
            torch.distributed.barrier()
        sync()

    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    barrier()
    own = time.perf_counter() - t0
    elapsed = own
    if world > 1:
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.distributed.get_backend() == "nccl" \
            else torch.device("cpu")
        t = torch.tensor([own], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, own


def dry_run(args, world: int, rank: int) -> None:
    """--dry-run: the multi-rank orchestration of main() on the CPU with the gloo backend and a placeholder
    step, so that the N > 1 path (spawn_ranks, barriers, MAX over ranks, frame accounting) runs where no GPU
    exists.  Rank r's step sleeps (r + 1) x 5 ms: the MAX-reduced time must be the slowest rank's."""
    if world > 1:
        torch.distributed.init_process_group("gloo")
        world = torch.distributed.get_world_size()
    delay = 0.005 * (rank + 1)

    def step(record):
        time.sleep(delay)

    for _ in range(args.warmup):
        step(False)
    elapsed, own = timed_steps(step, args.steps, lambda: None, world)
    owns = [own]
    if world > 1:
        g = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        torch.distributed.all_gather(g, torch.tensor([own], dtype=torch.float64))
        owns = [float(x.item()) for x in g]
    frames = world * args.batch * args.steps
    if rank == 0:
        print(json.dumps({
            "metric": "dry-run (bench.py orchestration only; no hot path ran)", "value": round(frames / elapsed, 3),
            "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "none", "data": "none (placeholder step)",
            "config": {"workload": "placeholder", "frames_per_gpu_per_step": args.batch,
                       "frames_per_step": world * args.batch, "backend": "gloo" if world > 1 else "none"},
            "frames": frames, "elapsed_s": elapsed, "rank_elapsed_s": owns}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(world_env or 1)
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if args.dry_run:
        return dry_run(args, world, rank)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if dist:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=dev)
        world = tdist.get_world_size()  # what RCCL actually formed

    import bev_dist
    import bev_native as nat
    import bev_rig
    from models.encoders.cnn_encoder import CNNEncoder
    from models.fusion.geometry import GeometryTransformer

    B, V, C = args.batch, args.views, args.channels
    H, W = args.img
    if args.camera_shard:
        B = 1
        v0, v1 = bev_dist.camera_shard(V, rank, world)
    else:
        v0, v1 = 0, V
    VL = v1 - v0
    torch.manual_seed(1234)  # same weights on every rank (camera sharding shares one trunk)
    enc = CNNEncoder(out_channels=C, backbone=args.backbone, pretrained=False).eval().to(dev)
    if hasattr(enc.backbone, "stream_groups"):
        if args.stream_groups is not None:
            enc.backbone.stream_groups = args.stream_groups
        if args.stem_f32 or args.no_stem_pool:
            import models.encoders.resnet as _resnet
            _resnet.STEM_X6 = _resnet.STEM_X6 and not args.stem_f32
            _resnet.STEM_POOL = _resnet.STEM_POOL and not args.no_stem_pool
        if args.stream_offset is not None:
            enc.backbone.stream_offset = args.stream_offset
    geom = GeometryTransformer(args.bev[0], args.bev[1], BOUNDS)
    K, Rt = bev_rig.rig(V, H, W, B)
    Kd, Rtd = torch.from_numpy(K[:, v0:v1]).to(dev), torch.from_numpy(Rt[:, v0:v1]).to(dev)
    gen = torch.Generator(device=dev).manual_seed(rank)
    images = torch.randn(B, VL, 3, H, W, device=dev, generator=gen)

    nat.tune(nat.TUNE_WARP_KERNEL, {"dma": 0, "register": 1, "rows": 3}[args.warp_kernel])
    for kv in args.tune:
        name, v = kv.split("=")
        nat.tune(getattr(nat, "TUNE_" + name.upper()), int(v))
    nat.set_conv_arith(args.conv_arith)
    stream = torch.cuda.current_stream(dev)
    bev_format = torch.channels_last if args.warp_nhwc else torch.contiguous_format
    ev = []  # (t0, t1, t2) per timed step: backbone [t0,t1], geometry (+ exchange) [t1,t2]

    def step(record):
        with torch.no_grad():
            e0 = e1 = e2 = None
            if record:
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record(stream)
            if args.warp_only and step.feats is not None:
                feats = step.feats
            else:
                feats = enc(images)
            if record:
                e1.record(stream)
            if args.warp_touch == "sleep":  # experiment: an idle gap (~60 us of GPU sleep) instead of a read
                torch.cuda._sleep(150000)
            elif args.warp_touch != "none":  # experiment (--warp-touch): warm TLB / caches for the warp's gathers
                flat = feats.as_strided((feats.numel(),), (1,))
                step.sink = (flat[::1024] if args.warp_touch == "tlb" else flat).sum()
            if args.camera_shard:
                bev = bev_dist.camera_sharded_forward(geom, feats, Kd, Rtd, (H, W), V, "mean")
            else:
                bev = geom.forward_fused(feats, Kd, Rtd, (H, W), "mean", memory_format=bev_format)
            if record:
                e2.record(stream)
                ev.append((e0, e1, e2))
            return feats, bev

    step.feats = None
    feats, bev = step(False)
    step.feats = feats
    for _ in range(args.warmup):
        step(False)

    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    nat.spans_start()  # HIP events around every conv / warp launch, on the launch stream
    elapsed, _ = timed_steps(step, args.steps, lambda: torch.cuda.synchronize(dev), world)
    spans = nat.spans_stop()

    h2d = None
    if world == 1 and not args.warp_only:
        # side figure (never `value`): the same step with the images first copied H2D from pinned host memory
        host = images.cpu().pin_memory()
        n_h2d = min(args.steps, 20)
        barrier()
        t1 = time.perf_counter()
        for _ in range(n_h2d):
            images.copy_(host, non_blocking=True)
            step(False)
        barrier()
        h2d = {"value": round(B * n_h2d / (time.perf_counter() - t1), 3), "unit": "frames/s",
               "note": f"pinned host images ({B}x{VL}x3x{H}x{W} f32) copied H2D inside each of {n_h2d} steps"}

    bb_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))  # encoder stage (convs + pool + layout)
    stage_wp_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))  # geometry stage (+ reduce-scatter)
    # conv kernels only, per step (EfficientNet: + its depthwise convs, which the FLOP count includes)
    conv_ms = float(np.sum(spans.get("conv", [0.0])) + np.sum(spans.get("dwconv", [0.0]))) / args.steps
    wp_ms = float(np.mean(spans["warp_fuse"]))  # the fused warp kernel only
    box_ms = float(np.mean(spans["warp_boxes"])) if spans.get("warp_boxes") else 0.0  # its footprint-box pre-pass
    frames = (B if args.camera_shard else world * B) * args.steps
    value = frames / elapsed

    if rank == 0:
        pmc = pmc_traffic(args, world)
        flops = backbone_flops(enc, H, W) * VL * B
        # under the bf16x6 arithmetic every trunk conv and the proj run on the bf16 matrix cores (6 partial products
        # per fp32 product); the ResNet stem too (k_stem_x6) unless --stem-f32 keeps the exact-f32 MFMA stem kernel
        x6 = nat.conv_arith() == "bf16x6" and not args.backbone.startswith("efficient") and enc._use_timm
        import models.encoders.resnet as _resnet
        stem6 = x6 and _resnet.STEM_X6
        f_stem = 0 if stem6 else stem_flops(enc, H, W) * VL * B if x6 else flops
        peak_mfma = flops / (f_stem / PEAK_F32_MFMA_TF + (flops - f_stem) / PEAK_X6_TF) if x6 else PEAK_F32_MFMA_TF
        Hm = geom.homographies(Kd, Rtd, B, VL, dev)
        alg, out_b, touched = warp_alg_bytes(geom, Hm, feats.shape, (H, W), B)
        groups = int(getattr(enc.backbone, "stream_groups", 1)) if not args.backbone.startswith("efficient") else 1
        groups = min(groups, VL * B)
        # with >1 stream group the conv launches of the groups overlap: their HIP-event spans sum to more
        # than the wall time, so the kernel time is the encoder stage's wall time (convs + max-pool)
        kern_ms = conv_ms if groups <= 1 else bb_ms
        ach_tf = flops / (kern_ms * 1e-3) / 1e12
        roof_bb = None if args.warp_only else {
            "kernel": ("k_conv_x6* + k_stem_x6 (fp32 as 3-way split bf16, 6 partial products on "
                       "v_mfma_f32_32x32x16_bf16), every backbone conv launch of one step" if stem6 else
                       "k_conv_x6* (fp32 as 3-way split bf16, 6 partial products on v_mfma_f32_32x32x16_bf16) + "
                       "k_stem (exact-f32 MFMA), every backbone conv launch of one step" if x6 else
                       "k_conv + k_stem (fp32 MFMA implicit GEMM, every backbone conv launch of one step)"),
            "bound": "mfma", "achieved": round(ach_tf, 3), "peak": round(peak_mfma, 1),
            "unit": "TFLOP/s", "frac": round(ach_tf / peak_mfma, 4),
            "arith": nat.conv_arith() if x6 else "f32",
            "peak_basis": (f"algorithmic fp32 FLOPs at bf16 dense {PEAK_BF16_MFMA_TF:.0f} / 6 = {PEAK_X6_TF:.1f}"
                           if stem6 else
                           "algorithmic fp32 FLOPs; peak blended by FLOP share: stem at the fp32 MFMA peak 157.3, "
                           f"the rest at bf16 dense {PEAK_BF16_MFMA_TF:.0f} / 6 = {PEAK_X6_TF:.1f}" if x6 else
                           "fp32 MFMA dense peak"),
            "frac_of_fp32_mfma_peak": round(ach_tf / PEAK_F32_MFMA_TF, 4),
            "traffic": pmc.get("conv"), "flops_per_step": flops, "kernel_ms_per_step": round(kern_ms, 4),
            "conv_span_sum_ms_per_step": round(conv_ms, 4), "encoder_stage_ms": round(bb_ms, 4),
            "stream_groups": groups,
            "timing": ("HIP events around every conv launch on its stream, summed" if groups <= 1 else
                       f"{groups} image groups on separate streams overlap: encoder-stage wall time (HIP events on "
                       "the caller stream around the whole encoder, incl. the max-pool); per-launch spans sum "
                       "higher because launches of the two groups run concurrently")}
        ach = alg / (wp_ms * 1e-3) / 1e9
        wk = {"rows": "k_warp_fuse_v3", "register": "k_warp_fuse", "dma": "k_warp_fuse_v2"}[args.warp_kernel]
        roof_wp = {"kernel": f"{wk} (IPM warp + {'sum' if args.camera_shard else 'mean'}, fused)", "bound": "hbm",
                   "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
                   "traffic": pmc.get("warp"), "alg_bytes_per_launch": alg, "out_bytes": out_b,
                   "touched_src_pixels": touched, "avg_us": round(wp_ms * 1e3, 2),
                   "boxes_prepass_us": round(box_ms * 1e3, 2),
                   "frac_incl_prepass": round(alg / ((wp_ms + box_ms) * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                   "geometry_stage_us": round(stage_wp_ms * 1e3, 2),
                   "timing": "HIP events on the launch stream around the fused kernel launch alone (its footprint-box "
                             "pre-pass, k_warp_boxes, and the homographies run before the span, inside the geometry "
                             "stage)"}
        label, wl = workload(args, world)
        roof_bb_hbm = None
        if not args.warp_only and args.backbone.startswith("efficientnet"):
            # EfficientNet trunk: depthwise / pointwise layers stream their tensors -- HBM-bound, not MFMA-bound
            nbytes = backbone_bytes(enc, H, W) * VL * B
            ach_bb = nbytes / (bb_ms * 1e-3) / 1e9
            roof_bb_hbm = {"kernel": "k_conv + k_dwconv(_t) + k_se_gate (EfficientNet trunk + proj, every launch of "
                                     "one step)", "bound": "hbm", "achieved": round(ach_bb, 1), "peak": PEAK_HBM_GBS,
                           "unit": "GB/s", "frac": round(ach_bb / PEAK_HBM_GBS, 4), "traffic": pmc.get("conv"),
                           "alg_bytes_per_step": nbytes, "encoder_stage_ms": round(bb_ms, 4),
                           "timing": "HIP events on the caller stream around the whole encoder stage",
                           "bytes": "each launch reads its input once and writes its output once (+ residual), "
                                    "fp32 NHWC (bench.backbone_bytes)"}
        line = {
            "metric": "multi-cam frames/sec (7-cam→480×1440 BEV)" if label == "BASELINE configs[1]" else
                      f"multi-cam frames/sec ({V}-cam→{args.bev[0]}×{args.bev[1]} BEV)",
            "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if args.camera_shard else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{wl} ({label})", "baseline_config": label,
                       "frames_per_gpu_per_step": None if args.camera_shard else B,
                       "batch_source": ("camera-sharded: one frame per step" if args.camera_shard else
                                        "reference inference batch: inference.py:27, configs/wildtrack.yaml:2"
                                        if B == 2 else "--batch"),
                       "frames_per_step": B if args.camera_shard else world * B, "cameras": V,
                       "cameras_per_gpu": VL, "bev": list(args.bev), "channels": C,
                       "bev_memory_format": ("n/a" if args.camera_shard else
                                             "channels_last (--warp-nhwc)" if args.warp_nhwc else "NCHW"),
                       "parallelism": (f"camera-sharded x{world} (reduce-scatter over BEV rows)" if args.camera_shard
                                       else f"frame-sharded x{world} (no collective)")},
            "roofline": roof_bb_hbm or roof_bb or roof_wp,
            "roofline_warp": roof_wp,
        }
        if roof_bb_hbm:
            line["roofline_mfma"] = roof_bb
        if args.camera_shard:
            line["roofline_warp"]["note"] = "per-rank partial-sum warp of this rank's cameras; geometry_stage_us " \
                                            "includes the reduce-scatter and the /V"
        if pmc:
            line["traffic_source"] = pmc["source"]
        prov = nat.provenance()  # the library this run loaded, and whether it was built from this tree's sources
        line["build"] = {"lib_source_hash": prov["lib_source_hash"], "tree_source_hash": prov["tree_source_hash"],
                         "matches_tree": prov["matches_tree"]}
        if h2d:
            line["h2d_inclusive"] = h2d
        if args.warp_only:
            line["metric"] = "IPM warp+mean launches/sec (warp-only profiling mode)"
        if world == 1 and args.cpu_iters > 0 and not args.warp_only:
            line["cpu_baseline"] = cpu_baseline(enc, args, K, Rt)
            if not args.camera_shard and args.views == 7 and tuple(args.img) == (1080, 1920):
                line["cpu_k1"] = cpu_k1(args, K, Rt)
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
