"""BASELINE config 3 as the reference's train.py runs it.

The reference trains BEVNet with RUNTIME.USE_AMP: true (configs/wildtrack.yaml:45): forward and loss under
`autocast(dtype=torch.float16)`, then `scaler.scale(loss).backward()`, `scaler.step(optimizer)`,
`scaler.update()` (train.py:168-173,238-247).  The drop-in's native autograd Functions run their forward with
autocast disabled and fp32 inputs (bev_native.amp_fwd: torch's custom-extension contract), so under AMP every
kernel still computes in fp32 -- wider than the reference's fp16 convs -- and the gradients that reach the
optimizer are the fp32 gradients times the loss scale, which scaler.unscale_ removes exactly (a power of two).

Tolerances: the fixture pin (bevnet_small.npz, the reference BEVNet's own gradients) uses test_bevnet_gpu's
fp32 tolerances unchanged (rtol 1e-3, atol 1e-3 x max|ref|); the ResNet-50 BEVNet step is compared with a
float64 torch restatement of the reference graph (oracle/bevnet_ref.py; its loss evaluated in fp32 like the
native run's): outputs and losses rel 1e-4, every
parameter gradient max|d| <= 1e-3 x max(its own max|ref|, 1e-4 x the largest gradient), BN running statistics
rel 1e-4.
"""
import copy
import json
import os
import socket
import warnings

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from conftest import GOLDEN, PKG, gather_results

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _autocast():
    """The exact context train.py:239 opens (`from torch.cuda.amp import autocast`; deprecated alias of
    torch.autocast('cuda', ...))."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", FutureWarning)
        return torch.cuda.amp.autocast(dtype=torch.float16)


@pytest.mark.timeout(240)
def test_bevnet_amp_step_matches_reference_fp32_gradients():
    """train.py:238-247 on the pinned reference BEVNet (bevnet_small.npz): the AMP branch's losses and its
    unscaled gradients equal the reference's own fp32 values within the fp32 tolerances; scaler.step then
    takes the step (no inf / NaN found) and every parameter stays finite."""
    from test_bevnet_gpu import PATH, build, close, targets_of
    d = np.load(PATH)
    net, batch, cfg = build(d)
    net.train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    scaler = torch.amp.GradScaler("cuda")
    opt.zero_grad(set_to_none=True)
    with _autocast():
        preds = net(batch)
        losses = net.loss(preds, targets_of(d), cfg["LOSS"])
        loss = losses["total_loss"] / 1.0
    for k in ("heatmap_loss", "offset_loss", "size_loss", "total_loss"):
        assert losses[k].dtype == torch.float32
        close(float(losses[k].detach()), float(d["loss_" + k]), 1e-4, 0.0, k)
    scale0 = scaler.get_scale()
    scaler.scale(loss).backward()
    scaler.unscale_(opt)
    params = dict(net.named_parameters())
    checked = 0
    for key in d.files:
        if key.startswith("g_"):
            g = params[key[2:]].grad
            assert g is not None and g.dtype == torch.float32, key
            close(g.cpu().numpy(), d[key], 1e-3, 1e-3, "amp grad " + key[2:])
            checked += 1
    assert checked >= 15
    before = {k: p.detach().clone() for k, p in params.items()}
    scaler.step(opt)
    scaler.update()
    assert scaler.get_scale() == scale0  # no inf / NaN gradient: the step was taken, the scale kept
    moved = sum(int(not torch.equal(before[k], p.detach())) for k, p in params.items())
    assert moved >= 15 and all(bool(torch.isfinite(p).all()) for p in params.values())


def _r50_cfg():
    return {"MODEL": {"BACKBONE": "resnet50", "PRETRAINED": False, "FEAT_DIM": 64, "OUT_INDEX": 2,
                      "BEV_SIZE": [32, 60, 180], "BEV_BOUNDS": [-24.0, 24.0, -7.2, 7.2], "BEV_PROJ_CH": 32},
            "LOSS": {}, "EVAL": {"CONF_THRESH": 0.4, "NMS_DIST_M": 0.5}}


def _r50_batch(B, V, H, W, seed=1):
    import bev_rig
    K, Rt = bev_rig.rig(V, H, W, B)
    g = torch.Generator().manual_seed(seed)
    imgs = torch.randn(B, V, 3, H, W, generator=g)
    boxes = [torch.tensor([[1.0, 0.5, 0.6, 0.6], [-3.0, 2.0, 0.6, 0.6]]), torch.tensor([[4.0, -1.0, 0.6, 0.6]])]
    return imgs, torch.from_numpy(K), torch.from_numpy(Rt), boxes[:B]


def _randomize_bn(model, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.running_mean.copy_(torch.rand(m.num_features, generator=g) * 0.4 - 0.2)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.rand(m.num_features, generator=g) * 0.4 - 0.2)
        for m in (model.detector.stem[1], model.detector.stem[4], model.detector.stem[7]):
            m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
            m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.2)
        w = model.detector.offset_head.weight  # the CenterNet init zeroes it
        w.copy_(torch.randn(w.shape, generator=g) * 0.05)


def _reference_copy(model, cfg):
    """A CPU float64 BEVNet with the lazy modules built at the same shapes and `model`'s state loaded."""
    from models.encoders.resnet import FoldedConv  # noqa: F401  (module import only)
    from models.heads.detector import BEVDetector
    from models.model_wrapper import BEVNet
    ref = BEVNet(cfg)
    enc = model.encoder
    ref.encoder._feature_channels = enc._feature_channels
    ref.encoder.proj = nn.Conv2d(enc.proj.in_channels, enc.proj.out_channels, 1)
    ref.proj = nn.Conv2d(model.proj.in_channels, model.proj.out_channels, 1)
    ref.detector = BEVDetector(in_channels=model.detector.in_channels, bev_bounds=model.bounds,
                               bev_size=(model.bev_h, model.bev_w), default_box_wh=model.default_box_wh)
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()}, strict=True)
    return ref.double()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("amp", [False, True], ids=["fp32", "amp"])
def test_bevnet_r50_training_step_vs_float64_reference(amp):
    """One BEVNet training step on the K3 graph (ResNet-50 trunk trainable with batch-statistics BN, encoder
    proj, ConcatFusion -> BEV proj -> pos-enc -> CenterNet head, focal / L1 loss) vs the float64 torch
    restatement of the reference's graph on the same parameters: outputs, the four losses, EVERY parameter's
    gradient and the BN running-stat update.  amp: the train.py:238-247 branch (autocast float16 +
    GradScaler), whose unscaled gradients must meet the same bar."""
    import bev_dist
    import bev_native as nat
    import bevnet_ref
    from models.model_wrapper import BEVNet
    torch.manual_seed(0)
    cfg = _r50_cfg()
    B, V, H, W = 2, 3, 128, 224
    imgs, K, Rt, boxes = _r50_batch(B, V, H, W)
    batch = {"images": imgs.to(DEV), "calib": {"intrinsic": K.to(DEV), "extrinsic": Rt.to(DEV)}}
    targets = [{"boxes_world": b.to(DEV)} for b in boxes]
    model = BEVNet(cfg).to(DEV)
    bev_dist.materialize_lazy(model, batch)
    _randomize_bn(model, 7)
    ref = _reference_copy(model, cfg)
    model.train()
    ref.train()

    trunk_masks, head_masks = [], []
    bn_apply, gn_apply = nat.batchnorm_apply, nat.groupnorm_apply

    def rec_bn(z, scale, shift, residual=None, act=0):
        out = bn_apply(z, scale, shift, residual, act)
        if act == 1:
            trunk_masks.append((out > 0).permute(0, 3, 1, 2).double().cpu())
        return out

    def rec_gn(x, scale, shift, relu):
        out = gn_apply(x, scale, shift, relu)
        if relu:
            head_masks.append((out > 0).permute(0, 3, 1, 2).double().cpu())
        return out

    nat.batchnorm_apply, nat.groupnorm_apply = rec_bn, rec_gn
    scaler = torch.amp.GradScaler("cuda") if amp else None
    try:
        model.zero_grad(set_to_none=True)
        if amp:
            with _autocast():
                preds = model(batch)
                losses = model.loss(preds, targets, cfg["LOSS"])
            scaler.scale(losses["total_loss"]).backward()
        else:
            preds = model(batch)
            losses = model.loss(preds, targets, cfg["LOSS"])
            losses["total_loss"].backward()
    finally:
        nat.batchnorm_apply, nat.groupnorm_apply = bn_apply, gn_apply
    if amp:
        opt = torch.optim.SGD(model.parameters(), lr=0.0)
        scaler.unscale_(opt)
    got = {k: p.grad.detach().double().cpu() for k, p in model.named_parameters() if p.grad is not None}
    stats = {k: b.detach().double().cpu() for k, b in model.named_buffers() if "running" in k}

    n_trunk = len(trunk_masks)
    it = iter(trunk_masks)
    out = bevnet_ref.bevnet_train_forward(ref, imgs.double(), K, Rt, trunk_act=lambda t: t * next(it),
                                          head_masks=head_masks)
    assert n_trunk > 20 and len(head_masks) == 3
    for k in ("heatmap_logits", "offset_raw", "size_raw", "bev_feat"):
        a, r = preds[k].detach().double().cpu(), out[k].detach()
        err = (a - r).abs().max().item() / max(r.abs().max().item(), 1e-12)
        assert err < 1e-4, (k, err)
    # the loss is torch code in both (BEVNet.loss); evaluate it in fp32 on the reference graph's outputs, as the
    # native run does (the focal loss's log(1 - p) near p = 1 is only as precise as fp32 p), so that the
    # comparison measures the kernels, not fp32-vs-float64 loss arithmetic
    out32 = {k: v.float() for k, v in out.items()}
    ref_losses = ref.loss(out32, [{"boxes_world": b} for b in boxes], cfg["LOSS"])
    for k in ("heatmap_loss", "offset_loss", "size_loss", "total_loss"):
        a, r = float(losses[k].detach()), float(ref_losses[k].detach())
        assert abs(a - r) <= 1e-4 * abs(r) + 1e-7, (k, a, r)
    ref_losses["total_loss"].backward()
    gmax = max(p.grad.abs().max().item() for p in ref.parameters() if p.grad is not None)
    errs = {}
    for k, p in ref.named_parameters():
        if p.grad is None:
            assert k not in got, k
            continue
        assert k in got, f"no native gradient for {k}"
        errs[k] = (got[k] - p.grad).abs().max().item() / max(p.grad.abs().max().item(), 1e-4 * gmax)
    trunk = [k for k in errs if k.startswith("encoder.backbone.")]
    assert len(trunk) > 40 and any(k.startswith("detector.") for k in errs) and "proj.weight" in errs
    assert max(errs.values()) < 1e-3, sorted(errs.items(), key=lambda t: -t[1])[:6]
    for k, b in ref.named_buffers():
        if k in stats:
            err = (stats[k] - b).abs().max().item() / max(b.abs().max().item(), 1e-12)
            assert err < 1e-4, (k, err)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _r50_ddp_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # both ranks share the box's one GPU
    try:
        import bev_dist
        from models.model_wrapper import BEVNet
        torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's parameters
        B, V, H, W = 2, 3, 128, 224
        imgs, K, Rt, boxes = _r50_batch(B, V, H, W)
        sl = bev_dist.frame_shard(B, rank, world)
        batch = {"images": imgs[sl.start:sl.stop].to(DEV),
                 "calib": {"intrinsic": K[sl.start:sl.stop].to(DEV), "extrinsic": Rt[sl.start:sl.stop].to(DEV)}}
        targets = [{"boxes_world": b.to(DEV)} for b in boxes[sl.start:sl.stop]]
        model = BEVNet(_r50_cfg()).to(DEV)
        bev_dist.materialize_lazy(model, batch)
        ddp = bev_dist.ddp_wrap(model, torch.device(DEV))
        bufs = lambda: {k: v.detach().cpu().numpy().copy() for k, v in model.named_buffers()  # noqa: E731
                        if "running" in k}
        init = {k: v.detach().cpu().numpy().copy() for k, v in model.named_parameters()}
        init_bufs = bufs()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        scaler = torch.amp.GradScaler("cuda")
        model.train()
        losses = [bev_dist.train_step(ddp, batch, targets, opt, scaler=scaler)["total_loss"] for _ in range(2)]
        # an eval forward through DDP broadcasts rank 0's buffers (broadcast_buffers=True) and updates none
        model.eval()
        with torch.no_grad():
            ddp(batch)
        skip = set(bev_dist.unexecuted_parameters(model))  # never run, never synchronised
        q.put((rank, {k: v for k, v in init.items() if k not in skip},
               {k: v.detach().cpu().numpy().copy() for k, v in model.named_parameters() if k not in skip}, losses,
               init_bufs, bufs(), scaler.get_scale()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(420)
def test_bevnet_r50_ddp_world2_trainable_trunk_amp():
    """K3 at world 2 as train.py would run it under DDP: ResNet-50 BEVNet with the TRUNK trainable (batch-
    statistics BN), autocast(float16) + GradScaler, one frame per rank, gradients all-reduced (gloo; both ranks
    on the box's single GPU).  Rank 0's parameters are broadcast at wrap time; after the steps both replicas'
    parameters are bit-identical and moved (trunk included), the scaler found no inf, and rank 0's BN running
    statistics -- broadcast at each forward (bev_dist.ddp_wrap) -- are what both ranks hold."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_r50_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for r, init, after, losses, b0, b1, scale in gather_results(procs, q, 2, 360):
        res[r] = (init, after, losses, b0, b1, scale)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    moved_trunk = 0
    for k in res[0][0]:
        assert np.array_equal(res[0][0][k], res[1][0][k]), k
        assert np.array_equal(res[0][1][k], res[1][1][k]), k
        moved_trunk += k.startswith("encoder.backbone.") and not np.array_equal(res[0][0][k], res[0][1][k])
    assert moved_trunk > 40
    for k in res[0][4]:
        assert np.array_equal(res[0][4][k], res[1][4][k]), k
    assert any(not np.array_equal(res[0][3][k], res[0][4][k]) for k in res[0][3])  # batch statistics moved
    assert all(np.isfinite(res[r][2]).all() for r in (0, 1))
    assert res[0][5] == res[1][5] == 65536.0
