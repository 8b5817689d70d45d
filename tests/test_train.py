"""BASELINE config 3 (training): DDP harness, trainable encoder proj, warp backward in the loop.

CPU (gloo, world 2): bev_dist's harness (materialise lazy modules, wrap in DDP, one step) on a
small torch stand-in model -- both ranks end identical and equal to ONE full-batch step on one
process (gradient averaging over the all-reduce).
GPU: the native Proj1x1 backward vs torch fp32 autograd (floating point: rtol 1e-4), and BEVNet
training steps with a frozen trunk: the loss gradient reaches encoder.proj through the native
warp backward, under DDP (RCCL, world 1).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from conftest import PKG, gather_results


class _Stand(nn.Module):
    """Lazily built head like BEVNet's (model_wrapper.py:70-84), plain torch ops."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(4, 8)
        self.head = None

    def forward(self, batch):
        h = torch.tanh(self.a(batch["x"]))
        if self.head is None:
            self.head = nn.Linear(8, 1)
        return {"y": self.head(h)}

    def loss(self, preds, targets, cfg):
        return {"total_loss": ((preds["y"] - targets) ** 2).mean()}


def _data():
    g = torch.Generator().manual_seed(5)
    return torch.randn(8, 4, generator=g), torch.randn(8, 1, generator=g)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bev_dist
        torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's
        m = _Stand()
        x, y = _data()
        sl = bev_dist.frame_shard(x.shape[0], rank, world)
        batch = {"x": x[sl.start:sl.stop]}
        bev_dist.materialize_lazy(m, batch)
        ddp = bev_dist.ddp_wrap(m)
        init = {k: v.numpy().copy() for k, v in m.state_dict().items()}
        opt = torch.optim.SGD(m.parameters(), lr=0.1)
        bev_dist.train_step(ddp, batch, y[sl.start:sl.stop], opt)
        q.put((rank, init, {k: v.numpy().copy() for k, v in m.state_dict().items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_train_step_world2_matches_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, init, after = q.get(timeout=240)
        res[r] = (init, after)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for k in res[0][0]:
        assert np.array_equal(res[0][0][k], res[1][0][k]), k  # DDP broadcast rank 0's parameters
        assert np.array_equal(res[0][1][k], res[1][1][k]), k  # identical replicas after the step
    ref = _Stand()
    ref.head = nn.Linear(8, 1)
    ref.load_state_dict({k: torch.from_numpy(v) for k, v in res[0][0].items()})
    x, y = _data()
    opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    opt.zero_grad()
    ref.loss(ref({"x": x}), y, None)["total_loss"].backward()
    opt.step()
    for k, v in ref.state_dict().items():
        torch.testing.assert_close(torch.from_numpy(res[0][1][k]), v, rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
DEV = "cuda:0"


@pytest.mark.gpu
def test_proj1x1_backward_vs_torch_fp32():
    from models.encoders.proj import Proj1x1
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 5, 7, 48, generator=g)
    w = torch.randn(16, 48, 1, 1, generator=g) * 0.2
    b = torch.randn(16, generator=g) * 0.1
    r = torch.randn(2, 5, 7, 16, generator=g)
    xg, wg, bg = (t.to(DEV).requires_grad_() for t in (x, w, b))
    y = Proj1x1.apply(xg, wg, bg)
    (y * r.to(DEV)).sum().backward()
    xc, wc, bc = (t.clone().requires_grad_() for t in (x, w, b))
    yc = F.conv2d(xc.permute(0, 3, 1, 2), wc, bc).permute(0, 2, 3, 1)
    (yc * r).sum().backward()
    torch.testing.assert_close(y.detach().cpu(), yc.detach(), rtol=1e-4, atol=1e-5)
    for got, ref in ((xg, xc), (wg, wc), (bg, bc)):
        torch.testing.assert_close(got.grad.cpu(), ref.grad, rtol=1e-4, atol=1e-4)


def _bevnet_cfg():
    return {"MODEL": {"BACKBONE": "resnet18", "PRETRAINED": False, "FEAT_DIM": 16, "OUT_INDEX": 2,
                      "BEV_SIZE": [32, 40, 120], "BEV_BOUNDS": [-24.0, 24.0, -7.2, 7.2], "BEV_PROJ_CH": 16},
            "LOSS": {}, "EVAL": {"CONF_THRESH": 0.99}}


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_bevnet_ddp_training_frozen_trunk():
    """BEVNet training steps (frozen trunk, trainable encoder proj + BEV proj + head) under DDP
    world 1 over RCCL: gradients flow through the native warp backward into encoder.proj."""
    import bev_dist
    import bev_rig
    from models.model_wrapper import BEVNet
    torch.manual_seed(0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV))
    try:
        B, V, H, W = 1, 3, 128, 224
        model = BEVNet(_bevnet_cfg()).to(DEV)
        model.encoder.freeze()  # ViewEncoder.freeze (base.py:26-28): before the lazy proj exists
        K, Rt = bev_rig.rig(V, H, W, B)
        g = torch.Generator().manual_seed(1)
        batch = {"images": torch.randn(B, V, 3, H, W, generator=g).to(DEV),
                 "calib": {"intrinsic": torch.from_numpy(K).to(DEV), "extrinsic": torch.from_numpy(Rt).to(DEV)}}
        targets = [{"boxes_world": torch.tensor([[1.0, 0.5, 0.6, 0.6], [-3.0, 2.0, 0.6, 0.6]], device=DEV)}]
        bev_dist.materialize_lazy(model, batch)
        assert model.encoder.proj.weight.requires_grad
        assert not any(p.requires_grad for p in model.encoder.backbone.parameters())
        ddp = bev_dist.ddp_wrap(model, torch.device(DEV))
        opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=1e-3)
        w0 = model.encoder.proj.weight.detach().clone()
        model.train()
        losses = [bev_dist.train_step(ddp, batch, targets, opt)["total_loss"] for _ in range(4)]
        assert all(np.isfinite(losses)), losses
        assert model.encoder.proj.weight.grad is not None
        assert model.encoder.proj.weight.grad.abs().sum().item() > 0  # reached through the warp backward
        assert not torch.equal(model.encoder.proj.weight.detach(), w0)
        assert losses[-1] < losses[0], losses
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("bn_mode", ["batch", "frozen"])
@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
def test_trunk_backward_vs_torch_autograd(name, bn_mode):
    """Native trunk training path vs torch CPU autograd on the same weights: the loss gradient w.r.t. every
    trunk parameter and the encoder proj (floating point, atomics in wgrad: rel 1e-3).
    bn_mode "batch": model.train() as the reference's train.py:222 -- BatchNorm with batch statistics, and the
    running statistics updated by the momentum rule (checked too); "frozen": BN modules in eval() inside the
    training model -- running statistics folded into the conv."""
    import backbone_ref
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(0)
    enc = CNNEncoder(out_channels=16, backbone=name, pretrained=False)
    g = torch.Generator().manual_seed(3)
    for m in enc.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.running_mean.copy_(torch.rand(m.num_features, generator=g) * 0.4 - 0.2)
            m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.bias.data.copy_(torch.rand(m.num_features, generator=g) * 0.4 - 0.2)
    imgs = torch.randn(1, 2, 3, 70, 98, generator=g)
    with torch.no_grad():
        enc.eval().to(DEV)(imgs.to(DEV))  # builds the lazy proj
    enc.train()
    if bn_mode == "frozen":
        for m in enc.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()
    stats0 = {k: b.detach().cpu().clone() for k, b in enc.named_buffers() if "running" in k}
    # record the native ReLU decisions (batch mode: every ReLU is in bev_batchnorm_apply_f32) so the float64
    # reference takes the same ones -- an element within fp32 rounding of 0 may switch sides and then carries
    # its full upstream gradient, and through the batch statistics that reaches a whole channel
    import bev_native as nat
    masks, apply0 = [], nat.batchnorm_apply

    def recording_apply(z, scale, shift, residual=None, act=0):
        out = apply0(z, scale, shift, residual, act)
        if act == 1:
            masks.append((out > 0).permute(0, 3, 1, 2).double().cpu())
        return out

    nat.batchnorm_apply = recording_apply
    try:
        y = enc(imgs.to(DEV))
    finally:
        nat.batchnorm_apply = apply0
    r = torch.randn(y.shape, generator=g)
    (y * r.to(DEV)).sum().backward()
    got = {k: p.grad.detach().cpu() for k, p in enc.named_parameters() if p.grad is not None}
    stats1 = {k: b.detach().cpu().clone() for k, b in enc.named_buffers() if "running" in k}
    enc_c = enc.to("cpu").double()  # float64 reference: the error measured is the native path's
    enc_c.zero_grad(set_to_none=True)
    with torch.no_grad():
        for k, b in enc_c.named_buffers():
            if k in stats0:
                b.copy_(stats0[k])
    r = r.double()
    act = F.relu
    if bn_mode == "batch":
        act = lambda t: t * masks.pop(0)  # noqa: E731
    f = backbone_ref.resnet_features(enc_c.backbone, imgs.double().reshape(-1, 3, 70, 98), enc_c.out_index, grad=True,
                                     act=act)
    yc = F.conv2d(f, enc_c.proj.weight, enc_c.proj.bias)
    close_y = (y.detach().cpu() - yc.detach().reshape(y.shape)).abs().max() / yc.abs().max()
    assert float(close_y) < 1e-4, float(close_y)
    (yc.reshape(y.shape) * r).sum().backward()
    worst, n, errs = 0.0, 0, {}
    for k, p in enc_c.named_parameters():
        ref = p.grad
        if ref is None:  # stages past out_index are not executed (features_only, cnn_encoder.py:41-42)
            assert k not in got, k
            continue
        assert k in got, k
        n += 1
        err = (got[k].double() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-12)
        worst = max(worst, err)
        errs[k] = err
    assert n > 20 and worst > 0.0 and not masks
    assert worst < 1e-3, sorted(errs.items(), key=lambda t: -t[1])[:6]
    moved = 0
    for k, b in enc_c.named_buffers():  # the reference's own running-stat update, from the same start
        if k in stats1:
            err = (stats1[k].double() - b).abs().max().item() / max(b.abs().max().item(), 1e-12)
            assert err < 1e-4, (k, err)
            moved += int(not torch.equal(stats1[k], stats0[k]))
    assert (moved > 0) == (bn_mode == "batch")


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_bevnet_training_trunk_end_to_end():
    """The reference's training step (train.py:249-255, fp32) on BEVNet with the TRUNK trainable: every
    trunk conv / BN parameter up to out_index receives a gradient through the native backward."""
    import bev_dist
    import bev_rig
    from models.model_wrapper import BEVNet
    torch.manual_seed(0)
    B, V, H, W = 1, 3, 128, 224
    model = BEVNet(_bevnet_cfg()).to(DEV)
    K, Rt = bev_rig.rig(V, H, W, B)
    g = torch.Generator().manual_seed(1)
    batch = {"images": torch.randn(B, V, 3, H, W, generator=g).to(DEV),
             "calib": {"intrinsic": torch.from_numpy(K).to(DEV), "extrinsic": torch.from_numpy(Rt).to(DEV)}}
    targets = [{"boxes_world": torch.tensor([[1.0, 0.5, 0.6, 0.6], [-3.0, 2.0, 0.6, 0.6]], device=DEV)}]
    bev_dist.materialize_lazy(model, batch)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    w0 = model.encoder.backbone.conv1.weight.detach().clone()
    losses = [bev_dist.train_step(model, batch, targets, opt)["total_loss"] for _ in range(4)]
    assert all(np.isfinite(losses)), losses
    bb = model.encoder.backbone
    for name in ("conv1.weight", "bn1.weight", "layer1.0.conv1.weight", "layer2.0.downsample.0.weight"):
        p = dict(bb.named_parameters())[name]
        assert p.grad is not None and p.grad.abs().sum().item() > 0, name
    assert dict(bb.named_parameters())["layer4.0.conv1.weight"].grad is None  # past out_index: not executed
    assert not torch.equal(bb.conv1.weight.detach(), w0)
    assert losses[-1] < losses[0], losses


WGRAD_CASES = [
    # N, Ci, H, W, Co, k, stride, pad -- the host pads Ci / Co to multiples of 4, every case runs k_wgrad_v4
    (2, 64, 13, 17, 64, 3, 1, 1),     # layer1 3x3 (v4)
    (1, 128, 15, 21, 128, 3, 2, 1),   # strided 3x3 (v4), Wo < 16 rows wrap several output rows per step
    (2, 64, 9, 11, 256, 1, 1, 0),     # 1x1 expand (v4)
    (1, 256, 15, 21, 512, 1, 2, 0),   # strided 1x1 downsample (v4)
    (1, 64, 5, 7, 200, 1, 1, 0),      # ragged Co (v4, partial co block)
    (1, 3, 37, 53, 64, 7, 2, 3),      # stem (Ci padded 3 -> 4)
    (1, 48, 9, 10, 24, 3, 1, 1),      # Ci % 64 != 0: 64-wide k blocks straddle taps
    (1, 96, 11, 13, 512, 3, 1, 1),    # BEV head conv1 operand (66 channels padded to 96)
    (1, 128, 9, 10, 5, 3, 1, 1),      # the head's 5 outputs (Co padded to 8)
    (2, 24, 12, 14, 16, 3, 1, 2),     # pad 2 (dilated head geometry without dilation)
    (2, 64, 70, 90, 192, 3, 1, 1),    # many m splits and co / k tiles (ragged last tile of 128)
]


@pytest.mark.gpu
@pytest.mark.parametrize("mfma", [2, 1, 0], ids=["mfma_nat", "mfma_transposed", "valu"])
@pytest.mark.parametrize("case", WGRAD_CASES, ids=[f"ci{c[1]}_co{c[4]}_k{c[5]}s{c[6]}" for c in WGRAD_CASES])
def test_wgrad_and_colsum_vs_torch(case, mfma):
    """bev_conv_wgrad_f32 (the natural-layout LDS-DMA MFMA kernel, the transposed-staging MFMA kernel, the VALU
    float4 kernel) / bev_colsum_f32 vs torch's conv2d weight /
    bias gradients (fp32; float atomics change the summation order: rtol 1e-4 of the gradient scale)."""
    import bev_native as nat
    N, Ci, H, W, Co, k, s, p = case
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, Ci, H, W, generator=g)
    w = torch.randn(Co, Ci, k, k, generator=g, requires_grad=True)
    b = torch.zeros(Co, requires_grad=True)
    y = F.conv2d(x, w, b, s, p)
    dz = torch.randn(y.shape, generator=g)
    y.backward(dz)
    dzn = dz.permute(0, 2, 3, 1).contiguous().to("cuda:0")
    with nat.tuned(WGRAD_MFMA=mfma):
        dW = nat.conv_wgrad(x.permute(0, 2, 3, 1).contiguous().to("cuda:0"), dzn, k, k, s, p).cpu()
    db = nat.colsum(dzn).cpu()
    scale = float(w.grad.abs().max())
    np.testing.assert_allclose(dW.numpy(), w.grad.numpy(), rtol=0, atol=1e-4 * scale)
    np.testing.assert_allclose(db.numpy(), b.grad.numpy(), rtol=0, atol=1e-4 * float(b.grad.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("M,C", [(907200, 64), (5000, 512), (3000, 256), (4097, 128), (100000, 24)])
def test_colsum_sizes(M, C):
    """Column sums over layer-sized and ragged row counts (k_colsum_v4 and the generic kernel)."""
    import bev_native as nat
    g = torch.Generator().manual_seed(M)
    dz = torch.randn(M, C, generator=g)
    ref = dz.double().sum(0)
    got = nat.colsum(dz.to("cuda:0")).cpu().double()
    tol = 1e-5 * float(dz.abs().sum(0).max())
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=0, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,W", [(2, 64, 37, 53), (1, 8, 16, 16), (1, 6, 11, 13), (1, 4, 9, 7)])
def test_maxpool_bwd_vs_torch_ties(N, C, H, W):
    """bev_maxpool2d_bwd_nhwc_f32 (3x3 / stride 2 / pad 1, the ResNet stem pool) vs torch CPU autograd on
    integer-valued inputs, so windows hold tied maxima: the FIRST maximum in scan order takes the
    gradient (ATen semantics).  C % 4 == 0 runs the float4 kernel, C = 6 the scalar one.  Exact."""
    import bev_native as nat
    g = torch.Generator().manual_seed(C * 100 + H)
    x = torch.randint(-3, 4, (N, C, H, W), generator=g).float().requires_grad_(True)
    y = F.max_pool2d(x, 3, 2, 1)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    got = nat.maxpool_bwd_nhwc(x.detach().permute(0, 2, 3, 1).contiguous().to("cuda:0"),
                               dy.permute(0, 2, 3, 1).contiguous().to("cuda:0"), 3, 2, 1)
    ref = x.grad.permute(0, 2, 3, 1).contiguous()
    np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,W", [(2, 64, 37, 53), (1, 8, 16, 16), (3, 4, 9, 7)])
def test_maxpool_bwd_two_pass_bit_identical(N, C, H, W):
    """bev_maxpool2d_bwd_ws_nhwc_f32 (argmax bytes, then the gather: what maxpool_bwd_nhwc runs for C % 4 == 0)
    == the single-pass bev_maxpool2d_bwd_nhwc_f32 bit for bit, with tied maxima and NaNs in the windows."""
    import bev_native as nat
    g = torch.Generator().manual_seed(C + H)
    x = torch.randint(-2, 3, (N, H, W, C), generator=g).float()
    x.view(-1)[::97] = float("nan")
    dy = torch.randn(N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, C, generator=g)
    xd, dyd = x.to(DEV), dy.to(DEV)
    Ho, Wo = dy.shape[1], dy.shape[2]
    one = torch.empty_like(xd)
    assert nat.lib().bev_maxpool2d_bwd_nhwc_f32(nat._ptr(xd), nat._ptr(dyd), N, H, W, C, 3, 2, 1, Ho, Wo,
                                                nat._ptr(one), nat._stream(xd)) == 0
    two = nat.maxpool_bwd_nhwc(xd, dyd, 3, 2, 1)
    assert torch.equal(one.view(torch.int32), two.view(torch.int32))
    # the training form: argmax bytes kept by the forward pool (whose values equal maxpool_nhwc's), the row-grid gather
    y, arg = nat.maxpool_fwd_arg_nhwc(xd, 3, 2, 1)
    assert torch.equal(y.view(torch.int32), nat.maxpool_nhwc(xd, 3, 2, 1).view(torch.int32))
    three = nat.maxpool_bwd_arg_nhwc(arg, dyd, H, W, 3, 2, 1)
    assert torch.equal(one.view(torch.int32), three.view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("k,s,p", [(2, 3, 0), (3, 1, 1), (3, 2, 0), (5, 2, 2)])
def test_maxpool_argmax_training_form_other_windows(k, s, p):
    """The training max-pool pair (forward argmax bytes, then the gather) == the single-pass x-based backward for
    windows the stem pool does not use: uncovered inputs (s > k), 3 windows per axis (the looped gather), no padding,
    5 x 5."""
    import bev_native as nat
    g = torch.Generator().manual_seed(k * 10 + s)
    N, C, H, W = 2, 8, 13, 11
    x = torch.randint(-2, 3, (N, H, W, C), generator=g).float()
    x.view(-1)[::53] = float("nan")
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, Ho, Wo, C, generator=g)
    xd, dyd = x.to(DEV), dy.to(DEV)
    one = torch.empty_like(xd)
    assert nat.lib().bev_maxpool2d_bwd_nhwc_f32(nat._ptr(xd), nat._ptr(dyd), N, H, W, C, k, s, p, Ho, Wo,
                                                nat._ptr(one), nat._stream(xd)) == 0
    y, arg = nat.maxpool_fwd_arg_nhwc(xd, k, s, p)
    assert torch.equal(y.view(torch.int32), nat.maxpool_nhwc(xd, k, s, p).view(torch.int32))
    two = nat.maxpool_bwd_arg_nhwc(arg, dyd, H, W, k, s, p)
    assert torch.equal(one.view(torch.int32), two.view(torch.int32))


BN_CASES = [(2, 64, 13, 17, 1, True, False), (1, 384, 9, 11, 1, False, False), (3, 24, 7, 5, 0, False, False),
            (2, 512, 40, 60, 1, True, False), (1, 4, 1, 3, 0, True, False), (2, 144, 11, 13, 2, False, False),
            (1, 96, 9, 7, 2, False, True), (2, 64, 6, 9, 1, True, True)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", BN_CASES, ids=[f"n{c[0]}c{c[1]}_{c[2]}x{c[3]}_a{c[4]}r{int(c[5])}f{int(c[6])}"
                                                for c in BN_CASES])
def test_batchnorm_train_kernels_vs_torch(case):
    """bev_batchnorm_train_fwd / apply / bwd vs torch's F.batch_norm (+ residual) (+ ReLU / SiLU) autograd in
    float64: output, dz, d residual, dgamma, dbeta and the running-stat update; "frozen" = running statistics
    (a BN module in eval() inside a training model)."""
    import bev_native as nat
    N, C, H, W, act, res, frozen = case
    g = torch.Generator().manual_seed(C + H)
    z = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.3
    r = torch.randn(N, C, H, W, generator=g) if res else None
    dy = torch.randn(N, C, H, W, generator=g)
    rm0, rv0 = torch.rand(C, generator=g), torch.rand(C, generator=g) + 0.5
    zd = z.double().requires_grad_(True)
    gd, bd = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    rd = r.double().requires_grad_(True) if res else None
    rm, rv = rm0.double().clone(), rv0.double().clone()
    ref = F.batch_norm(zd, rm, rv, gd, bd, not frozen, 0.1, 1e-5)
    if res:
        ref = ref + rd
    ref = torch.relu(ref) if act == 1 else F.silu(ref) if act == 2 else ref
    ref.backward(dy.double())

    def nhwc(t):
        return t.permute(0, 2, 3, 1).contiguous().to(DEV)

    zg = nhwc(z)
    grm, grv = rm0.to(DEV), rv0.to(DEV)
    if frozen:
        mean, rstd = grm.clone(), torch.rsqrt(grv + 1e-5)
        scale = gamma.to(DEV) * rstd
        shift = beta.to(DEV) - mean * scale
    else:
        mean, rstd, scale, shift = nat.batchnorm_train_fwd(zg, gamma.to(DEV), beta.to(DEV), grm, grv, 1e-5, 0.1)
    y = nat.batchnorm_apply(zg, scale, shift, nhwc(r) if res else None, act)
    dz, dres, dgm, dbt = nat.batchnorm_bwd(nhwc(dy), y if act == 1 else None, zg, mean, rstd, gamma.to(DEV), res,
                                           act, scale, shift, frozen)

    def chk(got, want, tol, what):
        got = got.detach().double().cpu()
        if got.dim() == 4:
            got = got.permute(0, 3, 1, 2)
        want = want.detach()
        err = (got - want).abs().max().item() / max(want.abs().max().item(), 1e-12)
        assert err < tol, (what, err)

    chk(y, ref, 1e-5, "y")
    if act == 1:  # gradient checks need the same ReLU decisions: drop elements within rounding of 0
        assert int(((y.permute(0, 3, 1, 2).cpu() > 0) != (ref.detach() > 0)).sum()) == 0
    chk(dz, zd.grad, 1e-4, "dz")
    chk(dgm, gd.grad, 1e-4, "dgamma")
    chk(dbt, bd.grad, 1e-5, "dbeta")
    if res:
        chk(dres, rd.grad, 1e-5, "dres")
    chk(grm, rm, 1e-5, "running_mean")
    chk(grv, rv, 1e-5, "running_var")


BNSTAT_CASES = [(2, 64, 64, 31, 45, 3, 1), (1, 128, 256, 20, 33, 1, 1), (3, 64, 128, 17, 26, 3, 2),
                (1, 256, 64, 9, 14, 1, 1), (2, 64, 320, 16, 8, 3, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", BNSTAT_CASES, ids=[f"n{c[0]}ci{c[1]}co{c[2]}_{c[3]}x{c[4]}_k{c[5]}s{c[6]}"
                                                    for c in BNSTAT_CASES])
def test_conv_h16_epilogue_batchnorm_stats(case):
    """The autocast trunk conv with the train-mode BN statistics in its epilogue (bev_conv2d_h16_bnstats_f32 +
    bev_batchnorm_finalize_tiles_f32, what ConvBNTrain runs under autocast): z bit-identical to the plain fp16
    conv (same kernel, same K order), and mean / rstd / scale / shift / running stats equal to the separate pass
    over z (bev_batchnorm_train_fwd_f32) and to float64 statistics of z -- ragged row tiles (M % 128), Co of 64..320
    (partial 128-column tiles), 1x1 and 3x3, stride 1 / 2."""
    import bev_native as nat
    N, Ci, Co, H, W, k, st = case
    g = torch.Generator().manual_seed(Ci + Co + H)
    x = (torch.randn(N, H, W, Ci, generator=g) + 0.3).to(DEV)
    w = (torch.randn(Co, Ci, k, k, generator=g) / (Ci * k * k) ** 0.5).to(DEV)
    gamma, beta = (torch.rand(Co, generator=g) + 0.5).to(DEV), (torch.randn(Co, generator=g) * 0.3).to(DEV)
    rm0, rv0 = torch.rand(Co, generator=g).to(DEV), (torch.rand(Co, generator=g) + 0.5).to(DEV)
    p = k // 2
    with nat._half_mode(True):  # what a native Function sets under autocast(float16)
        packed = nat.pack_conv_weight(w)
    assert packed.dtype == torch.float16
    z0 = nat.conv2d_nhwc_h16(x, packed, torch.zeros(Co, device=DEV), Co, k, k, st, p)
    z, tiles = nat.conv2d_nhwc_h16_bnstats(x, packed, Co, k, k, st, p)
    assert torch.equal(z, z0)
    M = z.numel() // Co
    assert tiles.shape == (Co, (M + 127) // 128, 2)
    rm1, rv1, rm2, rv2 = rm0.clone(), rv0.clone(), rm0.clone(), rv0.clone()
    a = nat.batchnorm_finalize_tiles(tiles, M, gamma, beta, rm1, rv1, 1e-5, 0.1)
    b = nat.batchnorm_train_fwd(z, gamma, beta, rm2, rv2, 1e-5, 0.1)
    zd = z.double().reshape(M, Co)
    mu, var = zd.mean(0), zd.var(0, unbiased=False)
    for name, u, v in zip(("mean", "rstd", "scale", "shift"), a, b):
        np.testing.assert_allclose(u.cpu().numpy(), v.cpu().numpy(), rtol=2e-6, atol=2e-6 * float(v.abs().max()),
                                   err_msg=name)
    np.testing.assert_allclose(a[0].double().cpu().numpy(), mu.cpu().numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(a[1].double().cpu().numpy(), (1 / torch.sqrt(var + 1e-5)).cpu().numpy(), rtol=1e-6)
    np.testing.assert_allclose(rm1.cpu().numpy(), rm2.cpu().numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(rv1.cpu().numpy(), rv2.cpu().numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_batchnorm_bwd_relu_mask_from_z():
    """bev_batchnorm_bwd_f32 act 3 (ReLU without residual, mask recomputed from z as z * scale + shift > 0)
    == act 1 (mask from the saved output y of bev_batchnorm_apply_f32) bit for bit -- including elements whose
    pre-activation rounds to exactly 0 or a tiny value of either sign; act 3 with a residual is rejected."""
    import bev_native as nat
    g = torch.Generator().manual_seed(5)
    N, H, W, C = 2, 19, 23, 64
    z = torch.randn(N, H, W, C, generator=g).to(DEV)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), (torch.randn(C, generator=g) * 0.3).to(DEV)
    mean, rstd, scale, shift = nat.batchnorm_train_fwd(z, gamma, beta, None, None, 1e-5, 0.1)
    z.view(-1, C)[::7] = -shift / scale  # pre-activations at / around the ReLU kink
    dy = torch.randn(N, H, W, C, generator=g).to(DEV)
    y = nat.batchnorm_apply(z, scale, shift, None, 1)
    a = nat.batchnorm_bwd(dy, y, z, mean, rstd, gamma, False, 1, scale, shift)
    b = nat.batchnorm_bwd(dy, None, z, mean, rstd, gamma, False, nat.ACT_RELU_FROM_Z, scale, shift)
    for u, v in zip((a[0], a[2], a[3]), (b[0], b[2], b[3])):
        assert torch.equal(u, v)
    with pytest.raises(nat.HipError):
        nat.batchnorm_bwd(dy, None, z, mean, rstd, gamma, True, nat.ACT_RELU_FROM_Z, scale, shift)


@pytest.mark.gpu
@pytest.mark.parametrize("C", [64, 256, 512])
def test_batchnorm_relu_mask_bytes(C):
    """bev_batchnorm_apply_mask_f32 (ReLU with a residual, mask bytes: bit u of byte k = y[4k + u] > 0) writes the
    y of bev_batchnorm_apply_f32 bit for bit and the mask of that y; the backward with act 4 (mask bytes passed as
    y) == act 1 (mask from y) bit for bit in dz (fp32 and fp16 storage), the residual gradient, dgamma and dbeta --
    including pre-activations at / around the ReLU kink."""
    import bev_native as nat
    g = torch.Generator().manual_seed(C)
    N, H, W = 2, 13, 17
    z = torch.randn(N, H, W, C, generator=g).to(DEV)
    res = torch.randn(N, H, W, C, generator=g).to(DEV)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), (torch.randn(C, generator=g) * 0.3).to(DEV)
    mean, rstd, scale, shift = nat.batchnorm_train_fwd(z, gamma, beta, None, None, 1e-5, 0.1)
    z.view(-1, C)[::5] = -shift / scale
    res.view(-1, C)[::5] = 0.0
    dy = torch.randn(N, H, W, C, generator=g).to(DEV)
    y = nat.batchnorm_apply(z, scale, shift, res, 1)
    y2, mask = nat.batchnorm_apply_mask(z, scale, shift, res)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    bits = (y.view(-1, 4) > 0).to(torch.uint8)
    ref_mask = bits[:, 0] | (bits[:, 1] << 1) | (bits[:, 2] << 2) | (bits[:, 3] << 3)
    assert torch.equal(mask, ref_mask)
    a = nat.batchnorm_bwd(dy, y, z, mean, rstd, gamma, True, 1, scale, shift)
    b = nat.batchnorm_bwd_half(dy, mask, z, mean, rstd, gamma, True, nat.ACT_RELU_MASK, scale, shift)
    c = nat.batchnorm_bwd_half(dy, y, z, mean, rstd, gamma, True, 1, scale, shift)
    for u, v in zip((c[0], a[1], a[2], a[3]), (b[0], b[1], b[2], b[3])):
        assert torch.equal(u, v)


DW_CASES = [(2, 96, 17, 23, 3, 1), (1, 144, 20, 31, 3, 2), (2, 40, 13, 11, 5, 1), (1, 240, 18, 22, 5, 2),
            (1, 1152, 5, 7, 3, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DW_CASES, ids=[f"c{c[1]}_k{c[4]}s{c[5]}" for c in DW_CASES])
def test_dwconv_wgrad_and_channel_ops_vs_torch(case):
    """bev_dwconv_wgrad_f32 vs torch's grouped-conv weight gradient; bev_channel_sums_f32 (of x and of x * x2)
    and bev_channel_affine_f32 vs torch (float64 references)."""
    import bev_native as nat
    N, C, H, W, K, s = case
    g = torch.Generator().manual_seed(C + K)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.zeros(C, 1, K, K, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x.double(), w, stride=s, padding=K // 2, groups=C)
    dz = torch.randn(y.shape, generator=g)
    y.backward(dz.double())
    dW = nat.dwconv_wgrad(x.permute(0, 2, 3, 1).contiguous().to(DEV), dz.permute(0, 2, 3, 1).contiguous().to(DEV),
                          K, s, K // 2)
    got = dW.t().reshape(C, 1, K, K).double().cpu()
    assert (got - w.grad).abs().max().item() <= 1e-4 * w.grad.abs().max().item()
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    x2 = torch.randn(N, H, W, C, generator=g)
    sums = nat.channel_sums(xn).double().cpu()
    assert (sums - x.double().sum((2, 3))).abs().max().item() <= 1e-5 * x.abs().sum((2, 3)).max().item()
    prod = nat.channel_sums(xn, x2.to(DEV)).double().cpu()
    want = (x.permute(0, 2, 3, 1).double() * x2.double()).sum((1, 2))
    assert (prod - want).abs().max().item() <= 1e-5 * (x.permute(0, 2, 3, 1) * x2).abs().sum((1, 2)).max().item()
    a, b = torch.randn(N, C, generator=g), torch.randn(N, C, generator=g)
    aff = nat.channel_affine(xn, a.to(DEV), b.to(DEV)).cpu()
    assert torch.equal(aff, x.permute(0, 2, 3, 1) * a[:, None, None, :] + b[:, None, None, :])


def _bevnet_ddp_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # both ranks share the box's one GPU
    try:
        import bev_dist
        import bev_rig
        from models.model_wrapper import BEVNet
        torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's parameters
        B, V, H, W = 2, 3, 128, 224
        K, Rt = bev_rig.rig(V, H, W, B)
        g = torch.Generator().manual_seed(1)
        imgs = torch.randn(B, V, 3, H, W, generator=g)
        boxes = [torch.tensor([[1.0, 0.5, 0.6, 0.6], [-3.0, 2.0, 0.6, 0.6]]), torch.tensor([[4.0, -1.0, 0.6, 0.6]])]
        sl = bev_dist.frame_shard(B, rank, world)
        batch = {"images": imgs[sl.start:sl.stop].to(DEV),
                 "calib": {"intrinsic": torch.from_numpy(K[sl.start:sl.stop]).to(DEV),
                           "extrinsic": torch.from_numpy(Rt[sl.start:sl.stop]).to(DEV)}}
        targets = [{"boxes_world": b.to(DEV)} for b in boxes[sl.start:sl.stop]]
        model = BEVNet(_bevnet_cfg()).to(DEV)
        model.encoder.freeze()
        bev_dist.materialize_lazy(model, batch)
        ddp = bev_dist.ddp_wrap(model, torch.device(DEV))
        # parameters: BN running statistics are updated from each rank's own frame and broadcast from rank 0
        # at the next forward (ddp_wrap: broadcast_buffers=True), so after the last step they may differ
        skip = set(bev_dist.unexecuted_parameters(model))  # trunk stages past OUT_INDEX: never run, never synced
        init = {k: v.detach().cpu().numpy().copy() for k, v in model.named_parameters() if k not in skip}
        opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=1e-3)
        model.train()
        losses = [bev_dist.train_step(ddp, batch, targets, opt)["total_loss"] for _ in range(2)]
        q.put((rank, init, {k: v.detach().cpu().numpy().copy() for k, v in model.named_parameters() if k not in skip},
               losses))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bevnet_ddp_world2_replicas_identical():
    """The real BEVNet (native encoder / warp / head) under DDP at world 2: two rank processes, one frame each,
    gradients all-reduced (gloo; both ranks on the box's single GPU).  Rank 0's parameters are broadcast at
    wrap time and both replicas' parameters are bit-identical after the steps; the trainable ones moved."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bevnet_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for r, init, after, losses in gather_results(procs, q, 2, 240):
        res[r] = (init, after, losses)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    moved = 0
    for k in res[0][0]:
        assert np.array_equal(res[0][0][k], res[1][0][k]), k  # broadcast from rank 0
        assert np.array_equal(res[0][1][k], res[1][1][k]), k  # identical replicas after the steps
        moved += not np.array_equal(res[0][0][k], res[0][1][k])
    assert moved > 0
    assert all(np.isfinite(res[r][2]).all() for r in (0, 1))


@pytest.mark.gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("bn_mode", ["batch", "frozen"])
@pytest.mark.parametrize("name", ["efficientnet_b0", "efficientnet_b3"])
def test_effnet_trunk_backward_vs_torch_autograd(name, bn_mode):
    """Native EfficientNet training path (stem / pointwise conv + BN + SiLU, depthwise conv, SqueezeExcite,
    skip) vs float64 torch autograd of the timm graph on the same weights: every trunk parameter's gradient
    and the running-stat updates.  SiLU is smooth, so no activation decision can flip: rel 1e-3."""
    import backbone_ref
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(1)
    enc = CNNEncoder(out_channels=16, backbone=name, pretrained=False)
    g = torch.Generator().manual_seed(5)
    for m in enc.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.running_mean.copy_(torch.rand(m.num_features, generator=g) * 0.4 - 0.2)
            m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.bias.data.copy_(torch.rand(m.num_features, generator=g) * 0.4 - 0.2)
    imgs = torch.randn(1, 2, 3, 64, 96, generator=g)
    with torch.no_grad():
        enc.eval().to(DEV)(imgs.to(DEV))  # builds the lazy proj
    enc.train()
    if bn_mode == "frozen":
        for m in enc.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()
    stats0 = {k: b.detach().cpu().clone() for k, b in enc.named_buffers() if "running" in k}
    y = enc(imgs.to(DEV))
    r = torch.randn(y.shape, generator=g)
    (y * r.to(DEV)).sum().backward()
    got = {k: p.grad.detach().cpu() for k, p in enc.named_parameters() if p.grad is not None}
    stats1 = {k: b.detach().cpu().clone() for k, b in enc.named_buffers() if "running" in k}
    enc_c = enc.to("cpu").double()
    enc_c.zero_grad(set_to_none=True)
    with torch.no_grad():
        for k, b in enc_c.named_buffers():
            if k in stats0:
                b.copy_(stats0[k])
    f = backbone_ref.efficientnet_features(enc_c.backbone, imgs.double().reshape(-1, 3, 64, 96), enc_c.out_index,
                                           grad=True)
    yc = F.conv2d(f, enc_c.proj.weight, enc_c.proj.bias)
    fwd = (y.detach().cpu().double() - yc.detach().reshape(y.shape)).abs().max() / yc.abs().max()
    assert float(fwd) < 1e-4, float(fwd)
    (yc.reshape(y.shape) * r.double()).sum().backward()
    # The bias of a projection BN (no activation) whose output feeds a conv + batch-statistics BN has an
    # (exactly) vanishing gradient apart from the skip path -- the next BN removes any per-channel shift -- so
    # each error is taken relative to max(its own scale, 1e-4 of the largest parameter gradient: fp32 leaves a
    # ~1e-7 residue of the cancelled part).
    floor = 1e-4 * max(p.grad.abs().max().item() for p in enc_c.parameters() if p.grad is not None)
    errs = {}
    for k, p in enc_c.named_parameters():
        if p.grad is None:
            assert k not in got, k
            continue
        assert k in got, k
        errs[k] = (got[k].double() - p.grad).abs().max().item() / max(p.grad.abs().max().item(), floor)
    assert len(errs) > 30
    worst = sorted(errs.items(), key=lambda t: -t[1])[:3]
    print(f"effnet trunk gradient worst relative errors ({name}, {bn_mode}): {worst}")
    assert max(errs.values()) < 1e-3, sorted(errs.items(), key=lambda t: -t[1])[:6]
    moved = 0
    for k, b in enc_c.named_buffers():
        if k in stats1:
            assert (stats1[k].double() - b).abs().max().item() <= 1e-4 * max(b.abs().max().item(), 1e-12), k
            moved += int(not torch.equal(stats1[k], stats0[k]))
    assert (moved > 0) == (bn_mode == "batch")


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W,Ci,Co,res", [(2, 17, 23, 64, 128, True), (1, 40, 30, 256, 512, False),
                                            (3, 9, 12, 32, 64, True)])
def test_dgrad_1x1_strided_placement(N, H, W, Ci, Co, res):
    """Input gradient of a 1x1 / stride-2 conv (the downsample) as dz W on the Ho x Wo pixels placed at the strided
    positions (bev_place_strided_f32, + the residual gradient) against torch.nn.grad.conv2d_input in float64 --
    including odd H / W (the last row / column of x receives no gradient) -- and equal to the zero-inserted
    (dilated) form it replaces."""
    import bev_native as nat
    from models.encoders import trunk_grad
    g = torch.Generator().manual_seed(H * W + Ci)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dz = torch.randn(N, Ho, Wo, Co, generator=g)
    w = torch.randn(Co, Ci, 1, 1, generator=g) / Ci ** 0.5
    r = torch.randn(N, H, W, Ci, generator=g) if res else None
    got = trunk_grad._dgrad(dz.to(DEV), w.to(DEV), H, W, 2, 0, residual=r.to(DEV) if res else None)
    ref = torch.nn.grad.conv2d_input((N, Ci, H, W), w.double(), dz.double().permute(0, 3, 1, 2), stride=2)
    ref = ref.permute(0, 2, 3, 1) + (r.double() if res else 0)
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    assert float((got.cpu().double() - ref).abs().max()) <= 1e-5 * scale
    d = nat.dilate_nhwc(dz.to(DEV), 2, 0, 0, 2 * (Ho - 1) + 1 + (H - 1) % 2, 2 * (Wo - 1) + 1 + (W - 1) % 2)
    wt = nat.pack_conv_weight(w.flip(2, 3).transpose(0, 1).contiguous().to(DEV))
    old = nat.conv2d_nhwc(d, wt, torch.zeros(Ci, device=DEV), Ci, 1, 1, 1, 0, False)
    if res:
        old = old + r.to(DEV)
    assert torch.equal(got, old)
