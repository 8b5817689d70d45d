"""EfficientNet-B3 trunk (BASELINE config 4 backbone): module layout on the CPU, kernels on the GPU.

The module restates timm's efficientnet_b3 `features_only` trunk
(cnn_encoder.py:26); timm is absent offline, so parity with timm itself is
UNPINNED -- the layout test checks the published structure (block counts,
channel widths, SE widths, feature channels) and the GPU tests compare the
HIP kernels with torch fp32 CPU ops on the same weights (floating point:
tolerance stated per test, accumulation order differs).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

DEV = "cuda:0"


def _rand(shape, seed, scale=1.0):
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(size=shape, dtype=np.float32) * scale)


def _perturb_bn(module):
    g = torch.Generator().manual_seed(3)
    for m in module.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            n = m.num_features
            m.running_mean.copy_(torch.rand(n, generator=g) * 0.4 - 0.2)
            m.running_var.copy_(torch.rand(n, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(n, generator=g) + 0.5)
            m.bias.data.copy_(torch.rand(n, generator=g) * 0.4 - 0.2)


def test_effnet_b3_layout():
    """Published efficientnet_b3 structure: stem 40, stages [2,3,3,5,5,6,2] blocks, widths
    [24,32,48,96,136,232,384], SE rd = block input / 4, features_only channels [24,32,48,136,384]."""
    from models.encoders.efficientnet import efficientnet_b3
    m = efficientnet_b3()
    sd = m.state_dict()
    assert sd["conv_stem.weight"].shape == (40, 3, 3, 3)
    assert [len(s) for s in m.blocks] == [2, 3, 3, 5, 5, 6, 2]
    widths = [s[-1].bn2.num_features if i == 0 else s[-1].bn3.num_features for i, s in enumerate(m.blocks)]
    assert widths == [24, 32, 48, 96, 136, 232, 384]
    assert m.feature_channels == [24, 32, 48, 136, 384]
    assert sd["blocks.0.0.se.conv_reduce.weight"].shape == (10, 40, 1, 1)
    assert sd["blocks.1.0.conv_pw.weight"].shape == (144, 24, 1, 1)
    assert sd["blocks.1.0.se.conv_reduce.weight"].shape == (6, 144, 1, 1)
    assert sd["blocks.2.0.conv_dw.weight"].shape == (192, 1, 5, 5)
    assert sd["blocks.2.1.se.conv_expand.weight"].shape == (288, 12, 1, 1)
    assert sd["blocks.6.1.conv_pwl.weight"].shape == (384, 2304, 1, 1)
    n = sum(p.numel() for p in m.parameters())
    assert 10.0e6 < n < 10.2e6, n  # timm efficientnet_b3 (12.23 M) minus conv_head / bn2 / classifier


def test_effnet_b0_b1_b2_layout():
    """Published widths / depths of the other timm EfficientNets (b0 is configs/wildtrack.yaml:8's backbone)."""
    from models.encoders.efficientnet import EFFICIENTNETS
    exp = {"efficientnet_b0": ([1, 2, 2, 3, 3, 4, 1], [16, 24, 40, 112, 320], 3.595e6),
           "efficientnet_b1": ([2, 3, 3, 4, 4, 5, 2], [16, 24, 40, 112, 320], 6.101e6),
           "efficientnet_b2": ([2, 3, 3, 4, 4, 5, 2], [16, 24, 48, 120, 352], 7.203e6)}
    for name, (depths, feats, n) in exp.items():
        m = EFFICIENTNETS[name]()
        assert [len(s) for s in m.blocks] == depths, name
        assert m.feature_channels == feats, name
        assert abs(sum(p.numel() for p in m.parameters()) - n) < 2e3, name  # timm total minus head / classifier


def test_effnet_encoder_selected():
    from models.encoders.cnn_encoder import CNNEncoder
    enc = CNNEncoder(out_channels=16, backbone="efficientnet_b3", pretrained=False)
    assert enc._use_timm and hasattr(enc.backbone, "conv_stem")


DW_CASES = [  # N, C, H, W, K, stride, act
    (2, 40, 19, 33, 3, 1, 2),
    (1, 144, 21, 30, 3, 2, 2),
    (1, 192, 17, 26, 5, 2, 2),
    (2, 288, 9, 14, 5, 1, 0),
    (1, 1392, 6, 7, 3, 1, 2),  # > 1024 channels: channel chunks (blockIdx.z)
    (1, 64, 19, 23, 3, 1, 2),    # LDS-tiled kernel (8-quad chunks), partial 8 x 8 tiles
    (2, 96, 13, 11, 3, 2, 0),    # tiled, stride 2
    (1, 320, 10, 9, 5, 2, 2),    # tiled, 10 channel chunks, k5 s2
    (1, 20, 9, 12, 3, 1, 2),     # odd channel-quad count: per-pixel kernel
    (1, 36, 11, 7, 5, 2, 0),     # odd quads, k5 s2: row-run kernel
    (2, 24, 13, 37, 3, 1, 2),    # row runs of 8, ragged last run
    (1, 40, 10, 29, 3, 2, 2),    # row runs of 4 at stride 2, ragged
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DW_CASES, ids=[f"c{c[1]}_k{c[4]}s{c[5]}" for c in DW_CASES])
def test_dwconv_and_se_vs_torch_fp32(case):
    import bev_native as nat
    N, C, H, W, K, s, act = case
    x = _rand((N, C, H, W), 1)
    w = _rand((C, 1, K, K), 2, 0.3)
    b = _rand((C,), 3, 0.1)
    ref = F.conv2d(x, w, b, s, K // 2, groups=C)
    ref = F.silu(ref) if act == 2 else ref
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    wt = w.reshape(C, K * K).t().contiguous().to(DEV)
    y, ps = nat.dwconv2d_nhwc(xd, wt, b.to(DEV), K, s, K // 2, act, want_psum=True)
    got = y.permute(0, 3, 1, 2).cpu()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    # SE: squeeze from the fused partials, excite in place
    rd = max(1, C // 24)
    w1, b1 = _rand((rd, C), 4, 0.2), _rand((rd,), 5, 0.1)
    w2, b2 = _rand((C, rd), 6, 0.2), _rand((C,), 7, 0.1)
    m = ref.mean((2, 3))
    g_ref = torch.sigmoid(F.silu(m @ w1.t() + b1) @ w2.t() + b2)
    gate = nat.se_gate(ps, y.shape[1] * y.shape[2], w1.to(DEV), b1.to(DEV), w2.to(DEV), b2.to(DEV))
    np.testing.assert_allclose(gate.cpu().numpy(), g_ref.numpy(), rtol=1e-5, atol=1e-6)
    nat.channel_scale_(y, gate)
    exc = (ref * g_ref[:, :, None, None]).numpy()
    np.testing.assert_allclose(y.permute(0, 3, 1, 2).cpu().numpy(), exc, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(2, 24, 13, 37, 3, 1, 2), (1, 40, 10, 29, 3, 2, 2), (1, 144, 17, 21, 3, 2, 2),
                                  (1, 20, 9, 12, 3, 1, 0), (1, 36, 11, 7, 5, 2, 2), (1, 28, 12, 19, 5, 1, 2),
                                  (1, 192, 11, 19, 5, 2, 2), (1, 288, 9, 13, 5, 1, 2), (1, 384, 7, 9, 3, 1, 2)],
                         ids=lambda c: f"c{c[1]}_k{c[4]}s{c[5]}")
def test_dwconv_row_runs_match_per_pixel(case):
    """k_dwconv_r (BEV_TUNE_DW_RUN=1) == k_dwconv (=0): same taps in the same order, so y is identical up to the
    sign of an exact zero (compared after + 0.0); the SE partials sum the same outputs in another grouping
    (per-image totals within fp32 tolerance)."""
    import bev_native as nat
    N, C, H, W, K, s, act = case
    xd = _rand((N, H, W, C), 31).to(DEV)
    wt = _rand((K * K, C), 32, 0.3).to(DEV)
    b = _rand((C,), 33, 0.1).to(DEV)
    with nat.tuned(DW_RUN=0):
        y0, p0 = nat.dwconv2d_nhwc(xd, wt, b, K, s, K // 2, act, want_psum=True)
    for run in (1, 2, 3):  # 2: every kernel row's loads issued up front (3 x 3); 3: row runs for every width
        with nat.tuned(DW_RUN=run):
            y1, p1 = nat.dwconv2d_nhwc(xd, wt, b, K, s, K // 2, act, want_psum=True)
        assert torch.equal(y1 + 0.0, y0 + 0.0)
        np.testing.assert_allclose(p1.sum(1).cpu().numpy(), p0.sum(1).cpu().numpy(), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_conv_silu_epilogue():
    import bev_native as nat
    from models.encoders.resnet import FoldedConv
    conv = torch.nn.Conv2d(24, 144, 1, bias=False)
    x = _rand((2, 24, 11, 13), 8)
    fc = FoldedConv(conv.to(DEV))
    y = fc(x.permute(0, 2, 3, 1).contiguous().to(DEV), relu=nat.ACT_SILU)
    ref = F.silu(F.conv2d(x, conv.weight.detach().cpu()))
    np.testing.assert_allclose(y.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("Ci,Cm,K,S,N,H,W", [(24, 144, 3, 2, 2, 37, 70), (32, 192, 3, 1, 1, 33, 61),
                                             (32, 192, 5, 2, 1, 40, 47), (48, 288, 5, 1, 2, 19, 35),
                                             (16, 96, 3, 1, 1, 5, 3), (40, 240, 5, 2, 1, 17, 100)])
def test_ir_expand_dw_fused_vs_float64_and_separate(Ci, Cm, K, S, N, H, W):
    """bev_ir_expand_dw_f32 (an inverted residual's expansion + depthwise conv in one pass, h never stored) against
    float64 torch of conv_pw -> bn1 -> SiLU -> conv_dw -> bn2 -> SiLU (<= 1e-5 of max|ref|) and against the separate
    native launches (1x1 conv + bev_dwconv2d_f32, same bound), plus the SE squeeze: the partial sums add up to the
    channel sums of y -- ragged strips / row segments, tiny maps, every (K, stride) and Ci."""
    import bev_native as nat
    from models.encoders.efficientnet import FoldedDW
    from models.encoders.resnet import FoldedConv
    torch.manual_seed(Ci + K + S + H)
    pw, bn1 = torch.nn.Conv2d(Ci, Cm, 1, bias=False), torch.nn.BatchNorm2d(Cm)
    dw, bn2 = torch.nn.Conv2d(Cm, Cm, K, S, K // 2, groups=Cm, bias=False), torch.nn.BatchNorm2d(Cm)
    with torch.no_grad():
        for bn in (bn1, bn2):
            bn.weight.uniform_(0.5, 1.5), bn.bias.uniform_(-0.5, 0.5)
            bn.running_mean.uniform_(-0.2, 0.2), bn.running_var.uniform_(0.5, 2.0)
    for m in (bn1, bn2):
        m.eval()
    x = _rand((N, Ci, H, W), Ci + H)
    with torch.no_grad():
        h = F.silu(bn1.double()(F.conv2d(x.double(), pw.weight.double())))
        ref = F.silu(bn2.double()(F.conv2d(h, dw.weight.double(), stride=S, padding=K // 2, groups=Cm)))
    fc = FoldedConv(pw.to(DEV), bn1.float().to(DEV))
    fdw = FoldedDW(dw.to(DEV), bn2.float().to(DEV))
    fdw.prepare(DEV)
    w, b = fc.folded(DEV)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    y, ps = nat.ir_expand_dw(xn, w.reshape(Cm, Ci).contiguous(), b, fdw.wt, fdw.bias, K, S)
    y2, _ = fdw(fc(xn, relu=nat.ACT_SILU), want_psum=True)
    torch.cuda.synchronize()
    ref = ref.permute(0, 2, 3, 1)
    scale = ref.abs().max().item()
    assert y.shape == ref.shape
    assert (y.double().cpu() - ref).abs().max().item() <= 1e-5 * scale
    assert (y - y2).abs().max().item() <= 1e-5 * scale
    sums = y.double().sum(dim=(1, 2))
    assert (ps.double().sum(1) - sums).abs().max().item() <= 1e-5 * max(1.0, sums.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("Co,N,H,W", [(40, 2, 37, 70), (32, 1, 16, 128), (48, 1, 9, 250), (64, 3, 30, 3)])
def test_stem3_vs_float64_and_generic_conv(Co, N, H, W):
    """bev_conv2d_stem3_f32 (the EfficientNet stem on the vector ALU) == torch's conv_stem -> bn1 -> SiLU in float64
    within 2e-6 of max|ref| (27-term fp32 FMA chain + the hardware SiLU), and the generic implicit-GEMM path it
    replaces within the same bound -- ragged tiles (rows % 8, columns % 64), tiny widths, every supported Co."""
    import bev_native as nat
    from models.encoders.resnet import FoldedConv
    torch.manual_seed(Co + H)
    conv, bn = torch.nn.Conv2d(3, Co, 3, 2, 1, bias=False), torch.nn.BatchNorm2d(Co)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5), bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2), bn.running_var.uniform_(0.5, 2.0)
    bn.eval()
    x = _rand((N, 3, H, W), Co)
    with torch.no_grad():
        ref = F.silu(bn.double()(F.conv2d(x.double(), conv.weight.double(), stride=2, padding=1)))
    fc = FoldedConv(conv.to(DEV), bn.float().to(DEV))
    w, b = fc.folded(DEV)
    got = nat.conv2d_stem3(x.to(DEV), w.permute(1, 2, 3, 0).reshape(27, Co).contiguous(), b, nat.ACT_SILU)
    gen = fc(x.to(DEV), relu=nat.ACT_SILU, in_nchw=True)
    torch.cuda.synchronize()
    ref = ref.permute(0, 2, 3, 1)
    scale = ref.abs().max().item()
    assert got.shape == ref.shape
    assert (got.double().cpu() - ref).abs().max().item() <= 2e-6 * scale
    assert (got - gen).abs().max().item() <= 2e-6 * scale


@pytest.mark.gpu
@pytest.mark.parametrize("name,out_index", [("efficientnet_b3", 0), ("efficientnet_b3", 2), ("efficientnet_b3", 3),
                                            ("efficientnet_b0", 2)])
def test_effnet_encoder_vs_torch_fp32(name, out_index):
    """Native EfficientNet trunk to features_only[out_index] + proj vs torch fp32 CPU ops, same weights
    (b3: BASELINE config 4; b0: configs/wildtrack.yaml:8)."""
    from models.encoders.cnn_encoder import CNNEncoder
    import backbone_ref
    torch.manual_seed(0)
    enc = CNNEncoder(out_channels=32, backbone=name, pretrained=False, out_index=out_index)
    _perturb_bn(enc)
    enc.eval()
    imgs = _rand((1, 3, 3, 96, 160), 9)
    with torch.no_grad():
        y = enc.to(DEV)(imgs.to(DEV)).cpu()
        ref = backbone_ref.encoder_forward(enc.to("cpu"), imgs)
    stride = {0: 2, 2: 8, 3: 16}[out_index]
    assert tuple(y.shape) == tuple(ref.shape) == (1, 3, 32, 96 // stride, 160 // stride)
    err = (y - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-4, err


@pytest.mark.gpu
@pytest.mark.parametrize("Ci,Co,act,gated,res", [(40, 24, 0, False, False), (24, 24, 0, True, True),
                                                  (144, 32, 0, True, False), (24, 16, 2, False, True),
                                                  (288, 48, 1, True, True), (1024, 16, 0, False, False),
                                                  (96, 40, 2, True, False), (24, 144, 2, False, False),
                                                  (48, 288, 2, False, False), (32, 192, 2, True, True)])
def test_pw_small_matches_mfma_tiles(Ci, Co, act, gated, res):
    """Narrow 1x1 convs on the per-pixel VALU kernel (BEV_TUNE_CONV_PW_SMALL=1) == the MFMA tiles (=0) and torch
    fp32 within fp32 tolerance (rtol/atol 1e-4; same products, accumulation order differs), with the SE gate,
    bias, residual and activation of the EfficientNet projections; ragged pixel count (not a multiple of 256)."""
    import bev_native as nat
    from models.encoders.resnet import FoldedConv
    N, H, W = 2, 37, 29
    x = _rand((N, H, W, Ci), 21).to(DEV)
    gate = torch.sigmoid(_rand((N, Ci), 22)).to(DEV) if gated else None
    r = _rand((N, H, W, Co), 23).to(DEV) if res else None
    conv = torch.nn.Conv2d(Ci, Co, 1, bias=True).to(DEV)
    fc = FoldedConv(conv)
    with nat.tuned(CONV_PW_SMALL=0):
        b = fc(x, relu=act, residual=r, ascale=gate)
    xin = x * gate[:, None, None, :] if gated else x
    ref = F.conv2d(xin.permute(0, 3, 1, 2).cpu(), conv.weight.detach().cpu(), conv.bias.detach().cpu())
    ref = ref.permute(0, 2, 3, 1) + (r.cpu() if res else 0)
    ref = {0: ref, 1: torch.relu(ref), 2: F.silu(ref)}[act]
    for kern in (1, 2, 3, 4):  # 1: per-pixel VALU (Co <= 48); 2-4: wave-streaming MFMA (Ci in {24, 32, 40, 48})
        with nat.tuned(CONV_PW_SMALL=kern):
            a = fc(x, relu=act, residual=r, ascale=gate)
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(a.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("Ci", [144, 192, 40])
def test_conv_chscale_equals_separate_excitation(Ci):
    """SE excitation folded into the projection conv's operand load == x * gate, then the conv (bit-exact:
    the same fp32 product feeds the same MFMA chain), and == torch fp32 within tolerance."""
    import bev_native as nat
    from models.encoders.resnet import FoldedConv
    N, H, W, Co = 2, 9, 13, 48
    x = _rand((N, H, W, Ci), 11).to(DEV)
    gate = torch.sigmoid(_rand((N, Ci), 12)).to(DEV)
    res = _rand((N, H, W, Co), 13).to(DEV)
    conv = torch.nn.Conv2d(Ci, Co, 1, bias=False).to(DEV)
    fc = FoldedConv(conv)
    fused = fc(x, relu=nat.ACT_NONE, residual=res, ascale=gate)
    sep = fc(nat.channel_scale_(x.clone(), gate), relu=nat.ACT_NONE, residual=res)
    assert torch.equal(fused, sep)
    ref = F.conv2d((x * gate[:, None, None, :]).permute(0, 3, 1, 2).cpu(), conv.weight.detach().cpu())
    ref = ref.permute(0, 2, 3, 1) + res.cpu()
    np.testing.assert_allclose(fused.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_effnet_b3_encoder_full_1080p_bench_geometry():
    """The EfficientNet-B3 bench call (BASELINE configs[3]: 2 frames x 7 cameras x 3 x 1080 x 1920 through
    CNNEncoder('efficientnet_b3', out_index=2) + proj to C=64, cnn_encoder.py:26,41-46), so the dispatch picks the
    kernels the B3 bench line times (k_pw_mfma on the narrow projections, k_dwconv_r with channel chunks, the
    64 x 64 pointwise tiles, k_se_gate and the excitation folded into the projection load), vs the torch fp32 CPU
    restatement (oracle/backbone_ref.py) on the first and the last image of the batch (images are independent):
    max |err| <= 1e-4 * max |ref| per image (SURVEY §8d rtol)."""
    from models.encoders.cnn_encoder import CNNEncoder
    import backbone_ref
    torch.manual_seed(1234)
    enc = CNNEncoder(out_channels=64, backbone="efficientnet_b3", pretrained=False, out_index=2)
    _perturb_bn(enc)
    enc.eval()
    imgs = torch.randn(2, 7, 3, 1080, 1920, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        y = enc.to(DEV)(imgs.to(DEV))
        torch.cuda.synchronize()
    assert tuple(y.shape) == (2, 7, 64, 135, 240)
    pick = ((0, 0), (1, 6))
    got = torch.stack([y[b, v] for b, v in pick]).cpu()
    enc_cpu = enc.to("cpu")
    with torch.no_grad():
        ref = backbone_ref.encoder_forward(enc_cpu, torch.stack([imgs[b, v] for b, v in pick]).unsqueeze(0))[0]
    for i in range(len(pick)):
        err = (got[i] - ref[i]).abs().max().item() / ref[i].abs().max().item()
        assert err <= 1e-4, (pick[i], err)
