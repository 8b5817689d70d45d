"""GPU parity of the backbone conv kernels (fp32 MFMA implicit GEMM) and the encoder.

Floating-point kernel: compared with a torch fp32 CPU reference of the same
op and weights (tolerances stated per test; accumulation order differs).
The fallback encoder (cnn_encoder.py:31-37) is also checked against the
reference's own outputs in tests/golden/encoder_fallback.npz.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rand(shape, seed, scale=1.0):
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(size=shape, dtype=np.float32) * scale)


CASES = [
    # N, Ci, H, W, Co, K, stride, pad, nchw_in, residual, relu
    (2, 3, 37, 53, 64, 7, 2, 3, True, False, True),    # stem (k_stem: LDS patch, even/odd planes)
    (1, 3, 45, 301, 24, 7, 2, 3, True, False, False),  # stem, ragged Co / partial tiles, no relu
    (2, 3, 541, 963, 64, 7, 2, 3, True, False, True),  # stem, > 2 tiles per persistent workgroup, odd edges
    (1, 16, 20, 30, 24, 3, 2, 1, False, False, True),   # fallback encoder 2nd conv
    (2, 64, 17, 23, 64, 3, 1, 1, False, True, True),    # layer1 3x3 + residual
    (2, 64, 17, 23, 256, 1, 1, 0, False, True, True),   # 1x1 expand + residual
    (1, 256, 15, 21, 128, 1, 1, 0, False, False, True),
    (1, 128, 15, 21, 128, 3, 2, 1, False, False, False),  # strided 3x3
    (1, 256, 15, 21, 512, 1, 2, 0, False, False, False),  # strided 1x1 downsample
    (1, 512, 9, 11, 64, 1, 1, 0, False, False, False),    # encoder proj
    (1, 48, 9, 10, 200, 3, 1, 1, False, False, True),     # ragged Co, Ci % 16 == 0
    (1, 20, 9, 10, 33, 3, 1, 1, False, False, True),      # Ci % 16 != 0 NHWC generic
    (2, 24, 13, 17, 144, 1, 1, 0, False, False, True),    # contiguous 1x1 loader (Ci % 4), EfficientNet expand
    (1, 144, 9, 11, 32, 1, 1, 0, False, True, False),     # contiguous 1x1, K tail (144 = 4.5 K steps) + residual
    (1, 40, 7, 9, 24, 1, 1, 0, False, False, False),      # contiguous 1x1, Ci < BK
]


@pytest.mark.parametrize("case", CASES, ids=[f"ci{c[1]}_co{c[4]}_k{c[5]}s{c[6]}" for c in CASES])
def test_conv_vs_torch_fp32(case):
    import bev_native as nat
    N, Ci, H, W, Co, k, s, p, nchw, resid, relu = case
    x = _rand((N, Ci, H, W), 1)
    w = _rand((Co, Ci, k, k), 2, scale=(2.0 / (Ci * k * k)) ** 0.5)
    b = _rand((Co,), 3)
    ref = F.conv2d(x, w, b, s, p)
    r = _rand(tuple(ref.shape), 4) if resid else None
    if resid:
        ref = ref + r
    if relu:
        ref = F.relu(ref)
    packed = nat.pack_conv_weight(w.to(DEV))
    xin = x.to(DEV) if nchw else x.permute(0, 2, 3, 1).contiguous().to(DEV)
    rin = r.permute(0, 2, 3, 1).contiguous().to(DEV) if resid else None
    y = nat.conv2d_nhwc(xin, packed, b.to(DEV), Co, k, k, s, p, relu, residual=rin, in_nchw=nchw)
    got = y.permute(0, 3, 1, 2).cpu()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("tile", [1, 2, 3, 4])
@pytest.mark.parametrize("case", [CASES[3], CASES[4], CASES[6], CASES[8], CASES[9], CASES[11]],
                         ids=["l1c2_res", "l1c3_res", "s2_3x3", "proj", "ragged_co", "contig"])
def test_conv_every_tile_vs_torch_fp32(case, tile):
    """Every output tile shape (128x128, 128x64, 64x128, 64x64; bev_tune BEV_TUNE_CONV_TILE) forced on
    layers the automatic choice routes elsewhere: same results within the conv tolerance."""
    import bev_native as nat
    old = nat.tune(1, tile)
    try:
        test_conv_vs_torch_fp32(case)
    finally:
        nat.tune(1, old)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("case", [CASES[4], CASES[5], CASES[6], CASES[7], CASES[8], CASES[9], CASES[10]],
                         ids=["l1c2_res", "l1c3_res", "1x1", "s2_3x3", "s2_1x1", "proj", "ragged_co"])
def test_conv_lds_dma_bit_exact_vs_register_staging(case, tile):
    """BEV_TUNE_CONV_DMA: operands staged global -> LDS by LDS-DMA (k_conv_dma, swizzled 128-B rows) ==
    staged through registers (k_conv), bit for bit, on every tile shape (same MFMA order)."""
    import bev_native as nat
    N, Ci, H, W, Co, k, s, p, nchw, resid, relu = case
    x = _rand((N, H, W, Ci), 41).to(DEV)
    w = _rand((Co, Ci, k, k), 42, scale=(2.0 / (Ci * k * k)) ** 0.5).to(DEV)
    b = _rand((Co,), 43).to(DEV)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    r = _rand((N, Ho, Wo, Co), 44).to(DEV) if resid else None
    packed = nat.pack_conv_weight(w)
    outs = []
    old_t = nat.tune(nat.TUNE_CONV_TILE, tile)
    try:
        for dma in (0, 2):
            old = nat.tune(nat.TUNE_CONV_DMA, dma)
            try:
                outs.append(nat.conv2d_nhwc(x, packed, b, Co, k, k, s, p, relu, residual=r))
            finally:
                nat.tune(nat.TUNE_CONV_DMA, old)
    finally:
        nat.tune(nat.TUNE_CONV_TILE, old_t)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


DUAL_CASES = [
    # N, Ci (conv3 input), Ci2 (block input), H2, W2, s2, Co
    (2, 64, 64, 17, 23, 1, 256),     # layer1 block 0: conv3 64->256 + downsample 64->256
    (1, 128, 256, 15, 21, 2, 512),   # layer2 block 0: conv3 128->512 + downsample 256->512, stride 2
    (1, 32, 96, 9, 10, 3, 200),      # ragged Co, stride 3, odd sizes
]


@pytest.mark.parametrize("case", DUAL_CASES, ids=[f"ci{c[1]}+{c[2]}_s{c[5]}_co{c[6]}" for c in DUAL_CASES])
def test_conv_dual_vs_torch_fp32(case):
    """bev_conv2d_dual_f32 == relu(conv1x1(h, W1) + conv1x1(x, W2, stride) + b) (timm Bottleneck tail)."""
    import bev_native as nat
    N, Ci, Ci2, H2, W2, s2, Co = case
    Ho, Wo = (H2 - 1) // s2 + 1, (W2 - 1) // s2 + 1
    h = _rand((N, Ci, Ho, Wo), 11)
    x = _rand((N, Ci2, H2, W2), 12)
    w1 = _rand((Co, Ci, 1, 1), 13, scale=(2.0 / Ci) ** 0.5)
    w2 = _rand((Co, Ci2, 1, 1), 14, scale=(2.0 / Ci2) ** 0.5)
    b = _rand((Co,), 15)
    ref = F.relu(F.conv2d(h, w1) + F.conv2d(x, w2, stride=s2) + b.view(1, -1, 1, 1))
    packed = nat.pack_conv_weight(torch.cat([w1, w2], 1).to(DEV))
    y = nat.conv2d_dual_nhwc(h.permute(0, 2, 3, 1).contiguous().to(DEV), x.permute(0, 2, 3, 1).contiguous().to(DEV),
                             s2, packed, b.to(DEV), Co, relu=True)
    np.testing.assert_allclose(y.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


CHAIN_CASES = [
    # N, Ci, H, W, Co (conv2 out), K, stride, Co2, residual
    (2, 64, 17, 23, 64, 3, 1, 256, True),     # ResNet-50 layer1 blocks 1-2: 3x3 64->64, 1x1 64->256 + x
    (1, 128, 15, 21, 128, 3, 1, 512, True),   # layer2 blocks 1-3: 3x3 128->128, 1x1 128->512 + x
    (3, 64, 9, 37, 64, 3, 2, 128, False),     # strided, no residual, ragged last block (M = 3 * 5 * 19)
    (1, 96, 7, 5, 128, 1, 1, 384, True),      # 1x1 first conv, M < one block, 3 chunks per wave
]


@pytest.mark.parametrize("case", CHAIN_CASES, ids=[f"ci{c[1]}_co{c[4]}_k{c[5]}s{c[6]}_co2{c[7]}" for c in CHAIN_CASES])
def test_conv_chain_bit_exact_vs_two_launches(case):
    """bev_conv2d_chain_f32 (conv -> LDS -> 1x1 conv in one launch) == the two separate bev_conv2d_f32
    launches bit for bit (same K order for both GEMMs), and both == torch fp32 within the conv tolerance."""
    import bev_native as nat
    N, Ci, H, W, Co, k, s, Co2, resid = case
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = _rand((N, Ci, H, W), 21)
    w1 = _rand((Co, Ci, k, k), 22, scale=(2.0 / (Ci * k * k)) ** 0.5)
    b1 = _rand((Co,), 23)
    w2 = _rand((Co2, Co, 1, 1), 24, scale=(2.0 / Co) ** 0.5)
    b2 = _rand((Co2,), 25)
    r = _rand((N, Co2, Ho, Wo), 26) if resid else None
    xin = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    rin = r.permute(0, 2, 3, 1).contiguous().to(DEV) if resid else None
    pk1, pk2 = nat.pack_conv_weight(w1.to(DEV)), nat.pack_conv_weight(w2.to(DEV))
    h = nat.conv2d_nhwc(xin, pk1, b1.to(DEV), Co, k, k, s, p, True)
    two = nat.conv2d_nhwc(h, pk2, b2.to(DEV), Co2, 1, 1, 1, 0, True, residual=rin)
    for dma in (0, 2):  # chain kernel with register-staged and LDS-DMA operands
        old = nat.tune(nat.TUNE_CONV_DMA, dma)
        try:
            one = nat.conv2d_chain_nhwc(xin, pk1, b1.to(DEV), Co, k, k, s, p, 1, pk2, b2.to(DEV), Co2, 1, residual=rin)
        finally:
            nat.tune(nat.TUNE_CONV_DMA, old)
        torch.cuda.synchronize()
        assert torch.equal(one.view(torch.int32), two.view(torch.int32)), dma
    ref = F.conv2d(F.relu(F.conv2d(x, w1, b1, s, p)), w2, b2)
    ref = F.relu(ref + r if resid else ref)
    np.testing.assert_allclose(one.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


CHAIN_DUAL_CASES = [
    # N, Ci (conv2 in), H, W, Co, stride (conv2), Ci2 (block input), H2, W2, s2, Co2
    (2, 64, 17, 23, 64, 1, 64, 17, 23, 1, 256),      # layer1 block 0 (downsample 64 -> 256, stride 1)
    (1, 128, 15, 21, 128, 2, 256, 15, 21, 2, 512),   # layer2 block 0 (3x3 stride 2, downsample stride 2)
    (3, 32, 9, 10, 64, 3, 96, 9, 10, 3, 128),        # stride 3, odd sizes, ragged last block
]


@pytest.mark.parametrize("case", CHAIN_DUAL_CASES, ids=[f"co{c[4]}_s{c[5]}_ci2{c[6]}_co2{c[10]}" for c in CHAIN_DUAL_CASES])
def test_conv_chain_dual_bit_exact_vs_two_launches(case):
    """bev_conv2d_chain_dual_f32 == bev_conv2d_f32 (3x3) then bev_conv2d_dual_f32 (conv3 + downsample), bit for
    bit, and == torch fp32 relu(conv3(h) + ds(x) + b) within the conv tolerance."""
    import bev_native as nat
    N, Ci, H, W, Co, s, Ci2, H2, W2, s2, Co2 = case
    x = _rand((N, Ci, H, W), 31)
    xb = _rand((N, Ci2, H2, W2), 32)
    w1 = _rand((Co, Ci, 3, 3), 33, scale=(2.0 / (Ci * 9)) ** 0.5)
    b1 = _rand((Co,), 34)
    w3 = _rand((Co2, Co, 1, 1), 35, scale=(2.0 / Co) ** 0.5)
    wd = _rand((Co2, Ci2, 1, 1), 36, scale=(2.0 / Ci2) ** 0.5)
    b2 = _rand((Co2,), 37)
    xin = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    xbin = xb.permute(0, 2, 3, 1).contiguous().to(DEV)
    pk1 = nat.pack_conv_weight(w1.to(DEV))
    pk2 = nat.pack_conv_weight(torch.cat([w3, wd], 1).to(DEV))
    h = nat.conv2d_nhwc(xin, pk1, b1.to(DEV), Co, 3, 3, s, 1, True)
    two = nat.conv2d_dual_nhwc(h, xbin, s2, pk2, b2.to(DEV), Co2, True)
    one = nat.conv2d_chain_dual_nhwc(xin, pk1, b1.to(DEV), Co, 3, 3, s, 1, 1, xbin, s2, pk2, b2.to(DEV), Co2, 1)
    torch.cuda.synchronize()
    assert one.shape == two.shape
    assert torch.equal(one.view(torch.int32), two.view(torch.int32))
    ref = F.relu(F.conv2d(F.relu(F.conv2d(x, w1, b1, s, 1)), w3) + F.conv2d(xb, wd, stride=s2) + b2.view(1, -1, 1, 1))
    np.testing.assert_allclose(one.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


def test_conv_chain_rejects_unsupported_shapes():
    import bev_native as nat
    x = torch.zeros(1, 5, 5, 64, device=DEV)
    pk = nat.pack_conv_weight(torch.zeros(96, 64, 3, 3, device=DEV))
    pk2 = nat.pack_conv_weight(torch.zeros(256, 96, 1, 1, device=DEV))
    with pytest.raises(nat.HipError):  # Co must be 64 or 128 (one workgroup holds every channel of h)
        nat.conv2d_chain_nhwc(x, pk, None, 96, 3, 3, 1, 1, 1, pk2, None, 256, 1)


def test_maxpool_and_layouts_exact():
    import bev_native as nat
    x = _rand((2, 64, 31, 45), 5)
    xn = nat.nchw_to_nhwc(x.to(DEV))
    assert torch.equal(xn.cpu(), x.permute(0, 2, 3, 1).contiguous())
    assert torch.equal(nat.nhwc_to_nchw(xn).cpu(), x)
    y = nat.maxpool_nhwc(xn, 3, 2, 1)
    assert torch.equal(y.permute(0, 3, 1, 2).cpu(), F.max_pool2d(x, 3, 2, 1))
    for shape in ((3, 3, 36, 20), (2, 3, 7, 5)):  # 3-channel images: the 4-pixel kernel (H*W % 4 == 0) and the tiles
        x3 = _rand(shape, 6)
        assert torch.equal(nat.nchw_to_nhwc(x3.to(DEV)).cpu(), x3.permute(0, 2, 3, 1).contiguous())
        x4 = nat.nchw_to_nhwc4(x3.to(DEV)).cpu()  # 4-channel pixels with a zero channel (the stem's wgrad operand)
        assert torch.equal(x4[..., :3], x3.permute(0, 2, 3, 1)) and not x4[..., 3].any()


def test_encoder_proj_streaming_loads_same_result():
    """CNNEncoder's projection with non-temporal activation loads (proj_stream_nt, BEV_TUNE_CONV_X6_NT) gives the
    same bits as with cached loads (same kernel arithmetic), at a full 1080p camera."""
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(3)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(DEV)
    x = _rand((1, 2, 3, 1080, 1920), 4).to(DEV)
    with torch.no_grad():
        enc.proj_stream_nt = True
        a = enc(x)
        enc.proj_stream_nt = False
        b = enc(x)
    assert torch.equal(a, b)


@pytest.mark.parametrize("shape,k,s,p", [((2, 64, 31, 45), 3, 2, 1), ((1, 12, 17, 9), 2, 2, 0), ((3, 4, 8, 11), 3, 1, 1),
                                         ((1, 64, 540, 960), 3, 2, 1)])
def test_maxpool_rows_kernel_exact(shape, k, s, p):
    """k_maxpool_rows (the float4 row-grid kernel) vs torch max_pool2d, NaNs included (torch propagates them)."""
    import bev_native as nat
    x = _rand(shape, 11)
    x.view(-1)[:: 997] = float("nan")
    y = nat.maxpool_nhwc(nat.nchw_to_nhwc(x.to(DEV)), k, s, p)
    ref = F.max_pool2d(x, k, s, p)
    got = y.permute(0, 3, 1, 2).cpu()
    assert torch.equal(torch.isnan(got), torch.isnan(ref))
    assert torch.equal(torch.nan_to_num(got, nan=7.0), torch.nan_to_num(ref, nan=7.0))


def test_fallback_encoder_matches_reference_fixture():
    """cnn_encoder.py:31-37 (the branch the reference takes without timm) vs its recorded outputs."""
    from models.encoders.cnn_encoder import CNNEncoder
    d = np.load(os.path.join(GOLDEN, "encoder_fallback.npz"))
    enc = CNNEncoder(out_channels=8, backbone="resnet18", pretrained=False, backbone_impl="fallback")
    sd = {k: torch.from_numpy(d["w_" + k.replace(".", "_")]) for k in d["keys"]}
    enc.load_state_dict(sd)
    enc = enc.to(DEV).eval()
    with torch.no_grad():
        y5 = enc(torch.from_numpy(d["x5"]).to(DEV)).cpu().numpy()
        y4 = enc(torch.from_numpy(d["x4"]).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(y5, d["y5"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(y4, d["y4"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
def test_resnet_encoder_vs_torch_fp32(name):
    """Native ResNet trunk to layer2 + proj vs torch fp32 CPU ops on the same weights."""
    from models.encoders.cnn_encoder import CNNEncoder
    import backbone_ref
    torch.manual_seed(0)
    enc = CNNEncoder(out_channels=64, backbone=name, pretrained=False)
    for m in enc.modules():  # non-trivial BN statistics so the folding is exercised
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    enc.eval()
    imgs = _rand((1, 3, 3, 96, 160), 6)
    with torch.no_grad():
        enc_gpu = enc.to(DEV)
        y = enc_gpu(imgs.to(DEV)).cpu()
        enc_cpu = enc.to("cpu")
        ref = backbone_ref.encoder_forward(enc_cpu, imgs)
    assert tuple(y.shape) == tuple(ref.shape) == (1, 3, 64, 12, 20)
    err = (y - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-4, err


def test_resnet_chain_fusion_bit_exact():
    """ResNet-50 trunk with the bottleneck conv2 -> conv3 chains in one launch (FoldedChain) == the
    unchained launches, bit for bit."""
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(2)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(DEV)
    imgs = _rand((1, 3, 3, 90, 150), 10).to(DEV)
    with torch.no_grad():
        enc.backbone.fuse_chain = False
        ref = enc(imgs).clone()
        enc.backbone.fuse_chain = True
        got = enc(imgs)
        torch.cuda.synchronize()
    assert torch.equal(got.contiguous().view(torch.int32), ref.contiguous().view(torch.int32))


@pytest.mark.parametrize("groups,offset", [(2, 0), (3, 0), (2, 1), (3, 3)])
def test_resnet_stream_groups_bit_exact(groups, offset):
    """Inference split over image groups on separate streams == one stream, bit for bit (same kernels,
    same per-element accumulation order), including an uneven split and the output written in place."""
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(1)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(DEV)
    imgs = _rand((1, 5, 3, 90, 150), 9).to(DEV)
    with torch.no_grad():
        ref = enc(imgs).clone()
        enc.backbone.stream_groups, enc.backbone.stream_offset = groups, offset
        got = enc(imgs)
        torch.cuda.synchronize()
        enc.backbone.stream_groups, enc.backbone.stream_offset = 1, 0
    assert got.shape == ref.shape
    assert torch.equal(got.contiguous().view(torch.int32), ref.contiguous().view(torch.int32))


def test_resnet_stream_groups_cold_cache_and_repack():
    """a fresh model run straight away with 2 stream groups (every folded panel packed during this
    call) and again after in-place weight / BN-statistic updates (re-pack) == the single-stream trunk, bit for bit.
    The panels are packed on the caller's stream before the groups fork (ResNet._prepare_eval)."""
    import copy
    from models.encoders.resnet import resnet50
    torch.manual_seed(3)
    a = resnet50().eval()
    b = copy.deepcopy(a)
    a.to(DEV)
    b.to(DEV)
    a.stream_groups, b.stream_groups = 2, 1
    x = _rand((6, 3, 90, 150), 12).to(DEV)
    outs = []
    with torch.no_grad():
        for it in range(2):
            if it == 1:
                for m in (a, b):
                    m.layer1[0].conv2.weight.mul_(1.5)
                    m.layer2[1].bn2.running_var.mul_(2.0)
                    m.bn1.bias.add_(0.1)
            ya = a.forward_features_nhwc(x, 2)
            yb = b.forward_features_nhwc(x, 2)
            torch.cuda.synchronize()
            assert torch.equal(ya.view(torch.int32), yb.view(torch.int32))
            outs.append(ya.clone())
    assert not torch.equal(outs[0], outs[1])


@pytest.mark.gpu
def test_resnet50_encoder_full_1080p_bench_geometry():
    """The bench's exact encoder call (BASELINE configs[1]: 2 frames x 7 cameras x 3 x 1080 x 1920, ResNet-50 to
    layer2 + proj to C=64, two stream groups of 7 images, so the same tiles, chains, LDS-DMA staging and XCD
    order the bench times) vs the torch fp32 CPU restatement (oracle/backbone_ref.py) on the first and last image
    of each stream group (images are independent), max |err| <= 1e-4 * max |ref| per image (SURVEY §8d rtol)."""
    from models.encoders.cnn_encoder import CNNEncoder
    import backbone_ref
    torch.manual_seed(1234)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False)
    g = torch.Generator().manual_seed(5)
    for m in enc.modules():  # non-trivial BN statistics so the folding is exercised
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2, generator=g)
            m.running_var.uniform_(0.5, 1.5, generator=g)
            m.weight.data.uniform_(0.5, 1.5, generator=g)
            m.bias.data.uniform_(-0.2, 0.2, generator=g)
    enc.eval()
    imgs = torch.randn(2, 7, 3, 1080, 1920, generator=torch.Generator().manual_seed(0))
    enc_gpu = enc.to(DEV)
    assert enc_gpu.backbone.stream_groups == 2
    with torch.no_grad():
        y = enc_gpu(imgs.to(DEV))
        torch.cuda.synchronize()
    assert tuple(y.shape) == (2, 7, 64, 135, 240)
    pick = ((0, 0), (0, 6), (1, 0), (1, 6))  # group 0 = images 0..6, group 1 = images 7..13
    got = torch.stack([y[b, v] for b, v in pick]).cpu()
    enc_cpu = enc.to("cpu")
    ref = backbone_ref.encoder_forward(enc_cpu, torch.stack([imgs[b, v] for b, v in pick]).unsqueeze(0))[0]
    for i in range(len(pick)):
        err = (got[i] - ref[i]).abs().max().item() / ref[i].abs().max().item()
        assert err <= 1e-4, (pick[i], err)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_resnet50_encoder_4k_camera_shard_geometry():
    """The camera-shard bench's exact encoder call (BASELINE configs[4]: 1 frame x 16 cameras x 3 x 2160 x 3840,
    ResNet-50 to layer2 + proj to C=64, bench.py --camera-shard at world 1) vs the torch fp32 CPU restatement
    (oracle/backbone_ref.py) on the first and last camera, max |err| <= 1e-4 * max |ref| per image (SURVEY §8d
    rtol).  At this size ResNet-50's layer1 output holds 16 * 540 * 960 * 256 = 2.12e9 elements (98.9 % of
    INT32_MAX), so the M-dependent paths -- buffer-descriptor rebasing of the split-bf16 convs, grid sizes, tile
    rounds, the 64-bit pixel offsets of the stem and the max-pool -- run at the largest extent the bench uses."""
    from models.encoders.cnn_encoder import CNNEncoder
    import backbone_ref
    torch.manual_seed(1234)  # bench.py's weight seed
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False)
    g = torch.Generator().manual_seed(6)
    for m in enc.modules():  # non-trivial BN statistics so the folding is exercised
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2, generator=g)
            m.running_var.uniform_(0.5, 1.5, generator=g)
            m.weight.data.uniform_(0.5, 1.5, generator=g)
            m.bias.data.uniform_(-0.2, 0.2, generator=g)
    enc.eval()
    enc_gpu = enc.to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)  # bench.py: rank 0's image generator
    imgs = torch.randn(1, 16, 3, 2160, 3840, device=DEV, generator=gen)
    with torch.no_grad():
        y = enc_gpu(imgs)
        torch.cuda.synchronize()
    assert tuple(y.shape) == (1, 16, 64, 270, 480)
    pick = (0, 15)
    got = torch.stack([y[0, v] for v in pick]).cpu()
    x_ref = torch.stack([imgs[0, v] for v in pick]).cpu()
    del y, imgs
    torch.cuda.empty_cache()
    enc_cpu = enc.to("cpu")
    for i, v in enumerate(pick):  # one camera at a time (host memory)
        ref = backbone_ref.encoder_forward(enc_cpu, x_ref[i][None, None])[0, 0]
        err = (got[i] - ref).abs().max().item() / ref.abs().max().item()
        assert err <= 1e-4, (v, err)
