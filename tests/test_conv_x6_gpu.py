"""fp32 convolutions on the bf16 matrix cores by exact three-way operand split (bev_conv2d_x6_f32,
bev_conv2d_dual_x6_f32; csrc/bev_conv_x6.hip) -- the default arithmetic of the inference trunk.

The reference runs these convs (timm trunk + lazy 1x1 proj, cnn_encoder.py:26,41-46) as fp32 nn.Conv2d.  The
split kernels must be an fp32 convolution: every case is compared against float64 torch, and their error must not
exceed the exact-f32 MFMA kernel's (bev_conv2d_f32) by more than a small factor -- fp32 accuracy, not bf16
accuracy.  The tolerance (fp32 rtol 1e-4 vs torch fp32) is asserted too.
"""
import pytest
import torch
import torch.nn.functional as F

import bev_native as nat

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _case(N, H, W, Ci, Co, K, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, Ci, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Co, Ci, K, K, generator=g, dtype=torch.float64) / (Ci * K * K) ** 0.5
    b = torch.randn(Co, generator=g, dtype=torch.float64) * 0.1
    return x, w, b


def _ref(x, w, b, stride, pad, dil, act, res=None):
    y = F.conv2d(x, w, b, stride=stride, padding=pad, dilation=dil)
    if res is not None:
        y = y + res
    if act == 1:
        y = torch.relu(y)
    elif act == 2:
        y = F.silu(y)
    return y


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


CASES = [
    # N, H, W, Ci, Co, K, stride, pad, dil, act, residual
    (2, 23, 37, 64, 64, 3, 1, 1, 1, 1, False),    # layer1 conv2 shape class, ragged M
    (1, 30, 41, 128, 128, 3, 2, 1, 1, 1, False),  # layer2 block-0 conv2 (stride 2)
    (2, 17, 19, 256, 64, 1, 1, 0, 1, 1, False),   # conv1 (1x1 reduce)
    (2, 17, 19, 64, 256, 1, 1, 0, 1, 1, True),    # conv3 + identity residual + ReLU
    (1, 21, 22, 48, 80, 3, 1, 2, 2, 2, False),    # dilation 2, SiLU, Co not a multiple of 64
    (1, 9, 13, 512, 64, 1, 1, 0, 1, 0, False),    # the encoder's 1x1 proj (no activation)
    (3, 15, 16, 16, 200, 3, 1, 1, 1, 1, True),    # Ci = 16 (one K step per tap), three N tiles
]


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_x6_conv_fp32_accuracy_vs_float64(case):
    N, H, W, Ci, Co, K, s, p, d, act, with_res = case
    x, w, b = _case(N, H, W, Ci, Co, K, 1234 + Ci + Co)
    Ho, Wo = (H + 2 * p - d * (K - 1) - 1) // s + 1, (W + 2 * p - d * (K - 1) - 1) // s + 1
    res = torch.randn(N, Co, Ho, Wo, dtype=torch.float64, generator=torch.Generator().manual_seed(7)) if with_res else None
    # float64 reference on the fp32-rounded operands (what both kernels see)
    x32, w32, b32 = x.float(), w.float(), b.float()
    res32 = res.float() if res is not None else None
    ref = _ref(x32.double(), w32.double(), b32.double(), s, p, d, act, res32.double() if res is not None else None)
    ref = _nhwc(ref)
    xd = _nhwc(x32).to(DEV)
    rd = _nhwc(res32).to(DEV) if res is not None else None
    bd = b32.to(DEV)
    p6 = nat.pack_conv_weight_x6(w32.to(DEV))
    assert p6.dtype == torch.bfloat16
    y6 = nat.conv2d_nhwc_x6(xd, p6, bd, Co, K, K, s, p, d, act, residual=rd)
    torch.cuda.synchronize()
    e6 = (y6.cpu().double() - ref).abs()
    scale = ref.abs().max().item()
    assert torch.isfinite(y6).all()
    assert e6.max().item() <= 1e-5 * scale, (e6.max().item(), scale)
    torch.testing.assert_close(y6.cpu().double(), ref, rtol=1e-4, atol=1e-4 * scale)
    if d == 1:  # the exact-f32 MFMA kernel on the same operands: the split kernel is no less accurate (within 4x)
        pf = nat.pack_conv_weight(w32.to(DEV))
        yf = nat.conv2d_nhwc(xd, pf, bd, Co, K, K, s, p, act == 1, residual=rd) if act != 2 else None
        if yf is not None:
            ef = (yf.cpu().double() - ref).abs()
            assert e6.max().item() <= 4 * ef.max().item() + 1e-7 * scale, (e6.max().item(), ef.max().item())
            assert e6.mean().item() <= 4 * ef.mean().item() + 1e-9 * scale, (e6.mean().item(), ef.mean().item())


def test_x6_tiles_bit_identical():
    """Both output tiles (BEV_TUNE_CONV_X6_TILE 1 = 128x128, 2 = 128x64) and both kernels (BEV_TUNE_CONV_X6_KERNEL:
    32-deep steps with B from the panel, 16-deep steps with B through LDS) sum every output in the same K order."""
    N, H, W, Ci, Co = 2, 19, 29, 64, 192
    x, w, b = _case(N, H, W, Ci, Co, 3, 5)
    xd, bd = _nhwc(x.float()).to(DEV), b.float().to(DEV)
    p6 = nat.pack_conv_weight_x6(w.float().to(DEV))
    outs = []
    for t in (1, 2):
        for kern in (0, 1, 2):
            with nat.tuned(CONV_X6_TILE=t, CONV_X6_KERNEL=kern):
                outs.append(nat.conv2d_nhwc_x6(xd, p6, bd, Co, 3, 3, 1, 1, 1, 1))
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)


@pytest.mark.parametrize("Ci,Co,K,stride,tile", [(64, 64, 3, 1, 0), (128, 128, 3, 2, 0), (64, 192, 3, 1, 1),
                                                  (64, 192, 3, 1, 2), (32, 64, 1, 1, 0)])
def test_x6_split_operand_bit_identical(Ci, Co, K, stride, tile):
    """Pre-split operand planes (bev_split3_f32 -> k_conv_x6s, LDS-DMA staging) give bit-for-bit the result of the
    fp32 operand split in-kernel, and a split output (ys) holds exactly the split of the fp32 output."""
    N, H, W = 2, 23, 35
    x, w, b = _case(N, H, W, Ci, Co, K, 77 + Ci)
    xd, bd = _nhwc(x.float()).to(DEV), b.float().to(DEV)
    p6 = nat.pack_conv_weight_x6(w.float().to(DEV))
    pad = K // 2
    xs = nat.split3(xd)
    assert torch.equal(xs.to_float(), xd)  # exact split
    with nat.tuned(CONV_X6_TILE=tile):
        ref = nat.conv2d_nhwc_x6(xd, p6, bd, Co, K, K, stride, pad, 1, 1)
        got = nat.conv2d_nhwc_x6(xs, p6, bd, Co, K, K, stride, pad, 1, 1)
        ys = nat.conv2d_nhwc_x6(xs, p6, bd, Co, K, K, stride, pad, 1, 1, split_out=True)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert torch.equal(ys.to_float(), ref)
    assert torch.equal(ys.planes, nat.split3(ref).planes)


@pytest.mark.parametrize("stride2,Ci,Ci2,Co", [(1, 64, 64, 256), (2, 128, 256, 512)])
def test_x6_dual_accuracy(stride2, Ci, Ci2, Co):
    """Bottleneck conv3 + downsample shortcut as one split-bf16 GEMM (FoldedTail) vs float64."""
    g = torch.Generator().manual_seed(11 + Ci2)
    N, H2, W2 = 2, 21, 26
    Ho, Wo = (H2 - 1) // stride2 + 1, (W2 - 1) // stride2 + 1
    h = torch.randn(N, Ci, Ho, Wo, generator=g).float()
    x2 = torch.randn(N, Ci2, H2, W2, generator=g).float()
    w1 = (torch.randn(Co, Ci, 1, 1, generator=g) / Ci ** 0.5).float()
    w2 = (torch.randn(Co, Ci2, 1, 1, generator=g) / Ci2 ** 0.5).float()
    b = (torch.randn(Co, generator=g) * 0.1).float()
    ref = torch.relu(F.conv2d(h.double(), w1.double(), b.double()) + F.conv2d(x2.double(), w2.double(), stride=stride2))
    ref = _nhwc(ref)
    wcat = torch.cat([w1.reshape(Co, -1), w2.reshape(Co, -1)], 1).reshape(Co, Ci + Ci2, 1, 1).contiguous()
    p6 = nat.pack_conv_weight_x6(wcat.to(DEV))
    y = nat.conv2d_dual_nhwc(_nhwc(h).to(DEV), _nhwc(x2).to(DEV), stride2, p6, b.to(DEV), Co, relu=True)
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    e = (y.cpu().double() - ref).abs().max().item()
    assert e <= 1e-5 * scale, (e, scale)


@pytest.mark.parametrize("Ci,Co,Co2,stride", [(64, 64, 256, 1), (128, 128, 512, 1), (256, 64, 256, 2)])
def test_x6_chain_bit_identical_to_two_launches(Ci, Co, Co2, stride):
    """bev_conv2d_chain_x6_f32 (conv2 -> conv3 + residual, h2 split in LDS) == the two split-bf16 launches."""
    g = torch.Generator().manual_seed(Ci + Co2)
    N, H, W = 2, 25, 37
    x = torch.randn(N, H, W, Ci, generator=g).to(DEV)
    w2 = (torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5).to(DEV)
    w3 = (torch.randn(Co2, Co, 1, 1, generator=g) / Co ** 0.5).to(DEV)
    b2, b3 = (torch.randn(Co, generator=g) * 0.1).to(DEV), (torch.randn(Co2, generator=g) * 0.1).to(DEV)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    res = torch.randn(N, Ho, Wo, Co2, generator=g).to(DEV)
    p2, p3 = nat.pack_conv_weight_x6(w2), nat.pack_conv_weight_x6(w3)
    h2 = nat.conv2d_nhwc_x6(x, p2, b2, Co, 3, 3, stride, 1, 1, 1)
    ref = nat.conv2d_nhwc_x6(h2, p3, b3, Co2, 1, 1, 1, 0, 1, 1, residual=res)
    got = nat.conv2d_chain_nhwc(x, p2, b2, Co, 3, 3, stride, 1, 1, p3, b3, Co2, 1, residual=res)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_x6_chain_dual_bit_identical_to_two_launches():
    """bev_conv2d_chain_dual_x6_f32 (layer1 block 0: conv2 -> [conv3 | downsample], h2 split in LDS, the shortcut
    operand split in registers) == the split conv2 launch + the split dual tail launch."""
    g = torch.Generator().manual_seed(3)
    N, H, W, Ci, Co, Co2 = 2, 25, 37, 64, 64, 256
    x = torch.randn(N, H, W, Ci, generator=g).to(DEV)        # conv2 input (conv1's output)
    xb = torch.randn(N, H, W, 64, generator=g).to(DEV)       # block input (the downsample's operand)
    w2 = (torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5).to(DEV)
    w3 = (torch.randn(Co2, Co + 64, 1, 1, generator=g) / (Co + 64) ** 0.5).to(DEV)
    b2, b3 = (torch.randn(Co, generator=g) * 0.1).to(DEV), (torch.randn(Co2, generator=g) * 0.1).to(DEV)
    p2, p3 = nat.pack_conv_weight_x6(w2), nat.pack_conv_weight_x6(w3)
    h2 = nat.conv2d_nhwc_x6(x, p2, b2, Co, 3, 3, 1, 1, 1, 1)
    ref = nat.conv2d_dual_nhwc(h2, xb, 1, p3, b3, Co2, relu=True)
    got = nat.conv2d_chain_dual_nhwc(x, p2, b2, Co, 3, 3, 1, 1, 1, xb, 1, p3, b3, Co2, 1)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("Ci,Co,Co2,stride,N,H,W", [(64, 64, 256, 1, 2, 25, 37), (128, 128, 512, 1, 2, 25, 37),
                                                    (64, 64, 256, 2, 1, 31, 20), (64, 64, 256, 1, 3, 7, 130)])
def test_x6_chain_pre_split_operand_bit_identical(Ci, Co, Co2, stride, N, H, W):
    """The chain with conv2's operand handed over split (conv1's ys planes -> LDS-DMA staging, k_conv_x6s CHAIN)
    == the chain splitting the fp32 operand per tap (k_conv_x6b CHAIN), bit for bit; ragged M (the last tile's
    rows past M), W past one 128-row tile, stride 2."""
    g = torch.Generator().manual_seed(5 * Ci + Co2 + H)
    x = torch.randn(N, H, W, Ci, generator=g).to(DEV)
    w2 = (torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5).to(DEV)
    w3 = (torch.randn(Co2, Co, 1, 1, generator=g) / Co ** 0.5).to(DEV)
    b2, b3 = (torch.randn(Co, generator=g) * 0.1).to(DEV), (torch.randn(Co2, generator=g) * 0.1).to(DEV)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    res = torch.randn(N, Ho, Wo, Co2, generator=g).to(DEV)
    p2, p3 = nat.pack_conv_weight_x6(w2), nat.pack_conv_weight_x6(w3)
    ref = nat.conv2d_chain_nhwc(x, p2, b2, Co, 3, 3, stride, 1, 1, p3, b3, Co2, 1, residual=res)
    got = nat.conv2d_chain_nhwc(nat.split3(x), p2, b2, Co, 3, 3, stride, 1, 1, p3, b3, Co2, 1, residual=res)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_x6_chain_dual_pre_split_operand_bit_identical():
    """bev_conv2d_chain_dual_x6_f32 with conv2's operand pre-split == with it fp32 (layer1 block 0 shape)."""
    g = torch.Generator().manual_seed(31)
    N, H, W, Ci, Co, Co2 = 2, 27, 45, 64, 64, 256
    x = torch.randn(N, H, W, Ci, generator=g).to(DEV)
    xb = torch.randn(N, H, W, 64, generator=g).to(DEV)
    w2 = (torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5).to(DEV)
    w3 = (torch.randn(Co2, Co + 64, 1, 1, generator=g) / (Co + 64) ** 0.5).to(DEV)
    b2, b3 = (torch.randn(Co, generator=g) * 0.1).to(DEV), (torch.randn(Co2, generator=g) * 0.1).to(DEV)
    p2, p3 = nat.pack_conv_weight_x6(w2), nat.pack_conv_weight_x6(w3)
    ref = nat.conv2d_chain_dual_nhwc(x, p2, b2, Co, 3, 3, 1, 1, 1, xb, 1, p3, b3, Co2, 1)
    got = nat.conv2d_chain_dual_nhwc(nat.split3(x), p2, b2, Co, 3, 3, 1, 1, 1, xb, 1, p3, b3, Co2, 1)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("Co3,dual,split_out,N,H,W", [(64, False, True, 2, 25, 37), (128, False, False, 1, 31, 70),
                                                      (64, True, True, 2, 27, 45), (128, False, True, 3, 7, 130)])
def test_x6_chain_next_conv_bit_identical(Co3, dual, split_out, N, H, W):
    """bev_conv2d_chain_next_x6_f32 (a pre-split chain that also runs the next block's 1x1 conv in its epilogue, conv3
    computed transposed): y == the pre-split chain's y, and h3 == bev_conv2d_x6_f32 over y (split or fp32 output),
    bit for bit -- ragged M, 7-pixel-row images.  The dual (block 0) form is refused (BEV_ERR_ARGS)."""
    g = torch.Generator().manual_seed(Co3 + 3 * H + dual)
    Ci, Co, Co2 = 64, 64, 256
    x = torch.randn(N, H, W, Ci, generator=g).to(DEV)
    w2 = (torch.randn(Co, Ci, 3, 3, generator=g) / (9 * Ci) ** 0.5).to(DEV)
    w3 = (torch.randn(Co2, Co + (64 if dual else 0), 1, 1, generator=g) / Co ** 0.5).to(DEV)
    wn = (torch.randn(Co3, Co2, 1, 1, generator=g) / Co2 ** 0.5).to(DEV)
    b2, b3 = (torch.randn(Co, generator=g) * 0.1).to(DEV), (torch.randn(Co2, generator=g) * 0.1).to(DEV)
    bn = (torch.randn(Co3, generator=g) * 0.1).to(DEV)
    p2, p3, pn = nat.pack_conv_weight_x6(w2), nat.pack_conv_weight_x6(w3), nat.pack_conv_weight_x6(wn)
    xs = nat.split3(x)
    if dual:
        xb = torch.randn(N, H, W, 64, generator=g).to(DEV)
        with pytest.raises(nat.HipError):
            nat.conv2d_chain_next_nhwc(xs, p2, b2, Co, 3, 3, 1, 1, 1, p3, b3, Co2, 1, pn, bn, Co3, 1, x2=xb,
                                       split3_out=split_out)
        return
    else:
        res = torch.randn(N, H, W, Co2, generator=g).to(DEV)
        ref = nat.conv2d_chain_nhwc(xs, p2, b2, Co, 3, 3, 1, 1, 1, p3, b3, Co2, 1, residual=res)
        y, h3 = nat.conv2d_chain_next_nhwc(xs, p2, b2, Co, 3, 3, 1, 1, 1, p3, b3, Co2, 1, pn, bn, Co3, 1, residual=res,
                                           split3_out=split_out)
    ref3 = nat.conv2d_nhwc_x6(ref, pn, bn, Co3, 1, 1, 1, 0, 1, 1, split_out=split_out)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    if split_out:
        assert torch.equal(h3.planes, ref3.planes)
    else:
        assert torch.equal(h3, ref3)


def test_x6_resnet50_encoder_fused_next_conv1_bit_identical():
    """The ResNet-50 encoder with the layer1 chains running the next block's conv1 (resnet.FUSE_NEXT_CONV1, default)
    == with every conv1 its own launch, bit for bit."""
    from models.encoders import resnet
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(2)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(DEV)
    imgs = torch.randn(2, 3, 3, 120, 200, device=DEV)
    old = resnet.FUSE_NEXT_CONV1
    try:
        with torch.no_grad(), nat.conv_arith_mode("bf16x6"):
            resnet.FUSE_NEXT_CONV1 = False
            ref = enc(imgs).float().clone()
            resnet.FUSE_NEXT_CONV1 = True
            got = enc(imgs).float().clone()
    finally:
        resnet.FUSE_NEXT_CONV1 = old
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_x6_resnet50_encoder_split_chain_bit_identical():
    """The ResNet-50 encoder with conv1 -> chain edges pre-split (resnet.SPLIT_CHAIN, the default) == with them fp32."""
    from models.encoders import resnet
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(1)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(DEV)
    imgs = torch.randn(1, 3, 3, 96, 160, device=DEV)
    old = resnet.SPLIT_CHAIN
    try:
        with torch.no_grad(), nat.conv_arith_mode("bf16x6"):
            resnet.SPLIT_CHAIN = False
            ref = enc(imgs).float().clone()
            resnet.SPLIT_CHAIN = True
            got = enc(imgs).float().clone()
    finally:
        resnet.SPLIT_CHAIN = old
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_x6_resnet50_encoder_matches_f32_path():
    """The ResNet-50 CNNEncoder (the bench's trunk) in the split-bf16 arithmetic vs the exact-f32 MFMA chains."""
    from models.encoders.cnn_encoder import CNNEncoder
    torch.manual_seed(0)
    enc = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False).eval().to(DEV)
    imgs = torch.randn(1, 3, 3, 96, 160, device=DEV)
    with torch.no_grad():
        with nat.conv_arith_mode("f32"):
            ref = enc(imgs).float().clone()
        with nat.conv_arith_mode("bf16x6"):
            got = enc(imgs).float().clone()
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4 * scale)


@pytest.mark.parametrize("N,H,W,Co,relu", [(2, 45, 140, 64, True), (1, 1080, 1920, 64, True), (1, 33, 70, 40, False)],
                         ids=["ragged", "bench-frame", "co40-norelu"])
def test_stem_x6_vs_float64_and_exact_stem(N, H, W, Co, relu):
    """The ResNet stem on the split arithmetic (bev_conv2d_stem_x6_f32: 7x7 / s2 / p3 over NCHW Ci = 3) against the
    float64 conv of the fp32 operands, with the x6 bar (max error <= 1e-5 max|ref|) and no less accurate than the
    exact-f32 stem kernel (bev_conv2d_f32 with the NCHW loader) within 4x -- ragged tiles (Ho, Wo not multiples of
    8 / 64), one full 1080p image, and Co < 64."""
    x, w, b = _case(N, H, W, 3, Co, 7, 99 + Co)
    x32, w32, b32 = x.float(), w.float(), b.float()
    ref = _nhwc(_ref(x32.double(), w32.double(), b32.double(), 2, 3, 1, 1 if relu else 0))
    xd, bd = x32.to(DEV), b32.to(DEV)
    y6 = nat.conv2d_stem_x6(xd, nat.pack_conv_weight_x6(w32.to(DEV)), bd, Co, relu)
    yf = nat.conv2d_nhwc(xd, nat.pack_conv_weight(w32.to(DEV)), bd, Co, 7, 7, 2, 3, relu, in_nchw=True)
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    e6, ef = (y6.cpu().double() - ref).abs(), (yf.cpu().double() - ref).abs()
    assert torch.isfinite(y6).all()
    assert e6.max().item() <= 1e-5 * scale, (e6.max().item(), scale)
    assert e6.max().item() <= 4 * ef.max().item() + 1e-7 * scale, (e6.max().item(), ef.max().item())


@pytest.mark.parametrize("N,H,W", [(2, 45, 140), (3, 37, 131), (1, 1080, 1920), (2, 8, 8)],
                         ids=["ragged", "odd-sizes", "bench-frame", "one-tile"])
def test_stem_pool_x6_bit_identical_to_stem_then_maxpool(N, H, W):
    """The stem with timm's max-pool fused into its epilogue (bev_conv2d_stem_pool_x6_f32: tile seams exported and
    folded in by k_stem_pool_seams) equals bev_conv2d_stem_x6_f32 (ReLU) + bev_maxpool2d_nhwc_f32(3, 2, 1) bit for bit
    -- ragged and odd image sizes (pooled rows / columns past a tile, seams on both axes and their corners), several
    images, one 1080p frame, an image smaller than one tile."""
    x, w, b = _case(N, H, W, 3, 64, 7, 321 + H)
    xd, bd = x.float().to(DEV), b.float().to(DEV)
    packed = nat.pack_conv_weight_x6(w.float().to(DEV))
    ref = nat.maxpool_nhwc(nat.conv2d_stem_x6(xd, packed, bd, 64, True), 3, 2, 1)
    got = nat.conv2d_stem_pool_x6(xd, packed, bd)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), (got - ref).abs().max().item()
