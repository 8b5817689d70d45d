"""bev_conv2d_h16_f32: the autocast(float16) convolution (fp16 operands, fp32 accumulation) on the fp16 matrix
cores, against a float64 convolution of the fp16-rounded operands.

The products of two fp16 values are exact in fp32, so the kernel's only error is the fp32 summation order: the
bar is the worst-case fp32 summation bound K * 2^-24 * sum_k |x_k w_k| per output (K = Ci * KH * KW), and the
typical error must sit far below it (max err / sum|terms| < 2e-6).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(N, H, W, Ci, Co, K, stride, pad, dil, act, residual=False, ldy=None, seed=0):
    import bev_native as nat
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, W, Ci, generator=g)
    w = torch.randn(Co, Ci, K, K, generator=g) / (Ci * K * K) ** 0.5
    b = torch.randn(Co, generator=g)
    Ho = (H + 2 * pad - dil * (K - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (K - 1) - 1) // stride + 1
    r = torch.randn(N, Ho, Wo, Co, generator=g) if residual else None
    with nat._half_mode(True):
        packed = nat.pack_conv_weight(w.to(DEV))
    assert packed.dtype == torch.float16
    out = None
    if ldy is not None:
        out = torch.full((N, Ho, Wo, ldy), 7.0, device=DEV)
    y = nat.conv2d_nhwc_h16(x.to(DEV), packed, b.to(DEV), Co, K, K, stride, pad, dil, act,
                            residual=None if r is None else r.to(DEV), out=out)
    torch.cuda.synchronize()
    y = y.cpu().double()
    # float64 reference of the fp16-rounded operands
    xh, wh = x.half().double().permute(0, 3, 1, 2), w.half().double()
    z = F.conv2d(xh, wh, None, stride, pad, dil).permute(0, 2, 3, 1)
    mag = F.conv2d(xh.abs(), wh.abs(), None, stride, pad, dil).permute(0, 2, 3, 1)
    ref = z + b.double()
    if r is not None:
        ref = ref + r.double()
    if act == 1:
        ref = ref.clamp_min(0)
    elif act == 2:
        ref = ref * torch.sigmoid(ref)
    if ldy is not None:
        assert bool((y[..., Co:] == 7.0).all()), "columns past Co written"
        y = y[..., :Co]
    Kt = Ci * K * K
    err = (y - ref).abs()
    bound = Kt * 2.0 ** -24 * (mag + b.double().abs() + (r.double().abs() if r is not None else 0)) + 1e-6
    if act == 2:
        bound = bound * 1.2 + 1e-6
    assert bool((err <= bound).all()), float((err - bound).max())
    assert float((err / (mag + 1e-3)).max()) < 2e-6
    # and it is the fp16 arithmetic, not fp32: the fp32 conv of the raw operands differs
    z32 = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), None, stride, pad, dil).permute(0, 2, 3, 1)
    assert float((z32 - z).abs().max()) > 10 * float(err.max())


@pytest.mark.parametrize("shape", [
    dict(N=2, H=20, W=24, Ci=64, Co=128, K=3, stride=1, pad=1, dil=1, act=0),
    dict(N=1, H=17, W=33, Ci=32, Co=200, K=3, stride=2, pad=1, dil=1, act=1),
    dict(N=2, H=16, W=19, Ci=128, Co=128, K=3, stride=1, pad=2, dil=2, act=1),
    dict(N=3, H=9, W=11, Ci=96, Co=5, K=1, stride=1, pad=0, dil=1, act=0),
    dict(N=1, H=14, W=14, Ci=256, Co=64, K=1, stride=1, pad=0, dil=1, act=1, residual=True),
    dict(N=1, H=12, W=13, Ci=32, Co=40, K=3, stride=1, pad=1, dil=1, act=2),
    dict(N=1, H=10, W=10, Ci=64, Co=30, K=3, stride=1, pad=1, dil=1, act=0, ldy=64),
    dict(N=1, H=23, W=29, Ci=64, Co=64, K=7, stride=2, pad=3, dil=1, act=1),
], ids=lambda d: f"{d['Ci']}to{d['Co']}k{d['K']}s{d['stride']}d{d['dil']}a{d['act']}")
def test_conv_h16_vs_float64_of_rounded_operands(shape):
    _case(**shape)


@pytest.mark.parametrize("Ci,K,stride,Co", [(64, 3, 1, 192), (128, 3, 2, 192), (256, 1, 1, 192), (64, 3, 1, 64),
                                            (256, 1, 1, 40), (128, 3, 2, 64)])
def test_conv_h16_kernels_bit_identical(Ci, K, stride, Co):
    """The 64-deep-step kernel (default for Ci % 64 == 0; 64-column tiles when Co <= 64), the same with 128-column
    tiles always (CONV_H16_KERNEL 2) or 64-column tiles always (3), and the 32-deep one (1) sum every output in the
    same order; and fp16-stored
    operands (bev_conv2d_h16_ex_f32 x_half) give the same bits as the fp32 operand they round."""
    import bev_native as nat
    g = torch.Generator().manual_seed(Ci + Co)
    N, H, W = 2, 19, 27
    x = torch.randn(N, H, W, Ci, generator=g).to(DEV)
    w = (torch.randn(Co, Ci, K, K, generator=g) / (Ci * K * K) ** 0.5).to(DEV)
    b = torch.randn(Co, generator=g).to(DEV)
    with nat._half_mode(True):
        packed = nat.pack_conv_weight(w)
    outs = []
    for kern in (0, 1, 2, 3):
        with nat.tuned(CONV_H16_KERNEL=kern):
            outs.append(nat.conv2d_nhwc_h16(x, packed, b, Co, K, K, stride, K // 2, 1, 1))
    torch.cuda.synchronize()
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    # fp16-stored operand (the conv_h16_any path), default and 128-column kernels, against the fp32 operand
    z0 = nat.conv2d_nhwc_h16(x, packed, b, Co, K, K, stride, K // 2, 1, 0)
    for kern in (0, 2):
        with nat.tuned(CONV_H16_KERNEL=kern):
            z = nat.conv2d_h16_any(x.half(), packed, Co, K, K, stride, K // 2, bias=b)
        assert torch.equal(z, z0)


def test_conv_h16_rejects_bad_arguments():
    import bev_native as nat
    x = torch.zeros(1, 4, 4, 48, device=DEV)
    with nat._half_mode(True):
        assert nat.pack_conv_weight(torch.zeros(8, 48, 3, 3, device=DEV)).dtype == torch.float32  # 48 % 32 != 0
        packed = nat.pack_conv_weight(torch.zeros(8, 64, 3, 3, device=DEV))
    with pytest.raises(nat.HipError):  # Ci of x is not the panel's and not a multiple of 32
        nat.conv2d_nhwc_h16(x, packed, torch.zeros(8, device=DEV), 8, 3, 3, 1, 1)
    with pytest.raises(nat.HipError):
        nat.conv2d_nhwc_h16(x, packed.float(), torch.zeros(8, device=DEV), 8, 3, 3, 1, 1)


def test_amp_functions_take_half_convs_only_under_autocast():
    """The native Functions pick the fp16 panel exactly when called under autocast(float16) with
    AMP_HALF_CONVS on."""
    import bev_native as nat
    from models.encoders import trunk_grad
    conv = torch.nn.Conv2d(64, 64, 3, padding=1, bias=True).to(DEV)
    x = torch.randn(1, 8, 8, 64, device=DEV, requires_grad=True)
    seen = []
    orig = nat.conv2d_nhwc_h16

    def spy(*a, **k):
        seen.append(True)
        return orig(*a, **k)

    nat.conv2d_nhwc_h16 = spy
    try:
        trunk_grad.conv_act(conv, x, True).sum().backward()
        assert not seen
        with torch.autocast("cuda", dtype=torch.float16):
            y = trunk_grad.conv_act(conv, x, True)
        assert y.dtype == torch.float32 and len(seen) == 1
        y.sum().backward()
        assert len(seen) == 2  # the dgrad conv too
        old, nat.AMP_HALF_CONVS = nat.AMP_HALF_CONVS, False
        try:
            with torch.autocast("cuda", dtype=torch.float16):
                trunk_grad.conv_act(conv, x, True)
        finally:
            nat.AMP_HALF_CONVS = old
        assert len(seen) == 2
    finally:
        nat.conv2d_nhwc_h16 = orig


@pytest.mark.parametrize("shape", [
    dict(N=2, H=20, W=24, Ci=64, Co=128, K=3, stride=1, pad=1, dil=1),
    dict(N=1, H=33, W=17, Ci=32, Co=200, K=3, stride=2, pad=1, dil=1),
    dict(N=2, H=16, W=19, Ci=128, Co=36, K=3, stride=1, pad=2, dil=2),
    dict(N=3, H=9, W=11, Ci=96, Co=8, K=1, stride=1, pad=0, dil=1),
    dict(N=1, H=40, W=40, Ci=256, Co=64, K=1, stride=1, pad=0, dil=1),
    dict(N=1, H=110, W=110, Ci=256, Co=256, K=3, stride=1, pad=1, dil=1),  # 7 K steps per workgroup in the 64-px kernel
], ids=lambda d: f"{d['Ci']}to{d['Co']}k{d['K']}s{d['stride']}d{d['dil']}h{d['H']}")
@pytest.mark.parametrize("kern", [0, 1], ids=["wgrad64", "wgrad32"])
def test_wgrad_h16_vs_float64_of_rounded_operands(shape, kern):
    """conv_wgrad_ex under half_convs(): fp16 operands, fp32 sums (split over pixels, float atomics) against the
    float64 weight gradient of the fp16-rounded operands; relative to sum |terms| < 2e-6.  kern: bev_tune
    CONV_H16_KERNEL 0 = k_wgrad_h16b (64-pixel steps, two in flight), 1 = k_wgrad_h16 (32-pixel steps)."""
    import bev_native as nat
    N, H, W, Ci, Co, K = shape["N"], shape["H"], shape["W"], shape["Ci"], shape["Co"], shape["K"]
    st, pad, dil = shape["stride"], shape["pad"], shape["dil"]
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, H, W, Ci, generator=g)
    Ho = (H + 2 * pad - dil * (K - 1) - 1) // st + 1
    Wo = (W + 2 * pad - dil * (K - 1) - 1) // st + 1
    dz = torch.randn(N, Ho, Wo, Co, generator=g) * 1e-3
    with nat._half_mode(True), nat.tuned(CONV_H16_KERNEL=kern):
        dw = nat.conv_wgrad_ex(x.to(DEV), dz.to(DEV), K, pad, dil, stride=st)
    torch.cuda.synchronize()
    xh, dh = x.half().double().permute(0, 3, 1, 2), dz.half().double().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xh, (Co, Ci, K, K), dh, st, pad, dil)
    mag = torch.nn.grad.conv2d_weight(xh.abs(), (Co, Ci, K, K), dh.abs(), st, pad, dil)
    err = (dw.cpu().double() - ref).abs()
    assert dw.shape == (Co, Ci, K, K)
    assert float((err / (mag + 1e-12)).max()) < 2e-6
    # and it is the fp16 arithmetic: the float64 gradient of the raw operands differs by more
    raw = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (Co, Ci, K, K), dz.double().permute(0, 3, 1, 2),
                                      st, pad, dil)
    assert float((raw - ref).abs().max()) > 10 * float(err.max())


@pytest.mark.parametrize("shape", [
    dict(N=2, H=20, W=24, Ci=64, Co=128, K=3, stride=1, pad=1, dil=1),
    dict(N=1, H=33, W=17, Ci=32, Co=200, K=3, stride=2, pad=1, dil=1),
    dict(N=1, H=24, W=72, Ci=160, Co=512, K=3, stride=1, pad=1, dil=1),   # the head's conv1: taps inside 128-k tiles
    dict(N=1, H=16, W=70, Ci=512, Co=128, K=3, stride=1, pad=2, dil=2),   # head conv2 (dilated)
    dict(N=2, H=16, W=19, Ci=128, Co=36, K=3, stride=1, pad=2, dil=2),    # Co % 8 != 0: the register-transpose kernel
    dict(N=3, H=9, W=11, Ci=96, Co=8, K=1, stride=1, pad=0, dil=1),
    dict(N=1, H=45, W=60, Ci=256, Co=64, K=1, stride=2, pad=0, dil=1),    # the trunk's strided 1x1 downsample
    dict(N=1, H=110, W=110, Ci=64, Co=64, K=3, stride=1, pad=1, dil=1),   # many 64-pixel steps per workgroup
], ids=lambda d: f"{d['Ci']}to{d['Co']}k{d['K']}s{d['stride']}d{d['dil']}h{d['H']}")
@pytest.mark.parametrize("x_half", [True, False], ids=["xh", "xf"])
def test_wgrad_h16_fp16_gradient_vs_float64(shape, x_half):
    """conv_wgrad_h16_any with the gradient stored in fp16 (the AMP training step's dgrad / BatchNorm-backward
    outputs) and x in fp16 or fp32: k_wgrad_h16c (natural [pixel][channel] LDS images, transposing
    ds_read_b64_tr_b16 fragment reads) where Ci, Co % 8 == 0, else k_wgrad_h16b; against the float64 weight gradient
    of the fp16 operands, relative to sum |terms| < 2e-6."""
    import bev_native as nat
    N, H, W, Ci, Co, K = shape["N"], shape["H"], shape["W"], shape["Ci"], shape["Co"], shape["K"]
    st, pad, dil = shape["stride"], shape["pad"], shape["dil"]
    g = torch.Generator().manual_seed(Ci + Co + K)
    x = torch.randn(N, H, W, Ci, generator=g)
    Ho = (H + 2 * pad - dil * (K - 1) - 1) // st + 1
    Wo = (W + 2 * pad - dil * (K - 1) - 1) // st + 1
    dz = (torch.randn(N, Ho, Wo, Co, generator=g) * 1e-3).half()
    xd = x.to(DEV).half() if x_half else x.to(DEV)
    dw = nat.conv_wgrad_h16_any(xd, dz.to(DEV), K, K, st, pad, dilation=dil)
    torch.cuda.synchronize()
    xh, dh = x.half().double().permute(0, 3, 1, 2), dz.double().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xh, (Co, Ci, K, K), dh, st, pad, dil)
    mag = torch.nn.grad.conv2d_weight(xh.abs(), (Co, Ci, K, K), dh.abs(), st, pad, dil)
    err = (dw.cpu().double() - ref).abs()
    assert dw.shape == (Co, Ci, K, K)
    assert float((err / (mag + 1e-12)).max()) < 2e-6


@pytest.mark.parametrize("N,H,W,Ci,K,dil,Co,res", [(2, 19, 70, 64, 3, 1, 128, False), (1, 21, 96, 128, 3, 2, 64, True),
                                                   (1, 9, 40, 64, 3, 1, 192, True)])
def test_conv_h16_wide_rows_bit_identical(N, H, W, Ci, K, dil, Co, res):
    """Row tiles spanning image rows (Wo 40-96, ragged last tile), dilation 2, a residual and ReLU: the 64-deep kernel
    (k_conv_h16b, buffer staging) gives the bits of the 32-deep one (CONV_H16_KERNEL 1) with fp32 operands, and of
    the fp16-stored operand path.  (Round 5 also measured 2-D 8 x 16 output tiles for these convs: slower on every
    spatial shape, profiles/r05y_conv_h16_tile2d_ab.txt, not kept.)"""
    import bev_native as nat
    g = torch.Generator().manual_seed(Ci + Co + W)
    x = torch.randn(N, H, W, Ci, generator=g).to(DEV)
    w = (torch.randn(Co, Ci, K, K, generator=g) / (Ci * K * K) ** 0.5).to(DEV)
    b = torch.randn(Co, generator=g).to(DEV)
    r = torch.randn(N, H, W, Co, generator=g).to(DEV) if res else None
    with nat._half_mode(True):
        packed = nat.pack_conv_weight(w)
    pad = dil * (K // 2)
    z2d = nat.conv2d_nhwc_h16(x, packed, b, Co, K, K, 1, pad, dil, 1, residual=r)
    with nat.tuned(CONV_H16_KERNEL=1):
        z32 = nat.conv2d_nhwc_h16(x, packed, b, Co, K, K, 1, pad, dil, 1, residual=r)
    zh = nat.conv2d_h16_any(x.half(), packed, Co, K, K, 1, pad, bias=b, residual=r, dilation=dil)
    torch.cuda.synchronize()
    assert torch.equal(z2d, z32)
    assert torch.equal(torch.relu(zh), z2d)
