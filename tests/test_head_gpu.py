"""Native BEV head against a float64 torch restatement of the reference head.

The reference head is detector.py:7-62: 3 x [3x3 conv (no bias), GroupNorm(32), ReLU] (512 / 128 / 128 channels,
dilation 2 in the middle conv) + three 3x3 heads.  These tests check each native piece (dilated conv with the
GroupNorm affine + ReLU applied in the operand load, dilated weight gradient, GroupNorm forward / backward) and
the whole BEVDetector, forward and backward, against torch's own F.conv2d / F.group_norm evaluated in float64 on
the CPU with the same parameters.

Tolerance (fp32 MFMA vs float64, sums over up to 9 * 512 terms): |got - ref| <= 1e-4 * |ref| + 1e-4 * max|ref|
for activations, 1e-3 / 1e-3 for gradients (sums over every BEV cell).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def close(got, ref, rtol, atol_frac, what):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    assert got.shape == ref.shape, (what, tuple(got.shape), tuple(ref.shape))
    atol = atol_frac * max(float(ref.abs().max()), 1e-12)
    excess = ((got - ref).abs() - (atol + rtol * ref.abs())).max()
    assert float(excess) <= 0, f"{what}: max excess {float(excess):.3g}, max|d| {float((got - ref).abs().max()):.3g}"


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2)


@pytest.mark.parametrize("Ci,Co,dil,affine", [(160, 512, 1, False), (512, 128, 2, True), (128, 128, 1, True),
                                              (128, 5, 1, True), (32, 64, 3, False), (24, 16, 2, False)])
def test_conv_ex_matches_torch(Ci, Co, dil, affine):
    import bev_native as nat
    g = torch.Generator().manual_seed(Ci * 7 + Co + dil)
    N, H, W = 2, 13, 37
    x = torch.randn(N, Ci, H, W, generator=g)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / (3 * Ci ** 0.5)
    b = torch.randn(Co, generator=g)
    scale = torch.rand(N, Ci, generator=g) + 0.5 if affine else None
    shift = torch.randn(N, Ci, generator=g) if affine else None
    xin = x.double()
    if affine:
        xin = torch.relu(xin * scale.double()[:, :, None, None] + shift.double()[:, :, None, None])
    ref = F.conv2d(xin, w.double(), b.double(), padding=dil, dilation=dil)
    # write into a wider channels-last buffer (ldy > Co) to check the strided epilogue
    ldy = Co + 4 if Co % 4 == 0 else Co
    out = torch.full((N, H, W, ldy), 7.0, device=DEV)
    y = nat.conv2d_nhwc_ex(nhwc(x).to(DEV), nat.pack_conv_weight(w.to(DEV)), b.to(DEV), Co, 3, dil, dil,
                           in_scale=scale.to(DEV) if affine else None, in_shift=shift.to(DEV) if affine else None,
                           in_relu=affine, out=out)
    torch.cuda.synchronize()
    close(nchw(y[..., :Co]), ref, 1e-4, 1e-4, "conv_ex")
    if ldy > Co:
        assert bool((y[..., Co:] == 7.0).all()), "conv wrote past Co in the wide output buffer"


@pytest.mark.parametrize("Ci,Co,dil", [(128, 128, 2), (32, 512, 1), (128, 5, 1), (24, 16, 3)])
def test_conv_wgrad_ex_matches_torch(Ci, Co, dil):
    import bev_native as nat
    g = torch.Generator().manual_seed(Ci + Co * 3 + dil)
    N, H, W = 2, 11, 29
    x = torch.randn(N, Ci, H, W, generator=g)
    dz = torch.randn(N, Co, H, W, generator=g)
    w = torch.zeros(Co, Ci, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double(), w, padding=dil, dilation=dil).backward(dz.double())
    dW = nat.conv_wgrad_ex(nhwc(x).to(DEV), nhwc(dz).to(DEV), 3, dil, dil)
    close(dW, w.grad, 1e-4, 1e-4, "wgrad_ex")


@pytest.mark.parametrize("C", [512, 128])
def test_groupnorm_fwd_bwd_matches_torch(C):
    import bev_native as nat
    g = torch.Generator().manual_seed(C)
    N, H, W, G, eps = 2, 17, 23, 32, 1e-5
    x = torch.randn(N, C, H, W, generator=g) * 3 + 1
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    dy = torch.randn(N, C, H, W, generator=g)
    xd = x.double().requires_grad_(True)
    gd = gamma.double().requires_grad_(True)
    bd = beta.double().requires_grad_(True)
    ref = torch.relu(F.group_norm(xd, G, gd, bd, eps))
    ref.backward(dy.double())
    xg = nhwc(x).to(DEV)
    mean, rstd, scale, shift = nat.groupnorm_fwd(xg, G, gamma.to(DEV), beta.to(DEV), eps)
    y = nat.groupnorm_apply(xg, scale, shift, True)
    close(nchw(y), ref, 1e-4, 1e-5, "groupnorm fwd")
    dx, dg, db = nat.groupnorm_bwd(xg, nhwc(dy).to(DEV), G, mean, rstd, gamma.to(DEV), scale, shift, True)
    close(nchw(dx), xd.grad, 1e-3, 1e-4, "groupnorm dx")
    close(dg, gd.grad, 1e-4, 1e-5, "groupnorm dgamma")
    close(db, bd.grad, 1e-4, 1e-5, "groupnorm dbeta")


def reference_head(det, x, masks=None):
    """detector.py:47-62 in float64 on the CPU with det's parameters.  `masks` (one per GroupNorm + ReLU) replaces
    the ReLU decision by the native forward's: an element within fp32 rounding of 0 may switch sides between
    float64 and fp32 and then carries its full upstream gradient on one side only -- the forward outputs are
    checked separately, the masks only keep the gradient comparison well-conditioned."""
    p = {k: v.detach().double().cpu().requires_grad_(True) for k, v in det.named_parameters()}
    a = x
    for j, (i, d) in enumerate(((0, 1), (3, 2), (6, 1))):
        a = F.conv2d(a, p[f"stem.{i}.weight"], padding=d, dilation=d)
        a = F.group_norm(a, 32, p[f"stem.{i + 1}.weight"], p[f"stem.{i + 1}.bias"], 1e-5)
        a = torch.relu(a) if masks is None else a * masks[j]
    hm = F.conv2d(a, p["heatmap_head.weight"], p["heatmap_head.bias"], padding=1)
    off = F.conv2d(a, p["offset_head.weight"], p["offset_head.bias"], padding=1)
    size = F.conv2d(a, p["size_head.weight"], p["size_head.bias"], padding=1)
    return {"heatmap_logits": hm, "offset_raw": off, "size_raw": size}, p


def native_masks(det, x):
    """ReLU masks of the native training forward (same kernels BEVDetector.forward_nhwc runs)."""
    from models.heads import detector as D
    a = torch.zeros(x.shape[0], x.shape[2], x.shape[3], det.input_channels_padded, device=DEV)
    a[..., :x.shape[1]] = x.permute(0, 2, 3, 1).to(DEV)
    masks = []
    with torch.no_grad():
        for conv, gn in zip(*det._convs()):
            a = D._GroupNormReLU.apply(D._HeadConv.apply(a, conv.weight, None, conv.dilation[0]), gn.weight, gn.bias,
                                       gn.eps)
            masks.append((a > 0).permute(0, 3, 1, 2).double().cpu())
    return masks


@pytest.mark.parametrize("cin", [18, 130])
def test_detector_forward_backward_matches_torch(cin):
    from models.heads.detector import BEVDetector
    torch.manual_seed(cin)
    det = BEVDetector(in_channels=cin, bev_bounds=(-6.0, 6.0, -2.0, 2.0), bev_size=(20, 44)).to(DEV)
    with torch.no_grad():  # non-trivial offset head (the CenterNet init zeroes it)
        det.offset_head.weight.normal_(0, 0.05)
        for m in (det.stem[1], det.stem[4], det.stem[7]):
            m.weight.uniform_(0.5, 1.5)
            m.bias.normal_(0, 0.2)
    x = torch.randn(2, cin, 20, 44)
    ref, p = reference_head(det, x.double())

    with torch.no_grad():
        out = det(x.to(DEV))
    for k in ref:
        close(out[k], ref[k], 1e-4, 1e-4, "inference " + k)

    det.zero_grad()
    xg = x.to(DEV).requires_grad_(True)
    out = det(xg)
    g = torch.Generator().manual_seed(1)
    upstream = {k: torch.randn(ref[k].shape, generator=g) for k in ref}
    loss = sum((out[k] * upstream[k].to(DEV)).sum() for k in ref)
    loss.backward()
    for k in ref:
        close(out[k], ref[k], 1e-4, 1e-4, "train " + k)
    xr = x.double().requires_grad_(True)
    ref2, p = reference_head(det, xr, native_masks(det, x))
    sum((ref2[k] * upstream[k].double()).sum() for k in ref2).backward()
    for name, prm in det.named_parameters():
        close(prm.grad, p[name].grad, 1e-3, 1e-3, "grad " + name)
    close(xg.grad, xr.grad, 1e-3, 1e-3, "grad input")


def test_detector_decode_roundtrip():
    """forward -> decode on an input with a planted peak returns a box at that cell."""
    from models.heads.detector import BEVDetector
    det = BEVDetector(in_channels=18, bev_bounds=(-6.0, 6.0, -2.0, 2.0), bev_size=(16, 48)).to(DEV)
    hm = torch.zeros(1, 1, 16, 48, device=DEV)
    hm[0, 0, 5, 17] = 0.9
    off = torch.full((1, 2, 16, 48), 0.5, device=DEV)
    size = torch.full((1, 2, 16, 48), 2.0, device=DEV)
    boxes, scores = det.decode(hm, off, size, conf_thresh=0.4, nms_dist_m=0.5)
    assert boxes[0].shape == (1, 4) and abs(float(scores[0][0]) - 0.9) < 1e-6
    np.testing.assert_allclose(boxes[0][0].cpu().numpy(), [-6 + 17.5 * 0.25, -2 + 5.5 * 0.25, 0.5, 0.5], rtol=1e-6)
