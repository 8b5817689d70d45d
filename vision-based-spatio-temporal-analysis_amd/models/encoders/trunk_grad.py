"""Autograd for the backbone trunk on the HIP kernels (training; BASELINE config 3).

The reference trains the timm trunk through torch autograd (train.py:249-255; its optimizer holds
exactly the trunk parameters, quirk Q2).  Here every conv + BN (+ residual) (+ ReLU) of the trunk is
ONE autograd node, `ConvBNAct`, whose forward is the same folded MFMA conv as inference and whose
backward runs native kernels:

  dz  = dy * (y > 0)                         bev_relu_bwd_f32 (from the saved output)
  dx  = conv(dilate(dz), flip(W_f)^T)        bev_dilate_nhwc_f32 + bev_conv2d_f32 (stride 1, MFMA)
  dWf = sum_m dz (x) im2col(x)               bev_conv_wgrad_f32
  dbf = sum_m dz                             bev_colsum_f32
  residual gradient = dz

BatchNorm follows the module's own mode, as torch does:

* `bn.training` (model.train(), what the reference's train.py:222 runs): BATCH statistics --
  `ConvBNTrain`: z = conv(x, W) (MFMA), per-channel batch mean / variance of z
  (bev_batchnorm_train_fwd_f32, which also updates running_mean / running_var with the momentum
  rule and counts num_batches_tracked; under autocast the fp16 conv writes per-tile partials in its
  epilogue instead, bev_conv2d_h16_bnstats_f32 + bev_batchnorm_finalize_tiles_f32, so z is not read
  back), y = act(z * scale + shift (+ residual)) (bev_batchnorm_apply_f32); backward
  bev_batchnorm_bwd_f32 (dz, d residual, dgamma, dbeta; a ReLU layer without residual takes its mask
  from z, so y is neither saved nor read) then the conv dgrad / wgrad above.
* `bn.eval()` inside a training model (the usual way to freeze BN when fine-tuning): running
  statistics folded into the conv -- `ConvBNAct`: W_f = W * s, b_f = beta - mean * s with
  s = gamma / sqrt(var + eps), so dW = dWf * s, dgamma = (sum dWf * W - mean * dbf) / sqrt(var + eps),
  dbeta = dbf (tiny parameter-sized ops).

`MaxPool` backward: bev_maxpool2d_bwd_nhwc_f32.
"""
from __future__ import annotations

import torch
import torch.nn as nn

import bev_native as _nat

__all__ = ["ConvBNAct", "ConvBNTrain", "DWConvBNTrain", "SqueezeExcite", "ConvAct", "MaxPool", "conv_bn_act",
           "conv_act"]


EPILOGUE_BN_STATS = True  # autocast: train-mode BN statistics from the fp16 conv's epilogue (else a pass over z)


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d):
    with torch.no_grad():
        w = conv.weight.detach().float()
        r = torch.rsqrt(bn.running_var.detach().float() + bn.eps)
        s = bn.weight.detach().float() * r
        wf = (w * s.view(-1, 1, 1, 1)).contiguous()
        bf = (bn.bias.detach().float() - bn.running_mean.detach().float() * s).contiguous()
    return wf, bf, s, r


class GradSink:
    """Carries a bottleneck's identity-shortcut gradient from its last conv node to its first conv node, which the
    backward runs later (it is upstream): the first conv's input-gradient conv then adds it in its epilogue instead
    of autograd summing the block input's two gradients in a separate pass (a full read-read-write of the block
    input's size: 0.2-0.5 ms per block at the bench size).  It assumes the backward runs through the whole block
    (conv3's node sets the hand-off, conv1's node consumes it); after a partial backward that stops between the two
    (torch.autograd.grad with inputs inside the block) the hand-off is simply not consumed -- the gradient it carries
    belongs to the block input, which that backward does not ask for -- and the block's next forward clears it."""
    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None


def _dgrad(dz: torch.Tensor, wf: torch.Tensor, H: int, W: int, stride: int, pad: int,
           residual: torch.Tensor = None) -> torch.Tensor:
    """Input gradient of conv(x, wf, stride, pad) for x [N,H,W,Ci] NHWC, as a stride-1 MFMA conv (+ residual, a
    gradient of x from elsewhere, added in the epilogue)."""
    Co, Ci, K, _ = wf.shape
    wt = wf.flip(2, 3).transpose(0, 1).contiguous()  # [Ci][Co][K][K]
    packed = _nat.pack_conv_weight(wt)
    zero = torch.zeros(Ci, device=dz.device, dtype=torch.float32)
    q = K - 1 - pad
    if stride == 1:
        return _nat.conv2d_nhwc(dz, packed, zero, Ci, K, K, 1, q, False, residual=residual)
    if K == 1 and pad == 0 and Ci % 4 == 0 and 256 % (Ci // 4) == 0:
        # 1x1 strided (the downsample): y = dz W on the Ho x Wo pixels, placed at the strided positions of the
        # gradient (+ the residual) -- no zero-inserted map, a quarter of the MACs at stride 2
        y = _nat.conv2d_nhwc(dz, packed, zero, Ci, 1, 1, 1, 0, False)
        return _nat.place_strided(y, stride, H, W, residual)
    if residual is not None:
        return _dgrad(dz, wf, H, W, stride, pad).add_(residual)
    N, Ho, Wo, _ = dz.shape
    ry, rx = (H + 2 * pad - K) % stride, (W + 2 * pad - K) % stride
    Hd, Wd = stride * (Ho - 1) + 1 + 2 * q + ry, stride * (Wo - 1) + 1 + 2 * q + rx
    d = _nat.dilate_nhwc(dz, stride, q, q, Hd, Wd)
    return _nat.conv2d_nhwc(d, packed, zero, Ci, K, K, 1, 0, False)


def _stem_operand(x: torch.Tensor) -> torch.Tensor:
    """The NCHW input of an in_nchw conv (the stem) as the NHWC operand of its weight gradient: 3-channel images
    straight to 4-channel pixels with a zero channel (the float4 kernel's operand; no separate pad copy)."""
    return _nat.nchw_to_nhwc4(x) if x.shape[1] <= 4 else _nat.nchw_to_nhwc(x)


class ConvBNAct(torch.autograd.Function):
    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, weight, gamma, beta, conv, bn, relu: bool, in_nchw: bool, residual, sink_in=None,
                sink_out=None):
        ctx.sinks = (sink_in, sink_out)
        if sink_in is not None:
            sink_in.grad = None  # a stale hand-off of an earlier, partial backward (conv1's backward never ran)
        wf, bf, s, r = _fold(conv, bn)
        k, st, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        y = _nat.conv2d_nhwc(x, _nat.pack_conv_weight(wf), bf, conv.out_channels, k, k, st, p, relu,
                             residual=residual, in_nchw=in_nchw)
        ctx.save_for_backward(x, y if relu else None, wf, s, r, weight)
        ctx.meta = (conv, bn, relu, in_nchw, residual is not None)
        return y

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        x, y, wf, s, r, weight = ctx.saved_tensors
        conv, bn, relu, in_nchw, has_res = ctx.meta
        k, st, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        dy = dy.contiguous().float()
        dz = _nat.relu_bwd(dy, y) if relu else dy
        sink_in, sink_out = ctx.sinks
        dres = dz if has_res else None
        if sink_out is not None and dres is not None:  # the block's first conv adds it (GradSink)
            sink_out.grad, dres = dres, None
        res_in = None
        if sink_in is not None:
            res_in, sink_in.grad = sink_in.grad, None
        xn = _stem_operand(x) if in_nchw else x
        H, W = xn.shape[1], xn.shape[2]
        dx = _dgrad(dz, wf, H, W, st, p, residual=res_in) if (ctx.needs_input_grad[0] and not in_nchw) else (
            res_in if ctx.needs_input_grad[0] else None)
        dwf = _nat.conv_wgrad(xn, dz, k, k, st, p)
        if dwf.shape[1] != wf.shape[1]:  # the zero channel of the 4-channel stem operand
            dwf = dwf[:, :wf.shape[1]].contiguous()
        dbf = _nat.colsum(dz)
        dw = dwf * s.view(-1, 1, 1, 1)
        ds = (dwf * weight.detach().float()).sum((1, 2, 3)) - bn.running_mean.detach().float() * dbf
        dgamma = ds * r
        return dx, dw, dgamma, dbf, None, None, None, None, dres, None, None


def _bn_affine(bn: nn.BatchNorm2d, z: torch.Tensor, gamma, beta, tiles: torch.Tensor = None):
    """(mean, rstd, scale, shift, frozen) of BN over NHWC z: batch statistics (+ running-stat update) when the
    module is training -- from the conv epilogue's per-tile partials when given (`tiles`, z is not read), else by a
    pass over z -- and its running statistics (constants) when it is in eval()."""
    if bn.training:
        track = bn.track_running_stats and bn.running_mean is not None
        if track:
            bn.num_batches_tracked.add_(1)
        momentum = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
        rm, rv = (bn.running_mean, bn.running_var) if track else (None, None)
        if tiles is not None:
            mean, rstd, scale, shift = _nat.batchnorm_finalize_tiles(tiles, z.numel() // z.shape[-1], gamma, beta, rm,
                                                                     rv, bn.eps, momentum)
        else:
            mean, rstd, scale, shift = _nat.batchnorm_train_fwd(z, gamma, beta, rm, rv, bn.eps, momentum)
        return mean, rstd, scale, shift, False
    with torch.no_grad():
        mean = bn.running_mean.detach().float().contiguous()
        rstd = torch.rsqrt(bn.running_var.detach().float() + bn.eps)
        scale = (gamma.detach().float() * rstd).contiguous()
        shift = (beta.detach().float() - mean * scale).contiguous()
    return mean, rstd, scale, shift, True


class ConvBNTrain(torch.autograd.Function):
    """act(BN(conv(x, W)) (+ residual)), act 0 none / 1 ReLU / 2 SiLU; BN with batch statistics (train-mode
    BatchNorm2d) or, for a BN module in eval(), its running statistics."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, weight, gamma, beta, conv, bn, act: int, in_nchw: bool, residual, sink_in=None,
                sink_out=None):
        ctx.sinks = (sink_in, sink_out)
        if sink_in is not None:
            sink_in.grad = None  # a stale hand-off of an earlier, partial backward (conv1's backward never ran)
        k, st, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        w = weight.detach().float().contiguous()
        Co = conv.out_channels
        packed = _nat.pack_conv_weight(w)
        tiles = None
        if (EPILOGUE_BN_STATS and packed.dtype == torch.float16 and bn.training and not in_nchw and x.shape[-1] % 64 == 0
                and conv.dilation[0] == 1):  # autocast: the fp16 conv takes the BN statistics in its epilogue
            z, tiles = _nat.conv2d_nhwc_h16_bnstats(x, packed, Co, k, k, st, p)
        else:
            z = _nat.conv2d_nhwc(x, packed, torch.zeros(Co, device=x.device), Co, k, k, st, p, False, in_nchw=in_nchw)
        mean, rstd, scale, shift, frozen = _bn_affine(bn, z, gamma, beta, tiles)
        y = _nat.batchnorm_apply(z, scale, shift, residual, act)
        # ReLU without residual: the backward recomputes the mask from z (y > 0 <=> fmaf(z, scale, shift) > 0)
        ctx.save_for_backward(x, z, y if (act == 1 and residual is not None) else None, w, mean, rstd, gamma, scale,
                              shift)
        ctx.meta = (k, st, p, in_nchw, residual is not None, int(act), frozen)
        return y

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        x, z, y, w, mean, rstd, gamma, scale, shift = ctx.saved_tensors
        k, st, p, in_nchw, has_res, act, frozen = ctx.meta
        bact = _nat.ACT_RELU_FROM_Z if (act == 1 and not has_res) else act
        dz, dres, dgamma, dbeta = _nat.batchnorm_bwd(dy.float(), y, z, mean, rstd, gamma, has_res, bact, scale, shift,
                                                     frozen)
        sink_in, sink_out = ctx.sinks
        if sink_out is not None and dres is not None:  # the block's first conv adds it (GradSink)
            sink_out.grad, dres = dres, None
        res_in = None
        if sink_in is not None:
            res_in, sink_in.grad = sink_in.grad, None
        xn = _stem_operand(x) if in_nchw else x
        H, W = xn.shape[1], xn.shape[2]
        dx = _dgrad(dz, w, H, W, st, p, residual=res_in) if (ctx.needs_input_grad[0] and not in_nchw) else (
            res_in if ctx.needs_input_grad[0] else None)
        dw = _nat.conv_wgrad(xn, dz, k, k, st, p)
        if dw.shape[1] != w.shape[1]:  # the zero channel of the 4-channel stem operand
            dw = dw[:, :w.shape[1]].contiguous()
        return dx, dw, dgamma, dbeta, None, None, None, None, dres, None, None


class DWConvBNTrain(torch.autograd.Function):
    """act(BN(depthwise_conv(x, W))) for the EfficientNet trunk (timm conv_dw -> bn -> SiLU), NHWC.
    Forward: bev_dwconv2d_f32 (raw, no bias), BatchNorm kernels.  Backward: BN backward, dgrad = depthwise
    conv of the (zero-inserted) gradient with the flipped taps, wgrad = bev_dwconv_wgrad_f32."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, weight, gamma, beta, conv, bn, act: int):
        C, K, st, p = conv.out_channels, conv.kernel_size[0], conv.stride[0], conv.padding[0]
        wt = weight.detach().float().reshape(C, K * K).t().contiguous()  # [K*K, C] tap-major
        zero = torch.zeros(C, device=x.device)
        z, _ = _nat.dwconv2d_nhwc(x, wt, zero, K, st, p, _nat.ACT_NONE)
        mean, rstd, scale, shift, frozen = _bn_affine(bn, z, gamma, beta)
        y = _nat.batchnorm_apply(z, scale, shift, None, act)
        ctx.save_for_backward(x, z, y if act == 1 else None, wt, mean, rstd, gamma, scale, shift)
        ctx.meta = (K, st, p, int(act), frozen)
        return y

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        x, z, y, wt, mean, rstd, gamma, scale, shift = ctx.saved_tensors
        K, st, p, act, frozen = ctx.meta
        dz, _, dgamma, dbeta = _nat.batchnorm_bwd(dy.float(), y, z, mean, rstd, gamma, False, act, scale, shift,
                                                  frozen)
        N, H, W, C = x.shape
        dx = None
        if ctx.needs_input_grad[0]:
            wf = wt.view(K, K, C).flip(0, 1).reshape(K * K, C).contiguous()
            zero = torch.zeros(C, device=x.device)
            q = K - 1 - p
            if st == 1:
                dx, _ = _nat.dwconv2d_nhwc(dz, wf, zero, K, 1, q, _nat.ACT_NONE)
            else:
                Ho, Wo = dz.shape[1], dz.shape[2]
                ry, rx = (H + 2 * p - K) % st, (W + 2 * p - K) % st
                Hd, Wd = st * (Ho - 1) + 1 + 2 * q + ry, st * (Wo - 1) + 1 + 2 * q + rx
                dx, _ = _nat.dwconv2d_nhwc(_nat.dilate_nhwc(dz, st, q, q, Hd, Wd), wf, zero, K, 1, 0, _nat.ACT_NONE)
        dW = _nat.dwconv_wgrad(x, dz, K, st, p).t().reshape(C, 1, K, K)
        return dx, dW, dgamma, dbeta, None, None, None


class SqueezeExcite(torch.autograd.Function):
    """timm SqueezeExcite: y * sigmoid(expand(silu(reduce(mean_hw(y))))) over NHWC y.  The big-tensor work is
    native (per-image channel sums, the excitation as a channel affine); the [N, C] MLP is parameter-sized."""

    @staticmethod
    def _gate(s, w1, b1, w2, b2):
        r = torch.nn.functional.silu(s @ w1.reshape(w1.shape[0], -1).t() + b1)
        return torch.sigmoid(r @ w2.reshape(w2.shape[0], -1).t() + b2)

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, y, w1, b1, w2, b2):
        P = y.shape[1] * y.shape[2]
        s = _nat.channel_sums(y) / P
        g = SqueezeExcite._gate(s, w1.detach(), b1.detach(), w2.detach(), b2.detach()).contiguous()
        ctx.save_for_backward(y, s, g, w1, b1, w2, b2)
        return _nat.channel_affine(y, g)

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dout):
        y, s, g, w1, b1, w2, b2 = ctx.saved_tensors
        P = y.shape[1] * y.shape[2]
        dout = dout.contiguous().float()
        dg = _nat.channel_sums(dout, y)  # d gate = sum_p dout * y
        leaves = [t.detach().requires_grad_(True) for t in (s, w1, b1, w2, b2)]
        with torch.enable_grad():
            gate = SqueezeExcite._gate(*leaves)
            ds, dw1, db1, dw2, db2 = torch.autograd.grad(gate, leaves, dg)
        dy = _nat.channel_affine(dout, g, ds / P)  # dout * gate + d mean / P (broadcast over pixels)
        return dy, dw1, db1, dw2, db2


def _dgrad_h16(dz: torch.Tensor, wf: torch.Tensor, H: int, W: int, stride: int, pad: int,
               residual: torch.Tensor = None) -> torch.Tensor:
    """_dgrad under autocast with dz stored in fp16 (the fp16 conv rounds it to exactly these values)."""
    Co, Ci, K, _ = wf.shape
    packed = _nat.pack_conv_weight(wf.flip(2, 3).transpose(0, 1).contiguous())
    q = K - 1 - pad
    if stride == 1:
        return _nat.conv2d_h16_any(dz, packed, Ci, K, K, 1, q, residual=residual)
    N, Ho, Wo, _ = dz.shape
    ry, rx = (H + 2 * pad - K) % stride, (W + 2 * pad - K) % stride
    Hd, Wd = stride * (Ho - 1) + 1 + 2 * q + ry, stride * (Wo - 1) + 1 + 2 * q + rx
    d = _nat.dilate_nhwc_any(dz, stride, q, q, Hd, Wd)
    return _nat.conv2d_h16_any(d, packed, Ci, K, K, 1, 0, residual=residual)


# BottleneckTrainH16: keep the block output's ReLU mask as bytes for bn3's backward (default), or the fp32 output
# itself (A/B: tools/train_step_bench.py --no-mask-bytes; bit-identical results)
RELU_MASK_BYTES = True


class BottleneckTrainH16(torch.autograd.Function):
    """One timm Bottleneck (conv1 1x1 -> BN -> ReLU -> conv2 3x3 -> BN -> ReLU -> conv3 1x1 -> BN, + shortcut, ReLU)
    in training with batch-statistics BN under autocast(float16), as ONE autograd node, so the tensors that live
    between its layers can be stored in the precision their readers compute in:
      * y1, y2 (the ReLU outputs feeding conv2 / conv3) are read only by the fp16 convs and their weight gradients,
        which round them to fp16 -- stored in fp16 (`batchnorm_apply_half`);
      * dz1..dz3 (BN backward outputs) are read only by the fp16 dgrad convs and weight gradients -- fp16
        (`batchnorm_bwd_half`);
    both are exactly the values the fp32-stored path rounds them to, so every result is bit-identical to the
    per-layer `ConvBNTrain` chain (`tests/test_train_amp_gpu.py::test_bottleneck_h16_block_bit_identical`), with
    half the bytes on those tensors; the block output's ReLU mask is kept as bytes (1 B per 4 elements) for bn3's
    backward instead of re-reading the fp32 output twice.  The statistics come from the conv epilogues, the ReLU masks of y1 / y2 from
    z, and an identity shortcut's gradient is added in conv1's dgrad epilogue.  `sc`: the shortcut tensor (the
    downsample branch's output), or None for the identity (x).  `x_sink` (downsample blocks): the node's gradient of x
    is handed to the downsample conv's node (which consumes it as its dgrad epilogue's residual; that node's backward
    runs after this one, since it needs d sc), instead of autograd summing the two gradients of x in a separate pass."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, sc, w1, g1, b1, w2, g2, b2, w3, g3, b3, blk, x_sink=None):
        assert _nat.half_convs()
        ctx.x_sink = x_sink  # downsample block: x's gradient from this node goes to the downsample conv's dgrad
        layers = ((blk.conv1, blk.bn1), (blk.conv2, blk.bn2), (blk.conv3, blk.bn3))
        ws = (w1, w2, w3)
        gb = ((g1, b1), (g2, b2), (g3, b3))
        h = x
        saved, meta = [], []
        for i, ((conv, bn), w, (g, b)) in enumerate(zip(layers, ws, gb)):
            k, st, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            wd = w.detach().float().contiguous()
            Co = conv.out_channels
            z, tiles = _nat.conv2d_h16_any(h, _nat.pack_conv_weight(wd), Co, k, k, st, p, stats=True)
            mean, rstd, scale, shift, _ = _bn_affine(bn, z, g, b, tiles)
            if i < 2:
                y = _nat.batchnorm_apply_half(z, scale, shift, 1)
            elif RELU_MASK_BYTES:  # the block output, and its ReLU mask as bytes for the backward (not the 4-B y,
                y, mask = _nat.batchnorm_apply_mask(z, scale, shift, x if sc is None else sc)  # read twice there)
            else:
                y = mask = _nat.batchnorm_apply(z, scale, shift, x if sc is None else sc, 1)
            saved += [h, z, wd, mean, rstd, g, scale, shift]
            meta.append((k, st, p))
            h = y
        ctx.save_for_backward(*saved, mask)
        ctx.meta = (meta, sc is not None)
        return h

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        t = ctx.saved_tensors
        meta, has_sc = ctx.meta
        mask3 = t[24]
        g = dy.contiguous().float()
        grads = [None] * 3
        dres = None
        for i in (2, 1, 0):
            h, z, wd, mean, rstd, gamma, scale, shift = t[8 * i: 8 * i + 8]
            k, st, p = meta[i]
            if i == 2:
                act = _nat.ACT_RELU_MASK if mask3.dtype == torch.uint8 else 1  # mask bytes, or y itself
                dz, dres, dgm, dbt = _nat.batchnorm_bwd_half(g, mask3, z, mean, rstd, gamma, True, act, scale, shift)
            else:
                dz, _, dgm, dbt = _nat.batchnorm_bwd_half(g, None, z, mean, rstd, gamma, False,
                                                          _nat.ACT_RELU_FROM_Z, scale, shift)
            dw = _nat.conv_wgrad_h16_any(h, dz, k, k, st, p)
            res = dres if (i == 0 and not has_sc) else None
            need = i > 0 or ctx.needs_input_grad[0]
            g = _dgrad_h16(dz, wd, h.shape[1], h.shape[2], st, p, residual=res) if need else None
            grads[i] = (dw, dgm, dbt)
        dx = g
        if ctx.x_sink is not None and dx is not None:  # added in the downsample conv's dgrad epilogue instead
            ctx.x_sink.grad, dx = dx, None
        return (dx, dres if has_sc else None, *grads[0], *grads[1], *grads[2], None, None)


def bottleneck_h16_ok(blk) -> bool:
    """The BottleneckTrainH16 node applies: a 3-conv bottleneck, every BN in training mode, AMP fp16 convs active,
    channel counts the fp16-operand kernels take (Ci % 64), no dilation."""
    if not _nat.amp_half_active() or not hasattr(blk, "conv3"):
        return False
    convs = (blk.conv1, blk.conv2, blk.conv3)
    return (all(bn.training for bn in (blk.bn1, blk.bn2, blk.bn3))
            and all(c.in_channels % 64 == 0 and c.dilation[0] == 1 and c.groups == 1 and c.bias is None
                    for c in convs))


def conv_bn_act(conv: nn.Conv2d, bn: nn.BatchNorm2d, x, relu: bool, residual=None, in_nchw: bool = False,
                sink_in: GradSink = None, sink_out: GradSink = None):
    """One ResNet layer in training: batch-statistics BN when `bn.training`, else the folded frozen BN.  sink_out
    (the identity bottleneck's last conv) hands the residual's gradient to sink_in (its first conv)."""
    if bn.training:
        return ConvBNTrain.apply(x, conv.weight, bn.weight, bn.bias, conv, bn, 1 if relu else 0, in_nchw, residual,
                                 sink_in, sink_out)
    return ConvBNAct.apply(x, conv.weight, bn.weight, bn.bias, conv, bn, relu, in_nchw, residual, sink_in, sink_out)


class ConvAct(torch.autograd.Function):
    """conv2d(x, W, b) (+ ReLU) without BatchNorm -- the fallback encoder's layers (cnn_encoder.py:31-37)
    and the BEV head's plain convs: forward on the MFMA conv kernel, backward as ConvBNAct's (ReLU mask,
    dgrad as a stride-1 conv, wgrad, bias column sums)."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, weight, bias, stride: int, pad: int, relu: bool, in_nchw: bool):
        Co, Ci, k, _ = weight.shape
        w = weight.detach().float().contiguous()
        b = bias.detach().float().contiguous() if bias is not None else torch.zeros(Co, device=x.device)
        y = _nat.conv2d_nhwc(x, _nat.pack_conv_weight(w), b, Co, k, k, stride, pad, relu, in_nchw=in_nchw)
        ctx.save_for_backward(x, y if relu else None, w)
        ctx.meta = (stride, pad, relu, in_nchw, bias is not None)
        return y

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        x, y, w = ctx.saved_tensors
        stride, pad, relu, in_nchw, has_b = ctx.meta
        k = w.shape[2]
        dy = dy.contiguous().float()
        dz = _nat.relu_bwd(dy, y) if relu else dy
        xn = _nat.nchw_to_nhwc(x) if in_nchw else x
        H, W = xn.shape[1], xn.shape[2]
        dx = _dgrad(dz, w, H, W, stride, pad) if (ctx.needs_input_grad[0] and not in_nchw) else None
        dw = _nat.conv_wgrad(xn, dz, k, k, stride, pad) if ctx.needs_input_grad[1] else None
        db = _nat.colsum(dz) if (has_b and ctx.needs_input_grad[2]) else None
        return dx, dw, db, None, None, None, None


def conv_act(conv: nn.Conv2d, x, relu: bool, in_nchw: bool = False):
    return ConvAct.apply(x, conv.weight, conv.bias, conv.stride[0], conv.padding[0], relu, in_nchw)


# MaxPool: the forward keeps the window argmax bytes for the backward (default), or saves x (A/B:
# tools/train_step_bench.py --no-pool-arg; bit-identical results)
MAXPOOL_ARG = True


class MaxPool(torch.autograd.Function):
    """Max-pool (timm's stem pool).  C % 4 == 0: the forward keeps the window argmax bytes (1 B per output instead
    of the 4-B input per input element saved) and the backward gathers from them (bit-identical to the x-based
    backward); else x is saved and the backward re-scans it."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, k: int, stride: int, pad: int):
        ctx.meta = (k, stride, pad, x.shape[1], x.shape[2])
        if MAXPOOL_ARG and x.shape[-1] % 4 == 0 and k * k <= 255:
            y, arg = _nat.maxpool_fwd_arg_nhwc(x, k, stride, pad)
            ctx.save_for_backward(arg)
            ctx.arg = True
            return y
        ctx.save_for_backward(x)
        ctx.arg = False
        return _nat.maxpool_nhwc(x, k, stride, pad)

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        (t,) = ctx.saved_tensors
        k, stride, pad, H, W = ctx.meta
        dy = dy.contiguous().float()
        if ctx.arg:
            return _nat.maxpool_bwd_arg_nhwc(t, dy, H, W, k, stride, pad), None, None, None
        return _nat.maxpool_bwd_nhwc(t, dy, k, stride, pad), None, None, None
