"""EfficientNet-B3 trunk (timm-compatible module names) executed by the HIP kernels.

The reference's per-camera backbone is `timm.create_model(name, pretrained,
features_only=True)` (cnn_encoder.py:26) and CNNEncoder keeps
`feats_list[out_index]` (cnn_encoder.py:41-42, out_index=2).  BASELINE
config 4 names `efficientnet_b3`.  timm is an unpinned dependency absent from
this image, so the graph is restated from timm's published definition of
efficientnet_b3 (channel multiplier 1.2, depth multiplier 1.4, SiLU, SE with
rd = block-input channels / 4, symmetric padding, BN eps 1e-5) with timm's
parameter names (conv_stem / bn1 / blocks.S.B.{conv_dw,bn1,se,conv_pw,bn2} for
the depthwise-separable stage, {conv_pw,bn1,conv_dw,bn2,se,conv_pwl,bn3} for
inverted residuals), so a timm state_dict loads unchanged.  Parity with timm
itself is therefore UNPINNED; the kernels are pinned against a torch fp32
reference of the same weights (oracle/backbone_ref.py, tests/).

features_only feature indices (timm feature_info, 'bottleneck' location):
0 -> blocks.0 (24 ch, stride 2), 1 -> blocks.1 (32, 4), 2 -> blocks.2 (48, 8),
3 -> blocks.4 (136, 16), 4 -> blocks.6 (384, 32).

Execution (eval): NHWC on the device; stem / pointwise convs are MFMA
implicit GEMMs with BN folded and SiLU in the epilogue (bev_conv2d_f32,
act=2), the depthwise convs are `bev_dwconv2d_f32` (BN folded, SiLU, SE
squeeze partials fused), the SE gate is `bev_se_gate_f32`, and the excitation
`x * gate` is applied inside the projection conv's operand load (`bev_conv2d_chscale_f32`), which also adds
the skip in its epilogue.

Training (model.train()): the same graph on autograd nodes with native backward kernels (trunk_grad.py:
ConvBNTrain with SiLU, DWConvBNTrain, SqueezeExcite); BN with batch statistics.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

import bev_native as _nat
from .resnet import FoldedConv

__all__ = ["EfficientNet", "efficientnet_b0", "efficientnet_b1", "efficientnet_b2", "efficientnet_b3",
           "EFFICIENTNETS", "make_divisible"]

FEATURE_STAGE = {0: 0, 1: 1, 2: 2, 3: 4, 4: 6}  # features_only index -> last stage executed


def make_divisible(v, divisor=8, min_value=None, round_limit=0.9):
    """timm.layers.make_divisible."""
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < round_limit * v:
        new_v += divisor
    return new_v


class SqueezeExcite(nn.Module):
    def __init__(self, chs, rd):
        super().__init__()
        self.conv_reduce = nn.Conv2d(chs, rd, 1, bias=True)
        self.act1 = nn.SiLU(inplace=True)
        self.conv_expand = nn.Conv2d(rd, chs, 1, bias=True)
        self.gate = nn.Sigmoid()


class DepthwiseSeparableConv(nn.Module):
    def __init__(self, in_chs, out_chs, k, stride, se_ratio):
        super().__init__()
        self.has_skip = stride == 1 and in_chs == out_chs
        self.conv_dw = nn.Conv2d(in_chs, in_chs, k, stride, k // 2, groups=in_chs, bias=False)
        self.bn1 = nn.BatchNorm2d(in_chs)
        self.se = SqueezeExcite(in_chs, round(in_chs * se_ratio))
        self.conv_pw = nn.Conv2d(in_chs, out_chs, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_chs)


class InvertedResidual(nn.Module):
    def __init__(self, in_chs, out_chs, k, stride, exp_ratio, se_ratio):
        super().__init__()
        mid = make_divisible(in_chs * exp_ratio)
        self.has_skip = stride == 1 and in_chs == out_chs
        self.conv_pw = nn.Conv2d(in_chs, mid, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(mid)
        self.conv_dw = nn.Conv2d(mid, mid, k, stride, k // 2, groups=mid, bias=False)
        self.bn2 = nn.BatchNorm2d(mid)
        self.se = SqueezeExcite(mid, round(mid * se_ratio / exp_ratio))  # se_from_exp=False
        self.conv_pwl = nn.Conv2d(mid, out_chs, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(out_chs)


# (block type, repeats, kernel, stride, expansion, channels) of EfficientNet-B0; se 0.25 everywhere
_ARCH_B0 = [("ds", 1, 3, 1, 1, 16), ("ir", 2, 3, 2, 6, 24), ("ir", 2, 5, 2, 6, 40), ("ir", 3, 3, 2, 6, 80),
            ("ir", 3, 5, 1, 6, 112), ("ir", 4, 5, 2, 6, 192), ("ir", 1, 3, 1, 6, 320)]


class FoldedDW:
    """Depthwise conv + eval BN folded into tap-major weights [K*K, C] and a bias, cached on device."""

    def __init__(self, conv: nn.Conv2d, bn: nn.BatchNorm2d):
        self.fc = FoldedConv(conv, bn)
        self._key = None
        self.wt = self.bias = None

    def prepare(self, device):
        key = tuple((t.data_ptr(), t._version) for t in self.fc._tensors()) + (str(device),)
        if key == self._key:
            return
        w, b = self.fc.folded(device)  # [C, 1, K, K]
        C, _, K, _ = w.shape
        self.wt = w.reshape(C, K * K).t().contiguous()
        self.bias = b.contiguous().float()
        self._key = key

    def __call__(self, x, want_psum):
        self.prepare(x.device)
        c = self.fc.conv
        return _nat.dwconv2d_nhwc(x, self.wt, self.bias, c.kernel_size[0], c.stride[0], c.padding[0], _nat.ACT_SILU,
                                  want_psum=want_psum)


class EfficientNet(nn.Module):
    def __init__(self, channel_multiplier: float, depth_multiplier: float):
        super().__init__()
        stem = make_divisible(32 * channel_multiplier)
        self.conv_stem = nn.Conv2d(3, stem, 3, 2, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(stem)
        stages, cin = [], stem
        for kind, r, k, s, e, c in _ARCH_B0:
            cout = make_divisible(c * channel_multiplier)
            reps = int(math.ceil(r * depth_multiplier))
            blocks = []
            for i in range(reps):
                stride = s if i == 0 else 1
                if kind == "ds":
                    blocks.append(DepthwiseSeparableConv(cin, cout, k, stride, 0.25))
                else:
                    blocks.append(InvertedResidual(cin, cout, k, stride, e, 0.25))
                cin = cout
            stages.append(nn.Sequential(*blocks))
        self.blocks = nn.Sequential(*stages)
        self.feature_channels = [self.blocks[FEATURE_STAGE[i]][-1].bn2.num_features
                                 if isinstance(self.blocks[FEATURE_STAGE[i]][-1], DepthwiseSeparableConv)
                                 else self.blocks[FEATURE_STAGE[i]][-1].bn3.num_features for i in range(5)]
        self._folded = {}
        # the expansion 1x1 convs on the split-bf16 kernels: measured slower (r06q A/B, B3 encoder ms per 2-frame step:
        # split 13.81, exact-f32 13.67), so off
        self.x6_expand = False
        self.stem3 = True  # the stem on its vector-ALU kernel (bev_conv2d_stem3_f32) instead of the implicit GEMM
        self.pw_stream = True  # eval: the wide tiny-K expansions on k_pw_mfma too (see forward_features_nhwc)
        self.ir_fuse = True  # eval: expansion + depthwise conv of an inverted residual as one kernel (_ir_fused)
        self._stem3_key = None

    def _fc(self, conv, bn):
        """Pointwise / stem convs: exact-f32 kernels.  The trunk is HBM-bound; its Ci % 16 == 0 pointwise convs on the
        split-bf16 kernels measured slower (r03: EfficientNet-B3 bench 109.7 vs 112.9 frames/s)."""
        k = id(conv)
        if k not in self._folded:
            self._folded[k] = FoldedConv(conv, bn)
        return self._folded[k]

    def _stem(self, x):
        """conv_stem -> bn1 -> SiLU: the vector-ALU stem kernel (bev_conv2d_stem3_f32) for the timm 3x3 / s2 / p1
        shape when `stem3`, else the generic implicit GEMM (in_nchw)."""
        c = self.conv_stem
        fc = self._fc(c, self.bn1)
        if not (self.stem3 and c.in_channels == 3 and c.kernel_size == (3, 3) and c.stride == (2, 2)
                and c.padding == (1, 1) and c.groups == 1 and c.dilation == (1, 1)
                and c.out_channels in (32, 40, 48, 64)):
            return fc(x, relu=_nat.ACT_SILU, in_nchw=True)
        key = tuple((t.data_ptr(), t._version) for t in fc._tensors()) + (str(x.device),)
        if self._stem3_key != key:
            w, b = fc.folded(x.device)
            self._stem3_w = w.permute(1, 2, 3, 0).reshape(27, c.out_channels).contiguous()  # [(ci, ky, kx)][Co]
            self._stem3_b = b.contiguous().float()
            self._stem3_key = key
        return _nat.conv2d_stem3(x, self._stem3_w, self._stem3_b, _nat.ACT_SILU)

    def _ir_fusable(self, blk, x) -> bool:
        return self.ir_fused_block(blk, x.shape[-1])

    def ir_fused_block(self, blk, cin: int) -> bool:
        """The inverted residual's expansion + depthwise conv take the fused kernel (bev_ir_expand_dw_f32) for a
        `cin`-channel input (eval path)?"""
        if not isinstance(blk, InvertedResidual):
            return False
        pw, dw = blk.conv_pw, blk.conv_dw
        return (self.ir_fuse and not self.x6_expand and cin in (16, 24, 32, 40, 48)
                and pw.out_channels % 48 == 0 and pw.kernel_size == (1, 1) and pw.stride == (1, 1)
                and dw.kernel_size[0] == dw.kernel_size[1] and dw.kernel_size[0] in (3, 5) and dw.stride[0] in (1, 2)
                and dw.stride[0] == dw.stride[1] and dw.padding == (dw.kernel_size[0] // 2,) * 2
                and dw.groups == dw.in_channels == pw.out_channels and dw.dilation == (1, 1))

    def _ir_fused(self, blk, x):
        fc, fdw = self._fc(blk.conv_pw, blk.bn1), self._fdw(blk.conv_dw, blk.bn2)
        fdw.prepare(x.device)
        key = ("irw", id(blk.conv_pw))
        tkey = tuple((t.data_ptr(), t._version) for t in fc._tensors()) + (str(x.device),)
        ent = self._folded.get(key)
        if ent is None or ent[0] != tkey:
            w, b = fc.folded(x.device)
            ent = (tkey, w.reshape(w.shape[0], -1).contiguous(), b.contiguous().float())
            self._folded[key] = ent
        dw = blk.conv_dw
        return _nat.ir_expand_dw(x, ent[1], ent[2], fdw.wt, fdw.bias, dw.kernel_size[0], dw.stride[0])

    def _fc_expand(self, conv, bn):
        """The inverted-residual expansion (1x1, Ci -> 6 Ci, SiLU): on the split-bf16 kernels (bev_conv2d_x6_f32, fp32
        class) when `x6_expand` and the arithmetic is bf16x6 and Ci % 16 == 0, else as _fc."""
        if not self.x6_expand:
            return self._fc(conv, bn)
        k = ("x6", id(conv))
        if k not in self._folded:
            self._folded[k] = FoldedConv(conv, bn, split_ok=True)
        return self._folded[k]

    def _fdw(self, conv, bn):
        k = ("dw", id(conv))
        if k not in self._folded:
            self._folded[k] = FoldedDW(conv, bn)
        return self._folded[k]

    def _gate(self, se: SqueezeExcite, y, psum):
        """SqueezeExcite gate sigmoid(conv_expand(SiLU(conv_reduce(mean(y))))) [N, C]; the excitation
        y * gate is applied by the following projection conv's operand loader (bev_conv2d_chscale_f32)."""
        w1 = se.conv_reduce.weight.detach().reshape(se.conv_reduce.out_channels, -1).float()
        w2 = se.conv_expand.weight.detach().reshape(se.conv_expand.out_channels, -1).float()
        return _nat.se_gate(psum, y.shape[1] * y.shape[2], w1, se.conv_reduce.bias.detach().float(), w2,
                            se.conv_expand.bias.detach().float())

    def _project(self, conv, bn, y, gate, residual):
        C = y.shape[-1]
        if C % 32 == 0 or C % 4 == 0:  # fast / contiguous 1x1 loader: fold the excitation in
            return self._fc(conv, bn)(y, relu=_nat.ACT_NONE, residual=residual, ascale=gate)
        return self._fc(conv, bn)(_nat.channel_scale_(y, gate), relu=_nat.ACT_NONE, residual=residual)

    def _block(self, blk, x):
        if isinstance(blk, DepthwiseSeparableConv):
            y, ps = self._fdw(blk.conv_dw, blk.bn1)(x, want_psum=True)
            return self._project(blk.conv_pw, blk.bn2, y, self._gate(blk.se, y, ps), x if blk.has_skip else None)
        y, ps = self._ir_fused(blk, x) if self._ir_fusable(blk, x) else (None, None)
        if y is None:
            h = self._fc_expand(blk.conv_pw, blk.bn1)(x, relu=_nat.ACT_SILU)
            y, ps = self._fdw(blk.conv_dw, blk.bn2)(h, want_psum=True)
        return self._project(blk.conv_pwl, blk.bn3, y, self._gate(blk.se, y, ps), x if blk.has_skip else None)

    def unexecuted_parameter_names(self, out_index: int):
        """Parameters of the stages past features_only[out_index]: never run, so never given a gradient
        (DistributedDataParallel must not wait for them)."""
        last = FEATURE_STAGE[out_index]
        return [f"blocks.{si}.{n}" for si in range(last + 1, len(self.blocks))
                for n, _ in self.blocks[si].named_parameters()]

    def forward_features_nhwc(self, x: torch.Tensor, out_index: int) -> torch.Tensor:
        """x: images [N,3,H,W] NCHW fp32 on the device -> NHWC features_only[out_index]."""
        if out_index not in FEATURE_STAGE:
            raise IndexError(f"efficientnet feature index {out_index} out of range 0..4")
        if self.training:  # torch semantics: train-mode BN uses batch statistics, with or without autograd
            return self._forward_train(x, out_index)
        y = self._stem(x)
        # inference: every tiny-K (Ci 24-48) 1x1 conv on the wave-streaming k_pw_mfma (BEV_TUNE_CONV_PW_SMALL 3), the
        # wide expansions included; training keeps the default (2: narrow outputs only), whose k order the float64
        # gradient bounds were set on (bev_conv.hip try_pw_mfma)
        with torch.no_grad(), _nat.tuned(CONV_PW_SMALL=3 if self.pw_stream else 2):
            for si in range(FEATURE_STAGE[out_index] + 1):
                for blk in self.blocks[si]:
                    y = self._block(blk, y)
        return y

    def _forward_train(self, x: torch.Tensor, out_index: int) -> torch.Tensor:
        """Training (model.train()): every conv + BN (+ SiLU) (+ skip), depthwise conv and SqueezeExcite is one
        autograd node on the native forward / backward kernels; BN with batch statistics (or running statistics
        for BN modules in eval()), like timm's trunk in the reference's train.py:222."""
        from .trunk_grad import ConvBNTrain
        y = ConvBNTrain.apply(x, self.conv_stem.weight, self.bn1.weight, self.bn1.bias, self.conv_stem, self.bn1, 2,
                              True, None)
        for si in range(FEATURE_STAGE[out_index] + 1):
            for blk in self.blocks[si]:
                y = _train_block(blk, y)
        return y


def _train_block(blk, y):
    """timm DepthwiseSeparableConv / InvertedResidual forward on the training autograd nodes (trunk_grad)."""
    from .trunk_grad import ConvBNTrain, DWConvBNTrain, SqueezeExcite
    se = blk.se
    res = y if blk.has_skip else None
    if isinstance(blk, DepthwiseSeparableConv):
        h = DWConvBNTrain.apply(y, blk.conv_dw.weight, blk.bn1.weight, blk.bn1.bias, blk.conv_dw, blk.bn1, 2)
        h = SqueezeExcite.apply(h, se.conv_reduce.weight, se.conv_reduce.bias, se.conv_expand.weight,
                                se.conv_expand.bias)
        return ConvBNTrain.apply(h, blk.conv_pw.weight, blk.bn2.weight, blk.bn2.bias, blk.conv_pw, blk.bn2, 0, False,
                                 res)
    h = ConvBNTrain.apply(y, blk.conv_pw.weight, blk.bn1.weight, blk.bn1.bias, blk.conv_pw, blk.bn1, 2, False, None)
    h = DWConvBNTrain.apply(h, blk.conv_dw.weight, blk.bn2.weight, blk.bn2.bias, blk.conv_dw, blk.bn2, 2)
    h = SqueezeExcite.apply(h, se.conv_reduce.weight, se.conv_reduce.bias, se.conv_expand.weight, se.conv_expand.bias)
    return ConvBNTrain.apply(h, blk.conv_pwl.weight, blk.bn3.weight, blk.bn3.bias, blk.conv_pwl, blk.bn3, 0, False, res)


def efficientnet_b0():
    """configs/wildtrack.yaml:8 (the reference's main training config)."""
    return EfficientNet(channel_multiplier=1.0, depth_multiplier=1.0)


def efficientnet_b1():
    return EfficientNet(channel_multiplier=1.0, depth_multiplier=1.1)


def efficientnet_b2():
    return EfficientNet(channel_multiplier=1.1, depth_multiplier=1.2)


def efficientnet_b3():
    """BASELINE config 4."""
    return EfficientNet(channel_multiplier=1.2, depth_multiplier=1.4)


EFFICIENTNETS = {"efficientnet_b0": efficientnet_b0, "efficientnet_b1": efficientnet_b1,
                 "efficientnet_b2": efficientnet_b2, "efficientnet_b3": efficientnet_b3}
