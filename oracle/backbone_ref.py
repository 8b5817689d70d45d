"""torch fp32 CPU reference of the backbone graphs (TEST INFRASTRUCTURE ONLY).

Restates, with plain torch CPU ops, what timm's `features_only` ResNet
computes up to feature index `out_index` (cnn_encoder.py:26,41-42) followed
by the encoder's 1x1 projection (cnn_encoder.py:43-46), reading the weights
of our timm-named module (models/encoders/resnet.py) so both sides use the
same parameters.  BatchNorm runs unfused (F.batch_norm; eval statistics, or batch statistics
with the running-stat update when the BN module is in training mode) -- the HIP path folds eval
BN into the conv, so the comparison is tolerance-based (fp32 order of
accumulation differs; rtol 1e-4 per SURVEY.md §8d).  Parity with timm itself
is unpinned (timm is absent offline).

Used by tests/ and by bench.py's cpu_baseline leg only.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _cbr(x, conv, bn, relu=True, act=F.relu):
    y = F.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding)
    if bn is not None:
        y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training,
                         bn.momentum if bn.momentum is not None else 0.0, bn.eps)
    return act(y) if relu else y


def resnet_features(net, x, out_index: int, grad: bool = False, act=F.relu):
    """features_only[out_index] of a timm-named ResNet `net` on NCHW x (any device; CPU in practice).
    BN follows each module's mode (eval: running statistics; training: batch statistics + running-stat
    update); with grad=True autograd records the graph (reference for the native trunk backward).
    `act` replaces every ReLU (in execution order), e.g. by the native run's masks for gradient checks."""
    with torch.set_grad_enabled(grad):
        y = _cbr(x, net.conv1, net.bn1, act=act)
        if out_index == 0:
            return y
        y = F.max_pool2d(y, 3, 2, 1)
        for li, layer in enumerate((net.layer1, net.layer2, net.layer3, net.layer4), start=1):
            for blk in layer:
                sc = x_in = y
                if blk.downsample is not None:
                    sc = _cbr(x_in, blk.downsample[0], blk.downsample[1], relu=False)
                chain = blk.convs()
                z = x_in
                for idx, (conv, bn, _) in enumerate(chain):
                    last = idx == len(chain) - 1
                    z = _cbr(z, conv, bn, relu=not last, act=act)
                y = act(z + sc)
            if li == out_index:
                return y
        return y


def _bn(y, bn):
    return F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training,
                        bn.momentum if bn.momentum is not None else 0.0, bn.eps)


def _se(y, se):
    s = y.mean((2, 3), keepdim=True)
    s = F.silu(F.conv2d(s, se.conv_reduce.weight, se.conv_reduce.bias))
    s = F.conv2d(s, se.conv_expand.weight, se.conv_expand.bias)
    return y * torch.sigmoid(s)


def _dw(y, conv):
    return F.conv2d(y, conv.weight, None, conv.stride, conv.padding, groups=conv.groups)


def efficientnet_features(net, x, out_index: int, grad: bool = False):
    """features_only[out_index] of a timm-named EfficientNet `net` (timm DepthwiseSeparableConv /
    InvertedResidual / SqueezeExcite forward, _efficientnet_blocks.py) on NCHW x.  BN follows each module's
    mode; with grad=True autograd records the graph (reference for the native trunk backward)."""
    from models.encoders.efficientnet import FEATURE_STAGE, DepthwiseSeparableConv
    with torch.set_grad_enabled(grad):
        y = F.silu(_bn(F.conv2d(x, net.conv_stem.weight, None, 2, 1), net.bn1))
        for si in range(FEATURE_STAGE[out_index] + 1):
            for blk in net.blocks[si]:
                sc = y
                if isinstance(blk, DepthwiseSeparableConv):
                    z = _se(F.silu(_bn(_dw(y, blk.conv_dw), blk.bn1)), blk.se)
                    z = _bn(F.conv2d(z, blk.conv_pw.weight), blk.bn2)
                else:
                    z = F.silu(_bn(F.conv2d(y, blk.conv_pw.weight), blk.bn1))
                    z = _se(F.silu(_bn(_dw(z, blk.conv_dw), blk.bn2)), blk.se)
                    z = _bn(F.conv2d(z, blk.conv_pwl.weight), blk.bn3)
                y = z + sc if blk.has_skip else z
        return y


def encoder_forward(enc, images):
    """CNNEncoder.forward restated on torch CPU ops: [B,V,3,H,W] -> [B,V,C,Hf,Wf] (contiguous)."""
    B, V = images.shape[:2]
    x = images.reshape(B * V, *images.shape[2:])
    with torch.no_grad():
        if enc._use_timm:
            if hasattr(enc.backbone, "conv_stem"):
                f = efficientnet_features(enc.backbone, x, enc.out_index)
            else:
                f = resnet_features(enc.backbone, x, enc.out_index)
            y = F.conv2d(f, enc.proj.weight, enc.proj.bias)
        else:
            s = enc.backbone
            y = F.relu(F.conv2d(F.relu(F.conv2d(x, s[0].weight, s[0].bias, 2, 1)), s[2].weight, s[2].bias, 2, 1))
    return y.reshape(B, V, *y.shape[1:])
