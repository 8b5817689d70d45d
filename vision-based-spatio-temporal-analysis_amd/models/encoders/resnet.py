"""ResNet backbones (timm-compatible module names) executed by the HIP conv kernels.

The reference builds its per-camera backbone with
`timm.create_model(name, pretrained, features_only=True)` (cnn_encoder.py:26)
and keeps `feats_list[out_index]` (cnn_encoder.py:41-42, out_index=2 ->
the stride-8 `layer2` output).  timm is an unpinned third-party dependency
absent from this image, so the graphs are restated here with timm's
parameter names (conv1 / bn1 / layer1..4 / downsample.0/1), so that a timm
state_dict loads unchanged.  Parity with timm itself is therefore UNPINNED;
the conv kernels are pinned against a torch fp32 reference of the same
weights (oracle/backbone_ref.py, tests/test_backbone_gpu.py).

Training (train mode with gradients): one autograd node per conv + BN on the native
forward / backward kernels (trunk_grad.py); BN uses batch statistics when its module is in
training mode (timm under model.train()), the folded running statistics when it is in eval().

Execution (inference / eval mode): activations stay channels-last (NHWC) on
the device; every conv+BN(+residual)(+ReLU) is ONE `bev_conv2d_f32` launch
with batch-norm folded into the packed weights and bias; the stem reads the
caller's NCHW images directly.  Stages past `out_index` are not executed:
features_only returns them but CNNEncoder discards them, so skipping them
leaves the output unchanged.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn

import bev_native as _nat

__all__ = ["ResNet", "resnet18", "resnet34", "resnet50", "NATIVE_BACKBONES", "FoldedConv", "stage_of"]


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def convs(self):
        """(conv, bn, relu, residual_from) chain for the native executor."""
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, True)]


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        outplanes = planes * self.expansion
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)  # timm: stride on the 3x3
        self.bn2 = nn.BatchNorm2d(width)
        self.act2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(width, outplanes, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(outplanes)
        self.act3 = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def convs(self):
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, True), (self.conv3, self.bn3, True)]


# The ResNet stem on the split arithmetic (FoldedConv.stem_x6); False keeps the exact-f32 stem kernel.
STEM_X6 = True
# ... and, in the eval chain, with the stem max-pool fused into its epilogue (bev_conv2d_stem_pool_x6_f32,
# bit-identical; False: the stem output is written and max-pooled by its own launch)
STEM_POOL = True
# The chained bottleneck bodies (chain6 / chaintail6) take conv1's output pre-split: conv1 writes h / m / l bf16 planes
# (bev_conv2d_x6_f32 ys) and the chain stages conv2's operand by LDS-DMA with no split in its mainloop (k_conv_x6s
# CHAIN).  Bit-identical either way; False: conv1 writes fp32 and the chain splits it once per tap (k_conv_x6b).
SPLIT_CHAIN = True
# ... and such a chain over a 64-channel conv2 (the 128-row tile: layer1) also runs the NEXT block's 1x1 conv1 on the
# block output it computes (bev_conv2d_chain_next_x6_f32: the next conv1's launch and its HBM read of the block output
# disappear; bit-identical).  False: the next block runs its conv1 itself.  Off: the fusion needs conv3 in the
# transposed epilogue layout, whose per-pixel stores cost what the saved launch gains (r06p A/B, encoder ms per 2-frame
# step: fused 15.82, separate conv1 15.76, no pre-split chains 16.00).
FUSE_NEXT_CONV1 = False


class FoldedConv:
    """conv (+ eval-mode BN) folded into a packed MFMA weight panel + bias, cached on device.

    The cache is keyed on the parameters' storage and version counters, so an
    optimizer step or load_state_dict triggers a re-pack on the next call.
    With `split_ok` (the ResNet trunk and the encoder proj) an NHWC conv with Ci % 16 == 0 runs in the
    arithmetic bev_native.conv_arith() selects: "bf16x6" packs the split-bf16 panel (bev_conv2d_x6_f32), "f32"
    the exact-f32 MFMA panel (bev_conv2d_f32).  The chained bottleneck kernels always take the fp32 panel.
    """

    def __init__(self, conv: nn.Conv2d, bn: nn.BatchNorm2d = None, split_ok: bool = False):
        self.conv, self.bn = conv, bn
        self.split_ok = split_ok
        self._keys = {}
        self.packed = self.packed6 = self.bias = None

    def _tensors(self):
        ts = [self.conv.weight] + ([self.conv.bias] if self.conv.bias is not None else [])
        if self.bn is not None:
            ts += [self.bn.weight, self.bn.bias, self.bn.running_mean, self.bn.running_var]
        return ts

    def arith(self) -> str:
        c = self.conv
        if (self.split_ok and _nat.conv_arith() == "bf16x6" and c.in_channels % 16 == 0 and c.groups == 1
                and c.dilation == (1, 1)):
            return "bf16x6"
        return "f32"

    def stem_x6(self) -> bool:
        """The ResNet stem (7x7 / s2 / p3, Ci 3, Co <= 64) under the bf16x6 arithmetic takes the split-arithmetic
        stem kernel (STEM_X6, default on; off: the exact-f32 stem, fp32-tolerance equal)."""
        c = self.conv
        return (STEM_X6 and self.split_ok and _nat.conv_arith() == "bf16x6" and c.in_channels == 3
                and c.out_channels <= 64 and c.kernel_size == (7, 7) and c.stride == (2, 2) and c.padding == (3, 3)
                and c.groups == 1 and c.dilation == (1, 1))

    def prepare(self, device, arith: str = None):
        arith = arith or self.arith()
        key = tuple((t.data_ptr(), t._version) for t in self._tensors()) + (str(device),)
        if self._keys.get(arith) == key:
            return
        w, b = self.folded(device)
        with torch.no_grad():
            if arith == "bf16x6":
                self.packed6 = _nat.pack_conv_weight_x6(w.contiguous())
            else:
                self.packed = _nat.pack_conv_weight(w.contiguous())
            self.bias = b.contiguous().float()
        self._keys[arith] = key

    def folded(self, device):
        """(w OIHW, b) with eval BN folded in, on `device`."""
        with torch.no_grad():
            w = self.conv.weight.detach().to(device=device, dtype=torch.float32)
            b = (self.conv.bias.detach().to(device=device, dtype=torch.float32) if self.conv.bias is not None
                 else torch.zeros(w.shape[0], device=device))
            if self.bn is not None:
                bn = self.bn
                scale = bn.weight.detach().to(device) / torch.sqrt(bn.running_var.detach().to(device) + bn.eps)
                w = w * scale.view(-1, 1, 1, 1)
                b = bn.bias.detach().to(device) + (b - bn.running_mean.detach().to(device)) * scale
        return w, b

    def __call__(self, x, relu: bool, residual=None, in_nchw: bool = False, ascale=None, out=None,
                 split_out: bool = False):
        """x: NHWC fp32 (NCHW with in_nchw) or, in the bf16x6 arithmetic, a bev_native.Split3; split_out (bf16x6
        only) returns the result as a Split3 -- the pre-split operand of the next conv."""
        c = self.conv
        if in_nchw and self.stem_x6():  # the stem on the split arithmetic (bev_conv2d_stem_x6_f32)
            self.prepare(x.device, "bf16x6")
            return _nat.conv2d_stem_x6(x, self.packed6, self.bias, c.out_channels, relu, out=out)
        arith = "f32" if (in_nchw or ascale is not None) else self.arith()
        self.prepare(x.device, arith)
        if arith == "bf16x6":
            return _nat.conv2d_nhwc_x6(x, self.packed6, self.bias, c.out_channels, c.kernel_size[0],
                                       c.kernel_size[1], c.stride[0], c.padding[0], 1, int(relu), residual=residual,
                                       out=out, split_out=split_out)
        assert not split_out and not isinstance(x, _nat.Split3)
        return _nat.conv2d_nhwc(x, self.packed, self.bias, c.out_channels, c.kernel_size[0], c.kernel_size[1],
                                c.stride[0], c.padding[0], relu, residual=residual, in_nchw=in_nchw, ascale=ascale,
                                out=out)


class FoldedTail:
    """Bottleneck tail conv3/bn3 + downsample conv/bn (+ add + ReLU) as ONE dual-source 1x1 GEMM.

    timm's Bottleneck.forward computes act3(bn3(conv3(h)) + bn_ds(conv_ds(x))); with both
    BNs folded this is act(h (*) W3 + x[::s] (*) Wds + (b3 + bds)), a single GEMM over the
    concatenated K = [h | x[::s]] -- the shortcut tensor is never written (bev_conv2d_dual_f32).
    Summation order differs from conv-then-add: fp32-tolerance equal, not bitwise.
    """

    def __init__(self, main: FoldedConv, short: FoldedConv):
        self.main, self.short = main, short
        self._keys = {}
        self.packed = self.packed6 = self.bias = None

    @staticmethod
    def applies(blk) -> bool:
        ds = blk.downsample
        c3 = blk.conv3
        return (ds is not None and isinstance(ds[0], nn.Conv2d) and ds[0].kernel_size == (1, 1)
                and ds[0].padding == (0, 0) and c3.kernel_size == (1, 1) and c3.stride == (1, 1)
                and c3.in_channels % 32 == 0 and ds[0].in_channels % 32 == 0 and ds[0].bias is None)

    def arith(self) -> str:
        return "bf16x6" if self.main.arith() == "bf16x6" and self.short.arith() == "bf16x6" else "f32"

    def prepare(self, device, arith: str = None):
        arith = arith or self.arith()
        key = tuple((t.data_ptr(), t._version) for f in (self.main, self.short) for t in f._tensors()) + (str(device),)
        if self._keys.get(arith) == key:
            return
        w1, b1 = self.main.folded(device)
        w2, b2 = self.short.folded(device)
        with torch.no_grad():
            w = torch.cat([w1.reshape(w1.shape[0], -1), w2.reshape(w2.shape[0], -1)], 1)
            w = w.reshape(w.shape[0], w.shape[1], 1, 1).contiguous()
            if arith == "bf16x6":
                self.packed6 = _nat.pack_conv_weight_x6(w)
            else:
                self.packed = _nat.pack_conv_weight(w)
            self.bias = (b1 + b2).contiguous().float()
        self._keys[arith] = key

    def __call__(self, h, x, out=None):
        arith = self.arith()
        self.prepare(h.device, arith)
        return _nat.conv2d_dual_nhwc(h, x, self.short.conv.stride[0], self.packed6 if arith == "bf16x6" else self.packed,
                                     self.bias, self.main.conv.out_channels, relu=True, out=out)


class FoldedChain:
    """Bottleneck conv2/bn2/act2 -> conv3/bn3 (+ identity shortcut) -> act3 as ONE launch.

    timm Bottleneck.forward for a block without a downsample computes
    act3(bn3(conv3(act2(bn2(conv2(h1))))) + x); with both BNs folded, bev_conv2d_chain_f32 keeps
    the conv2 output of each workgroup's pixels (all `width` channels) in LDS and runs conv3 on it,
    so that tensor is never written to HBM.  Bit-identical to the two separate launches.
    """

    def __init__(self, c2: FoldedConv, c3: FoldedConv):
        self.c2, self.c3 = c2, c3

    @staticmethod
    def applies(blk) -> bool:
        c2, c3 = blk.conv2, blk.conv3
        return (blk.downsample is None and c2.out_channels in (64, 128) and c2.in_channels % 32 == 0
                and c2.kernel_size[0] == c2.kernel_size[1] and c2.dilation == (1, 1) and c2.groups == 1
                and c3.kernel_size == (1, 1) and c3.stride == (1, 1) and c3.padding == (0, 0)
                and c3.out_channels % 128 == 0)

    def prepare(self, device, arith: str = "f32"):
        self.c2.prepare(device, arith)
        self.c3.prepare(device, arith)

    def __call__(self, h, x, out=None, arith: str = "f32"):
        """arith "f32": bev_conv2d_chain_f32 (exact-f32 MFMA, bit-identical to the two launches); "bf16x6":
        bev_conv2d_chain_x6_f32 (the split arithmetic, h2 kept split in LDS)."""
        self.prepare(h.device, arith)
        c2 = self.c2.conv
        x6 = arith == "bf16x6"
        return _nat.conv2d_chain_nhwc(h, self.c2.packed6 if x6 else self.c2.packed, self.c2.bias, c2.out_channels,
                                      c2.kernel_size[0], c2.kernel_size[1], c2.stride[0], c2.padding[0],
                                      _nat.ACT_RELU, self.c3.packed6 if x6 else self.c3.packed, self.c3.bias,
                                      self.c3.conv.out_channels, _nat.ACT_RELU, residual=x, out=out)

    def fused(self, h, x, nxt: "FoldedConv", out=None, split_out: bool = True):
        """The split-arithmetic chain that also runs the next block's 1x1 conv1 `nxt` on its output
        (bev_conv2d_chain_next_x6_f32): returns (y, h1 of the next block)."""
        self.prepare(h.device, "bf16x6")
        nxt.prepare(h.device, "bf16x6")
        c2 = self.c2.conv
        return _nat.conv2d_chain_next_nhwc(h, self.c2.packed6, self.c2.bias, c2.out_channels, c2.kernel_size[0],
                                           c2.kernel_size[1], c2.stride[0], c2.padding[0], _nat.ACT_RELU,
                                           self.c3.packed6, self.c3.bias, self.c3.conv.out_channels, _nat.ACT_RELU,
                                           nxt.packed6, nxt.bias, nxt.conv.out_channels, _nat.ACT_RELU, residual=x,
                                           out=out, split3_out=split_out)


class FoldedChainTail:
    """Bottleneck conv2/bn2/act2 -> [conv3/bn3 + downsample conv/bn] -> act3 as ONE launch (block 0).

    bev_conv2d_chain_dual_f32: conv2's output stays in LDS and the dual-source 1x1 GEMM of
    FoldedTail (K = [h2 | x[::s]]) runs on it.  Bit-identical to conv2 followed by FoldedTail.
    """

    def __init__(self, c2: FoldedConv, tail: FoldedTail):
        self.c2, self.tail = c2, tail

    @staticmethod
    def applies(blk) -> bool:
        c2 = blk.conv2
        # the shortcut operand streams from L2 once per 64-column chunk: measured (r02k, 7 x 1080p ResNet-50)
        # layer1 block 0 (64-channel shortcut) 1333 -> 1203 us, layer2 block 0 (256 channels) 1335 -> 1440 us
        return (FoldedTail.applies(blk) and blk.downsample[0].in_channels <= c2.out_channels
                and c2.out_channels in (64, 128) and c2.in_channels % 32 == 0
                and c2.kernel_size[0] == c2.kernel_size[1] and c2.dilation == (1, 1) and c2.groups == 1
                and blk.conv3.out_channels % 128 == 0)

    def prepare(self, device, arith: str = "f32"):
        self.c2.prepare(device, arith)
        self.tail.prepare(device, arith)

    def __call__(self, h, x, out=None, arith: str = "f32"):
        """arith "f32": bev_conv2d_chain_dual_f32; "bf16x6": bev_conv2d_chain_dual_x6_f32 (64-channel shapes)."""
        self.prepare(h.device, arith)
        c2 = self.c2.conv
        x6 = arith == "bf16x6"
        return _nat.conv2d_chain_dual_nhwc(h, self.c2.packed6 if x6 else self.c2.packed, self.c2.bias, c2.out_channels,
                                           c2.kernel_size[0], c2.kernel_size[1], c2.stride[0], c2.padding[0],
                                           _nat.ACT_RELU, x, self.tail.short.conv.stride[0],
                                           self.tail.packed6 if x6 else self.tail.packed, self.tail.bias,
                                           self.tail.main.conv.out_channels, _nat.ACT_RELU, out=out)


def stage_of(out_index: int) -> int:
    """features_only index -> number of residual stages to run (0: act1, 1: layer1, ...)."""
    return max(0, out_index)


class ResNet(nn.Module):
    """timm-named ResNet trunk.  forward_features_nhwc(x, out_index) runs natively."""

    def __init__(self, block, layers: List[int]):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.act1 = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0], 1)
        self.layer2 = self._make_layer(block, 128, layers[1], 2)
        self.layer3 = self._make_layer(block, 256, layers[2], 2)
        self.layer4 = self._make_layer(block, 512, layers[3], 2)
        self.feature_info = [64, 64 * block.expansion, 128 * block.expansion, 256 * block.expansion,
                             512 * block.expansion]
        for m in self.modules():  # timm's ResNet init
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        self._folded = {}
        self.fuse_shortcut = True  # bottleneck conv3 + downsample as one dual-source GEMM
        self.fuse_chain = True  # bottleneck conv2 -> conv3 (+ identity) in one launch (h2 stays in LDS)
        self.h16_blocks = True  # AMP training: bottlenecks as one node with fp16-stored inner tensors (bit-identical)
        # Inference: split the images into this many groups, each run on its own HIP stream, so the
        # HBM- / latency-bound 1x1 layers of one group overlap the MFMA-bound 3x3 layers of another (the
        # images are independent; every layer still runs as one kernel per group; bit-identical output).
        # r02h A/B (7-cam 1080p ResNet-50 bench): 1 group 87.6, 2 groups 89.4, 3 groups 88.4 frames/s;
        # staggering the groups' start (stream_offset) did not help.
        # bf16x6 arithmetic (bev_native.conv_arith()): the stages (1 = layer1 ...) whose bottlenecks keep the exact-f32
        # chained kernels (conv2 output in LDS, no HBM round trip) -- measured faster where the 1x1 tails are
        # HBM-bound -- and whether conv1 hands conv2 a pre-split operand (k_conv_x6s).
        self.f32_chain_stages = set()
        # stages whose bottleneck bodies run as one split-arithmetic chained launch (r03 tools/trunk_ab.py, encoder ms
        # per 2-frame step: none 17.06, {1} 16.02-16.21, {1, 2} 15.97-16.01)
        self.x6_chain_stages = {1, 2}
        self.split_edges = False
        self.stream_groups = 2
        self.stream_offset = 0  # > 0: group g waits for group g - 1 to pass this launch stage (staggered start)
        self._streams = {}

    def _make_layer(self, block, planes, blocks, stride):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def _fc(self, conv, bn):
        k = id(conv)
        if k not in self._folded:
            self._folded[k] = FoldedConv(conv, bn, split_ok=True)
        return self._folded[k]

    def unexecuted_parameter_names(self, out_index: int):
        """Parameters of the residual stages past features_only[out_index] (not run: stage_of), which never
        receive a gradient (DistributedDataParallel must not wait for them)."""
        return [f"layer{li}.{n}" for li in range(stage_of(out_index) + 1, 5)
                for n, _ in getattr(self, f"layer{li}").named_parameters()]

    def forward_features_nhwc(self, x: torch.Tensor, out_index: int) -> torch.Tensor:
        """x: images [N,3,H,W] NCHW fp32 on the device -> NHWC feature map of features_only[out_index]."""
        if self.training:  # torch semantics: train-mode BN uses batch statistics, with or without autograd
            return self._forward_train(x, out_index)
        G = min(int(self.stream_groups), x.shape[0])
        if G <= 1:
            return self._forward_eval(x, out_index)
        return self._forward_eval_streams(x, out_index, G)

    def _forward_eval(self, x: torch.Tensor, out_index: int, out: torch.Tensor = None, mark=None) -> torch.Tensor:
        """The eval chain; `out` (optional) receives the last layer's output; mark(i) is called after
        launch stage i (1 = stem, 2 = max-pool, 3.. = residual blocks)."""
        mark = mark or (lambda i: None)
        last_li = max(1, min(out_index, 4))
        fc = self._fc(self.conv1, self.bn1)
        if out_index > 0 and STEM_POOL and fc.stem_x6() and self.conv1.out_channels == 64:
            fc.prepare(x.device, "bf16x6")
            y = _nat.conv2d_stem_pool_x6(x, fc.packed6, fc.bias)  # stem + max-pool, one pass
            mark(1)
            mark(2)
        else:
            y = fc(x, relu=True, in_nchw=True, out=out if out_index == 0 else None)
            mark(1)
            if out_index == 0:
                return y
            y = _nat.maxpool_nhwc(y, 3, 2, 1)
            mark(2)
        stage = 2
        layers = (self.layer1, self.layer2, self.layer3, self.layer4)
        seq = [(li, bi, blk) for li, layer in enumerate(layers, start=1) if li <= max(out_index, 1)
               for bi, blk in enumerate(layer)]
        h1 = None  # the next block's conv1 output, computed by the previous chain's epilogue (FUSE_NEXT_CONV1)
        for k, (li, bi, blk) in enumerate(seq):
            last = li == last_li and bi == len(layers[li - 1]) - 1
            nxt = seq[k + 1][2] if k + 1 < len(seq) else None
            y, h1 = self._block(blk, y, out=out if last else None, h1=h1, nxt=nxt)
            stage += 1
            mark(stage)
            if li == out_index and bi == len(layers[li - 1]) - 1:
                return y
        return y

    def _out_shape(self, x: torch.Tensor, out_index: int):
        """[N, Hf, Wf, C] of features_only[out_index]: the stem, the max-pool and layer2..4 each halve
        (h -> (h - 1) // 2 + 1 for 7x7/s2/p3, 3x3/s2/p1 and the 3x3/s2/p1 convs)."""
        oi = max(0, min(out_index, 4))
        H, W = x.shape[-2:]
        for _ in range(1 + min(oi, 1) + max(0, oi - 1)):
            H, W = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        return x.shape[0], H, W, self.feature_info[oi]

    def _prepare_eval(self, device, out_index: int):
        """Fold + pack every conv the eval chain up to `out_index` runs, on the caller's stream.  Called
        before the image groups fork onto their side streams, so no group can read a panel (or a freed old
        one) while another group's stream is still re-packing it."""
        self._fc(self.conv1, self.bn1).prepare(device)
        if out_index == 0:
            return
        for li, layer in enumerate((self.layer1, self.layer2, self.layer3, self.layer4), start=1):
            for blk in layer:
                kind, fs = self._block_plan(blk)
                for f in fs:
                    if f is None:
                        continue
                    if kind in ("chain6", "chaintail6") and isinstance(f, (FoldedChain, FoldedChainTail)):
                        f.prepare(device, "bf16x6")
                    else:
                        f.prepare(device)
            if li == out_index:
                return

    def _forward_eval_streams(self, x: torch.Tensor, out_index: int, G: int) -> torch.Tensor:
        dev = x.device
        self._prepare_eval(dev, out_index)
        cur = torch.cuda.current_stream(dev)
        side = self._streams.setdefault(dev, [])
        while len(side) < G:
            side.append(torch.cuda.Stream(device=dev))
        out = torch.empty(self._out_shape(x, out_index), device=dev, dtype=torch.float32)
        bounds = [x.shape[0] * g // G for g in range(G + 1)]
        prev = None  # group g starts once group g - 1 has passed launch stage `stream_offset`
        for g in range(G):
            s = side[g]
            s.wait_stream(cur)  # x and out are ready on the caller's stream
            if prev is not None:
                s.wait_event(prev)
            ev = torch.cuda.Event() if (self.stream_offset > 0 and g + 1 < G) else None

            def mark(i, ev=ev, s=s):
                if ev is not None and i == self.stream_offset:
                    ev.record(s)
            with torch.cuda.stream(s):
                self._forward_eval(x[bounds[g]:bounds[g + 1]], out_index, out=out[bounds[g]:bounds[g + 1]],
                                   mark=mark)
            prev = ev
        for g in range(G):
            cur.wait_stream(side[g])
        x.record_stream(side[0])  # the caller may free x once its stream passes this point
        for g in range(1, G):
            x.record_stream(side[g])
            out.record_stream(side[g])
        out.record_stream(side[0])
        return out

    def _forward_train(self, x: torch.Tensor, out_index: int) -> torch.Tensor:
        """Training: the same graph with one autograd node per conv + BN (+ residual) (+ ReLU)
        and native backward kernels (trunk_grad.py; batch-statistics or frozen BN per module mode).  No
        bottleneck-tail fusion in the forward; in the backward an identity block's shortcut gradient is added in its
        first conv's dgrad epilogue (trunk_grad.GradSink), a downsample block's is a separate conv backward."""
        from .trunk_grad import BottleneckTrainH16, GradSink, MaxPool, bottleneck_h16_ok, conv_bn_act
        y = conv_bn_act(self.conv1, self.bn1, x, relu=True, in_nchw=True)
        if out_index == 0:
            return y
        y = MaxPool.apply(y, 3, 2, 1)
        for li, layer in enumerate((self.layer1, self.layer2, self.layer3, self.layer4), start=1):
            for blk in layer:
                sc = y
                h16 = self.h16_blocks and bottleneck_h16_ok(blk)
                # downsample block as one H16 node: the node's input gradient (conv1's dgrad) goes to the downsample
                # conv's dgrad epilogue (GradSink) instead of autograd adding the block input's two gradients
                ds_sink = GradSink() if (h16 and blk.downsample is not None) else None
                if blk.downsample is not None:
                    sc = conv_bn_act(blk.downsample[0], blk.downsample[1], y, relu=False, sink_in=ds_sink)
                if h16:  # AMP: one node, fp16-stored inner tensors
                    y = BottleneckTrainH16.apply(y, None if blk.downsample is None else sc, blk.conv1.weight,
                                                 blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
                                                 blk.bn2.bias, blk.conv3.weight, blk.bn3.weight, blk.bn3.bias, blk,
                                                 ds_sink)
                    continue
                chain = blk.convs()
                # identity shortcut: the residual's gradient goes to the first conv's dgrad epilogue (GradSink)
                sink = GradSink() if blk.downsample is None else None
                h = y
                for idx, (conv, bn, relu) in enumerate(chain):
                    last = idx == len(chain) - 1
                    h = conv_bn_act(conv, bn, h, relu=relu, residual=sc if last else None,
                                    sink_in=sink if idx == 0 else None, sink_out=sink if last else None)
                y = h
            if li == out_index:
                return y
        return y

    def _tail(self, blk):
        k = ("tail", id(blk))
        if k not in self._folded:
            self._folded[k] = FoldedTail(self._fc(blk.conv3, blk.bn3), self._fc(blk.downsample[0], blk.downsample[1]))
        return self._folded[k]

    def _chain(self, blk):
        k = ("chain", id(blk))
        if k not in self._folded:
            self._folded[k] = FoldedChain(self._fc(blk.conv2, blk.bn2), self._fc(blk.conv3, blk.bn3))
        return self._folded[k]

    def _block_plan(self, blk):
        """(kind, folded executors) of one residual block on the eval path.  The chained kernels are exact-f32
        MFMA kernels: with the split-bf16 arithmetic (bev_native.conv_arith() == "bf16x6") the block runs as
        separate split-bf16 launches (conv1, conv2, conv3 + shortcut as one dual GEMM) instead."""
        stage = self._stage_of_block(blk)
        chains = self.fuse_chain and (_nat.conv_arith() == "f32" or stage in self.f32_chain_stages)
        if (isinstance(blk, Bottleneck) and self.fuse_chain and not chains and stage in self.x6_chain_stages
                and FoldedChain.applies(blk) and self._fc(blk.conv2, blk.bn2).arith() == "bf16x6"
                and self._fc(blk.conv3, blk.bn3).arith() == "bf16x6"):
            return "chain6", [self._fc(blk.conv1, blk.bn1), self._chain(blk)]
        if (isinstance(blk, Bottleneck) and self.fuse_chain and self.fuse_shortcut and not chains
                and stage in self.x6_chain_stages and FoldedChainTail.applies(blk) and blk.conv2.out_channels == 64
                and blk.downsample[0].in_channels == 64 and self._fc(blk.conv2, blk.bn2).arith() == "bf16x6"
                and self._tail(blk).arith() == "bf16x6"):
            k = ("chaintail", id(blk))
            if k not in self._folded:
                self._folded[k] = FoldedChainTail(self._fc(blk.conv2, blk.bn2), self._tail(blk))
            return "chaintail6", [self._fc(blk.conv1, blk.bn1), self._folded[k]]
        if isinstance(blk, Bottleneck) and chains and FoldedChain.applies(blk):
            return "chain", [self._fc(blk.conv1, blk.bn1), self._chain(blk)]
        if isinstance(blk, Bottleneck) and chains and self.fuse_shortcut and FoldedChainTail.applies(blk):
            k = ("chaintail", id(blk))
            if k not in self._folded:
                self._folded[k] = FoldedChainTail(self._fc(blk.conv2, blk.bn2), self._tail(blk))
            return "chaintail", [self._fc(blk.conv1, blk.bn1), self._folded[k]]
        if isinstance(blk, Bottleneck) and self.fuse_shortcut and FoldedTail.applies(blk):
            return "tail", [self._fc(blk.conv1, blk.bn1), self._fc(blk.conv2, blk.bn2), self._tail(blk)]
        ds = self._fc(blk.downsample[0], blk.downsample[1]) if blk.downsample is not None else None
        return "plain", [ds] + [self._fc(conv, bn) for conv, bn, _ in blk.convs()]

    def _stage_of_block(self, blk) -> int:
        for li, layer in enumerate((self.layer1, self.layer2, self.layer3, self.layer4), start=1):
            if any(b is blk for b in layer):
                return li
        return 0

    def _split_edge(self, f1, f2) -> bool:
        """conv f1's output feeds only conv f2: with both in the bf16x6 arithmetic and f2 a KxK (K > 1) conv, f1
        writes it pre-split (f2 would otherwise split every input pixel once per tap)."""
        return (self.split_edges and f1.arith() == "bf16x6" and f2.arith() == "bf16x6" and f2.conv.kernel_size[0] > 1
                and f2.conv.in_channels % 32 == 0 and f1.conv.out_channels % 4 == 0)

    def _next_conv1(self, fs, nxt):
        """The next block's conv1 that this split chain (fs = its plan) may run in its epilogue, with whether the
        next block wants that output split (a chain) or fp32 (the tail plan's stride-2 conv2); (None, _) if not.
        Identity-shortcut chains only: the library refuses the dual (block 0) form (bev_mi355x.h)."""
        if not (FUSE_NEXT_CONV1 and SPLIT_CHAIN and nxt is not None and isinstance(fs[1], FoldedChain)
                and fs[1].c2.conv.out_channels == 64):
            return None, False
        kind, nf = self._block_plan(nxt)
        if kind not in ("chain6", "chaintail6", "tail"):
            return None, False
        c1 = nf[0]
        cv = c1.conv
        ok = (c1.arith() == "bf16x6" and cv.kernel_size == (1, 1) and cv.stride == (1, 1) and cv.padding == (0, 0)
              and cv.in_channels == fs[1].c3.conv.out_channels and cv.out_channels in (64, 128))
        return (c1, kind != "tail") if ok else (None, False)

    def _block(self, blk, x, out=None, h1=None, nxt=None):
        """One residual block of the eval chain -> (y, h1 of the next block if this block's chain computed it)."""
        kind, fs = self._block_plan(blk)
        if kind in ("chain", "chaintail"):
            h = fs[0](x, relu=True)
            return fs[1](h, x, out=out), None
        if kind in ("chain6", "chaintail6"):
            split = SPLIT_CHAIN and fs[0].arith() == "bf16x6" and fs[0].conv.out_channels % 32 == 0
            h = h1 if h1 is not None else fs[0](x, relu=True, split_out=split)
            if isinstance(h, _nat.Split3):
                c1n, split_n = self._next_conv1(fs, nxt)
                if c1n is not None:
                    return fs[1].fused(h, x, c1n, out=out, split_out=split_n)
            return fs[1](h, x, out=out, arith="bf16x6"), None
        if kind == "tail":
            h = h1 if h1 is not None else fs[0](x, relu=True, split_out=self._split_edge(fs[0], fs[1]))
            h = fs[1](h, relu=True)
            return fs[2](h, x, out=out), None
        sc = fs[0](x, relu=False) if fs[0] is not None else x
        chain = blk.convs()
        fl = fs[1:]
        y = x
        for idx, ((conv, bn, relu), f) in enumerate(zip(chain, fl)):
            last = idx == len(chain) - 1
            split = not last and self._split_edge(f, fl[idx + 1])
            y = f(y, relu=relu, residual=sc if last else None, out=out if last else None, split_out=split)
        return y, None


def resnet18():
    return ResNet(BasicBlock, [2, 2, 2, 2])


def resnet34():
    return ResNet(BasicBlock, [3, 4, 6, 3])


def resnet50():
    return ResNet(Bottleneck, [3, 4, 6, 3])


NATIVE_BACKBONES = {"resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50}
