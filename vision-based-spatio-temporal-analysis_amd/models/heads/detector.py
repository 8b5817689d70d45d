"""CenterNet-style BEV detection head -- drop-in for project/models/heads/detector.py.

Same constructor, module tree and parameter names as the reference's BEVDetector
(detector.py:7-45: `stem` = 3 x [3x3 conv (no bias), GroupNorm(32), ReLU] with 512 / 128 / 128
channels and dilation 2 in the middle conv, then 3x3 `heatmap_head` (1), `offset_head` (2) and
`size_head` (2) convs with the CenterNet initialisation), the same forward dict
(detector.py:47-62) and decode (detector.py:64-125), so state_dicts and callers carry over.

The computation is native and channels-last:

* every conv is the fp32 MFMA implicit GEMM (bev_conv2d_nhwc_ex_f32), dilation in the tap grid;
* GroupNorm statistics come from bev_groupnorm_fwd_f32, and in inference the normalisation + ReLU is
  applied by the NEXT conv while it loads its operand -- the 512- and 128-channel normalised maps are
  never written;
* the three heads are ONE 128 -> 5 conv (weights concatenated), split into the reference's outputs;
* training materialises each GroupNorm + ReLU output and runs the native backward (conv dgrad as a
  conv with the flipped, transposed kernel; dilated wgrad; GroupNorm backward kernels).
* decode: bev_decode_peaks_f32 + bev_decode_nms_f32 (peak test, threshold, sort, greedy NMS on the
  device; one host sync per batch instead of one per pair of detections).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

import bev_native as _nat

__all__ = ["BEVDetector", "AnchorDetector"]

_GROUPS = 32


def _ceil_to(c: int, m: int) -> int:
    return (c + m - 1) // m * m


class _Packed:
    """Packed MFMA panel of a conv weight (input channels zero-padded to `cin_pad`), rebuilt when the
    parameter changes (storage pointer + version counter)."""

    def __init__(self):
        self.key, self.panel = None, None

    def get(self, weight: torch.Tensor, cin_pad: int) -> torch.Tensor:
        key = (weight.data_ptr(), weight._version, cin_pad, str(weight.device))
        if key != self.key:
            with torch.no_grad():
                w = weight.detach().float()
                if cin_pad > w.shape[1]:
                    w = F.pad(w, (0, 0, 0, 0, 0, cin_pad - w.shape[1]))
                self.panel = _nat.pack_conv_weight(w.contiguous())
            self.key = key
        return self.panel


class _HeadConv(torch.autograd.Function):
    """Stride-1 'same' KxK conv of an NHWC operand (padding = dilation * (K // 2)), native both ways."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, weight, bias, dil: int):
        Co, Ci, K, _ = weight.shape
        cp = x.shape[-1]
        w = weight.detach().float()
        if cp > Ci:
            w = F.pad(w, (0, 0, 0, 0, 0, cp - Ci))
        w = w.contiguous()
        b = bias.detach().float().contiguous() if bias is not None else torch.zeros(Co, device=x.device)
        pad = dil * (K // 2)
        y = _nat.conv2d_nhwc_ex(x, _nat.pack_conv_weight(w), b, Co, K, pad, dil)
        ctx.save_for_backward(x, w)
        ctx.meta = (dil, Ci, bias is not None)
        return y

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dil, Ci, has_b = ctx.meta
        Co, cp, K, _ = w.shape
        pad = dil * (K // 2)
        dy = dy.contiguous().float()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:  # dgrad: the same conv with the flipped, transposed kernel
            wt = w.flip(2, 3).transpose(0, 1).contiguous()
            dx = _nat.conv2d_nhwc_ex(dy, _nat.pack_conv_weight(wt), torch.zeros(cp, device=dy.device), cp, K, pad, dil)
        if ctx.needs_input_grad[1]:
            dw = _nat.conv_wgrad_ex(x, dy, K, pad, dil)[:, :Ci]
        if has_b and ctx.needs_input_grad[2]:
            db = _nat.colsum(dy)
        return dx, dw, db, None


class _GroupNormReLU(torch.autograd.Function):
    """relu(GroupNorm(32)(z)) over NHWC z, materialised (training), native backward."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, z, gamma, beta, eps: float):
        mean, rstd, scale, shift = _nat.groupnorm_fwd(z, _GROUPS, gamma, beta, eps)
        ctx.save_for_backward(z, gamma, mean, rstd, scale, shift)
        return _nat.groupnorm_apply(z, scale, shift, True)

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, da):
        z, gamma, mean, rstd, scale, shift = ctx.saved_tensors
        dz, dg, db = _nat.groupnorm_bwd(z, da, _GROUPS, mean, rstd, gamma, scale, shift, True)
        return dz, dg, db, None


class _HeadTrainH16(torch.autograd.Function):
    """The whole training head under autocast(float16) as ONE autograd node: 3 x [conv -> GroupNorm -> ReLU] -> the
    heads conv, with the tensors that live between its layers stored in the precision their readers compute in --
    each GroupNorm + ReLU output (read only by the next fp16 conv and its weight gradient) and each GroupNorm
    backward output (read only by its conv's fp16 dgrad and weight gradient) in fp16: exactly the values the
    fp32-stored per-layer path (_HeadConv / _GroupNormReLU) rounds them to, so every result is bit-identical to it
    (`tests/test_train_amp_gpu.py::test_head_h16_node_bit_identical`) with half the bytes on those tensors."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, w1, g1, b1, w2, g2, b2, w3, g3, b3, wh, bh, head):
        assert _nat.half_convs()
        convs, gns = head._convs()
        ws, gbs = (w1, w2, w3), ((g1, b1), (g2, b2), (g3, b3))
        a = x
        saved, meta = [], []
        for i, (conv, gn) in enumerate(zip(convs, gns)):
            Co, Ci, K, _ = ws[i].shape
            cp = a.shape[-1]
            w = ws[i].detach().float()
            if cp > Ci:
                w = F.pad(w, (0, 0, 0, 0, 0, cp - Ci))
            w = w.contiguous()
            dil = conv.dilation[0]
            pad = dil * (K // 2)
            packed = _nat.pack_conv_weight(w)
            if a.dtype == torch.float16:
                z = _nat.conv2d_h16_any(a, packed, Co, K, K, 1, pad, dilation=dil)
            else:
                z = _nat.conv2d_nhwc_ex(a, packed, torch.zeros(Co, device=a.device), Co, K, pad, dil)
            g, b = gbs[i]
            mean, rstd, scale, shift = _nat.groupnorm_fwd(z, _GROUPS, g, b, gn.eps)
            saved += [a, w, z, g, mean, rstd, scale, shift]
            meta.append((dil, Ci))
            a = _nat.groupnorm_apply_half(z, scale, shift, True)
        w = wh.detach().float().contiguous()
        bb = bh.detach().float().contiguous()
        y = _nat.conv2d_h16_any(a, _nat.pack_conv_weight(w), w.shape[0], 3, 3, 1, 1, bias=bb)
        ctx.save_for_backward(*saved, a, w)
        ctx.meta = meta
        ctx.grad_channels = min(head.grad_channels or head.in_channels, x.shape[-1])
        return y

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dy):
        t = ctx.saved_tensors
        a3, wh = t[24], t[25]
        dy = dy.contiguous().float()
        Co_h, cp, K, _ = wh.shape
        # heads conv: colsum bias gradient, dgrad on the fp32 gradient, weight gradient (output channels padded to 4)
        dbh = _nat.colsum(dy)
        dyp = F.pad(dy, (0, (-Co_h) % 4)).contiguous()
        dwh = _nat.conv_wgrad_h16_any(a3, dyp, K, K, 1, 1)[:Co_h]
        wt = wh.flip(2, 3).transpose(0, 1).contiguous()
        da = _nat.conv2d_nhwc_ex(dy, _nat.pack_conv_weight(wt), torch.zeros(cp, device=dy.device), cp, K, 1, 1)
        grads = [None] * 3
        for i in (2, 1, 0):
            a, w, z, g, mean, rstd, scale, shift = t[8 * i: 8 * i + 8]
            dil, Ci = ctx.meta[i]
            Co, cpi, K, _ = w.shape
            pad = dil * (K // 2)
            dz, dg, db = _nat.groupnorm_bwd_half(z, da, _GROUPS, mean, rstd, g, scale, shift, True)
            dw = _nat.conv_wgrad_h16_any(a, dz, K, K, 1, pad, dil)[:, :Ci]
            if i > 0:
                wt = w.flip(2, 3).transpose(0, 1).contiguous()
                da = _nat.conv2d_h16_any(dz, _nat.pack_conv_weight(wt), cpi, K, K, 1, pad, dilation=dil)
            elif ctx.needs_input_grad[0]:
                # the operand's gradient is read only in its first `gc` channels (the BEV features; the position
                # encoding and the zero pad take none): the dgrad computes those alone, into a cp-wide buffer
                gc = ctx.grad_channels
                wt = w.flip(2, 3).transpose(0, 1)[:gc].contiguous()
                da = torch.empty(dz.shape[0], dz.shape[1], dz.shape[2], cpi, device=dz.device, dtype=torch.float32)
                if gc < cpi:  # the channels past gc are defined (zero), so a hook / anomaly check sees no garbage
                    da[..., gc:].zero_()
                _nat.conv2d_h16_any(dz, _nat.pack_conv_weight(wt), gc, K, K, 1, pad, dilation=dil, out=da)
            else:
                da = None
            grads[i] = (dw, dg, db)
        return (da, *grads[0], *grads[1], *grads[2], dwh, dbh, None)


def _head_h16_ok(head) -> bool:
    """_HeadTrainH16 applies: AMP fp16 convs active and the layers' channels fit the fp16-operand kernels."""
    if not _nat.amp_half_active():
        return False
    convs, _ = head._convs()
    return all(c.out_channels % 64 == 0 for c in convs) and head.input_channels_padded % 32 == 0


class BEVDetector(nn.Module):
    def __init__(self, in_channels: int = 32, bev_bounds: Tuple[float, float, float, float] = (-6.0, 6.0, -2.0, 2.0),
                 bev_size: Tuple[int, int] = (64, 64), default_box_wh: Tuple[float, float] = (0.6, 0.6)):
        super().__init__()
        layers = []
        for cin, cout, dil in ((in_channels, 512, 1), (512, 128, 2), (128, 128, 1)):
            layers += [nn.Conv2d(cin, cout, kernel_size=3, padding=dil, dilation=dil, bias=False),
                       nn.GroupNorm(num_groups=_GROUPS, num_channels=cout), nn.ReLU(inplace=True)]
        self.stem = nn.Sequential(*layers)
        # leading operand channels that need a gradient (BEVNet: the P BEV feature channels -- its position-encoding
        # channels are a buffer); the AMP node's input gradient is computed for these alone, the rest of its
        # channels are zero.  None: every input channel.  Owned by BEVNet (model_wrapper.py sets it when it builds
        # the head); a standalone BEVDetector leaves it None.
        self.grad_channels = None
        self.heatmap_head = nn.Conv2d(128, 1, kernel_size=3, padding=1)
        self.offset_head = nn.Conv2d(128, 2, kernel_size=3, padding=1)
        self.size_head = nn.Conv2d(128, 2, kernel_size=3, padding=1)
        # CenterNet initialisation (detector.py:33-45): heatmap prior, zero offsets, default footprint
        nn.init.constant_(self.heatmap_head.bias, -2.19)
        nn.init.zeros_(self.offset_head.weight)
        nn.init.zeros_(self.offset_head.bias)
        self.in_channels = in_channels
        self.bounds = bev_bounds
        self.bev_h, self.bev_w = bev_size
        self.res_x = (bev_bounds[1] - bev_bounds[0]) / float(self.bev_w)
        self.res_y = (bev_bounds[3] - bev_bounds[2]) / float(self.bev_h)
        cells = [max(default_box_wh[0] / max(self.res_x, 1e-6), 1e-3), max(default_box_wh[1] / max(self.res_y, 1e-6), 1e-3)]
        with torch.no_grad():
            self.size_head.bias.copy_(torch.log(torch.tensor(cells, dtype=torch.float32)))
        self._panels = [_Packed() for _ in range(3)]
        self.h16_node = True  # AMP training: the head as one node with fp16-stored inner tensors (bit-identical)

    # ---- layout helpers -----------------------------------------------------------------------
    @property
    def input_channels_padded(self) -> int:
        """Channel count of the NHWC operand forward_nhwc expects (in_channels rounded up to 32)."""
        return _ceil_to(self.in_channels, 32)

    def _convs(self):
        return (self.stem[0], self.stem[3], self.stem[6]), (self.stem[1], self.stem[4], self.stem[7])

    def _head_params(self):
        w = torch.cat([self.heatmap_head.weight, self.offset_head.weight, self.size_head.weight], dim=0)
        b = torch.cat([self.heatmap_head.bias, self.offset_head.bias, self.size_head.bias], dim=0)
        return w, b

    # ---- forward (detector.py:47-62) ------------------------------------------------------------
    def forward(self, bev_feat: torch.Tensor) -> Dict[str, torch.Tensor]:
        """bev_feat [B, in_channels, H, W] (any strides) -> heatmap_logits / heatmap [B,1,H,W],
        offset(_raw) / size(_raw) [B,2,H,W]."""
        B, C, H, W = bev_feat.shape
        x = torch.zeros(B, H, W, self.input_channels_padded, device=bev_feat.device, dtype=torch.float32)
        x[..., :C] = bev_feat.permute(0, 2, 3, 1)
        return self.forward_nhwc(x)

    def forward_nhwc(self, x: torch.Tensor) -> Dict[str, torch.Tensor]:
        """x [B, H, W, input_channels_padded] NHWC (channels >= in_channels zero)."""
        convs, gns = self._convs()
        train = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if train and self.h16_node and _head_h16_ok(self):  # AMP: one node, fp16-stored inner tensors (bit-identical)
            w, b = self._head_params()
            (c1, c2, c3), (n1, n2, n3) = convs, gns
            y = _HeadTrainH16.apply(x, c1.weight, n1.weight, n1.bias, c2.weight, n2.weight, n2.bias, c3.weight,
                                    n3.weight, n3.bias, w, b, self)
        elif train:
            a = x
            for conv, gn in zip(convs, gns):
                z = _HeadConv.apply(a, conv.weight, None, conv.dilation[0])
                a = _GroupNormReLU.apply(z, gn.weight, gn.bias, gn.eps)
            w, b = self._head_params()
            y = _HeadConv.apply(a, w, b, 1)
        else:
            with torch.no_grad():
                z, scale, shift = x, None, None
                for i, (conv, gn) in enumerate(zip(convs, gns)):
                    d = conv.dilation[0]
                    panel = self._panels[i].get(conv.weight, z.shape[-1])
                    z = _nat.conv2d_nhwc_ex(z, panel, torch.zeros(conv.out_channels, device=z.device),
                                            conv.out_channels, 3, d, d, in_scale=scale, in_shift=shift,
                                            in_relu=scale is not None)
                    _, _, scale, shift = _nat.groupnorm_fwd(z, _GROUPS, gn.weight, gn.bias, gn.eps)
                w, b = self._head_params()
                y = _nat.conv2d_nhwc_ex(z, _nat.pack_conv_weight(w.detach().float().contiguous()),
                                        b.detach().float().contiguous(), 5, 3, 1, 1, in_scale=scale, in_shift=shift,
                                        in_relu=True)
        logits = y[..., 0:1].permute(0, 3, 1, 2).contiguous()
        offset_raw = y[..., 1:3].permute(0, 3, 1, 2).contiguous()
        size_raw = y[..., 3:5].permute(0, 3, 1, 2).contiguous()
        return {"heatmap_logits": logits, "heatmap": torch.sigmoid(logits), "offset": torch.sigmoid(offset_raw),
                "offset_raw": offset_raw, "size": torch.exp(size_raw), "size_raw": size_raw}

    # ---- decode (detector.py:64-125) ------------------------------------------------------------
    @staticmethod
    def _nms2d(x: torch.Tensor, kernel: int = 3) -> torch.Tensor:
        """detector.py:65-69 (kept for callers; decode() does this on the device)."""
        peak = F.max_pool2d(x, kernel_size=kernel, stride=1, padding=kernel // 2)
        return x * (x == peak).float()

    def decode(self, heatmap, offset, size_cells, conf_thresh: float = 0.4, nms_dist_m: float = 0.5,
               lazy: bool = False):
        """Peaks -> world boxes [cx, cy, w, h] + scores per frame (detector.py:71-125) on the device:
        bev_decode_peaks_f32 (3x3 peak test + threshold + compaction) and bev_decode_nms_f32 (sort by
        score, box arithmetic, greedy centre-distance NMS).  One host sync per batch, not per pair; with `lazy`
        the per-frame lists are bev_native.DetectionList sequences that take that sync when first read."""
        return _nat.decode(heatmap, offset, size_cells, self.bounds, conf_thresh, nms_dist_m, lazy=lazy)


class AnchorDetector(nn.Module):
    """The reference's placeholder (detector.py:128-131): no parameters, no forward."""

    def __init__(self):
        super().__init__()
