"""Trainable 1x1 projection of the encoder (cnn_encoder.py:43-46) on the HIP conv kernel.

CNNEncoder's lazy `proj` maps the trunk's stride-8 features to FEAT_DIM.  In
eval it is folded into one MFMA conv launch (FoldedConv).  When it trains
(BASELINE config 3 with a `ViewEncoder.freeze()`d trunk -- in the reference
the lazily created proj stays trainable because it does not exist yet when
freeze() runs), this autograd Function keeps the data path native:

  forward   y  = x (*) W + b          bev_conv2d_f32 (1x1, NHWC)
  backward  dX = dY (*) W^T           bev_conv2d_f32 with the transposed panel
            dW = dY^T X               bev_conv_wgrad_f32 (1x1: MFMA GEMM over pixels)
            db = sum dY               bev_colsum_f32

so the loss gradient reaches the BEV features through the native warp
backward (geometry.py _WarpFn -> bev_ipm_warp_bwd_f32) and then this proj.
"""
from __future__ import annotations

import torch

import bev_native as _nat

__all__ = ["Proj1x1"]


class Proj1x1(torch.autograd.Function):
    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, feat: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
        """feat [N,H,W,Ci] NHWC, weight [Co,Ci,1,1], bias [Co] -> y [N,H,W,Co] NHWC."""
        Co = weight.shape[0]
        feat = feat.contiguous()
        packed = _nat.pack_conv_weight(weight.detach().float().contiguous())
        y = _nat.conv2d_nhwc(feat, packed, bias.detach().float().contiguous(), Co, 1, 1, 1, 0, False)
        ctx.save_for_backward(feat, weight)
        return y

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, gy: torch.Tensor):
        feat, weight = ctx.saved_tensors
        Co, Ci = weight.shape[0], weight.shape[1]
        gy = gy.contiguous().float()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            packed_t = _nat.pack_conv_weight(weight.detach().float().transpose(0, 1).contiguous())
            zero = torch.zeros(Ci, device=gy.device, dtype=torch.float32)
            dx = _nat.conv2d_nhwc(gy, packed_t, zero, Ci, 1, 1, 1, 0, False)
        if ctx.needs_input_grad[1]:
            # [Co, Ci] storage with the parameter's strides (DDP's bucket views compare strides exactly)
            dw = _nat.conv_wgrad(feat, gy, 1, 1, 1, 0).reshape(Co, Ci).clone().view(Co, Ci, 1, 1).to(weight.dtype)
        if ctx.needs_input_grad[2]:
            db = _nat.colsum(gy)
        return dx, dw, db
