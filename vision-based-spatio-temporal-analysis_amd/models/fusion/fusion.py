"""N-view BEV fusion modules -- drop-in for the reference's project/models/fusion/fusion.py.

FusionModule / SimpleFusion / AttentionFusion / ConcatFusion keep the
reference's names, constructor signatures, assertions and output shapes
(fusion.py:5-46).  SimpleFusion's reduction runs in the HIP kernel
`bev_view_fuse_f32` (bit-identical to torch's CPU sum / mean / max over dim
1: sequential v = 0..V-1 sum from +0, true division by V, NaN-propagating
max).  AttentionFusion is, as in the reference, a placeholder that prints
once and returns the mean (fusion.py:25-36, quirk Q8).  ConcatFusion is a
zero-copy reshape (fusion.py:39-46).

When the per-view maps come straight out of GeometryTransformer, prefer
`GeometryTransformer.forward_fused(..., mode)`: it fuses this reduction into
the warp and never materialises [B, V, C, H, W].
"""
from __future__ import annotations

import torch
import torch.nn as nn

import bev_native as _nat

__all__ = ["FusionModule", "SimpleFusion", "AttentionFusion", "ConcatFusion", "BEVFusion"]


class _FuseFn(torch.autograd.Function):
    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, x, mode):
        out = _nat.view_fuse(x, mode)
        ctx.mode = mode
        ctx.V = x.shape[1]
        if mode == "max":
            ctx.save_for_backward(x)
        return out

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, g):
        V = ctx.V
        if ctx.mode == "sum":
            return g.unsqueeze(1).expand(g.shape[0], V, *g.shape[1:]), None
        if ctx.mode == "mean":
            return (g / V).unsqueeze(1).expand(g.shape[0], V, *g.shape[1:]), None
        x, = ctx.saved_tensors
        # to the view torch's max(dim) returns: the first NaN, else the first maximal element (bev_view_max_bwd_f32)
        return _nat.view_max_bwd(x, g), None


class FusionModule(nn.Module):
    def forward(self, bev_maps: torch.Tensor) -> torch.Tensor:
        """bev_maps: Tensor[B, V, C, H, W] -> Tensor[B, C, H, W]"""
        raise NotImplementedError


class SimpleFusion(FusionModule):
    def __init__(self, mode: str = "sum"):
        super().__init__()
        assert mode in ("sum", "mean", "max")
        self.mode = mode

    def forward(self, bev_maps: torch.Tensor) -> torch.Tensor:
        return _FuseFn.apply(bev_maps, self.mode)


class AttentionFusion(FusionModule):
    def __init__(self):
        super().__init__()
        # placeholder, as in the reference: no attention is implemented there
        self._warned = False

    def forward(self, bev_maps: torch.Tensor) -> torch.Tensor:
        if not self._warned:
            print("[AttentionFusion] Placeholder only. Not implemented.")
            self._warned = True
        return _FuseFn.apply(bev_maps, "mean")


class ConcatFusion(FusionModule):
    def __init__(self):
        super().__init__()

    def forward(self, bev_maps: torch.Tensor) -> torch.Tensor:
        # [B, V, C, H, W] -> [B, V*C, H, W]
        B, V, C, H, W = bev_maps.shape
        return bev_maps.reshape(B, V * C, H, W)


# north_star vocabulary alias
BEVFusion = SimpleFusion
