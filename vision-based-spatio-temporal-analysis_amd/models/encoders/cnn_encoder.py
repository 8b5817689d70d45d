"""CNNEncoder -- per-camera 2D backbone; drop-in for project/models/encoders/cnn_encoder.py.

Same constructor `CNNEncoder(out_channels=32, backbone="resnet18",
pretrained=True, out_index=2)` (cnn_encoder.py:15), same input conventions
([B,V,3,H,W], or [N,3,H,W] treated as B=1, anything else ValueError;
cnn_encoder.py:50-72) and same state_dict layout:

* backbones restated in models/encoders/resnet.py (resnet18/34/50) and
  models/encoders/efficientnet.py (efficientnet_b3), with timm names, play
  the role of the timm `features_only` model: `backbone.*`
  weights, `feats_list[out_index]`, then a lazily created 1x1 `proj`
  (cnn_encoder.py:43-46);
* any other backbone name takes the reference's fallback stack
  Conv(3->16,k3,s2)+ReLU+Conv(16->C,k3,s2)+ReLU (cnn_encoder.py:31-37),
  printing the same notice the reference prints when timm cannot build it.
  `backbone_impl="fallback"` forces it (the configuration the golden
  fixtures pin, since timm is absent where they were generated).

All convolutions run on the HIP MFMA kernels (NHWC); the returned
[B,V,C,Hf,Wf] tensor is a channels-last view of the NHWC feature buffer,
which GeometryTransformer consumes through its strides without a copy.

Quirk Q2: the reference creates the lazy proj on the CPU
and never moves it; here it is created on the input's device.
"""
from __future__ import annotations


import torch
import torch.nn as nn

import bev_native as _nat
from .base import ViewEncoder
from .efficientnet import EFFICIENTNETS
from .proj import Proj1x1
from .resnet import NATIVE_BACKBONES as _RESNETS
from .resnet import FoldedConv
from .trunk_grad import conv_act

# backbones with a native (HIP) trunk: timm names of BASELINE configs 1-4
NATIVE_BACKBONES = dict(_RESNETS, **EFFICIENTNETS)

__all__ = ["CNNEncoder", "Backbone"]


class CNNEncoder(ViewEncoder):
    def __init__(self, out_channels: int = 32, backbone: str = "resnet18", pretrained: bool = True,
                 out_index: int = 2, backbone_impl: str = "auto"):
        super().__init__(out_channels)
        self.backbone_name = backbone
        self.pretrained = pretrained
        self.out_index = out_index
        self._use_timm = False  # True <=> the restated timm-style trunk is in use (name kept for parity)
        self._feature_channels = None
        if backbone_impl not in ("auto", "native", "fallback"):
            raise ValueError(f"backbone_impl must be auto|native|fallback, got {backbone_impl!r}")
        if backbone_impl != "fallback":
            if backbone in NATIVE_BACKBONES:
                self._use_timm = True
                self.backbone = NATIVE_BACKBONES[backbone]()
                self.proj = None
                if pretrained:
                    print(f"[CNNEncoder] pretrained weights for {backbone} are not available offline; "
                          "random init (load a state_dict to use trained weights)")
            else:
                if backbone_impl == "native":
                    raise ValueError(f"no native backbone {backbone!r}; have {sorted(NATIVE_BACKBONES)}")
                print(f"[CNNEncoder] timm unavailable (unknown backbone {backbone!r}), fallback to simple conv")
        if not self._use_timm:
            self.backbone = nn.Sequential(
                nn.Conv2d(3, 16, kernel_size=3, stride=2, padding=1),
                nn.ReLU(inplace=True),
                nn.Conv2d(16, out_channels, kernel_size=3, stride=2, padding=1),
                nn.ReLU(inplace=True),
            )
        self._fb = None
        self._fproj = None
        self.proj_stream_nt = True  # non-temporal activation loads in the inference projection (see forward)

    def _trunk_frozen(self) -> bool:
        return not any(p.requires_grad for p in self.backbone.parameters())

    def _encode_single_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        """x [N,3,H,W] NCHW -> NHWC features [N,Hf,Wf,C] (cnn_encoder.py:39-48)."""
        if self._use_timm:
            if self._trunk_frozen():  # ViewEncoder.freeze(): no trunk gradients (BN still follows train/eval)
                with torch.no_grad():
                    feat = self.backbone.forward_features_nhwc(x, self.out_index)
            else:
                feat = self.backbone.forward_features_nhwc(x, self.out_index)
            if self._feature_channels is None:
                self._feature_channels = feat.shape[-1]
                self.proj = nn.Conv2d(self._feature_channels, self.out_channels, kernel_size=1).to(feat.device)
                self._fproj = FoldedConv(self.proj, split_ok=True)
            if torch.is_grad_enabled() and (self.proj.weight.requires_grad or self.proj.bias.requires_grad):
                return Proj1x1.apply(feat, self.proj.weight, self.proj.bias)  # trainable proj (BASELINE config 3)
            if self.proj_stream_nt:
                # The projection is the last reader of the trunk output (~8x the feature maps' bytes): streamed
                # with non-temporal loads it no longer evicts the maps it writes from the Infinity Cache, and the
                # warp that follows reads them from there (bench: warp 179.5 -> 136.4 us, profiles/r04nt_proj_ab.txt)
                old = _nat.tune(_nat.TUNE_CONV_X6_NT, 1)
                try:
                    return self._fproj(feat, relu=False)
                finally:
                    _nat.tune(_nat.TUNE_CONV_X6_NT, old)
            return self._fproj(feat, relu=False)
        c0, c2 = self.backbone[0], self.backbone[2]
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.backbone.parameters()):
            # trainable fallback stack (the reference trains this nn.Sequential): native autograd nodes
            y = conv_act(c0, x, relu=True, in_nchw=True)
            return conv_act(c2, y, relu=True)
        if self._fb is None:
            self._fb = (FoldedConv(c0), FoldedConv(c2))
        y = self._fb[0](x, relu=True, in_nchw=True)
        return self._fb[1](y, relu=True)

    def _encode_single(self, x: torch.Tensor) -> torch.Tensor:
        y = self._encode_single_nhwc(x)
        return y.permute(0, 3, 1, 2)  # logical NCHW, channels-last storage

    def forward(self, images: torch.Tensor) -> torch.Tensor:
        """
        images: Tensor[B*V, 3, H, W] or Tensor[B, V, 3, H, W]
        Returns: Tensor[B, V, C, Hf, Wf]  (channels-last strides)
        """
        if images.dim() == 4:
            B, V = 1, images.shape[0]  # cnn_encoder.py:55-64: 4-D input is one frame (quirk Q9)
            x = images
        elif images.dim() == 5:
            B, V = images.shape[0], images.shape[1]
            x = images.reshape(B * V, *images.shape[2:])
        else:
            raise ValueError(f"[CNNEncoder] unexpected input shape: {tuple(images.shape)}")
        if x.dtype != torch.float32:
            x = x.float()
        y = self._encode_single_nhwc(x)  # [B*V, Hf, Wf, C]
        Hf, Wf, C = y.shape[1], y.shape[2], y.shape[3]
        return y.view(B, V, Hf, Wf, C).permute(0, 1, 4, 2, 3)

    def load_pretrained(self, weights_path: str):
        super().load_pretrained(weights_path)

    def freeze(self):
        super().freeze()


# north_star vocabulary alias
Backbone = CNNEncoder
