"""ViewEncoder ABC -- drop-in for project/models/encoders/base.py:6-28 (same contract)."""
import torch
import torch.nn as nn
from abc import ABC, abstractmethod


class ViewEncoder(nn.Module, ABC):
    def __init__(self, out_channels: int):
        super().__init__()
        self.out_channels = out_channels

    @abstractmethod
    def forward(self, images: torch.Tensor) -> torch.Tensor:
        """
        images: Tensor[B*V, 3, H, W] or Tensor[B, V, 3, H, W]
        Returns: Tensor[B, V, C, Hf, Wf]
        """
        raise NotImplementedError

    def load_pretrained(self, weights_path: str):
        # base.py:19-24 semantics (strict=False, print on failure); tensors only.
        try:
            state = torch.load(weights_path, map_location="cpu", weights_only=True)
            self.load_state_dict(state, strict=False)
        except Exception as e:
            print(f"[ViewEncoder] load_pretrained failed: {e}")

    def freeze(self):
        for p in self.parameters():
            p.requires_grad = False
