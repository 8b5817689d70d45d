"""Image transforms -- drop-in for project/data/transforms.py.

The reference builds `T.Compose([T.Resize(img_size), T.RandomApply([T.ColorJitter(0.2, 0.2, 0.2,
0.05)], p=0.5), T.ToTensor(), T.Normalize(IMAGENET_MEAN, IMAGENET_STD)])` (transforms.py:12-19)
from torchvision, which this image (and many ROCm deployments) does not ship.  This module restates
each step on PIL + torch with torchvision's semantics for PIL inputs, drawing its random numbers
from torch's global generator in the same order (RandomApply: `torch.rand(1)`; ColorJitter:
`torch.randperm(4)`, then one `uniform_` per enabled factor), so a seeded run makes the same
augmentation choices:

* Resize((H, W)): `img.resize((W, H), Image.BILINEAR)` (torchvision's PIL path);
* ColorJitter: brightness / contrast / saturation through `PIL.ImageEnhance` (Brightness,
  Contrast, Color) and hue by rotating the HSV hue byte (uint8 wrap-around), in the order of
  the drawn permutation;
* ToTensor + Normalize: `(float(u8) / 255 - mean) / std`.

The last two steps are split off by `build_transforms(..., normalize=False)`: the pipeline then
stops at an 8-bit HWC array, the batch crosses PCIe at a quarter of the fp32 bytes and
`normalize_on_device` (HIP kernel `bev_image_normalize_u8_f32`) produces the bit-identical fp32
[N, 3, H, W] input on the GPU.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import numpy as np
import torch
from PIL import Image, ImageEnhance

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)

__all__ = ["build_transforms", "Compose", "Resize", "RandomApply", "ColorJitter", "ToTensor", "Normalize",
           "ToUint8HWC", "normalize_on_device", "IMAGENET_MEAN", "IMAGENET_STD"]


class Compose:
    def __init__(self, fns: Sequence[Callable]):
        self.transforms = list(fns)

    def __call__(self, x):
        for f in self.transforms:
            x = f(x)
        return x


class Resize:
    """torchvision T.Resize((H, W)) on a PIL image: bilinear PIL resize to exactly (H, W)."""

    def __init__(self, size: Tuple[int, int]):
        self.size = (int(size[0]), int(size[1]))

    def __call__(self, img: Image.Image) -> Image.Image:
        H, W = self.size
        if img.size == (W, H):
            return img
        return img.resize((W, H), Image.BILINEAR)


class RandomApply:
    """Apply the transforms with probability p; one `torch.rand(1)` draw per call."""

    def __init__(self, fns: Sequence[Callable], p: float = 0.5):
        self.transforms = list(fns)
        self.p = float(p)

    def __call__(self, img):
        if self.p < torch.rand(1):
            return img
        for f in self.transforms:
            img = f(img)
        return img


def _range(value: float, center: float = 1.0, bound=(0.0, float("inf"))) -> Tuple[float, float]:
    lo, hi = center - float(value), center + float(value)
    return max(lo, bound[0]), min(hi, bound[1])


def _adjust_hue(img: Image.Image, hue_factor: float) -> Image.Image:
    if not -0.5 <= hue_factor <= 0.5:
        raise ValueError(f"hue_factor ({hue_factor}) is not in [-0.5, 0.5].")
    mode = img.mode
    if mode in {"L", "1", "I", "F"}:
        return img
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    with np.errstate(over="ignore"):
        np_h += np.array(hue_factor * 255).astype(np.uint8)  # uint8 wrap-around, as torchvision
    h = Image.fromarray(np_h, "L")
    return Image.merge("HSV", (h, s, v)).convert(mode)


class ColorJitter:
    """torchvision T.ColorJitter(brightness, contrast, saturation, hue) for PIL images."""

    def __init__(self, brightness: float = 0.0, contrast: float = 0.0, saturation: float = 0.0, hue: float = 0.0):
        self.brightness = _range(brightness) if brightness else None
        self.contrast = _range(contrast) if contrast else None
        self.saturation = _range(saturation) if saturation else None
        self.hue = _range(hue, center=0.0, bound=(-0.5, 0.5)) if hue else None

    def get_params(self):
        fn_idx = torch.randperm(4)
        b = None if self.brightness is None else float(torch.empty(1).uniform_(*self.brightness))
        c = None if self.contrast is None else float(torch.empty(1).uniform_(*self.contrast))
        s = None if self.saturation is None else float(torch.empty(1).uniform_(*self.saturation))
        h = None if self.hue is None else float(torch.empty(1).uniform_(*self.hue))
        return fn_idx, b, c, s, h

    def __call__(self, img: Image.Image) -> Image.Image:
        fn_idx, b, c, s, h = self.get_params()
        for fn_id in fn_idx.tolist():
            if fn_id == 0 and b is not None:
                img = ImageEnhance.Brightness(img).enhance(b)
            elif fn_id == 1 and c is not None:
                img = ImageEnhance.Contrast(img).enhance(c)
            elif fn_id == 2 and s is not None:
                img = ImageEnhance.Color(img).enhance(s)
            elif fn_id == 3 and h is not None:
                img = _adjust_hue(img, h)
        return img


class ToUint8HWC:
    """PIL RGB image -> [H, W, 3] uint8 tensor (what ToTensor reads, before the float conversion)."""

    def __call__(self, img: Image.Image) -> torch.Tensor:
        return torch.from_numpy(np.array(img.convert("RGB"), dtype=np.uint8, copy=True))


class ToTensor:
    """PIL RGB image -> [3, H, W] float32 in [0, 1]: permute, then `.float().div(255)`."""

    def __call__(self, img: Image.Image) -> torch.Tensor:
        t = ToUint8HWC()(img).permute(2, 0, 1).contiguous()
        return t.to(dtype=torch.float32).div(255)


class Normalize:
    def __init__(self, mean: Sequence[float], std: Sequence[float]):
        self.mean = torch.as_tensor(mean, dtype=torch.float32).view(-1, 1, 1)
        self.std = torch.as_tensor(std, dtype=torch.float32).view(-1, 1, 1)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return t.sub(self.mean).div(self.std)


def build_transforms(img_size=(256, 256), normalize: bool = True) -> Compose:
    """The reference pipeline (transforms.py:12-19).  normalize=False stops at uint8 HWC (see module doc)."""
    steps: List[Callable] = [
        Resize(img_size),
        RandomApply([ColorJitter(brightness=0.2, contrast=0.2, saturation=0.2, hue=0.05)], p=0.5),
    ]
    steps += [ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)] if normalize else [ToUint8HWC()]
    return Compose(steps)


def normalize_on_device(images_u8: torch.Tensor, mean=IMAGENET_MEAN, std=IMAGENET_STD) -> torch.Tensor:
    """[B, V, H, W, 3] (or [N, H, W, 3]) uint8 on the GPU -> [B, V, 3, H, W] fp32 ToTensor + Normalize.

    One HIP launch (`bev_image_normalize_u8_f32`); bit-identical to ToTensor + Normalize on the CPU.
    """
    import bev_native as nat

    lead = images_u8.shape[:-3]
    H, W = images_u8.shape[-3], images_u8.shape[-2]
    flat = images_u8.reshape(-1, H, W, 3)
    out = nat.image_normalize_u8(flat, mean, std)
    return out.view(*lead, 3, H, W)
