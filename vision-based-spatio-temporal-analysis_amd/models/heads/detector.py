"""CenterNet-style BEV detection head -- drop-in for project/models/heads/detector.py.

Same module names (stem / heatmap_head / offset_head / size_head), init and
outputs as the reference (detector.py:7-62), and the same decode (3x3
max-pool peak NMS, threshold, greedy distance NMS; detector.py:64-125).

Scope note: the head sits downstream of the BEV
fusion hot path; it runs on torch/MIOpen ops here.  Moving its 3x3 convs
onto the HIP MFMA conv kernel is the next step for BASELINE config 3.
"""
from typing import Dict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

import bev_native as _nat


def _conv_gn_relu(cin, cout, dilation=1):
    return [nn.Conv2d(cin, cout, kernel_size=3, padding=dilation, dilation=dilation, bias=False),
            nn.GroupNorm(num_groups=32, num_channels=cout), nn.ReLU(inplace=True)]


class BEVDetector(nn.Module):
    def __init__(self, in_channels: int = 32, bev_bounds: Tuple[float, float, float, float] = (-6.0, 6.0, -2.0, 2.0),
                 bev_size: Tuple[int, int] = (64, 64), default_box_wh: Tuple[float, float] = (0.6, 0.6)):
        super().__init__()
        mid1, mid2 = 512, 128
        self.stem = nn.Sequential(*_conv_gn_relu(in_channels, mid1), *_conv_gn_relu(mid1, mid2, dilation=2),
                                  *_conv_gn_relu(mid2, mid2))
        self.heatmap_head = nn.Conv2d(mid2, 1, kernel_size=3, padding=1)
        self.offset_head = nn.Conv2d(mid2, 2, kernel_size=3, padding=1)
        self.size_head = nn.Conv2d(mid2, 2, kernel_size=3, padding=1)
        nn.init.constant_(self.heatmap_head.bias, -2.19)  # CenterNet prior
        nn.init.constant_(self.offset_head.weight, 0.0)
        nn.init.constant_(self.offset_head.bias, 0.0)
        self.bounds = bev_bounds
        self.bev_h, self.bev_w = bev_size
        self.res_x = (bev_bounds[1] - bev_bounds[0]) / float(self.bev_w)
        self.res_y = (bev_bounds[3] - bev_bounds[2]) / float(self.bev_h)
        cells = [max(default_box_wh[0] / max(self.res_x, 1e-6), 1e-3), max(default_box_wh[1] / max(self.res_y, 1e-6), 1e-3)]
        with torch.no_grad():
            self.size_head.bias.copy_(torch.log(torch.tensor(cells, dtype=torch.float32)))

    def forward(self, bev_feat: torch.Tensor) -> Dict:
        shared = self.stem(bev_feat)
        logits = self.heatmap_head(shared)
        offset_raw = self.offset_head(shared)
        size_raw = self.size_head(shared)
        return {"heatmap_logits": logits, "heatmap": torch.sigmoid(logits), "offset": torch.sigmoid(offset_raw),
                "offset_raw": offset_raw, "size": torch.exp(size_raw), "size_raw": size_raw}

    @staticmethod
    def _nms2d(x: torch.Tensor, kernel: int = 3) -> torch.Tensor:
        """detector.py:65-69 (kept for callers; decode() does this on the device)."""
        peak = F.max_pool2d(x, kernel_size=kernel, stride=1, padding=kernel // 2)
        return x * (x == peak).float()

    def decode(self, heatmap, offset, size_cells, conf_thresh: float = 0.4, nms_dist_m: float = 0.5):
        """Peaks -> world boxes [cx, cy, w, h] + scores per frame (detector.py:71-125) on the device:
        bev_decode_peaks_f32 (3x3 peak test + threshold + compaction) and bev_decode_nms_f32 (sort by
        score, box arithmetic, greedy centre-distance NMS).  One host sync per batch, not per pair."""
        return _nat.decode(heatmap, offset, size_cells, self.bounds, conf_thresh, nms_dist_m)


class AnchorDetector(nn.Module):
    def __init__(self):
        super().__init__()
