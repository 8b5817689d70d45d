"""Metre <-> BEV-cell helpers -- drop-in for project/utils/geometry.py (utils/geometry.py:5-21).

Host-side conversions for targets and predictions (not on the hot path): cell (column x, row y) of
a point in metres, clamped to the map, and the metric centre of a cell.
"""
from __future__ import annotations

from typing import Tuple

import torch

__all__ = ["meters_to_bev_indices", "bev_indices_to_meters"]


def _cell_size(bev_bounds, bev_size) -> Tuple[float, float, float, float]:
    x_min, x_max, y_min, y_max = bev_bounds
    H, W = bev_size
    return x_min, y_min, (x_max - x_min) / float(W), (y_max - y_min) / float(H)


def meters_to_bev_indices(xy: torch.Tensor, bev_bounds, bev_size) -> torch.Tensor:
    """[N, 2] metres -> [N, 2] fractional (x, y) cell coordinates, clamped to [0, W-1] x [0, H-1]."""
    x_min, y_min, rx, ry = _cell_size(bev_bounds, bev_size)
    H, W = bev_size
    cols = ((xy[:, 0] - x_min) / rx).clamp(0, W - 1)
    rows = ((xy[:, 1] - y_min) / ry).clamp(0, H - 1)
    return torch.stack([cols, rows], dim=1)


def bev_indices_to_meters(idx: torch.Tensor, bev_bounds, bev_size) -> torch.Tensor:
    """[N, 2] (x, y) cell indices -> [N, 2] metres of the cell centres."""
    x_min, y_min, rx, ry = _cell_size(bev_bounds, bev_size)
    return torch.stack([x_min + (idx[:, 0] + 0.5) * rx, y_min + (idx[:, 1] + 0.5) * ry], dim=1)
