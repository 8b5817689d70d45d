"""Prediction output -- drop-in for project/utils/visualization.py.

`save_predictions_json` writes the inference output contract exactly as the reference does
(visualization.py:22-29): one `frame_{idx:06d}.json` per frame holding
{"frame_idx": int, "boxes": [[cx, cy, w, h], ...], "scores": [...]} with the fp32 values
widened to Python floats (the same text as json.dump of `tensor.tolist()`).
`save_bev_heatmap` renders a heatmap PNG like visualization.py:9-19 (matplotlib, optional).
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Sequence

import numpy as np


def _rows(t) -> list:
    if t is None:
        return []
    a = t.detach().cpu().numpy() if hasattr(t, "detach") else np.asarray(t)
    return a.tolist()


def save_predictions_json(boxes_list: Sequence, scores_list: Sequence, save_dir: str,
                          frame_indices: Sequence[int]) -> List[str]:
    """Write frame_{idx:06d}.json for every frame; returns the paths written."""
    os.makedirs(save_dir, exist_ok=True)
    paths = []
    for b, frame_idx in enumerate(frame_indices):
        rec = {"frame_idx": int(frame_idx), "boxes": _rows(boxes_list[b]), "scores": _rows(scores_list[b])}
        path = os.path.join(save_dir, f"frame_{int(frame_idx):06d}.json")
        with open(path, "w") as f:
            json.dump(rec, f)
        paths.append(path)
    return paths


def save_bev_heatmap(heatmap, save_path: str, figsize: Optional[tuple] = (4, 4)) -> None:
    """PNG of a [H, W] (or [B, 1, H, W]: the first frame) heatmap, 'hot' colormap."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    d = os.path.dirname(save_path)
    if d:
        os.makedirs(d, exist_ok=True)
    hm = heatmap.detach().cpu().numpy() if hasattr(heatmap, "detach") else np.asarray(heatmap)
    if hm.ndim == 4:
        hm = hm[0, 0]
    plt.figure(figsize=figsize)
    plt.imshow(hm, cmap="hot", interpolation="nearest")
    plt.colorbar()
    plt.tight_layout()
    plt.savefig(save_path)
    plt.close()
