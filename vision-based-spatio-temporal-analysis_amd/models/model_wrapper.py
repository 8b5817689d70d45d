"""BEVNet -- drop-in for project/models/model_wrapper.py (what train.py / inference.py import).

Wiring (model_wrapper.py:41-43, 53-69): CNNEncoder -> GeometryTransformer
(warp_impl='kornia', which -- as in the reference without kornia -- runs the
grid_sample semantics, quirk Q7) -> ConcatFusion -> lazy 1x1 BEV proj ->
2-channel positional encoding -> lazy BEVDetector -> decode.  The encoder and
the warp run on the HIP kernels; proj / head / decode / loss run on torch ops
(they are downstream of the fused BEV hot path).

Same cfg keys, attribute names (encoder, geom, fusion, proj, detector,
pos_enc) and output dict as the reference, so state_dicts and the train /
inference loops carry over.  Deliberate difference: lazily created modules
are placed on the feature device (the reference creates the encoder proj on
the CPU, quirk Q2).
"""
import math
from typing import Any, Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .encoders.cnn_encoder import CNNEncoder
from .fusion.fusion import ConcatFusion
from .fusion.geometry import GeometryTransformer
from .heads.detector import BEVDetector


class BEVNet(nn.Module):
    def __init__(self, cfg: Dict[str, Any]):
        super().__init__()
        m = cfg["MODEL"]
        feat_dim = int(m["FEAT_DIM"])
        bev_h, bev_w = m["BEV_SIZE"][1], m["BEV_SIZE"][2]
        bev_bounds = tuple(m["BEV_BOUNDS"])
        self.bev_proj_ch = int(m.get("BEV_PROJ_CH", 0))
        ev = cfg.get("EVAL", {})
        self.conf_thresh = float(ev.get("CONF_THRESH", 0.4))
        self.nms_dist_m = float(ev.get("NMS_DIST_M", 0.5))
        lc = cfg.get("LOSS", {})
        self.default_box_wh = tuple(lc.get("DEFAULT_BOX_WH", [0.6, 0.6]))
        self.max_objects = int(lc.get("MAX_OBJECTS", 64))
        self.hm_alpha = float(lc.get("HM_ALPHA", 2.0))
        self.hm_beta = float(lc.get("HM_BETA", 4.0))
        self.hm_weight = float(lc.get("HM_WEIGHT", 1.0))
        self.offset_weight = float(lc.get("OFFSET_WEIGHT", 1.0))
        self.size_weight = float(lc.get("SIZE_WEIGHT", 0.1))
        self.gaussian_min_radius = int(lc.get("GAUSSIAN_MIN_RADIUS", 2))
        self.gaussian_iou = float(lc.get("GAUSSIAN_IOU", 0.7))
        self.res_x = (bev_bounds[1] - bev_bounds[0]) / float(bev_w)
        self.res_y = (bev_bounds[3] - bev_bounds[2]) / float(bev_h)

        # MODEL.BACKBONE_IMPL (extension; default "auto"): "fallback" selects the reference's timm-less
        # 2-conv encoder for any backbone name (cnn_encoder.py:31-37) -- what the reference runs offline
        self.encoder = CNNEncoder(out_channels=feat_dim, backbone=m["BACKBONE"],
                                  pretrained=bool(m.get("PRETRAINED", False)), out_index=int(m.get("OUT_INDEX", 2)),
                                  backbone_impl=str(m.get("BACKBONE_IMPL", "auto")))
        self.geom = GeometryTransformer(bev_h=bev_h, bev_w=bev_w, bev_bounds=bev_bounds, warp_impl="kornia")
        self.fusion = ConcatFusion()
        self.detector = None  # in_channels = V*C (+proj) + 2, known at the first forward
        self.proj = None
        self.bev_h, self.bev_w = bev_h, bev_w
        self.bounds = bev_bounds
        self.register_buffer("pos_enc", self._create_pos_enc(bev_h, bev_w, bev_bounds), persistent=False)

    @staticmethod
    def _stack_calib(c):
        return torch.stack([torch.stack(v, dim=0) for v in c], dim=0) if isinstance(c, list) else c

    def forward(self, batch: Dict) -> Dict:
        images = batch["images"]  # [B, V, 3, H, W]
        B, V, _, H, W = images.shape
        feats = self.encoder(images)
        K = self._stack_calib(batch["calib"]["intrinsic"])
        Rt = self._stack_calib(batch["calib"]["extrinsic"])
        bev_per_view = self.geom(feats, K, Rt, img_size=(H, W))  # quirk Q1: network-input size
        bev_concat = self.fusion(bev_per_view)
        if self.proj is None and self.bev_proj_ch > 0:
            self.proj = nn.Conv2d(bev_concat.shape[1], self.bev_proj_ch, kernel_size=1).to(bev_concat.device)
        bev_main = self.proj(bev_concat) if self.proj is not None else bev_concat
        bev_feat = torch.cat([bev_main, self.pos_enc.unsqueeze(0).expand(B, -1, -1, -1)], dim=1)
        if self.detector is None:
            self.detector = BEVDetector(in_channels=bev_feat.shape[1], bev_bounds=self.bounds,
                                        bev_size=(self.bev_h, self.bev_w),
                                        default_box_wh=self.default_box_wh).to(bev_feat.device)
        det = self.detector(bev_feat)
        boxes, scores = self.detector.decode(det["heatmap"], det["offset"], det["size"],
                                             conf_thresh=self.conf_thresh, nms_dist_m=self.nms_dist_m)
        return {"heatmap": det["heatmap"], "heatmap_logits": det["heatmap_logits"], "boxes": boxes, "scores": scores,
                "offset": det["offset"], "offset_raw": det["offset_raw"], "size": det["size"],
                "size_raw": det["size_raw"], "bev_feat": bev_feat}

    # ---- training objective (model_wrapper.py:105-247) --------------------------
    def loss(self, preds: Dict, targets: List[Dict], loss_cfg: Dict[str, Any]) -> Dict[str, torch.Tensor]:
        t = self._build_training_targets(targets)
        hm_loss = self._heatmap_focal_loss(preds["heatmap_logits"], t["heatmap"])
        mask = t["mask"].unsqueeze(-1)
        denom = mask.sum() + 1e-4
        off = self._gather_feat(preds["offset"], t["indices"])
        off_loss = F.l1_loss(off * mask, t["offset"] * mask, reduction="sum") / denom
        siz = self._gather_feat(preds["size_raw"], t["indices"])
        size_loss = F.l1_loss(siz * mask, t["size_log"] * mask, reduction="sum") / denom
        total = self.hm_weight * hm_loss + self.offset_weight * off_loss + self.size_weight * size_loss
        return {"heatmap_loss": hm_loss, "offset_loss": off_loss, "size_loss": size_loss, "total_loss": total}

    def _build_training_targets(self, targets: List[Dict]) -> Dict[str, torch.Tensor]:
        dev = next(self.parameters()).device
        B = len(targets)
        hm = torch.zeros(B, 1, self.bev_h, self.bev_w, device=dev)
        indices = torch.zeros(B, self.max_objects, dtype=torch.long, device=dev)
        mask = torch.zeros(B, self.max_objects, dtype=torch.float32, device=dev)
        offset = torch.zeros(B, self.max_objects, 2, device=dev)
        size_log = torch.zeros(B, self.max_objects, 2, device=dev)
        x_min, _, y_min, _ = self.bounds
        wh = torch.tensor(self.default_box_wh, device=dev, dtype=torch.float32)
        for b, tgt in enumerate(targets):
            boxes = tgt.get("boxes_world", None)
            if boxes is None or boxes.numel() == 0:
                c = tgt.get("centers_world", None)
                if c is not None and c.numel() > 0:
                    boxes = torch.cat([c, wh.to(c.device).repeat(c.shape[0], 1)], dim=1)
            if boxes is None or boxes.numel() == 0:
                continue
            boxes = boxes.to(dev)
            rel = torch.stack([(boxes[:, 0] - x_min) / self.res_x, (boxes[:, 1] - y_min) / self.res_y], dim=1)
            ok = (rel[:, 0] >= 0) & (rel[:, 0] < self.bev_w) & (rel[:, 1] >= 0) & (rel[:, 1] < self.bev_h)
            if not torch.any(ok):
                continue
            keep = torch.nonzero(ok, as_tuple=False).squeeze(1)[: self.max_objects]
            rel, sizes = rel[keep], boxes[keep, 2:]
            gfl = torch.floor(rel)
            w_cells = (sizes[:, 0] / self.res_x).clamp(min=1e-3)
            h_cells = (sizes[:, 1] / self.res_y).clamp(min=1e-3)
            radii = self._gaussian_radius_tensor(w_cells, h_cells)
            gi = gfl.to(torch.long)
            n = rel.shape[0]
            indices[b, :n] = gi[:, 1] * self.bev_w + gi[:, 0]
            mask[b, :n] = 1.0
            offset[b, :n] = rel - gfl
            size_log[b, :n] = torch.stack([w_cells.log(), h_cells.log()], dim=1)
            for k in range(n):
                hm[b, 0] = self._draw_gaussian(hm[b, 0], (int(gi[k, 0]), int(gi[k, 1])), int(radii[k]))
        return {"heatmap": hm, "indices": indices, "mask": mask, "offset": offset, "size_log": size_log}

    def _gaussian_radius_tensor(self, width_cells: torch.Tensor, height_cells: torch.Tensor) -> torch.Tensor:
        """CenterNet radius, same tensor arithmetic (and rounding) as model_wrapper.py:205-233."""
        w = width_cells.clamp(min=1.0)
        h = height_cells.clamp(min=1.0)
        ov = self.gaussian_iou

        def root(a, b, c):  # larger root numerator of a x^2 + b x + c, clamped discriminant
            return b + torch.sqrt(torch.clamp(b ** 2 - 4 * a * c, min=0.0))

        r1 = root(torch.ones_like(w), h + w, w * h * (1 - ov) / (1 + ov)) / 2
        a2 = torch.full_like(w, 4.0)
        r2 = root(a2, 2 * (h + w), (1 - ov) * w * h) / (2 * a2)
        if ov == 0:
            r3 = torch.full_like(w, float("inf"))
        else:
            a3 = torch.full_like(w, 4 * ov)
            r3 = root(a3, -2 * ov * (h + w), (ov - 1) * w * h) / (2 * a3)
        r = torch.clamp(torch.min(torch.min(r1, r2), r3), min=float(self.gaussian_min_radius))
        return torch.floor(r).to(torch.long)

    def _heatmap_focal_loss(self, pred_logits: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
        p = torch.clamp(torch.sigmoid(pred_logits), min=1e-4, max=1 - 1e-4)
        pos = gt.eq(1.0)
        neg = gt.lt(1.0)
        pos_loss = torch.log(p) * torch.pow(1 - p, self.hm_alpha) * pos
        neg_loss = torch.log(1 - p) * torch.pow(p, self.hm_alpha) * torch.pow(1 - gt, self.hm_beta) * neg
        return -(pos_loss.sum() + neg_loss.sum()) / pos.float().sum().clamp(min=1.0)

    def _gaussian_radius(self, width_cells: float, height_cells: float) -> int:
        """Scalar variant (unused by loss()); keeps the reference's '/2' for r2 (quirk Q10)."""
        w, h = max(width_cells, 1.0), max(height_cells, 1.0)
        ov = self.gaussian_iou
        b1 = h + w
        r1 = (b1 + math.sqrt(max(0.0, b1 ** 2 - 4 * (w * h * (1 - ov) / (1 + ov))))) / 2
        b2 = 2 * (h + w)
        r2 = (b2 + math.sqrt(max(0.0, b2 ** 2 - 16 * (1 - ov) * w * h))) / 2
        a3 = 4 * ov
        r3 = float("inf") if a3 == 0 else (-2 * ov * (h + w) + math.sqrt(
            max(0.0, (2 * ov * (h + w)) ** 2 - 4 * a3 * (ov - 1) * w * h))) / (2 * a3)
        return max(self.gaussian_min_radius, int(min(r1, r2, r3)))

    def _draw_gaussian(self, heatmap: torch.Tensor, center: Tuple[int, int], radius: int) -> torch.Tensor:
        radius = int(radius)
        if radius <= 0:
            return heatmap
        sigma = (2 * radius + 1) / 6.0
        x, y = center
        H, W = heatmap.shape
        if x < 0 or y < 0 or x >= W or y >= H:
            return heatmap
        left, right = min(x, radius), min(W - x - 1, radius)
        top, bottom = min(y, radius), min(H - y - 1, radius)
        yr = torch.arange(-top, bottom + 1, device=heatmap.device, dtype=heatmap.dtype)
        xr = torch.arange(-left, right + 1, device=heatmap.device, dtype=heatmap.dtype)
        yy, xx = torch.meshgrid(yr, xr, indexing="ij")
        g = torch.exp(-(xx ** 2 + yy ** 2) / (2 * sigma * sigma))
        patch = heatmap[y - top:y + bottom + 1, x - left:x + right + 1]
        torch.maximum(patch, g, out=patch)
        return heatmap

    @staticmethod
    def _gather_feat(feat: torch.Tensor, indices: torch.Tensor) -> torch.Tensor:
        B, C, H, W = feat.shape
        flat = feat.view(B, C, -1).permute(0, 2, 1)
        return torch.gather(flat, 1, indices.unsqueeze(-1).expand(-1, -1, C))

    @staticmethod
    def _create_pos_enc(H: int, W: int, bounds: Tuple[float, float, float, float]) -> torch.Tensor:
        """[2, H, W]: sin over normalised x, cos over normalised y (model_wrapper.py:342-353)."""
        x_min, x_max, y_min, y_max = bounds
        yy, xx = torch.meshgrid(torch.linspace(y_min, y_max, H), torch.linspace(x_min, x_max, W), indexing="ij")
        return torch.stack([torch.sin(2.0 * torch.pi * ((xx - x_min) / (x_max - x_min))),
                            torch.cos(2.0 * torch.pi * ((yy - y_min) / (y_max - y_min)))], dim=0)
