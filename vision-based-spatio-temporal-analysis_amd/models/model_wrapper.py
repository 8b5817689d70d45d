"""BEVNet -- drop-in for project/models/model_wrapper.py (what train.py / inference.py import).

Same cfg keys, attribute names (encoder, geom, fusion, proj, detector, pos_enc), lazily created modules
(proj, detector) and output dict as the reference (model_wrapper.py:13-124), so state_dicts and the train /
inference loops carry over.  Deliberate difference: lazily created modules are placed on the feature device
(the reference creates the encoder proj on the CPU, quirk Q2).

The computation is reorganised for the GPU:

* BEV projection.  The reference warps every camera's C-channel map to the BEV grid, concatenates the
  V*C-channel result and applies the 1x1 `proj` (model_wrapper.py:74-81).  The bilinear IPM warp is linear
  and acts per channel, and the zero fill of out-of-image cells commutes with a channel mix, so
      proj(concat_v warp_v(f_v)) = sum_v warp_v(W_v f_v) + b,   W_v = proj.weight[:, v*C:(v+1)*C].
  Here each camera's features are first mixed down to P = BEV_PROJ_CH channels in image space (MFMA 1x1
  conv over Hf*Wf pixels instead of Hb*Wb cells) and the V projected maps are warped and summed by ONE fused
  kernel (bev_ipm_warp_fuse_f32, mode "sum") -- the [B, V*C, Hb, Wb] tensor is never formed.  Same value up
  to fp32 reassociation (the BEVNet parity test pins it against the reference's own outputs).
* The head input is assembled channels-last ([B, Hb, Wb, ceil32(P+2)]: projection, pos-enc, zero pad) and
  fed to BEVDetector.forward_nhwc; `bev_feat` is returned as an NCHW view of it.
* Training targets are built for the whole batch at once (no per-object Python loop / host syncs): gaussian
  splats are one scatter_reduce('amax') over every object's footprint.
"""
import math
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

import torch
import torch.nn as nn
import torch.nn.functional as F

import bev_native as _nat

from .encoders.cnn_encoder import CNNEncoder
from .fusion.fusion import ConcatFusion
from .fusion.geometry import GeometryTransformer, _WarpFuseFn
from .heads.detector import BEVDetector, _ceil_to


AMP_FWD_HALF_PANELS = True  # autocast: the projection's forward packs fp16 panels (its backward's arithmetic)


# BEVNet.forward queues its decode and returns bev_native.DetectionList sequences that synchronise when first read
# (A/B: tools/train_step_bench.py --eager-decode)
LAZY_DECODE = True


# BEVNet's focal heatmap and L1 offset / size losses on the GPU run on the native kernels (A/B:
# tools/train_step_bench.py --torch-loss)
NATIVE_LOSS = True

# BEVNet.loss in a training step replays the target construction + loss terms as one captured graph pair
# (torch.cuda.make_graphed_callables): ~50 small launches become two graph launches, so the loss no longer waits on
# the host between the forward and the backward.  Only with NATIVE_LOSS: in this PyTorch / ROCm build a torch
# reduction over more than one workgroup (x.sum() over the 691 k heatmap cells) gives wrong results when replayed
# from a HIP graph -- from the second replay on in isolation (tools/graph_reduce_check.py), the fifth inside the
# round-5 loss graph, whose torch-op focal loss returned -375 (profiles/r06e_loss_graph_cause.txt) -- while the
# native loss kernels (per-workgroup double partials, no cross-workgroup semaphore) replay bit-identically.
# A/B: tools/train_step_bench.py --loss-graph.
LOSS_GRAPHS = False  # measured neutral with the native losses (r06f: 52.3-52.4 vs 52.3-52.5 ms), kept as an A/B


class _FocalLoss(torch.autograd.Function):
    """The focal heatmap loss (model_wrapper.py:235-247) on the native kernels; gradient for the logits only (the
    heatmap targets carry none)."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, logits, gt, alpha: float, beta: float):
        loss, inv = _nat.focal_loss(logits, gt, alpha, beta)
        ctx.save_for_backward(logits, gt, inv)
        ctx.ab = (alpha, beta)
        return loss

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, g):
        logits, gt, inv = ctx.saved_tensors
        return _nat.focal_loss_bwd(logits, gt, *ctx.ab, g.reshape(1), inv), None, None, None


class _L1Losses(torch.autograd.Function):
    """model_wrapper.py:109-116's masked L1 offset and log-size losses on the native kernels -> [2]; gradients for the
    offset / size maps only."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, offset, size, indices, mask, off_t, size_t):
        out = _nat.l1_losses(offset, size, indices, mask, off_t, size_t)
        ctx.save_for_backward(offset, size, indices, mask, off_t, size_t, out)
        return out[:2].clone()

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, g):
        offset, size, indices, mask, off_t, size_t, out = ctx.saved_tensors
        d_off, d_size = _nat.l1_losses_bwd(offset, size, indices, mask, off_t, size_t, g, out)
        return d_off, d_size, None, None, None, None


class _HeadOperand(torch.autograd.Function):
    """x [B,Hb,Wb,cp] channels-last head operand = (s + bias, pos_enc, zeros) per cell (model_wrapper.py:69-75: the
    BEV projection's bias add and the pos-enc concat), s [B,P,Hb,Wb] the fused warp-sum of the projected views: one
    native transpose pass (bev_head_operand_f32) instead of torch's add, permuted cat and, backward, slice + permute;
    the values are the same (one fp32 add).  Gradients: s gets gx[..., :P] back in NCHW, bias its sum over (b, h, w)
    (torch's reduction of the broadcast add's gradient); pos_enc is a buffer."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, s, bias, pos, cp):
        ctx.P = s.shape[1]
        return _nat.head_operand(s, bias, pos, cp)

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, gx):
        if ctx.needs_input_grad[1]:  # the bias gradient from the same pass (block partials added in double)
            gs, gb = _nat.head_operand_bwd_bias(gx, ctx.P)
            if gb is None:
                gb = gs.sum((0, 2, 3))
        else:
            gs, gb = _nat.head_operand_bwd(gx, ctx.P), None
        return gs, gb, None, None


class _ViewProjection(torch.autograd.Function):
    """g[b, v] = W_v (1x1) f[b, v] for channels-last per-camera maps f [B,V,C,Hf,Wf]; returns the projected
    maps as a [B,V,P,Hf,Wf] view of a [B,V,Hf,Wf,P] buffer (the layout the fused warp reads)."""

    @staticmethod
    @_nat.amp_fwd
    def forward(ctx, feats, weight, panels):
        B, V, C, Hf, Wf = feats.shape
        P = weight.shape[0]
        fl = feats.permute(0, 1, 3, 4, 2)
        if not fl.is_contiguous():
            fl = fl.contiguous()
        g = torch.empty(B, V, Hf, Wf, P, device=feats.device, dtype=torch.float32)
        zero = torch.zeros(P, device=feats.device)
        if _nat.half_convs() and AMP_FWD_HALF_PANELS:
            # under autocast(float16) the projection runs in the fp16 arithmetic its backward uses (dgrad / wgrad
            # under the same half mode): pack the per-view slices here, in that precision
            wv = weight.detach().float().view(P, V, C)
            panels = [_nat.pack_conv_weight(wv[:, v].contiguous().view(P, C, 1, 1)) for v in range(V)]
        for v in range(V):
            for b in range(B):
                _nat.conv2d_nhwc_ex(fl[b, v][None], panels[v], zero, P, 1, 0, out=g[b, v][None])
        ctx.save_for_backward(fl, weight)
        return g.permute(0, 1, 4, 2, 3)

    @staticmethod
    @_nat.amp_bwd
    def backward(ctx, dg):
        fl, weight = ctx.saved_tensors
        B, V, Hf, Wf, C = fl.shape
        P = weight.shape[0]
        dgl = dg.permute(0, 1, 3, 4, 2)
        if dgl.is_contiguous():  # the fused-warp backward hands its gradient over channels-last: no transpose
            dgn = dgl
        else:
            dgn = _nat.nchw_to_nhwc(dg.reshape(B * V, P, Hf, Wf)).view(B, V, Hf, Wf, P)
        dfeat = dw = None
        w = weight.detach().float().view(P, V, C)
        if ctx.needs_input_grad[0]:
            dfeat = torch.empty(B, V, Hf, Wf, C, device=dg.device, dtype=torch.float32)
            zero = torch.zeros(C, device=dg.device)
            for v in range(V):
                wt = _nat.pack_conv_weight(w[:, v].t().contiguous().view(C, P, 1, 1))
                for b in range(B):
                    _nat.conv2d_nhwc_ex(dgn[b, v][None], wt, zero, C, 1, 0, out=dfeat[b, v][None])
            dfeat = dfeat.permute(0, 1, 4, 2, 3)
        if ctx.needs_input_grad[1]:
            parts = []
            for v in range(V):
                # one weight-gradient launch over the view's B images (the kernel reduces over every pixel of the
                # batch; conv_wgrad_ex gathers the view's slices, strided by V images, when B > 1)
                parts.append(_nat.conv_wgrad_ex(fl[:, v], dgn[:, v], 1, 0, 1).reshape(P, C))
            # [P, V*C] storage with the parameter's strides (the per-view OIHW views are channels-last-strided;
            # DDP's bucket views compare strides exactly)
            dw = torch.cat(parts, dim=1).view(P, V * C, 1, 1)
        return dfeat, dw, None


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
        self.detector = None  # in_channels = (BEV_PROJ_CH or V*C) + 2, known at the first forward
        self.proj = None
        self.bev_h, self.bev_w = bev_h, bev_w
        self.bounds = bev_bounds
        self.register_buffer("pos_enc", self._create_pos_enc(bev_h, bev_w, bev_bounds), persistent=False)
        self._proj_panels = (None, None)

    @staticmethod
    def _stack_calib(c):
        return torch.stack([torch.stack(v, dim=0) for v in c], dim=0) if isinstance(c, list) else c

    def _view_panels(self, V: int, C: int):
        """Packed per-camera slices W_v of proj.weight (cached until the parameter changes)."""
        w = self.proj.weight
        key = (w.data_ptr(), w._version, V, C)
        if self._proj_panels[0] != key:
            with torch.no_grad():
                wv = w.detach().float().view(w.shape[0], V, C)
                panels = [_nat.pack_conv_weight(wv[:, v].contiguous().view(-1, C, 1, 1)) for v in range(V)]
            self._proj_panels = (key, panels)
        return self._proj_panels[1]

    def _bev_main(self, feats, H, xs, ys, img_hw):
        """[B,V,C,Hf,Wf] features -> BEV map before pos-enc: proj(concat of per-view warps), NCHW (any strides)."""
        B, V, C = feats.shape[:3]
        if self.proj is None and self.bev_proj_ch > 0:
            self.proj = nn.Conv2d(V * C, self.bev_proj_ch, kernel_size=1).to(feats.device)
        if self.proj is None:  # no projection: the concatenated per-view warps (model_wrapper.py:80)
            per_view = _WarpFn_views(feats, H, xs, ys, img_hw)
            return self.fusion(per_view.view(B, V, C, self.bev_h, self.bev_w))
        g = _ViewProjection.apply(feats, self.proj.weight, self._view_panels(V, C))
        s = _WarpFuseFn.apply(g, H, xs, ys, img_hw, "sum")
        return s, self.proj.bias  # the bias is added where the head operand is assembled (_HeadOperand)

    def forward(self, batch: Dict) -> Dict:
        images = batch["images"]  # [B, V, 3, H, W]
        B, V, _, Hi, Wi = images.shape
        feats = self.encoder(images)
        K = self._stack_calib(batch["calib"]["intrinsic"])
        Rt = self._stack_calib(batch["calib"]["extrinsic"])
        # quirk Q1: network-input size; warp_impl='kornia' -> grid_sample semantics unless KORNIA_AVAILABLE
        H, xs, ys, hw = self.geom._sampling(feats, K, Rt, (Hi, Wi))
        main = self._bev_main(feats, H, xs, ys, hw)
        bias = None
        if isinstance(main, tuple):
            main, bias = main
        P = main.shape[1]
        if self.detector is None:
            self.detector = BEVDetector(in_channels=P + 2, bev_bounds=self.bounds, bev_size=(self.bev_h, self.bev_w),
                                        default_box_wh=self.default_box_wh).to(main.device)
        self.detector.grad_channels = P  # the position-encoding channels are a buffer: no gradient
        cp = self.detector.input_channels_padded
        if bias is not None and P <= 512 and main.is_cuda:
            x = _HeadOperand.apply(main, bias, self.pos_enc, cp)  # [B, Hb, Wb, cp] channels-last head operand
        else:
            if bias is not None:
                main = main + bias.view(1, -1, 1, 1)
            pos = self.pos_enc.permute(1, 2, 0).unsqueeze(0).expand(B, -1, -1, -1)
            parts = [main.permute(0, 2, 3, 1), pos]
            if cp > P + 2:
                parts.append(main.new_zeros(B, self.bev_h, self.bev_w, cp - P - 2))
            x = torch.cat(parts, dim=-1)  # [B, Hb, Wb, cp] channels-last head operand
        det = self.detector.forward_nhwc(x)
        # the detections are queued, and the host waits for them only when they are read (a training step reads
        # only the loss: its loss and backward launches then queue behind the forward instead of after a drain)
        boxes, scores = self.detector.decode(det["heatmap"], det["offset"], det["size"],
                                             conf_thresh=self.conf_thresh, nms_dist_m=self.nms_dist_m, lazy=LAZY_DECODE)
        return {"heatmap": det["heatmap"], "heatmap_logits": det["heatmap_logits"], "boxes": boxes, "scores": scores,
                "offset": det["offset"], "offset_raw": det["offset_raw"], "size": det["size"],
                "size_raw": det["size_raw"], "bev_feat": x[..., :P + 2].permute(0, 3, 1, 2)}

    # ---- training objective (model_wrapper.py:105-247) --------------------------
    def loss(self, preds: Dict, targets: List[Dict], loss_cfg: Dict[str, Any]) -> Dict[str, torch.Tensor]:
        pr = (preds["heatmap_logits"], preds["offset"], preds["size_raw"])
        if (LOSS_GRAPHS and NATIVE_LOSS and all(a.is_cuda for a in pr) and torch.is_grad_enabled()
                and any(a.requires_grad for a in pr)):
            boxes, frame, bound = self._target_boxes(targets, pr[0].device, pad=16)
            if bound is not None and boxes.shape[0] > 0:  # host targets: targets + loss terms as one graph pair
                B = len(targets)
                outs = self._graphed((B, bound), pr + (boxes, frame),
                                     lambda *a: self._loss_from_boxes(*a, B=B, bound=bound))
                # the graph's outputs live in its static buffers (overwritten by the next replay): one stack copies
                hm_loss, off_loss, size_loss, total = torch.stack(outs).unbind(0)
                return {"heatmap_loss": hm_loss, "offset_loss": off_loss, "size_loss": size_loss, "total_loss": total}
            t = self._targets_from_boxes(boxes, frame, bound, len(targets))
        else:
            t = self._build_training_targets(targets)
        hm_loss, off_loss, size_loss, total = self._loss_terms(
            *pr, t["heatmap"], t["indices"], t["mask"], t["offset"], t["size_log"])
        return {"heatmap_loss": hm_loss, "offset_loss": off_loss, "size_loss": size_loss, "total_loss": total}

    def _loss_from_boxes(self, logits, offset, size_raw, boxes, frame, B: int, bound: int):
        t = self._targets_from_boxes(boxes, frame, bound, B)
        return self._loss_terms(logits, offset, size_raw, t["heatmap"], t["indices"], t["mask"], t["offset"],
                                t["size_log"])

    def _graphed(self, extra: tuple, args, fn):
        """fn(*args) captured as a HIP graph pair (forward, backward) per input signature
        (torch.cuda.make_graphed_callables) and replayed -- the same kernels on the same values, bit-identical to the
        eager loss (tests/test_targets.py::test_graphed_loss_replays_bit_identical).  Captured with autocast off:
        every loss input is fp32 and the native loss kernels compute in fp32 under autocast(float16) as well."""
        key = extra + tuple((tuple(a.shape), a.dtype, a.requires_grad, a.device) for a in args)
        key += (self.hm_weight, self.offset_weight, self.size_weight, self.hm_alpha, self.hm_beta, self.max_objects)
        graphs = self.__dict__.setdefault("_loss_graphs", {})
        g = graphs.get(key)
        if g is None and len(graphs) >= 8:  # many target signatures (radius bounds, box counts): stay eager
            return fn(*args)
        if g is None:
            samples = tuple(a.detach().clone().requires_grad_(a.requires_grad) for a in args)
            with torch.autocast("cuda", enabled=False):
                g = torch.cuda.make_graphed_callables(fn, samples, allow_unused_input=True)
            graphs[key] = g
        return g(*args)

    def _loss_terms(self, logits, offset, size_raw, hm, indices, mask, off_t, size_t):
        """model_wrapper.py:105-124: the focal heatmap loss and the masked L1 offset / log-size losses."""
        hm_loss = self._heatmap_focal_loss(logits, hm)
        if NATIVE_LOSS and offset.is_cuda and size_raw.is_cuda and indices.is_cuda:
            off_loss, size_loss = _L1Losses.apply(offset, size_raw, indices, mask, off_t, size_t).unbind(0)
        else:
            m = mask.unsqueeze(-1)
            n = m.sum() + 1e-4
            off_loss = (self._gather_feat(offset, indices) - off_t).mul(m).abs().sum() / n
            size_loss = (self._gather_feat(size_raw, indices) - size_t).mul(m).abs().sum() / n
        total = self.hm_weight * hm_loss + self.offset_weight * off_loss + self.size_weight * size_loss
        return hm_loss, off_loss, size_loss, total

    def _target_boxes(self, targets: List[Dict], dev, pad: int = 0
                      ) -> Tuple[torch.Tensor, torch.Tensor, Optional[int]]:
        """All frames' boxes [N, 4] (cx, cy, w, h; centre-only targets get DEFAULT_BOX_WH) + frame index [N] on
        `dev`, and an upper bound of the objects' gaussian radii when it is known without waiting for the device.
        The reference's loader hands the targets over in host memory (train.py:228-243 moves only the images and
        calibration): then the boxes go over in one pinned, asynchronous copy and the bound comes from the host
        values; boxes already on the device give None (the splat then reads its bound back, one sync).  `pad`: host
        boxes are padded to a multiple of it by out-of-grid dummies of the last frame (no slot, no gaussian: the
        targets are unchanged), so a captured loss graph serves every box count up to that multiple."""
        boxes, frame = [], []
        for b, tgt in enumerate(targets):
            bx = tgt.get("boxes_world", None)
            if bx is None or bx.numel() == 0:
                c = tgt.get("centers_world", None)
                bx = None
                if c is not None and c.numel() > 0:
                    c = c.to(torch.float32).reshape(-1, 2)
                    bx = torch.cat([c, c.new_tensor(self.default_box_wh).expand(c.shape[0], 2)], dim=1)
            if bx is None:
                continue
            bx = bx.to(torch.float32).reshape(-1, bx.shape[-1])
            boxes.append(bx[:, :4])
            frame.append(torch.full((bx.shape[0],), b, device=bx.device, dtype=torch.long))
        if not boxes:
            return torch.zeros(0, 4, device=dev), torch.zeros(0, dtype=torch.long, device=dev), None
        if all(not t.is_cuda for t in boxes):
            bh, fh = torch.cat(boxes), torch.cat(frame)
            bound = self._radius_bound_host(bh)
            if pad and bh.shape[0] % pad:
                x_min, _, y_min, _ = self.bounds
                n = pad - bh.shape[0] % pad
                dummy = bh.new_tensor([x_min - 1e6 * self.res_x, y_min - 1e6 * self.res_y, self.res_x, self.res_y])
                bh = torch.cat([bh, dummy.expand(n, 4)])
                fh = torch.cat([fh, fh.new_full((n,), len(targets) - 1)])
            if dev.type == "cuda":
                bh, fh = bh.pin_memory(), fh.pin_memory()
            return bh.to(dev, non_blocking=True), fh.to(dev, non_blocking=True), bound
        return torch.cat([t.to(dev) for t in boxes]), torch.cat([t.to(dev) for t in frame]), None

    def _radius_bound_host(self, boxes: torch.Tensor) -> Optional[int]:
        """An integer >= every gaussian radius _gaussian_radius_tensor gives these (host) boxes: the same formula
        in float64 on the host, floored, plus one (the device's float32 result differs from it by ~1e-7
        relative, far below one cell).  None if a size is not finite."""
        bx = boxes.double().numpy()
        if not np.isfinite(bx).all():
            return None
        # only objects that can be in the grid draw (with a one-cell margin against float32 rounding)
        x_min, _, y_min, _ = self.bounds
        gx, gy = (bx[:, 0] - x_min) / self.res_x, (bx[:, 1] - y_min) / self.res_y
        near = (gx >= -1) & (gx < self.bev_w + 1) & (gy >= -1) & (gy < self.bev_h + 1)
        wh = bx[near, 2:4]
        if wh.shape[0] == 0:
            return 0
        w = np.maximum(np.maximum(wh[:, 0] / self.res_x, 1e-3), 1.0)
        h = np.maximum(np.maximum(wh[:, 1] / self.res_y, 1e-3), 1.0)
        ov = self.gaussian_iou
        r1 = (h + w + np.sqrt(np.maximum((h + w) ** 2 - 4 * w * h * (1 - ov) / (1 + ov), 0.0))) / 2
        r2 = (2 * (h + w) + np.sqrt(np.maximum(4 * (h + w) ** 2 - 16 * (1 - ov) * w * h, 0.0))) / 8
        r = np.minimum(r1, r2)
        if ov != 0:
            r3 = (-2 * ov * (h + w) + np.sqrt(np.maximum((2 * ov * (h + w)) ** 2 - 16 * ov * (ov - 1) * w * h,
                                                         0.0))) / (8 * ov)
            r = np.minimum(r, r3)
        r = np.maximum(r, float(self.gaussian_min_radius))
        return int(np.floor(r.max())) + 1

    def _build_training_targets(self, targets: List[Dict]) -> Dict[str, torch.Tensor]:
        """CenterNet targets (model_wrapper.py:127-203) for the whole batch at once: the first MAX_OBJECTS
        in-grid objects of each frame fill its slots in order; heatmap = per-cell max of their gaussians.
        No host synchronisation when the targets come in host memory: nothing is compacted by a boolean mask
        (objects outside the grid or past MAX_OBJECTS write a discarded slot M / a discarded heatmap cell), and
        the splat's window comes from the host bound (_target_boxes)."""
        dev = next(self.parameters()).device
        return self._targets_from_boxes(*self._target_boxes(targets, dev), len(targets))

    def _targets_from_boxes(self, boxes, frame, bound: Optional[int], B: int) -> Dict[str, torch.Tensor]:
        dev = next(self.parameters()).device
        M, Hb, Wb = self.max_objects, self.bev_h, self.bev_w
        hm_ext = torch.zeros(B * Hb * Wb + 1, device=dev)  # + one discarded cell
        hm = hm_ext[:-1].view(B, 1, Hb, Wb)
        if boxes.shape[0] == 0:
            z = torch.zeros
            return {"heatmap": hm, "indices": z(B, M, dtype=torch.long, device=dev), "mask": z(B, M, device=dev),
                    "offset": z(B, M, 2, device=dev), "size_log": z(B, M, 2, device=dev)}
        x_min, _, y_min, _ = self.bounds
        gx = (boxes[:, 0] - x_min) / self.res_x
        gy = (boxes[:, 1] - y_min) / self.res_y
        inside = (gx >= 0) & (gx < Wb) & (gy >= 0) & (gy < Hb)
        # slot = rank among the frame's in-grid objects (boxes are grouped by frame, in order)
        run = torch.cumsum(inside.long(), 0)
        first = torch.searchsorted(frame, torch.arange(B, device=dev))
        before = torch.where(first > 0, run[(first - 1).clamp(min=0)], torch.zeros_like(first))
        slot = run - 1 - before[frame]
        sel = inside & (slot < M)
        s = torch.where(sel, slot, torch.full_like(slot, M))  # slot M of each frame: discarded
        wh = boxes[:, 2:4]
        cx, cy = torch.floor(gx), torch.floor(gy)
        w_cells = (wh[:, 0] / self.res_x).clamp(min=1e-3)
        h_cells = (wh[:, 1] / self.res_y).clamp(min=1e-3)
        cxl, cyl = cx.long(), cy.long()
        indices = torch.zeros(B, M + 1, dtype=torch.long, device=dev)
        mask = torch.zeros(B, M + 1, device=dev)
        offset = torch.zeros(B, M + 1, 2, device=dev)
        size_log = torch.zeros(B, M + 1, 2, device=dev)
        indices[frame, s] = cyl * Wb + cxl
        mask[frame, s] = torch.ones((), device=dev)  # a device scalar: no host-to-device copy (graph capture)
        offset[frame, s] = torch.stack([gx - cx, gy - cy], dim=1)
        size_log[frame, s] = torch.stack([w_cells.log(), h_cells.log()], dim=1)
        if NATIVE_LOSS and w_cells.is_cuda:  # the same float32 op sequence in one launch
            radius = _nat.gaussian_radius(w_cells, h_cells, self.gaussian_iou, self.gaussian_min_radius)
        else:
            radius = self._gaussian_radius_tensor(w_cells, h_cells)
        self._splat_gaussians(hm_ext, frame, cxl, cyl, radius, sel, bound,
                              (B, Hb, Wb))
        return {"heatmap": hm, "indices": indices[:, :M], "mask": mask[:, :M], "offset": offset[:, :M],
                "size_log": size_log[:, :M]}

    @staticmethod
    def _splat_gaussians(hm_ext: torch.Tensor, b, cx, cy, radius, keep, bound: Optional[int], shape):
        """hm[b, 0] = max(hm, exp(-(dx^2+dy^2) / (2 sigma^2))) over each kept object's clipped (2r+1)^2 window,
        sigma = (2r+1)/6 (the splat of model_wrapper.py:250-276); radius <= 0 draws nothing.  hm_ext = the
        flat heatmap [B*Hb*Wb] + one discarded cell that every masked-out window position writes; `bound` >= the
        largest radius (None: read back from the device).  The maxima are order-free, so the result is the
        same for any bound."""
        B, Hb, Wb = shape
        keep = keep & (radius > 0)
        R = int(torch.where(keep, radius, torch.zeros_like(radius)).max()) if bound is None else bound
        if R <= 0:
            return
        d = torch.arange(-R, R + 1, device=hm_ext.device)
        dy, dx = d.view(-1, 1).expand(-1, d.numel()).reshape(-1), d.repeat(d.numel())
        x = cx[:, None] + dx[None]
        y = cy[:, None] + dy[None]
        r = radius[:, None]
        ok = (keep[:, None] & (dx.abs()[None] <= r) & (dy.abs()[None] <= r) & (x >= 0) & (x < Wb) & (y >= 0)
              & (y < Hb))
        two_s2 = ((2.0 * radius.double() + 1.0) / 6.0) ** 2 * 2.0  # the reference's python-float denominator
        val = torch.exp(-(dx * dx + dy * dy).float()[None] / two_s2.float()[:, None])
        flat = torch.where(ok, (b[:, None] * Hb + y) * Wb + x, B * Hb * Wb)
        hm_ext.scatter_reduce_(0, flat.reshape(-1), torch.where(ok, val, torch.zeros_like(val)).reshape(-1),
                               reduce="amax", include_self=True)

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
        """Penalty-reduced focal loss (model_wrapper.py:235-247), normalised by the number of gt peaks.  On the GPU:
        bev_focal_loss_fwd_f32 / _bwd_f32 (three launches for forward + backward instead of ~60 small torch ones;
        fp32 terms, double sums, so within fp32 rounding of the torch composition)."""
        if NATIVE_LOSS and pred_logits.is_cuda and gt.is_cuda:
            return _FocalLoss.apply(pred_logits.float(), gt.float(), float(self.hm_alpha), float(self.hm_beta))
        p = torch.sigmoid(pred_logits).clamp(1e-4, 1 - 1e-4)
        peak = gt == 1.0
        pos = torch.where(peak, p.log() * (1 - p).pow(self.hm_alpha), torch.zeros_like(p))
        neg = torch.where(gt < 1.0, (1 - p).log() * p.pow(self.hm_alpha) * (1 - gt).pow(self.hm_beta),
                          torch.zeros_like(p))
        return -(pos.sum() + neg.sum()) / peak.sum().float().clamp(min=1.0)

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
        """Single-object splat into a [H, W] map, in place (model_wrapper.py:250-276 API)."""
        x, y = int(center[0]), int(center[1])
        H, W = heatmap.shape
        if int(radius) > 0 and 0 <= x < W and 0 <= y < H:
            dev = heatmap.device
            ext = torch.cat([heatmap.reshape(-1), heatmap.new_zeros(1)])
            self._splat_gaussians(ext, torch.zeros(1, dtype=torch.long, device=dev), torch.tensor([x], device=dev),
                                  torch.tensor([y], device=dev), torch.tensor([int(radius)], device=dev),
                                  torch.ones(1, dtype=torch.bool, device=dev), int(radius), (1, H, W))
            heatmap.copy_(ext[:-1].view(H, W))
        return heatmap

    @staticmethod
    def _gather_feat(feat: torch.Tensor, indices: torch.Tensor) -> torch.Tensor:
        """feat [B, C, H, W], indices [B, K] flat cell ids -> [B, K, C]."""
        B, C = feat.shape[:2]
        return feat.reshape(B, C, -1).gather(2, indices[:, None, :].expand(B, C, -1)).transpose(1, 2)

    def _geom_consistency_loss(self, targets: List[Dict], num_samples: int = 128) -> torch.Tensor:
        """image -> world round trip of random BEV cell centres for the first target's cameras
        (model_wrapper.py:317-340, unused by loss(), kept for callers)."""
        dev = next(self.parameters()).device
        zero = torch.zeros((), device=dev)
        calib = targets[0].get("calib", None) if targets else None
        if calib is None:
            return zero
        Ks, Rts = calib.get("intrinsic", []), calib.get("extrinsic", [])
        x_min, x_max, y_min, y_max = self.bounds
        yy, xx = torch.meshgrid(torch.linspace(y_min, y_max, self.bev_h, device=dev),
                                torch.linspace(x_min, x_max, self.bev_w, device=dev), indexing="ij")
        pts = torch.stack([xx.reshape(-1), yy.reshape(-1), torch.ones_like(xx).reshape(-1)], dim=1)
        pts = pts[torch.randperm(pts.shape[0], device=dev)[:num_samples]]
        loss = zero
        for K, Rt in zip(Ks, Rts):
            fwd = GeometryTransformer._compute_homography(K.to(dev), Rt.to(dev))
            uvw = fwd @ pts.T
            w = torch.where(uvw[2:3].abs() < 1e-6, torch.ones_like(uvw[2:3]), uvw[2:3])
            img = torch.cat([uvw[:2] / w, torch.ones_like(w)], dim=0)
            back = GeometryTransformer._compute_img_to_world_homography(K.to(dev), Rt.to(dev)) @ img
            loss = loss + F.l1_loss(back[:2].T, pts[:, :2])
        return loss / max(1, len(Ks))

    @staticmethod
    def _create_pos_enc(H: int, W: int, bounds: Tuple[float, float, float, float]) -> torch.Tensor:
        """[2, H, W]: sin over normalised x, cos over normalised y (model_wrapper.py:342-353)."""
        x_min, x_max, y_min, y_max = bounds
        yy, xx = torch.meshgrid(torch.linspace(y_min, y_max, H), torch.linspace(x_min, x_max, W), indexing="ij")
        return torch.stack([torch.sin(2.0 * torch.pi * ((xx - x_min) / (x_max - x_min))),
                            torch.cos(2.0 * torch.pi * ((yy - y_min) / (y_max - y_min)))], dim=0)


def _WarpFn_views(feats, H, xs, ys, img_hw):
    """Per-view warps [B*V, C, Hb, Wb] with autograd (GeometryTransformer.forward without the calib step)."""
    from .fusion.geometry import _WarpFn
    B, V, C, Hf, Wf = feats.shape
    f4 = feats.reshape(B * V, C, Hf, Wf) if feats.is_contiguous() else feats.flatten(0, 1)
    return _WarpFn.apply(f4, H, xs, ys, tuple(img_hw))
