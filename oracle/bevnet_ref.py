"""float64 torch restatement of the reference BEVNet training forward (TEST INFRASTRUCTURE ONLY).

What the reference computes for `model(batch)` in train mode (model_wrapper.py:53-103) with a timm
ResNet trunk, restated with plain torch CPU ops so autograd gives the reference gradients:

  CNNEncoder      timm features_only[out_index] (oracle/backbone_ref.py, BN with batch statistics
                  when the module trains) + the 1x1 proj (cnn_encoder.py:41-46)
  GeometryTransformer  per-(b, v) F.grid_sample(bilinear, zeros, align_corners=False) on the reference's
                  fp32 grid (geometry.py:142-162; oracle.reference_grid_cpu)
  ConcatFusion    [B, V*C, Hb, Wb] (fusion.py:39-46), lazy 1x1 proj (model_wrapper.py:70-73), pos-enc
                  concat (:74-75)
  BEVDetector     3 x (3x3 conv + GroupNorm(32) + ReLU), heads, sigmoid / exp (detector.py:47-62)

It reads the parameters of a (double, CPU) copy of the drop-in's BEVNet, whose state_dict keys are the
reference's, so `.grad` of that copy is the reference gradient.  ReLU decisions can be injected (the
native forward's), as in the trunk tests: an element within fp32 rounding of 0 may switch sides and then
carries its full gradient on one side only.  Used by tests/ only.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

import backbone_ref
from oracle import reference_grid_cpu


def head_forward(det, x, masks=None, check=None):
    """detector.py:47-62 with det's parameters (any dtype / device of det).  `check(pre_activation, mask)`, when given,
    sees each injected ReLU mask beside the reference's own pre-activation (tests compare their signs)."""
    a = x
    for j, (i, d) in enumerate(((0, 1), (3, 2), (6, 1))):
        a = F.conv2d(a, det.stem[i].weight, padding=d, dilation=d)
        a = F.group_norm(a, 32, det.stem[i + 1].weight, det.stem[i + 1].bias, det.stem[i + 1].eps)
        if masks is not None and check is not None:
            check(a, masks[j])
        a = torch.relu(a) if masks is None else a * masks[j]
    hm = F.conv2d(a, det.heatmap_head.weight, det.heatmap_head.bias, padding=1)
    off = F.conv2d(a, det.offset_head.weight, det.offset_head.bias, padding=1)
    size = F.conv2d(a, det.size_head.weight, det.size_head.bias, padding=1)
    return {"heatmap_logits": hm, "heatmap": torch.sigmoid(hm), "offset": torch.sigmoid(off), "offset_raw": off,
            "size": torch.exp(size), "size_raw": size}


def bevnet_train_forward(net, images, K, Rt, trunk_act=None, head_masks=None, head_check=None):
    """net: a float64 CPU BEVNet (lazy modules materialised, timm ResNet trunk); images [B,V,3,H,W] f64;
    K [B,V,3,3], Rt [B,V,4,4] fp32 (the grid is built in fp32 like the reference).  Returns the prediction
    dict of BEVNet.forward without the decoded boxes."""
    enc = net.encoder
    B, V, _, Hi, Wi = images.shape
    x = images.reshape(B * V, *images.shape[2:])
    f = backbone_ref.resnet_features(enc.backbone, x, enc.out_index, grad=True, act=trunk_act or F.relu)
    f = F.conv2d(f, enc.proj.weight, enc.proj.bias)
    C, Hf, Wf = f.shape[1:]
    grid = reference_grid_cpu(K.float(), Rt.float(), (Hi, Wi), Hf, Wf, net.bev_h, net.bev_w, net.bounds)
    warped = F.grid_sample(f, grid.to(f.dtype).reshape(B * V, net.bev_h, net.bev_w, 2), mode="bilinear",
                           padding_mode="zeros", align_corners=False)
    cat = warped.reshape(B, V * C, net.bev_h, net.bev_w)
    main = F.conv2d(cat, net.proj.weight, net.proj.bias)
    bev = torch.cat([main, net.pos_enc.to(main.dtype).unsqueeze(0).expand(B, -1, -1, -1)], dim=1)
    out = head_forward(net.detector, bev, head_masks, head_check)
    out["bev_feat"] = bev
    return out
