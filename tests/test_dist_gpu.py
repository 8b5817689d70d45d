"""Camera sharding (BASELINE config 5) on the GPU through RCCL.

One GPU per box, so the process group has one rank: the fused HIP kernel produces the
partial SUM / MAX of all cameras, the reduce-scatter over BEV rows runs through RCCL
(identity at world 1) and the mean divides by the camera count -- which makes the
result bit-identical to the reference's warp + SimpleFusion on the same inputs.
Multi-rank exchanges are covered on the CPU with gloo (tests/test_dist_gloo.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_camera_sharded_forward_rccl_world1(oracle):
    """16-camera 4K rig (feature maps 270 x 480 -> 480 x 1440), C = 64 channels-last, sum / mean / max."""
    import bev_dist
    from models.fusion.geometry import GeometryTransformer
    d = np.load(os.path.join(GOLDEN, "warp_w5_16cam_4k.npz"))
    B, V, Hf, Wf = (int(d[k]) for k in ("B", "V", "Hf", "Wf"))
    g = GeometryTransformer(int(d["bev_h"]), int(d["bev_w"]), tuple(float(x) for x in d["bounds"]))
    img = (int(d["img_h"]), int(d["img_w"]))
    feats = np.random.default_rng(31).standard_normal(size=(B, V, 64, Hf, Wf), dtype=np.float32)
    refs = oracle.fused_stream(feats, d["K"], d["Rt"], img, g.bev_h, g.bev_w, g.bounds)
    f = torch.from_numpy(feats).to(DEV).permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)
    K, Rt = torch.from_numpy(d["K"]).to(DEV), torch.from_numpy(d["Rt"]).to(DEV)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device(DEV))
    try:
        for mode, ref in refs.items():
            v0, v1 = bev_dist.camera_shard(V, dist.get_rank(), dist.get_world_size())
            for gather in (False, True):
                out = bev_dist.camera_sharded_forward(g, f[:, v0:v1], K[:, v0:v1], Rt[:, v0:v1], img, V, mode,
                                                      gather=gather)
                torch.cuda.synchronize()
                assert np.array_equal(bits(out.cpu().numpy()), bits(ref)), (mode, gather)
    finally:
        dist.destroy_process_group()
    # without a process group the same call is the fused kernel itself
    out = bev_dist.camera_sharded_forward(g, f, K, Rt, img, V, "mean")
    assert np.array_equal(bits(out.cpu().numpy()), bits(refs["mean"]))
