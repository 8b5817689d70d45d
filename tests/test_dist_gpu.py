"""Camera sharding (BASELINE config 5) on the GPU through RCCL.

One GPU per box, so the process group has one rank: the fused HIP kernel produces the
partial SUM / MAX of all cameras, the reduce-scatter over BEV rows runs through RCCL
(identity at world 1) and the mean divides by the camera count -- which makes the
result bit-identical to the reference's warp + SimpleFusion on the same inputs.
At world 2 (two rank processes sharing the box's GPU, gloo over host memory -- RCCL cannot put two ranks on
one device) each rank's partial comes from the fused HIP kernel on its 8 cameras and the reduce-scatter
combines them: tolerance-equal to the reference (the view-sum order changes), max bit-exact.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG, gather_results

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


def _cam_worker(rank, world, port, ref_path, q):
    import sys
    sys.path.insert(0, PKG)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import bev_dist
        from models.fusion.geometry import GeometryTransformer
        d = np.load(os.path.join(GOLDEN, "warp_w5_16cam_4k.npz"))
        B, V, Hf, Wf = (int(d[k]) for k in ("B", "V", "Hf", "Wf"))
        g = GeometryTransformer(int(d["bev_h"]), int(d["bev_w"]), tuple(float(x) for x in d["bounds"]))
        img = (int(d["img_h"]), int(d["img_w"]))
        feats = np.random.default_rng(31).standard_normal(size=(B, V, 64, Hf, Wf), dtype=np.float32)
        v0, v1 = bev_dist.camera_shard(V, rank, world)
        f = torch.from_numpy(feats[:, v0:v1]).to(DEV).permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)
        K, Rt = torch.from_numpy(d["K"][:, v0:v1]).to(DEV), torch.from_numpy(d["Rt"][:, v0:v1]).to(DEV)
        refs = np.load(ref_path)
        res = {}
        for mode in ("mean", "max"):
            full = bev_dist.camera_sharded_forward(g, f, K, Rt, img, V, mode, gather=True)
            sl = bev_dist.camera_sharded_forward(g, f, K, Rt, img, V, mode, gather=False)
            torch.cuda.synchronize()
            assert full.is_cuda and sl.is_cuda
            full, sl = full.cpu().numpy(), sl.cpu().numpy()
            ref = refs[mode]
            rows = -(-ref.shape[2] // world)
            res[mode] = (float(np.abs(full - ref).max()), float(np.abs(ref).max()),
                         bool(np.array_equal(bits(full), bits(ref))),
                         bool(np.array_equal(sl, full[:, :, rank * rows:(rank + 1) * rows])))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_camera_sharded_forward_world2_kernel_partials(oracle, tmp_path):
    """BASELINE configs[4] exchange with real kernel outputs: 16 cameras at 4K (270 x 480 x 64 features ->
    480 x 1440), 8 cameras per rank, partial SUM / MAX from the fused HIP kernel, ONE reduce-scatter over BEV
    rows (+ all-gather) -> vs the oracle's fused mean / max over all 16 cameras: mean within 1e-5 x max|ref|
    (the view-sum order changes), max bit-exact; each rank's slice is its rows of the full map."""
    d = np.load(os.path.join(GOLDEN, "warp_w5_16cam_4k.npz"))
    B, V, Hf, Wf = (int(d[k]) for k in ("B", "V", "Hf", "Wf"))
    img = (int(d["img_h"]), int(d["img_w"]))
    feats = np.random.default_rng(31).standard_normal(size=(B, V, 64, Hf, Wf), dtype=np.float32)
    bounds = tuple(float(x) for x in d["bounds"])
    refs = oracle.fused_stream(feats, d["K"], d["Rt"], img, int(d["bev_h"]), int(d["bev_w"]), bounds)
    ref_path = str(tmp_path / "refs.npz")
    np.savez(ref_path, mean=refs["mean"], max=refs["max"])
    del feats, refs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cam_worker, args=(r, 2, port, ref_path, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(gather_results(procs, q, 2, 240))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank in (0, 1):
        err, scale, _, slice_ok = res[rank]["mean"]
        assert err <= 1e-5 * scale and slice_ok, (rank, err, scale)
        _, _, exact, slice_ok = res[rank]["max"]
        assert exact and slice_ok, rank


@pytest.mark.timeout(300)
def test_fused_warp_rank_chunk_major_layout():
    """bev_ipm_warp_fuse_chunked_f32 (the camera-shard partial written in reduce-scatter order) holds exactly the
    plain fused map's values: out[r, b, c, k, x] == plain[b, c, r * rpr + k, x] bit for bit, padding rows zero --
    16-camera 4K fixture geometry (sum / max / mean) at rows per rank 60 (8 ranks), 17 (ragged: 29 chunks, 13-row
    tail) and 240 (2 ranks), and the bench's 7-camera rig at batch 2."""
    import bev_native as nat
    import bev_rig
    from models.fusion.geometry import GeometryTransformer
    d = np.load(os.path.join(GOLDEN, "warp_w5_16cam_4k.npz"))
    B, V, Hf, Wf = (int(d[k]) for k in ("B", "V", "Hf", "Wf"))
    cases = [(GeometryTransformer(int(d["bev_h"]), int(d["bev_w"]), tuple(float(x) for x in d["bounds"])),
              (int(d["img_h"]), int(d["img_w"])), B, V, Hf, Wf, torch.from_numpy(d["K"]), torch.from_numpy(d["Rt"]))]
    K7, Rt7 = bev_rig.rig(7, 1080, 1920, 2)
    cases.append((GeometryTransformer(480, 1440, (-24.0, 24.0, -7.2, 7.2)), (1080, 1920), 2, 7, 135, 240,
                  torch.from_numpy(K7), torch.from_numpy(Rt7)))
    for g, img, B, V, Hf, Wf, K, Rt in cases:
        gen = torch.Generator(device=DEV).manual_seed(4)
        f = torch.randn(B, V, Hf, Wf, 64, device=DEV, generator=gen).permute(0, 1, 4, 2, 3)
        K, Rt = K.to(DEV), Rt.to(DEV)
        with torch.no_grad():
            for mode in ("sum", "max", "mean"):
                plain = g.forward_fused(f, K, Rt, img, mode)
                for rpr in (60, 17, 240):
                    ck = g.forward_fused(f, K, Rt, img, mode, rows_per_chunk=rpr)
                    n = -(-g.bev_h // rpr)
                    assert tuple(ck.shape) == (n, B, 64, rpr, g.bev_w)
                    flat = ck.permute(1, 2, 0, 3, 4).reshape(B, 64, n * rpr, g.bev_w)
                    assert torch.equal(flat[:, :, :g.bev_h].view(torch.int32), plain.view(torch.int32)), (mode, rpr)
                    assert not flat[:, :, g.bev_h:].any(), (mode, rpr)
    assert nat.lib().bev_abi_version() == nat.ABI_VERSION


@pytest.mark.timeout(300)
@pytest.mark.parametrize("Hb,world,C,nhwc", [(120, 16, 64, True), (9, 4, 64, True), (120, 16, 20, False),
                                             (97, 3, 64, False)])
def test_fused_warp_chunked_world_chunks_and_any_layout(Hb, world, C, nhwc):
    """camera_sharded_forward's partial: exactly `world` chunks of rows_per_rank(Hb, world) rows even when
    ceil(Hb / rpr) < world (Hb 120 at world 16: 15 map chunks + 1 zero chunk; Hb 9 at world 4: 3 + 1), and for
    feature layouts the chunk-major LDS-DMA kernel does not take (NCHW storage, C % 64 != 0), which run the plain
    fused launch + a rearranging copy -- all bit-equal to the plain map, the rows / chunks past it zero."""
    import bev_rig
    from bev_dist import rows_per_rank
    from models.fusion.geometry import GeometryTransformer
    g = GeometryTransformer(Hb, 3 * Hb + 5, (-24.0, 24.0, -7.2, 7.2))
    B, V, Hf, Wf = 2, 5, 34, 60
    K, Rt = bev_rig.rig(V, 270, 480, B)
    K, Rt = torch.from_numpy(K).to(DEV), torch.from_numpy(Rt).to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(Hb + C)
    if nhwc:
        f = torch.randn(B, V, Hf, Wf, C, device=DEV, generator=gen).permute(0, 1, 4, 2, 3)
    else:
        f = torch.randn(B, V, C, Hf, Wf, device=DEV, generator=gen)
    rpr = rows_per_rank(Hb, world)
    with torch.no_grad():
        for mode in ("sum", "max"):
            plain = g.forward_fused(f, K, Rt, (270, 480), mode)
            ck = g.forward_fused(f, K, Rt, (270, 480), mode, rows_per_chunk=rpr, num_chunks=world)
            assert tuple(ck.shape) == (world, B, C, rpr, g.bev_w)
            flat = ck.permute(1, 2, 0, 3, 4).reshape(B, C, world * rpr, g.bev_w)
            assert torch.equal(flat[:, :, :Hb].view(torch.int32), plain.view(torch.int32)), mode
            assert not flat[:, :, Hb:].any(), mode
