"""Multi-process (world_size 2, gloo, CPU) tests of the sharding logic.

Frame sharding has no collective; camera sharding's single exchange is a
reduce-scatter over BEV rows.  Partial per-rank BEV sums come from the CPU
oracle here (test infrastructure); on the GPU they come from the fused HIP
kernel in SUM mode (bev_dist.camera_sharded_forward).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG, REPO

ORACLE_DIR = os.path.join(os.path.dirname(GOLDEN), "..", "oracle")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    import sys
    for p in (PKG, os.path.abspath(ORACLE_DIR)):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bev_dist
        from oracle import Oracle
        o = Oracle()
        d = np.load(os.path.join(GOLDEN, "warp_w3_v3.npz"))
        B, V, C, Hf, Wf = (int(d[k]) for k in ("B", "V", "C", "Hf", "Wf"))
        feats = np.random.default_rng(int(d["seed"])).standard_normal(size=(B, V, C, Hf, Wf), dtype=np.float32)
        img = (int(d["img_h"]), int(d["img_w"]))
        bounds = tuple(float(x) for x in d["bounds"])
        per_view = o.geometry_forward(feats, d["K"], d["Rt"], img, int(d["bev_h"]), int(d["bev_w"]), bounds)
        v0, v1 = bev_dist.camera_shard(V, rank, world)
        out = {}
        for mode in ("mean", "sum", "max"):
            part = per_view[:, v0:v1]
            partial = o.fuse(part, "max" if mode == "max" else "sum") if v1 > v0 else np.full(
                (B, C) + per_view.shape[3:], -np.inf if mode == "max" else 0.0, np.float32)
            full = bev_dist.reduce_partial_bev(torch.from_numpy(partial), V, mode, gather=True)
            sl = bev_dist.reduce_partial_bev(torch.from_numpy(partial), V, mode, gather=False)
            # the same partial in the rank-chunk-major layout the fused kernel writes for device groups
            # (bev_ipm_warp_fuse_chunked_f32): [world, B, C, rows_per_rank, Wb], padding rows zero
            Hb = partial.shape[2]
            rpr = bev_dist.rows_per_rank(Hb, world)
            pad = np.zeros((B, C, rpr * world, partial.shape[3]), np.float32)
            pad[:, :, :Hb] = partial
            ck = torch.from_numpy(np.ascontiguousarray(pad.reshape(B, C, world, rpr, -1).transpose(2, 0, 1, 3, 4)))
            full_c = bev_dist.reduce_partial_bev(ck, V, mode, gather=True, bev_h=Hb)
            sl_c = bev_dist.reduce_partial_bev(ck, V, mode, gather=False, bev_h=Hb)
            same = bool(torch.equal(full_c, full) and torch.equal(sl_c, sl))
            out[mode] = (full.numpy(), sl.numpy(), o.fuse(per_view, mode), same)
        result_q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_frame_shard_partitions():
    import bev_dist
    for n in (0, 1, 7, 8, 13, 64):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                got.extend(bev_dist.frame_shard(n, r, world))
            assert got == list(range(n))
    assert bev_dist.camera_shard(16, 3, 8) == (6, 8)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_camera_sharded_reduce_scatter(world):
    """world 2: BEV rows split evenly; world 3: 3 cameras over 3 ranks and BEV rows NOT a multiple of the
    group size (zero-padded reduce-scatter, shorter last slice)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank in range(world):
        for mode, (full, sl, ref, same_chunked) in res[rank].items():
            assert same_chunked, (mode, "chunk-major partial gives another result")
            scale = max(np.abs(ref).max(), 1e-30)
            if mode == "max":
                assert np.array_equal(full, ref), mode  # max is order-independent
            else:
                assert np.abs(full - ref).max() <= 1e-5 * scale, mode
            rows = -(-ref.shape[2] // world)
            np.testing.assert_array_equal(sl, full[:, :, rank * rows:(rank + 1) * rows])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2])
def test_bench_orchestration_dry_run(world):
    """bench.py's multi-rank path itself (spawn_ranks -> torch.distributed.run -> one process per rank, the
    barrier-bracketed timed region, the MAX reduction of the elapsed time, rank 0's JSON line) on the CPU with
    gloo and a placeholder step: the same code the driver's 8-GPU run executes, minus the hot path."""
    import json
    import subprocess
    import sys
    steps, batch = 5, 2
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--gpus", str(world), "--steps", str(steps),
           "--warmup", "1", "--batch", str(batch)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == steps
    assert d["frames"] == world * batch * steps
    assert len(d["rank_elapsed_s"]) == world
    assert d["elapsed_s"] == max(d["rank_elapsed_s"])  # MAX over ranks
    # the slowest rank sleeps world x 5 ms per step: the reported time per step covers it
    assert d["ms_per_step"] >= 5.0 * world
    assert abs(d["value"] - d["frames"] / d["elapsed_s"]) <= 1e-3 * d["value"]
