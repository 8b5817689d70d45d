"""Multi-GPU sharding of the multi-view -> BEV hot path.

The reference is single-process (no torch.distributed anywhere).  Two ways to
spread the path over the GPUs of a node, one process per GPU:

* frame sharding (BASELINE configs 2/4, the benchmark): frames are
  independent, each rank runs Backbone -> warp -> fusion on its own frames.
  No data-path collective at all; `frame_shard` just splits the frame range.

* data-parallel training (BASELINE config 3): one replica of BEVNet per GPU,
  DistributedDataParallel with gradient all-reduce over RCCL/xGMI
  (`materialize_lazy` -> `ddp_wrap` -> `train_step`).  Per step the gradients
  of the trainable parameters (encoder proj, BEV proj, detector: ~2.9 M
  params, 11.6 MB fp32) fit one 25 MB bucket -> one all-reduce, overlapped
  with the tail of the backward by DDP's bucket hooks.

* camera sharding (BASELINE config 5, 16 cams at 4K, 2 cameras per GPU): each
  rank warps ITS cameras with the fused kernel in SUM mode (a partial BEV sum
  [B, C, Hb, Wb]), then ONE reduce-scatter over BEV rows gives every rank the
  full sum for its slice of rows; mean divides by the global camera count.
  This is the path's only exchange step (RCCL over xGMI; gloo in CPU tests).
  The view-summation order differs from the reference's sequential v = 0..V-1
  (partial sums are added across ranks), so this mode is tolerance-equal
  (max|d| <= 1e-5 * max|x|), not bit-equal -- except at world
  size 1, where the reduce-scatter is the identity and the result is bit-exact.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["frame_shard", "camera_shard", "rows_per_rank", "reduce_partial_bev", "camera_sharded_forward",
           "materialize_lazy", "ddp_wrap", "train_step"]


def frame_shard(num_frames: int, rank: int, world: int) -> range:
    """Contiguous block of frame indices owned by `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    q, r = divmod(num_frames, world)
    start = rank * q + min(rank, r)
    return range(start, start + q + (1 if rank < r else 0))


def camera_shard(num_views: int, rank: int, world: int) -> Tuple[int, int]:
    """[v0, v1) cameras owned by `rank`."""
    rg = frame_shard(num_views, rank, world)
    return rg.start, rg.stop


def rows_per_rank(Hb: int, world: int) -> int:
    """BEV rows of each rank's slice of the reduce-scatter (ceil; the last slices shorter when world does not
    divide Hb)."""
    return -(-Hb // world)


def reduce_partial_bev(partial: torch.Tensor, num_views: int, mode: str = "mean",
                       group: Optional[dist.ProcessGroup] = None, gather: bool = False,
                       bev_h: Optional[int] = None) -> torch.Tensor:
    """Combine per-rank partial BEV maps into the fused result.

    `partial` is this rank's SUM over its cameras (mode sum/mean) or MAX over them (mode max), either as a map
    [B, C, Hb, Wb] or already in rank-chunk-major row order [world, B, C, rows_per_rank(Hb, world), Wb] with zero
    padding rows (GeometryTransformer.forward_fused(rows_per_chunk=...), the fused kernel writing that order
    directly; then `bev_h` = Hb).  Returns this rank's row slice of the fused map (rows [r * rpr, ...)), or the
    whole map when `gather` (one extra all-gather).  One reduce-scatter over BEV rows is the only exchange; a
    map-layout partial is first permuted into chunk order (one extra read + write of it).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if partial.is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device collectives here: exchange through host memory (CPU-process-group tests and
        # hosts without RCCL); RCCL groups exchange device buffers directly over xGMI
        out = reduce_partial_bev(partial.cpu(), num_views, mode, group, gather, bev_h)
        return out.to(partial.device)
    if partial.dim() == 5:  # chunk-major already
        if bev_h is None or partial.shape[0] != world or partial.shape[3] != rows_per_rank(bev_h, world):
            raise ValueError("chunked partial: [world, B, C, rows_per_rank(bev_h, world), Wb] with bev_h given")
        _, B, C, rpr, Wb = partial.shape
        Hb = bev_h
        x = partial
    else:
        B, C, Hb, Wb = partial.shape
        rpr = rows_per_rank(Hb, world)  # the map is zero-padded to world * rpr rows
        if rpr * world != Hb:
            partial = torch.nn.functional.pad(partial, (0, 0, 0, rpr * world - Hb))
        # rows-major chunks so that rank r's slice is the r-th contiguous chunk
        x = partial.reshape(B, C, world, rpr, Wb).permute(2, 0, 1, 3, 4).contiguous()
    out = torch.empty(B, C, rpr, Wb, dtype=partial.dtype, device=partial.device)
    op = dist.ReduceOp.MAX if mode == "max" else dist.ReduceOp.SUM
    dist.reduce_scatter_tensor(out, x.reshape(world * B, C, rpr, Wb), op=op, group=group)
    if mode == "mean":
        out = out / float(num_views)
    if not gather:
        lo, hi = min(rank * rpr, Hb), min((rank + 1) * rpr, Hb)
        return out[:, :, : hi - lo]
    full = torch.empty(world, B, C, rpr, Wb, dtype=out.dtype, device=out.device)
    dist.all_gather_into_tensor(full.view(world * B, C, rpr, Wb), out.contiguous(), group=group)
    return full.permute(1, 2, 0, 3, 4).reshape(B, C, world * rpr, Wb)[:, :, :Hb]


def camera_sharded_forward(geom, feats_local: torch.Tensor, K_local, Rt_local, img_size, num_views: int,
                           mode: str = "mean", group: Optional[dist.ProcessGroup] = None,
                           gather: bool = False) -> torch.Tensor:
    """K5 path: this rank's cameras -> fused partial (HIP kernel) -> reduce-scatter over BEV rows.
    Without an initialised process group this process holds every camera: the fused kernel computes
    the reduction directly (bit-identical to the reference).  On a device (RCCL) group the fused kernel writes its
    partial in rank-chunk-major row order, so the reduce-scatter takes it without a permute copy."""
    if not dist.is_available() or not dist.is_initialized():
        if feats_local.shape[1] != num_views:
            raise ValueError("camera_sharded_forward without a process group needs all cameras")
        return geom.forward_fused(feats_local, K_local, Rt_local, img_size, mode)
    part_mode = "max" if mode == "max" else "sum"
    world = dist.get_world_size(group)
    chunked = world > 1 and feats_local.is_cuda and dist.get_backend(group) != "gloo" and not (
        torch.is_grad_enabled() and feats_local.requires_grad)
    if chunked:
        # exactly `world` chunks of rows_per_rank rows (ceil(Hb / rpr) can be < world, e.g. Hb 120 at world 16:
        # 15 map chunks + one all-zero chunk); layouts the chunk-major kernel does not take are rearranged by
        # warp_fuse itself, so the reduce-scatter always receives [world, B, C, rpr, Wb]
        rpr = rows_per_rank(geom.bev_h, world)
        partial = geom.forward_fused(feats_local, K_local, Rt_local, img_size, part_mode, rows_per_chunk=rpr,
                                     num_chunks=world)
        return reduce_partial_bev(partial, num_views, mode, group, gather, bev_h=geom.bev_h)
    partial = geom.forward_fused(feats_local, K_local, Rt_local, img_size, part_mode)
    return reduce_partial_bev(partial, num_views, mode, group, gather)


# ---------------------------------------------------------------------------
# data-parallel training (BASELINE config 3)
# ---------------------------------------------------------------------------
def materialize_lazy(model: torch.nn.Module, batch) -> None:
    """One no-grad forward so the lazily created submodules exist (encoder proj, BEVNet proj /
    detector: cnn_encoder.py:43-46, model_wrapper.py:70-84) before DDP and the optimizer see the
    parameters.  (The reference builds its optimizer before they exist, quirk Q2.)"""
    was = model.training
    model.eval()
    with torch.no_grad():
        model(batch)
    model.train(was)


def non_persistent_buffers(model: torch.nn.Module):
    """Fully qualified names of the buffers that are not state (ground grid, pos-enc): derived from the
    config, identical on every rank, never worth a broadcast."""
    names = []
    for mname, m in model.named_modules():
        for b in getattr(m, "_non_persistent_buffers_set", ()):
            names.append(f"{mname}.{b}" if mname else b)
    return names


def unexecuted_parameters(model: torch.nn.Module):
    """Fully qualified names of trunk parameters the forward never uses: timm features_only builds every
    stage, CNNEncoder keeps feats_list[out_index] (cnn_encoder.py:41-42) and the stages past it are not run.
    A single-GPU loop does not notice; DDP would wait for their gradients forever (or need
    find_unused_parameters, a graph walk every step), so they are excluded from synchronisation."""
    names = []
    for mname, m in model.named_modules():
        bb = getattr(m, "backbone", None)
        if bb is not None and hasattr(bb, "unexecuted_parameter_names") and hasattr(m, "out_index"):
            pre = f"{mname}.backbone." if mname else "backbone."
            names += [pre + n for n in bb.unexecuted_parameter_names(m.out_index)]
    return names


def ddp_wrap(model: torch.nn.Module, device: Optional[torch.device] = None, bucket_cap_mb: float = 25.0,
             broadcast_buffers: bool = True):
    """DistributedDataParallel over the default group (RCCL on ROCm, gloo on CPU).  Frozen parameters
    (requires_grad False) are not synchronised.

    Buffers: a trainable trunk's BatchNorm uses each rank's own batch statistics (per-rank batch = the
    reference's batch under weak scaling) and updates its running statistics from them.  With
    broadcast_buffers (DDP's default, kept) rank 0's running statistics are broadcast at every forward, so all
    replicas hold the same buffers and the checkpoint rank 0 writes (train.py:336-343) is what every rank would
    write; the ground grid / pos-enc (non-persistent, config-derived) are excluded from that broadcast, and so are
    the trunk stages the encoder never runs (unexecuted_parameters)."""
    from torch.nn.parallel import DistributedDataParallel
    DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(
        model, non_persistent_buffers(model) + unexecuted_parameters(model))
    ids = [device.index] if device is not None and device.type == "cuda" else None
    return DistributedDataParallel(model, device_ids=ids, broadcast_buffers=broadcast_buffers,
                                   bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)


def train_step(model, batch, targets, optimizer, loss_cfg=None, scaler=None) -> dict:
    """One optimisation step as train.py:238-255: forward, BEVNet.loss, backward (DDP all-reduces the
    gradients when `model` is wrapped), optimizer step.  With a `torch.amp.GradScaler` (the reference's
    default, RUNTIME.USE_AMP: true) the forward and loss run under autocast(float16) -- the native kernels
    compute in fp32 inside it (bev_native.amp_fwd) -- and the step goes through scaler.scale / step / update,
    which skips it when a gradient is not finite.  Returns the losses."""
    optimizer.zero_grad(set_to_none=True)
    core = getattr(model, "module", model)
    if scaler is not None:
        with torch.autocast("cuda", dtype=torch.float16):
            preds = model(batch)
            losses = core.loss(preds, targets, loss_cfg or {})
        scaler.scale(losses["total_loss"]).backward()
        scaler.step(optimizer)
        scaler.update()
    else:
        preds = model(batch)
        losses = core.loss(preds, targets, loss_cfg or {})
        losses["total_loss"].backward()
        optimizer.step()
    return {k: float(v.detach()) for k, v in losses.items()}
