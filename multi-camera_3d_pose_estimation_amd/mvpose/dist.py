"""Frame sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Frames are independent in the reference's 2D->3D loop (pose_estimation.py:184-190,
:27-53), so the only collectives are: one broadcast of the folded backbone
weights from rank 0 at start-up, and one gather of the per-frame results to
rank 0.  Nothing is exchanged inside a step; per-GPU work is fixed as ranks are
added (weak scaling).  The helpers are backend-agnostic (the CPU tests run them
on gloo).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world_rank():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard(n_total: int, world: int, rank: int):
    """Contiguous, balanced [start, stop) of n_total frames for `rank` (first n % world ranks
    take one extra)."""
    base, extra = divmod(int(n_total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_(tensors, src: int = 0):
    """In-place broadcast of each tensor from `src` (e.g. the backbone's packed weights)."""
    world, _ = world_rank()
    if world > 1:
        for t in tensors:
            dist.broadcast(t, src)
    return tensors


def gather_frames(local: torch.Tensor, n_total: int, root: int = 0):
    """Gather every rank's shard (leading dim = its frame count) into a (n_total, ...) tensor on
    `root` (None elsewhere).  Shards may differ by one frame: they are padded to the largest
    shard for the collective and trimmed on the root."""
    world, rank = world_rank()
    if world == 1:
        return local
    counts = [shard(n_total, world, r) for r in range(world)]
    cap = max(b - a for a, b in counts)
    buf = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, parts, dst=root)
    if rank != root:
        return None
    return torch.cat([p[: b - a] for p, (a, b) in zip(parts, counts)])


def process_sharded(process, frames_total: int, root: int = 0):
    """Run `process(start, stop) -> dict of tensors with leading frame dim` on this rank's
    shard and gather each output to `root`.  Returns the full dict on root, None elsewhere."""
    world, rank = world_rank()
    a, b = shard(frames_total, world, rank)
    local = process(a, b)
    out = {k: gather_frames(v.contiguous(), frames_total, root) for k, v in sorted(local.items())}
    return out if rank == root else None
