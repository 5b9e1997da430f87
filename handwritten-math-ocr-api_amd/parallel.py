"""Image-parallel sharding across GPUs.

Images are independent through the encoder and the greedy decoder, so a global batch
is split into contiguous per-rank shards, one process and one ``Engine`` per GPU,
with no collective on the data path.  The only exchange is the final gather of the
decoded token streams (``[B_local, S+1]`` int32 per rank) to every rank — RCCL over
xGMI with the ``nccl`` backend and CUDA tensors, or gloo on CPU.
"""
from __future__ import annotations


def shard_bounds(n_total: int, world: int, rank: int):
    """Contiguous [start, stop) of rank's shard; shards differ in size by at most one."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_ids(ids_local, world: int, group=None):
    """All-gather equal-shaped per-rank id tensors and concatenate them in rank order."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return ids_local
    if ids_local.is_cuda:
        out = torch.empty((world * ids_local.shape[0],) + tuple(ids_local.shape[1:]), dtype=ids_local.dtype,
                          device=ids_local.device)
        dist.all_gather_into_tensor(out, ids_local.contiguous(), group=group)
        return out
    parts = [torch.empty_like(ids_local) for _ in range(world)]
    dist.all_gather(parts, ids_local.contiguous(), group=group)
    return torch.cat(parts, 0)
