"""Image-parallel sharding across GPUs (BASELINE config 3).

Images are independent through the Swin encoder and the greedy decoder, so a global
batch is split into contiguous per-rank shards, one process and one ``Engine`` per GPU,
with no collective on the data path.  The only exchange is the final all-gather of the
decoded token streams (``[B_local, S+1]`` int32 per rank): ``RcclGroup`` runs it inside
libmathocr.so over RCCL (xGMI) on device memory (``mocr_group_*`` in include/mathocr.h).
``torch.distributed`` carries only host-side control -- the group's 128-byte unique id,
barriers, the max-over-ranks timing -- never token data.  ``gather_ids_host`` is the same
exchange over a host process group (gloo), for the multi-process CPU tests of the shard
logic.
"""
from __future__ import annotations

import ctypes


def shard_bounds(n_total: int, world: int, rank: int):
    """Contiguous [start, stop) of rank's shard; shards differ in size by at most one."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class RcclGroup:
    """One rank of an image-parallel group on HIP device ``device`` (mocr_group_create).

    ``id_bytes``: the 128-byte unique id rank 0 made with ``RcclGroup.unique_id()``; with
    ``pg`` (a torch.distributed process group, e.g. gloo) and no id, rank 0 makes it and
    broadcasts it over ``pg`` -- host bytes only.  Collective: every rank constructs it."""

    def __init__(self, world: int, rank: int, device: int, id_bytes: bytes | None = None, pg=None):
        from .engine import MocrError, load_library
        self.lib = load_library()
        self.world, self.rank, self.device = world, rank, device
        if id_bytes is None:
            if world == 1:
                id_bytes = self.unique_id()
            else:
                import torch.distributed as dist
                box = [self.unique_id() if rank == 0 else None]
                dist.broadcast_object_list(box, src=0, group=pg)
                id_bytes = box[0]
        if len(id_bytes) != 128:
            raise ValueError("unique id must be 128 bytes")
        h = ctypes.c_void_p()
        rc = self.lib.mocr_group_create(id_bytes, world, rank, device, ctypes.byref(h))
        if rc != 0:
            raise MocrError(f"mocr_group_create failed ({rc}): {self.lib.mocr_group_last_error().decode()}")
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        from .engine import MocrError, load_library
        lib = load_library()
        buf = ctypes.create_string_buffer(128)
        rc = lib.mocr_group_unique_id(buf)
        if rc != 0:
            raise MocrError(f"mocr_group_unique_id failed ({rc}): {lib.mocr_group_last_error().decode()}")
        return buf.raw

    def size(self) -> int:
        """Ranks RCCL's communicator counts (ncclCommCount via mocr_group_size)."""
        from .engine import MocrError
        n = ctypes.c_int(0)
        rc = self.lib.mocr_group_size(self._h, ctypes.byref(n))
        if rc != 0:
            raise MocrError(f"mocr_group_size failed ({rc}): {self.lib.mocr_group_last_error().decode()}")
        return n.value

    def gather_ids(self, ids_local, out=None):
        """All-gather a [rows, width] int32 CUDA tensor from every rank into [world*rows,
        width] (rank order), on the device; returns ``out``."""
        import torch
        from .engine import MocrError
        if not ids_local.is_cuda or ids_local.dtype != torch.int32 or ids_local.dim() != 2:
            raise ValueError("ids must be a 2-D int32 CUDA tensor")
        ids_local = ids_local.contiguous()
        rows, width = ids_local.shape
        if out is None:
            out = torch.empty((self.world * rows, width), dtype=torch.int32, device=ids_local.device)
        if tuple(out.shape) != (self.world * rows, width) or not out.is_contiguous():
            raise ValueError("out must be a contiguous [world*rows, width] int32 tensor")
        # the group stream waits for torch's current stream (the producer of ids_local, e.g.
        # the .contiguous() copy above, and the last user of out's memory)
        producer = torch.cuda.current_stream(ids_local.device).cuda_stream
        rc = self.lib.mocr_group_gather_ids(self._h, ctypes.c_void_p(ids_local.data_ptr()), rows, width,
                                            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(producer))
        if rc != 0:
            raise MocrError(f"mocr_group_gather_ids failed ({rc}): {self.lib.mocr_group_last_error().decode()}")
        return out

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mocr_group_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def global_stop(ids, eos: int):
    """SURVEY.md §8(e) option 2: the reference's batch-global stop over the WHOLE sharded
    batch (``src/inference.py:18-25``: the loop ends after the step at which every row of
    the batch has produced EOS; finished rows keep generating until then).

    ``ids``: the gathered ``[B, S+1]`` token streams of every shard, each shard decoded with
    ``stop="none"`` (column 0 = sos, step t's token in column t+1).  A row's tokens up to
    any step do not depend on when the loop ends, so the global decode is the first
    ``n + 1`` columns, where ``n - 1`` is the latest first-EOS step over all rows (``n = S``
    when some row never produced EOS).  No collective beyond the all-gather the ids already
    went through: every rank computes the same ``n`` from the same gathered tensor.
    Returns ``(ids[:, :n + 1], n)``; equal, columns and step count, to one process decoding
    the whole batch with ``stop="batch"``."""
    import numpy as np
    a = ids.cpu().numpy() if hasattr(ids, "cpu") else np.asarray(ids)
    S = a.shape[1] - 1
    hit = a[:, 1:] == eos
    if a.shape[0] == 0 or not hit.any(axis=1).all():
        n = S
    else:
        n = int(hit.argmax(axis=1).max()) + 1
    return ids[:, :n + 1], n


def shard_rows_max(n_total: int, world: int) -> int:
    """Rows of the largest shard ``shard_bounds`` makes (rank 0's)."""
    return -(-n_total // world) if n_total > 0 else 0


def gather_shards(ids_local, n_total: int, world: int, rank: int, gather, pad_id: int = 0):
    """Pad-and-trim all-gather of per-rank token streams whose shards may differ by a row.

    The reference accepts any batch size (``src/inference.py:7``), so ``shard_bounds``
    splits ``n_total`` images into shards of ``m`` or ``m - 1`` rows, while an all-gather
    (``RcclGroup.gather_ids``, ``gather_ids_host``) moves equal blocks.  Each rank's
    ``[rows, width]`` ids are padded with ``pad_id`` to ``m`` rows, gathered into
    ``[world * m, width]`` by ``gather`` (a callable on one equal-shaped block), and each
    rank's block is trimmed back to its shard; returns the ``[n_total, width]`` ids in
    global row order.  Equal shards skip the pad and the trim."""
    import torch
    a, b = shard_bounds(n_total, world, rank)
    rows = b - a
    if ids_local.dim() != 2 or ids_local.shape[0] != rows:
        raise ValueError(f"rank {rank}'s shard of {n_total} rows over {world} ranks has {rows} rows, "
                         f"got ids of shape {list(ids_local.shape)}")
    m = shard_rows_max(n_total, world)
    if n_total % world == 0:
        return gather(ids_local)
    padded = torch.full((m, ids_local.shape[1]), pad_id, dtype=ids_local.dtype, device=ids_local.device)
    padded[:rows].copy_(ids_local)
    full = gather(padded)
    if tuple(full.shape) != (world * m, ids_local.shape[1]):
        raise ValueError(f"gather returned {list(full.shape)}, expected {[world * m, ids_local.shape[1]]}")
    parts = []
    for r in range(world):
        ra, rb = shard_bounds(n_total, world, r)
        parts.append(full[r * m:r * m + (rb - ra)])
    return torch.cat(parts, 0)


def decode_sharded(engine, images, n_total: int, world: int, rank: int, gather, max_steps: int = 150,
                   stop: str = "batch"):
    """One rank's part of an image-parallel greedy decode of an ``n_total``-image batch.

    ``images``: this rank's shard (rows ``shard_bounds(n_total, world, rank)`` of the global
    batch, host array or device tensor) for ``engine``; ``gather``: the all-gather of one
    equal-shaped id block (``RcclGroup.gather_ids`` on device memory, or
    ``lambda t: gather_ids_host(t.cpu(), world)``).  The shard decodes ``stop="none"``
    into a device buffer padded to the largest shard's rows (``Engine.decode_into``), the
    blocks are gathered and trimmed (``gather_shards``), and with ``stop="batch"`` the
    reference's batch-global stop is applied over the whole gathered batch
    (``global_stop``, SURVEY §8(e) option 2).  Returns ``(ids [n_total, n + 1], n)`` on
    every rank."""
    import torch
    if stop not in ("batch", "none"):
        raise ValueError("stop must be 'batch' or 'none'")
    a, b = shard_bounds(n_total, world, rank)
    if len(images) != b - a:
        raise ValueError(f"rank {rank}'s shard is rows [{a}, {b}) of {n_total}, got {len(images)} images")
    dev = torch.device("cuda", engine.device)
    m = shard_rows_max(n_total, world)
    buf = torch.full((m, max_steps + 1), engine.pad, dtype=torch.int32, device=dev)
    if b > a:
        engine.encode(images)
        engine.decode_into(buf[:b - a], max_steps=max_steps, stop="none")
    ids = gather_shards(buf[:b - a], n_total, world, rank, gather, pad_id=engine.pad)
    if stop == "none":
        return ids, max_steps
    return global_stop(ids, engine.eos)


def gather_ids_host(ids_local, world: int, group=None):
    """All-gather equal-shaped per-rank CPU id tensors over a host process group (gloo)
    and concatenate them in rank order (multi-process CPU tests)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return ids_local
    if ids_local.is_cuda:
        raise ValueError("device ids go through RcclGroup.gather_ids")
    parts = [torch.empty_like(ids_local) for _ in range(world)]
    dist.all_gather(parts, ids_local.contiguous(), group=group)
    return torch.cat(parts, 0)
