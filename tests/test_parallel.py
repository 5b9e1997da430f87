"""CPU: the image-parallel N>1 path (shards + gather of token streams) with gloo,
world size 2, in spawned processes."""
import importlib
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_total, steps, q):
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("handwritten-math-ocr-api_amd")
    a, b = pkg.parallel.shard_bounds(n_total, world, rank)
    # stand-in for this rank's decoded ids: row i of the global batch is filled with i
    local = torch.arange(a, b, dtype=torch.int32)[:, None].repeat(1, steps + 1)
    gathered = pkg.parallel.gather_ids_host(local, world)
    if rank == 0:
        q.put(gathered.numpy().tolist())
    dist.barrier()
    dist.destroy_process_group()


def _ragged_worker(rank, world, port, n_total, steps, q):
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("handwritten-math-ocr-api_amd")
    out = {}
    for n in n_total:
        a, b = pkg.parallel.shard_bounds(n, world, rank)
        # row i of the global batch: [i, i + 1, ...] so a misplaced or padded row shows
        local = (torch.arange(a, b, dtype=torch.int32)[:, None] + torch.arange(steps + 1, dtype=torch.int32)[None])
        got = pkg.parallel.gather_shards(local, n, world, rank, lambda t: pkg.parallel.gather_ids_host(t, world),
                                         pad_id=-7)
        out[n] = got.numpy().tolist()
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_shards_uneven_gloo_world2():
    """the pad-and-trim gather of shards that differ by a row (the
    reference takes any B, src/inference.py:7): B = 131 and 3 over 2 ranks, plus the equal
    B = 130, gathered on both ranks in global row order with no pad row left."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_total, steps = (131, 130, 3, 1), 4
    procs = [ctx.Process(target=_ragged_worker, args=(r, 2, port, n_total, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for n in n_total:
        want = [[i + j for j in range(steps + 1)] for i in range(n)]
        assert res[0][n] == want and res[1][n] == want, n


def test_gather_shards_checks_shapes():
    import pytest
    sys.path.insert(0, REPO)
    pkg = importlib.import_module("handwritten-math-ocr-api_amd")
    ident = lambda t: t
    with pytest.raises(ValueError):  # rank 0 of 5 rows over 2 ranks holds 3 rows
        pkg.parallel.gather_shards(torch.zeros(2, 4, dtype=torch.int32), 5, 2, 0, ident)
    with pytest.raises(ValueError):  # the gather must return world * m rows
        pkg.parallel.gather_shards(torch.zeros(3, 4, dtype=torch.int32), 5, 2, 0, ident)
    # one rank: the gather is the identity
    x = torch.arange(12, dtype=torch.int32).reshape(3, 4)
    assert torch.equal(pkg.parallel.gather_shards(x, 3, 1, 0, ident), x)
    assert pkg.parallel.shard_rows_max(5, 2) == 3 and pkg.parallel.shard_rows_max(0, 4) == 0


def test_gather_ids_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_total, steps = 8, 5
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [row[0] for row in out] == list(range(n_total))
    assert all(len(row) == steps + 1 for row in out)
