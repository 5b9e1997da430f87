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
