"""GPU: the image-parallel path (BASELINE config 3) with the real engine.

* two fresh processes share cuda:0 (this pool's boxes have one GPU), each encodes and
  decodes its own shard of a fixture batch, and the token streams gathered over a host
  process group (gloo) equal the fixture's ids -- the shard/gather logic of bench.py's
  N>1 path with the engine in it;
* the RCCL gather inside libmathocr.so (mocr_group_*) on a one-rank group: RCCL refuses
  two ranks on one device, so its N>1 run is the driver's multi-GPU bench.
"""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, stop="none"):
    try:
        sys.path.insert(0, REPO)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pkg = importlib.import_module("handwritten-math-ocr-api_amd")
        from tests.conftest import load_golden
        from oracle.gen_golden import apply_eos_boost
        g = load_golden("g96x320_b4_eos")
        m = g["meta"]
        if stop == "ragged":
            # the product path for any B: 3 of the fixture's rows over 2 ranks (2 + 1), each
            # rank decoding its shard into a padded device buffer, the pad-and-trim gather,
            # then the batch-global stop over the whole gathered batch (parallel.decode_sharded)
            n = 3
            a, b = pkg.parallel.shard_bounds(n, world, rank)
            imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])[a:b]
            eng = pkg.Engine(img_hw=(m["H"], m["W"]), max_batch=b - a, precision="bf16x3", device=0)
            eng.load_weights(apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"]))
            ids, n_steps = pkg.parallel.decode_sharded(
                eng, imgs, n, world, rank, lambda t: pkg.parallel.gather_ids_host(t.cpu(), world),
                max_steps=m["steps"], stop="batch")
            eng.close()
            if rank == 0:
                q.put(("ok", (ids.cpu().numpy(), n_steps)))
            dist.barrier()
            dist.destroy_process_group()
            return
        a, b = pkg.parallel.shard_bounds(m["B"], world, rank)
        imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])[a:b]
        eng = pkg.Engine(img_hw=(m["H"], m["W"]), max_batch=b - a, precision="bf16x3", device=0)
        eng.load_weights(apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"]))
        eng.encode(imgs)
        steps = g["ids"].shape[1] - 1
        if stop == "global":  # SURVEY §8(e) option 2: decode without stopping, cut after the gather
            res = eng.decode(max_steps=m["steps"], stop="none")
        else:
            res = eng.decode(max_steps=steps if stop == "none" else m["steps"], stop=stop)
        eng.close()
        # a shard under the batch stop ends when its own rows have all finished (DESIGN.md
        # §6): pad its ids to the fixture's width for the gather, and report its step count
        ids = np.full((b - a, m["steps"] + 1), pkg.synth.PAD_ID, np.int32)
        ids[:, :res.ids.shape[1]] = res.ids
        gathered = pkg.parallel.gather_ids_host(torch.from_numpy(ids), world)
        n_steps = pkg.parallel.gather_ids_host(torch.tensor([[res.n_steps]], dtype=torch.int32), world)
        if rank == 0:
            q.put(("ok", (gathered.numpy(), n_steps.numpy().ravel())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # report instead of hanging the parent on the queue
        q.put(("error", f"rank {rank}: {ex!r}"))
        raise


def _run_shards(stop):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, stop)) for r in range(2)]
    for p in procs:
        p.start()
    status, out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", out
    assert all(p.exitcode == 0 for p in procs)
    return out


def test_two_shards_on_one_gpu_match_fixture(golden):
    out, _ = _run_shards("none")
    out = out[:, :golden("g96x320_b4_eos")["ids"].shape[1]]
    # rows are independent: the fixed-length decode of each shard equals the fixture's rows
    # (the fixture's batch-global stop only decides how many columns exist)
    g = golden("g96x320_b4_eos")
    bad = [(i, int(np.nonzero(out[i] != g["ids"][i])[0][0])) for i in range(out.shape[0])
           if not np.array_equal(out[i], g["ids"][i])]
    # (row, first differing column, the fixture's top-2 logit margin at the step before it)
    assert not bad, [(i, c, float(g["margins"][i, c - 1])) for i, c in bad]


def test_two_shards_batch_stop_each_shard_stops_on_its_own(pkg, golden):
    """SURVEY §8(e) option 1: under the reference's batch-global stop
    (src/inference.py:23-25) each shard stops once its own rows have all produced EOS, with
    no collective; every row's tokens up to and including its EOS (its string) equal the
    fixture's, whose stop was global over the 4 rows.  The shards' step counts may be
    shorter than the fixture's, never longer."""
    g = golden("g96x320_b4_eos")
    out, n_steps = _run_shards("batch")
    eos = pkg.synth.EOS_ID
    n_fix = g["ids"].shape[1] - 1
    assert (n_steps <= n_fix).all() and n_steps.max() == n_fix, (n_steps, n_fix)
    for i in range(g["ids"].shape[0]):
        ref = g["ids"][i]
        hit = np.flatnonzero(ref[1:] == eos)
        assert hit.size, f"fixture row {i} never reaches EOS"
        end = int(hit[0]) + 2  # through the EOS column
        np.testing.assert_array_equal(out[i, :end], ref[:end], err_msg=f"row {i}")
    # the detokenised strings (cut at EOS) are the fixture's
    vocab, idx2char = pkg.synth.synthetic_vocab()
    assert [pkg.utils.detokenize(r.tolist(), idx2char) for r in out] == g["meta"]["strings"]


def test_two_shards_global_stop_equals_one_process(pkg, golden):
    """SURVEY §8(e) option 2: each shard decodes all 150 steps without stopping, the ids are
    gathered, and `parallel.global_stop` cuts them after the step at which the last row of
    the whole batch produced EOS: every column, post-EOS tokens included, and the step
    count equal the fixture's single-process batch-stop decode."""
    g = golden("g96x320_b4_eos")
    gathered, _ = _run_shards("global")
    cut, n = pkg.parallel.global_stop(gathered, pkg.synth.EOS_ID)
    assert n == g["ids"].shape[1] - 1
    np.testing.assert_array_equal(cut, g["ids"])


def test_rccl_group_gather_one_rank(pkg):
    grp = pkg.parallel.RcclGroup(world=1, rank=0, device=0)
    ids = torch.arange(64 * 129, dtype=torch.int32, device="cuda:0").reshape(64, 129)
    out = grp.gather_ids(ids)
    torch.cuda.synchronize()
    assert torch.equal(out, ids)
    with pytest.raises(ValueError):
        grp.gather_ids(ids.float())
    grp.close()


def test_rccl_gather_of_engine_ids(pkg, golden):
    """decode_into writes the shard's ids to device memory; the group gathers them."""
    from oracle.gen_golden import apply_eos_boost
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    eng = pkg.Engine(img_hw=(m["H"], m["W"]), max_batch=m["B"], precision="bf16x3", device=0)
    eng.load_weights(apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"]))
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    steps = g["ids"].shape[1] - 1
    ids = torch.empty((m["B"], steps + 1), dtype=torch.int32, device="cuda:0")
    eng.decode_into(ids, max_steps=steps, stop="none")
    grp = pkg.parallel.RcclGroup(world=1, rank=0, device=0)
    out = grp.gather_ids(ids)
    np.testing.assert_array_equal(out.cpu().numpy(), g["ids"])
    grp.close()
    eng.close()


def test_bench_two_ranks_torchrun():
    """bench.py's N > 1 path under torch.distributed.run (2 ranks; on a one-GPU box both
    share cuda:0, so the token streams are gathered over the host group): one JSON line
    from rank 0 with the whole-job throughput."""
    import json
    import subprocess
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--replicas", "1", "--no-isolated", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    cfg = out["config"]
    assert out["n_gpus"] == 2 and out["value"] > 0 and cfg["global_batch"] == 2 * cfg["per_gpu_batch"]
    assert cfg["per_gpu_batch"] == cfg["batch_unit"] == 64
    assert cfg["images_per_call"] == cfg["batch_unit"] * cfg["batches_per_chain"]
    assert len(out["rank_elapsed_s"]["all"]) == 2 and out["rank_elapsed_s"]["max"] * 1e3 / out["steps"] == \
        pytest.approx(out["ms_per_step"])
    assert out["config"]["gather"] in ("rccl (mocr_group_gather_ids)", "gloo host (ranks share a device)")


def test_uneven_shards_decode_sharded(pkg, golden):
    """shards that differ by a row have a product path.  Rows 0-2 of
    the 96x320 EOS fixture over 2 ranks (2 + 1 images) through ``parallel.decode_sharded``:
    padded device buffers, the pad-and-trim gather, the batch-global stop over the 3 rows.
    Rows are independent, so the result is the fixture's rows 0-2 cut at the step where the
    last of THEM produced EOS (``global_stop`` of the fixture's own columns)."""
    g = golden("g96x320_b4_eos")
    ids, n = _run_shards("ragged")
    # the fixture's ids run to its own 4-row stop; the 3-row stop comes no later
    ref, n_ref = pkg.parallel.global_stop(g["ids"][:3], pkg.synth.EOS_ID)
    assert n == n_ref and ids.shape == (3, n_ref + 1), (ids.shape, n, n_ref)
    np.testing.assert_array_equal(ids, ref)
