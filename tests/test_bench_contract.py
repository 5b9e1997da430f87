"""CPU checks of bench.py's measurement helpers: the roofline lines are
computed from HIP-event kernel-class records exactly as documented in DESIGN.md §5, and
the committed PMC traffic profile maps to the kernel classes they name."""
import importlib.util
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def rec(launches, ms, flops, byts=0.0):
    return {"launches": launches, "total_ms": ms * launches, "flops": flops * launches, "bytes": byts * launches}


def stats():
    # per-launch: s3.fc1 162 us / 43.5 GF, s3.fc2 153 us / 43.5 GF, s3.attn 286 us / 35.4 GF
    return {
        "s3.fc1": rec(18, 0.162, 43.486543872e9, 285.5e6),
        "s3.fc2": rec(18, 0.153, 43.486543872e9),
        "s3.attn": rec(18, 0.286, 35.38944e9, 115.0e6),
        "s1.attn": rec(6, 0.465, 20.0e9),
        "stem": rec(3, 0.114, 1.0e9),
        "decode.greedy": rec(384, 0.2435, 0.95e9, 247.1e6),
        "host.graph_launch": rec(48, 0.11, 0.0),
    }


def test_gemm_roofline_is_the_dominant_gemm_class(bench):
    r = bench.roofline(stats(), "bf16x3", "bf16x3", 64)
    assert r["kernel"] == "gemm_bf16[bf16x3] s3.fc1" and r["bound"] == "mfma" and r["unit"] == "TFLOP/s"
    assert r["achieved"] == pytest.approx(43.486543872e9 / 162e-6 / 1e12)
    assert r["peak"] == 2500.0 and r["frac"] == pytest.approx(r["achieved"] / 2500.0)
    assert r["mfma_issue_frac"] == pytest.approx(3 * r["frac"])
    assert r["avg_launch_ms"] == pytest.approx(0.162)


def test_attention_roofline_is_the_dominant_attention_class(bench):
    r = bench.roofline(stats(), "bf16x3", "bf16x3", 64, attention=True)
    assert r["kernel"] == "attention[bf16x3] s3.attn"
    assert r["achieved"] == pytest.approx(35.38944e9 / 286e-6 / 1e12)
    assert bench.roofline({"s3.fc1": rec(1, 0.1, 1e9)}, "bf16x3", "bf16x3", 64, attention=True) is None


def test_decode_roofline_against_hbm(bench):
    r = bench.roofline_decode(stats(), "bf16x3", 64, 128)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    # SURVEY §8(d) at B = 64, bf16: weights 13.2 MB + cross K/V 75.5 MB + self K/V <= 67 MB per step
    survey = sum(bench.survey_decode_step_bytes(64, t) for t in range(128)) / 128
    assert bench.survey_decode_step_bytes(64, 0) == pytest.approx(13.08e6 + 75.50e6 + 1.05e6, rel=1e-3)
    assert r["algorithmic_bytes_per_step"] == pytest.approx(survey)
    assert r["achieved"] == pytest.approx(survey / 0.2435e-3 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0)
    assert r["as_built_achieved"] == pytest.approx(247.1e6 / 0.2435e-3 / 1e9)
    assert bench.roofline_decode({}, "bf16x3", 64, 128) is None


def test_e2e_roofline_is_baseline_md_section4(bench):
    # 1 / (26.39 GFLOP / 2.5 PF + 245 MB / 8 TB/s) ~ 24.3k img/s per GPU
    assert bench.E2E_ROOFLINE_IMG_S == pytest.approx(24.3e3, rel=0.01)


def test_committed_pmc_traffic_covers_the_roofline_classes(bench):
    # the bench's roofline classes at its default 8 x 64 and the driver's 10 x 64 images per
    # call (round 3's 4 x 64 profile kept, from before stage 3's fused attention ran at
    # every batch: its norm1 + qkv was s3.lnqkv; round 6's profiles have the block tail
    # s3.tail where the proj GEMM and s3.mlp were, and merge 1 as one kernel)
    for batch in (256, 512, 640):
        s3 = "s3.lnqkv" if batch == 256 else "s3.attn"
        tail = "s3.mlp" if batch == 256 else "s3.tail"
        for cls in (tail, "s1.attn", s3, "decode.step") + (("merge1",) if batch != 256 else ()):
            t = bench.pmc_traffic("bf16x3", cls, batch)
            assert t is not None and t > 0, (batch, cls)
    assert bench.pmc_traffic("bf16x3", "no.such.class", 512) is None
    assert bench.pmc_traffic("bf16x3", "s3.mlp", 333) is None


def test_default_run_is_one_gpu_minutes_scale(bench, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.gpus == 1 and a.steps == 64 and a.warmup == 4 and a.batch == 64 and a.tokens == 128
    assert a.chain == 8 and a.replicas == 2 and a.precision == "bf16x3" and a.image == [384, 384]
    assert a.cpu_sample == 64 and a.cpu_runs == 3  # B = 64, median of 3
    monkeypatch.setattr(sys, "argv", ["bench.py", "--arch", "res18trans"])
    a = bench.parse()
    assert a.chain == 1 and a.replicas == 4  # its encoder attends across its batch of 64


def test_auto_chain_keeps_timed_calls_even_over_replicas(bench, monkeypatch):
    # the largest chain <= 10 batches that gives every replica the same number of calls:
    # the driver's --steps 20 -> 2 calls of 10, the default 64 -> 8 calls of 8
    assert bench.auto_chain(20, 2) == 10 and bench.auto_chain(64, 2) == 8 and bench.auto_chain(8, 2) == 4
    assert bench.auto_chain(7, 2) == 4 and bench.auto_chain(40, 2) == 10 and bench.auto_chain(20, 4) == 5
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "20", "--warmup", "5"])
    a = bench.parse()
    assert (a.chain, a.replicas) == (10, 2)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "20", "--chain-batches", "4"])
    assert bench.parse().chain == 4


def test_gpus_without_launcher_starts_torchrun_child(bench, monkeypatch):
    """--gpus N > 1 with no WORLD_SIZE: bench.py runs N ranks under torch.distributed.run
    as a child process (not exec) and returns its exit status."""
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "8", "--warmup", "4"])
    a = bench.parse()
    rc = bench.launch_if_needed(a, ["--gpus", "2", "--steps", "8", "--warmup", "4"], env={})
    assert rc == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-7:] == [os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "8", "--warmup", "4"]
    # one GPU, or a rank under a launcher: no child
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.launch_if_needed(bench.parse(), [], env={}) is None
    assert bench.launch_if_needed(a, [], env={"WORLD_SIZE": "2"}) is None
    with pytest.raises(SystemExit):
        bench.launch_if_needed(a, [], env={"WORLD_SIZE": "4"})


def test_warmup_reaches_every_replica(bench, monkeypatch):
    """The driver's form (--steps 20 --warmup 5: 10-batch calls, 2 replicas, one pooled
    warm-up call) still warms BOTH replicas before the timed region: each engine's first
    decode captures its graphs."""
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "20", "--warmup", "5"])
    a = bench.parse()
    assert -(-a.warmup // a.chain) == 1 < a.replicas  # the pooled warm-up alone is one call

    class Pool:
        engines = [object() for _ in range(a.replicas)]

    seen = []
    warmed = bench.warm_replicas(Pool, lambda e, k: seen.append(e))
    assert seen == Pool.engines and warmed == Pool.engines


def test_decode_traffic_on_the_steps_it_was_measured(bench, monkeypatch):
    """`traffic` of the decode step comes from PMC passes over steps 0..7: its ratio is taken
    against the SURVEY §8(d) bytes of those steps, not the t = 0..127 average."""
    monkeypatch.setattr(bench, "pmc_traffic", lambda precision, cls, rows: 1.256e9)
    st = {"decode.greedy": rec(128, 0.52, 1e9, 9e8)}
    r = bench.roofline_decode(st, "bf16x3", 640, 128)
    early = sum(bench.survey_decode_step_bytes(640, t) for t in range(8)) / 8
    assert r["algorithmic_bytes_pmc_steps"] == pytest.approx(early)
    assert r["traffic_ratio"] == pytest.approx(1.256e9 / early)
    assert r["algorithmic_bytes_per_step"] > early  # the t = 0..127 average (longer caches)


def test_gpus8_without_launcher_starts_eight_ranks(bench, monkeypatch):
    """The driver's N = 8 form without a launcher: one torch.distributed.run child with 8
    local ranks on 127.0.0.1."""
    seen = {}

    class Done:
        returncode = 0

    monkeypatch.setattr(bench.subprocess, "run", lambda cmd, *a, **k: seen.setdefault("cmd", cmd) and Done())
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "5"])
    a = bench.parse()
    assert bench.launch_if_needed(a, ["--gpus", "8", "--steps", "20", "--warmup", "5"], env={}) == 0
    assert "--nproc-per-node=8" in seen["cmd"] and "--master-addr=127.0.0.1" in seen["cmd"]


def test_rank0_stdout_is_one_json_line_with_gloo(tmp_path):
    """Two gloo ranks (the driver's N > 1 form on CPU): gloo's C++ connect messages ("[Gloo]
    Rank r is connected to ...") go to the process's stdout; bench.py routes fd 1 to fd 2
    around the group's creation, so rank 0's stdout holds only its JSON line."""
    import json
    import socket
    import subprocess

    script = tmp_path / "ranks.py"
    script.write_text(
        "import importlib.util, json, os, sys\n"
        "import torch.distributed as dist\n"
        f"spec = importlib.util.spec_from_file_location('b', {os.path.join(REPO, 'bench.py')!r})\n"
        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
        "with b.stdout_to_stderr():\n"
        "    dist.init_process_group('gloo')\n"
        "    dist.barrier()\n"
        "dist.barrier()\n"
        "if dist.get_rank() == 0:\n"
        "    print(json.dumps({'metric': 'x', 'n': dist.get_world_size()}), flush=True)\n"
        "dist.destroy_process_group()\n")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    assert json.loads(lines[0]) == {"metric": "x", "n": 2}


def test_serving_latency_is_the_reference_serving_call(bench):
    """serving_latency_ms times im2latex.predict on one 96x320 image
    (batch stop, 150-step cap) and a fixed 128-step decode, median of >= 10 calls."""
    import types
    calls = {"predict": 0, "decode": []}

    class Eng:
        def __init__(self, img_hw, max_batch, precision, device):
            assert img_hw == (96, 320) and max_batch == 1
            self.closed = False

        def load_weights(self, w):
            pass

        def encode(self, img):
            assert img.shape == (1, 1, 96, 320)

        def decode(self, max_steps, stop):
            calls["decode"].append((max_steps, stop))
            return types.SimpleNamespace(n_steps=max_steps if stop == "none" else 37)

        def close(self):
            self.closed = True

    def predict(eng, img, vocab, idx2char):
        calls["predict"] += 1
        return ("x", 0.5)

    import numpy as np
    pkg = types.SimpleNamespace(
        Engine=Eng, im2latex=types.SimpleNamespace(predict=predict),
        synth=types.SimpleNamespace(synthetic_vocab=lambda: ({}, {}),
                                    make_images=lambda n, h, w, seed0: np.zeros((n, 1, h, w), np.float32)),
        config=types.SimpleNamespace(config=types.SimpleNamespace(max_seq_len=150)))
    r = bench.serving_latency(pkg, {}, "bf16x3", 0)
    assert r["samples"] >= 10 and calls["predict"] == r["samples"] + 2
    assert r["fixed_steps"] == 128 and r["im2latex_predict_steps"] == 37
    assert (150, "batch") in calls["decode"] and r["image"] == [96, 320] and r["batch"] == 1
    assert r["im2latex_predict"] >= 0 and r["fixed_128_steps"] >= 0


def test_latency_pass_has_at_least_16_samples():
    """The headline p50 comes from >= 16 loaded calls run after the timed region."""
    src = open(os.path.join(REPO, "bench.py")).read()
    assert "lat_pass = run(max(16, 2 * R))" in src
    assert '"p50_image_latency_ms": statistics.median(lat_pass) * 1e3' in src
    assert '"image_latency_samples": len(lat_pass)' in src
