"""Headline benchmark: Swin-T + 8-layer decoder greedy decode, 128 tokens, batch 64 of
384x384x1 images per GPU (BASELINE.json configs[1]; configs[2] when run with N ranks).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = encode + 128-step greedy decode of one 64-image batch per GPU, images already
resident in HBM; with N > 1 ranks the decoded token streams are all-gathered over RCCL
(image-parallel shards, no other collective).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "images/sec + p50 per-image latency, Swin-T+8L-dec greedy@128tok, 1/2/4/8 GPU"
PEAK = {"f32": ("mfma", 157.3, "TFLOP/s"), "bf16": ("mfma", 2500.0, "TFLOP/s"), "bf16x3": ("mfma", 2500.0 / 3, "TFLOP/s")}
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64, help="images per GPU")
    ap.add_argument("--image", type=int, nargs=2, default=[384, 384])
    ap.add_argument("--tokens", type=int, default=128)
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3", "bf16"])
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--cpu-sample", type=int, default=32, help="images in the CPU-baseline sample")
    ap.add_argument("--no-b1-latency", dest="b1", action="store_false", default=True)
    return ap.parse_args()


def cpu_baseline(args, pkg):
    """The oracle restatement of the reference CPU path (src/inference.py: full-prefix
    re-decode, fp32, torch CPU) on a bounded sample of the same workload."""
    from oracle import model_ref
    threads = torch.get_num_threads()
    w = pkg.synth.make_weights(1234, "init")
    model = model_ref.build_model(w)
    n = args.cpu_sample
    imgs = torch.from_numpy(pkg.synth.make_images(n, *args.image, seed0=1000))
    model_ref.greedy_decode(model, images=imgs[:1], max_steps=2, stop="none")  # warm-up
    t0 = time.perf_counter()
    model_ref.greedy_decode(model, images=imgs, max_steps=args.tokens, stop="none")
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"{n} images {args.image[0]}x{args.image[1]}, {args.tokens} greedy steps, "
                      f"full-prefix re-decode as src/inference.py, fp32 torch CPU, {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    pkg = importlib.import_module("handwritten-math-ocr-api_amd")
    H, W = args.image
    B = args.batch
    S = args.tokens

    eng = pkg.Engine(img_hw=(H, W), max_batch=B, precision=args.precision, device=local)
    eng.load_weights(pkg.synth.make_weights(1234, "init"))
    # this rank's shard of the global batch, uploaded once (resident in HBM)
    imgs = torch.from_numpy(pkg.synth.make_images(B, H, W, seed0=1000 + rank * B)).to(f"cuda:{local}")
    eng.set_images(imgs)
    ids_local = torch.empty((B, S + 1), dtype=torch.int32, device=f"cuda:{local}")

    def step():
        eng.encode()
        eng.decode_into(ids_local, max_steps=S, stop="none")
        return pkg.parallel.gather_ids(ids_local, world)  # RCCL all-gather of the token streams

    for _ in range(args.warmup):
        step()
    eng.set_timing(True)
    lat = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        step()
        lat.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = eng.timing()
    eng.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    lat_b1 = None
    if rank == 0 and args.b1:
        e1 = pkg.Engine(img_hw=(H, W), max_batch=1, precision=args.precision, device=local)
        e1.load_weights(pkg.synth.make_weights(1234, "init"))
        e1.set_images(imgs[:1].contiguous())
        ts = []
        for _ in range(4):
            t1 = time.perf_counter()
            e1.encode()
            e1.decode(max_steps=S, stop="none")
            ts.append(time.perf_counter() - t1)
        lat_b1 = statistics.median(ts[1:]) * 1e3
        e1.close()

    if rank != 0:
        eng.close()
        if world > 1:
            dist.destroy_process_group()
        return

    dtype = {"fp32": "f32", "bf16x3": "bf16x3", "bf16": "bf16"}[args.precision]
    # dominant kernel class = largest total event-timed GPU time among the encoder GEMMs
    gemms = {k: v for k, v in stats.items() if v["flops"] > 0 and "attn" not in k and k != "stem"}
    dom_name, dom = max(gemms.items(), key=lambda kv: kv[1]["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    flops_per_launch = dom["flops"] / dom["launches"]
    bound, peak, unit = PEAK[dtype]
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12
    enc_ms = sum(v["total_ms"] for v in stats.values()) / args.steps
    out = {
        "metric": METRIC,
        "value": world * B * args.steps / elapsed,
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic: U(-1,1) 384x384x1 images (PCG64 seeds 1000+i), random-init weights with the "
                "reference's init distributions (seed 1234); 128 greedy steps, no early stop",
        "config": {"workload": f"B{B}/GPU {H}x{W} Swin-T + 8L decoder greedy@{S}", "global_batch": world * B,
                   "per_gpu_batch": B, "image": [H, W], "max_tokens": S, "vocab": pkg.synth.VOCAB,
                   "decoder_layers": pkg.synth.N_LAYERS, "parallelism": f"image-parallel x{world}",
                   "precision": args.precision},
        "p50_image_latency_ms": statistics.median(lat) * 1e3,
        "p50_image_latency_b1_ms": lat_b1,
        "encoder_gemm_ms_per_step": enc_ms,
        "roofline": {"kernel": f"gemm_{'f32' if dtype == 'f32' else 'bf16'} {dtype} ({dom_name})", "bound": bound, "achieved": achieved, "peak": peak,
                     "unit": unit, "frac": achieved / peak, "traffic": None,
                     "avg_launch_ms": avg_ms, "flops_per_launch": flops_per_launch},
        "kernel_classes": {k: {"launches": v["launches"], "avg_ms": v["total_ms"] / v["launches"],
                               "tflops": v["flops"] / v["total_ms"] * 1e-9 if v["total_ms"] else None}
                           for k, v in sorted(stats.items())},
    }
    if args.cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(args, pkg)
    eng.close()
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
