"""Capacity of each half of the path under the bench's replica pipelining: R replicas
running only encodes, only decodes (memory encoded once), or both, for --steps batches.

    python tools/pipeline_probe.py --replicas 3 --steps 12
"""
import argparse
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=3)
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--precision", default="bf16x3")
ap.add_argument("--modes", default="encode,decode,both")
ap.add_argument("--lib", default=None, help="libmathocr.so to load (an A/B build from tools/build_variant.sh)")
ap.add_argument("--rows", type=int, default=64, help="images per engine call (decode chain rows)")
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
if a.lib:
    pkg.engine.load_library(a.lib, ab_build=True)
B, S = a.rows, 128
pool = pkg.pipeline.ReplicaPool(a.replicas, img_hw=(384, 384), max_batch=B, precision=a.precision, device=0)
pool.load_weights(pkg.synth.make_weights(1234, "init"))
for i, e in enumerate(pool.engines):
    e.set_images(torch.from_numpy(pkg.synth.make_images(B, 384, 384, seed0=1000 + i * B)).to("cuda:0"))
    e.encode()


def enc(e, _k):
    e.encode()


def dec(e, _k):
    ids = torch.empty((B, S + 1), dtype=torch.int32, device="cuda:0")
    e.decode_into(ids, max_steps=S, stop="none")


def both(e, k):
    enc(e, k)
    dec(e, k)


out = {"replicas": a.replicas, "rows": B, "lib": a.lib or "default"}
for name, fn in (("encode", enc), ("decode", dec), ("both", both)):
    if name not in a.modes.split(","):
        continue
    list(pool.imap(fn, range(a.replicas)))  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    list(pool.imap(fn, range(a.steps)))
    torch.cuda.synchronize()
    out[name + "_img_s"] = B * a.steps / (time.perf_counter() - t0)
pool.close()
print(json.dumps(out))
