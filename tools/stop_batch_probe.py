"""Wall time of a greedy decode under the batch-global stop (src/inference.py's rule) that
never fires (random-init weights, 128 steps), i.e. 16 graph chunks with a stop check
between them, at B = 1 and B = 64 (384x384).

    python tools/stop_batch_probe.py [--lib LIB] [--reps 10]
"""
import argparse
import importlib
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (shared HIP runtime)

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
if a.lib:
    pkg.engine.load_library(a.lib)
w = pkg.synth.make_weights(1234, "init")
out = {"lib": a.lib or "default"}
for B in (1, 64):
    eng = pkg.Engine(img_hw=(384, 384), max_batch=B, precision="bf16x3")
    eng.load_weights(w)
    eng.set_images(pkg.synth.make_images(B, 384, 384))
    eng.encode()
    for mode in ("none", "batch"):
        eng.decode(max_steps=128, stop=mode)  # warm (graphs)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r = eng.decode(max_steps=128, stop=mode)
            ts.append(time.perf_counter() - t0)
        out[f"B{B}_{mode}_ms"] = statistics.median(ts) * 1e3
        out[f"B{B}_{mode}_steps"] = int(r.n_steps)
    eng.close()
print(json.dumps(out))
