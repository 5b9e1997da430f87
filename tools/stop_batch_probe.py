"""Wall time of a greedy decode under the batch-global stop (src/inference.py's rule) that
never fires (random-init weights, 128 steps), i.e. 16 graph chunks with a stop check
between them, at B = 1 and B = 64 (384x384); with --eos-boost, the EOS logit's bias is
raised so the batch stops early (the serving case): the stop is detected up to two 8-step
chunks late (the check of chunk c runs once chunk c + 1 is queued), and the chunks queued
after the stop run as early-outs.  Reports the steps run and the wall time against the
no-stop decode's time per step.

    python tools/stop_batch_probe.py [--lib LIB] [--reps 10] [--eos-boost 0,6,8]
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
ap.add_argument("--eos-boost", default="0")
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
if a.lib:
    pkg.engine.load_library(a.lib, ab_build=True)
out = {"lib": a.lib or "default"}
for boost in [float(x) for x in a.eos_boost.split(",")]:
    w = pkg.synth.make_weights(1234, "init")
    if boost:
        w["decoder.fc_out.bias"] = w["decoder.fc_out.bias"].copy()
        w["decoder.fc_out.bias"][pkg.synth.EOS_ID] += boost
    for B in (1, 64):
        eng = pkg.Engine(img_hw=(384, 384), max_batch=B, precision="bf16x3")
        eng.load_weights(w)
        eng.set_images(pkg.synth.make_images(B, 384, 384))
        eng.encode()
        per_step = None
        for mode in ("none", "batch"):
            eng.decode(max_steps=128, stop=mode)  # warm (graphs)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                r = eng.decode(max_steps=128, stop=mode)
                ts.append(time.perf_counter() - t0)
            ms = statistics.median(ts) * 1e3
            if mode == "none":
                per_step = ms / 128
            key = f"boost{boost:g}_B{B}_{mode}"
            out[key + "_ms"] = round(ms, 3)
            out[key + "_steps"] = int(r.n_steps)
            if mode == "batch":
                out[key + "_ms_at_nostop_rate"] = round(per_step * r.n_steps, 3)
        eng.close()
print(json.dumps(out))
