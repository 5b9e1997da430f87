"""Greedy-decode capacity by rows per chain x concurrent chains, one tool for every cell
(VERDICT r02 "Next" 1: reconcile decode_batch_scaling.log with pipeline_probe).

Every chain is one engine (max_batch = rows) decoding its encoded batch for 128 steps
with ``decode_into`` (ids stay on the device, stop="none"), driven by its own host
thread; the encoder is outside the timed region.  Prints rows/s and us per step per chain.

    python tools/decode_chain_probe.py [--rows 64,128,256] [--chains 1,2,4] [--reps 3]
    python tools/decode_chain_probe.py --rows 256 --chains 1 --reps 1     # under rocprofv3
"""
import argparse
import importlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", default="64,128,256")
ap.add_argument("--chains", default="1,2,4")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--precision", default="bf16x3")
ap.add_argument("--lib", default=None)
ap.add_argument("--variant", default="", help="comma-separated engine.VARIANT names")
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
if a.lib:
    pkg.engine.load_library(a.lib, ab_build=True)
w = pkg.synth.make_weights(1234, "init")
S = a.steps
out = []
for rows in [int(x) for x in a.rows.split(",")]:
    for R in [int(x) for x in a.chains.split(",")]:
        engs, bufs = [], []
        for r in range(R):
            e = pkg.Engine(img_hw=(384, 384), max_batch=rows, precision=a.precision, device=0,
                           variant=tuple(v for v in a.variant.split(",") if v))
            e.load_weights(w)
            e.set_images(torch.from_numpy(pkg.synth.make_images(rows, 384, 384, seed0=1000 + r * rows)).to("cuda:0"))
            e.encode()
            b = torch.empty((rows, S + 1), dtype=torch.int32, device="cuda:0")
            e.decode_into(b, max_steps=S, stop="none")  # graphs captured, caches warm
            engs.append(e)
            bufs.append(b)
        torch.cuda.synchronize()
        bar = threading.Barrier(R + 1)

        def run(e, b):
            bar.wait()
            for _ in range(a.reps):
                e.decode_into(b, max_steps=S, stop="none")

        th = [threading.Thread(target=run, args=(e, b)) for e, b in zip(engs, bufs)]
        for t in th:
            t.start()
        bar.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.reps
        rec = {"rows": rows, "chains": R, "ms_per_round": dt * 1e3, "rows_per_s": R * rows / dt,
               "us_per_step_per_chain": dt / S * 1e6}
        out.append(rec)
        print(json.dumps(rec), flush=True)
        for e in engs:
            e.close()
        del engs, bufs
        torch.cuda.empty_cache()
