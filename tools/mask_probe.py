"""Decode-only throughput of R concurrent replicas, each on all CUs or on its own
contiguous CU range (mocr_set_cu_mask), to test whether per-XCD isolation removes the
replicas' mutual slowdown (docs/DESIGN_history_r01-r05.md §5.6)."""
import importlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

pkg = importlib.import_module("handwritten-math-ocr-api_amd")
w = pkg.synth.make_weights(1234, "init")
engs = []
for r in range(4):
    e = pkg.Engine(img_hw=(384, 384), max_batch=64, precision="bf16x3")
    e.load_weights(w)
    e.set_images(pkg.synth.make_images(64, 384, 384, seed0=1000 + 64 * r))
    e.encode()
    e.decode(max_steps=128, stop="none")
    engs.append(e)


def run(R, n=4):
    out = []

    def f(e):
        t0 = time.perf_counter()
        for _ in range(n):
            e.decode(max_steps=128, stop="none")
        out.append(time.perf_counter() - t0)
    th = [threading.Thread(target=f, args=(engs[i],)) for i in range(R)]
    [t.start() for t in th]
    [t.join() for t in th]
    return round(R * n * 64 / max(out), 1)


res = {}
for R in (1, 2, 3, 4):
    for e in engs:
        e.set_cu_mask(None)
    res[f"R={R} all CUs img/s"] = run(R)
    span = 256 // R
    for i, e in enumerate(engs[:R]):
        e.set_cu_mask(range(i * span, (i + 1) * span))
    res[f"R={R} own {span} CUs img/s"] = run(R)
    print(json.dumps(res), flush=True)
