"""Throughput of R engine replicas on one GPU, each driven by its own host thread
(ctypes releases the GIL): decode (latency-bound) of one batch overlaps the encoder
(throughput-bound) of another."""
import importlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: F401,E402

pkg = importlib.import_module("handwritten-math-ocr-api_amd")
B, S, N = 64, 128, 4
prec = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
w = pkg.synth.make_weights(1234, "init")
engs = []
for r in range(4):
    e = pkg.Engine(img_hw=(384, 384), max_batch=B, precision=prec, device=0)
    e.load_weights(w)
    e.set_images(pkg.synth.make_images(B, 384, 384, seed0=1000 + r * B))
    e.encode()
    e.decode(max_steps=S, stop="none")
    engs.append(e)


def run(e, n, out):
    for _ in range(n):
        t0 = time.perf_counter()
        e.encode()
        e.decode(max_steps=S, stop="none")
        out.append(time.perf_counter() - t0)


res = {}
for R in (1, 2, 3, 4):
    outs = [[] for _ in range(R)]
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(engs[i], N, outs[i])) for i in range(R)]
    [t.start() for t in th]
    [t.join() for t in th]
    dt = time.perf_counter() - t0
    res[R] = {"img_s": R * N * B / dt, "batch_ms": 1e3 * sum(sum(o) for o in outs) / (R * N)}
print(json.dumps(res))
