"""Does the encoder of one engine replica overlap the greedy decode of another?
Replica A loops encode() (B=64, 384², bf16x3), replica B loops 128-step decodes; each
loop is timed alone and then with the other running in its own host thread.  With no
overlap the concurrent loops take the sum of the alone times; with full overlap, each
takes its alone time.  Also E+E and D+D (two replicas of the same half)."""
import importlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

pkg = importlib.import_module("handwritten-math-ocr-api_amd")
B, S = 64, 128
w = pkg.synth.make_weights(1234, "init")
engs = []
for r in range(3):
    e = pkg.Engine(img_hw=(384, 384), max_batch=B, precision="bf16x3", device=0)
    e.load_weights(w)
    e.set_images(pkg.synth.make_images(B, 384, 384, seed0=1000 + r * B))
    e.encode()
    e.decode(max_steps=S, stop="none")
    engs.append(e)


def enc_loop(e, n, out):
    t0 = time.perf_counter()
    for _ in range(n):
        e.encode()
    out.append(time.perf_counter() - t0)


def dec_loop(e, n, out):
    t0 = time.perf_counter()
    for _ in range(n):
        e.decode(max_steps=S, stop="none")
    out.append(time.perf_counter() - t0)


def run(jobs):
    outs = [[] for _ in jobs]
    th = [threading.Thread(target=f, args=(engs[i], n, outs[i])) for i, (f, n) in enumerate(jobs)]
    [t.start() for t in th]
    [t.join() for t in th]
    return [round(o[0] * 1e3, 2) for o in outs]


NE, ND = 30, 10
res = {}
# host time inside hipGraphLaunch per decode, alone and with 3 concurrent decoders
for e in engs:
    e.set_timing(True)
run([(dec_loop, 4)])
st = {k: v for k, v in engs[0].timing().items() if k.startswith("host") or k.startswith("decode")}
print("alone", json.dumps(st), flush=True)
for e in engs:
    e.set_timing(True)
run([(dec_loop, 4), (dec_loop, 4), (dec_loop, 4)])
for e in engs:
    st = {k: v for k, v in e.timing().items() if k.startswith("host") or k.startswith("decode")}
    print("3 concurrent", json.dumps(st), flush=True)
    e.set_timing(False)
masks = {
    "hi32": (list(range(0, 224)), list(range(224, 256))),
    "stride8": ([i for i in range(256) if i % 8 != 7], [i for i in range(256) if i % 8 == 7]),
    "hi64": (list(range(0, 192)), list(range(192, 256))),
    "stride4": ([i for i in range(256) if i % 4 != 3], [i for i in range(256) if i % 4 == 3]),
}
for name, (me, md) in masks.items():
    engs[0].set_cu_mask(me)
    engs[1].set_cu_mask(md)
    res[f"{name}: E alone"] = run([(enc_loop, NE)])
    res[f"{name}: D alone"] = run([(dec_loop, ND)])
    res[f"{name}: E || D"] = run([(enc_loop, NE), (dec_loop, ND)])
    print(json.dumps(res), flush=True)
engs[0].set_cu_mask(None)
engs[1].set_cu_mask(None)
for rep in range(1):
    res[f"E alone ({NE} encodes) ms"] = run([(enc_loop, NE)])
    res[f"D alone ({ND} decodes) ms"] = run([(dec_loop, ND)])
    res["E || D ms"] = run([(enc_loop, NE), (dec_loop, ND)])
    res["E || E ms"] = run([(enc_loop, NE), (enc_loop, NE)])
    res["D || D ms"] = run([(dec_loop, ND), (dec_loop, ND)])
    res["D || D || D ms"] = run([(dec_loop, ND), (dec_loop, ND), (dec_loop, ND)])
    print(json.dumps(res), flush=True)
