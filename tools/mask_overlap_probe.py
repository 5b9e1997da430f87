"""Encoder / decoder overlap with the encoder's stream restricted to the first N CUs
(hipExtStreamCreateWithCUMask via Engine.set_cu_mask) and the decoder's on all CUs.
Replica E loops 256-image encodes, replica D loops 256-row 128-step decodes; each loop
alone, then both at once.  Perfect overlap: together = max(alone); none: the sum.

    python tools/mask_overlap_probe.py [--cus 256,224,192] [--ne 6] [--nd 4]
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
ap.add_argument("--cus", default="256,224,192")
ap.add_argument("--ne", type=int, default=6)
ap.add_argument("--nd", type=int, default=4)
ap.add_argument("--rows", type=int, default=256)
ap.add_argument("--dec-priority", type=int, default=0, help="decoder stream priority (> 0 high, < 0 low)")
ap.add_argument("--enc-priority", type=int, default=0)
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
R, S = a.rows, 128
w = pkg.synth.make_weights(1234, "init")
engs = []
for r in range(2):
    e = pkg.Engine(img_hw=(384, 384), max_batch=R, precision="bf16x3", device=0)
    e.load_weights(w)
    e.set_images(torch.from_numpy(pkg.synth.make_images(R, 384, 384, seed0=1000 + r * R)).to("cuda:0"))
    e.encode()
    engs.append(e)
ids = torch.empty((R, S + 1), dtype=torch.int32, device="cuda:0")
engs[0].set_stream_priority(a.enc_priority)
engs[1].set_stream_priority(a.dec_priority)
engs[1].decode_into(ids, max_steps=S, stop="none")
torch.cuda.synchronize()


def enc_loop(out):
    t0 = time.perf_counter()
    for _ in range(a.ne):
        engs[0].encode()
    out.append(time.perf_counter() - t0)


def dec_loop(out):
    t0 = time.perf_counter()
    for _ in range(a.nd):
        engs[1].decode_into(ids, max_steps=S, stop="none")
    torch.cuda.synchronize()
    out.append(time.perf_counter() - t0)


def run(fns):
    outs = [[] for _ in fns]
    th = [threading.Thread(target=f, args=(o,)) for f, o in zip(fns, outs)]
    [t.start() for t in th]
    [t.join() for t in th]
    return [round(o[0] * 1e3, 1) for o in outs]


for n in [int(x) for x in a.cus.split(",")]:
    if n < 256:
        engs[0].set_cu_mask(range(n))
    run([enc_loop])
    e_alone = run([enc_loop])[0]
    d_alone = run([dec_loop])[0]
    e_tog, d_tog = run([enc_loop, dec_loop])
    imgs = R * (a.ne + a.nd)
    print(json.dumps({"enc_cus": n, "dec_priority": a.dec_priority, "enc_priority": a.enc_priority, "enc_alone_ms": e_alone, "dec_alone_ms": d_alone, "enc_together_ms": e_tog,
                      "dec_together_ms": d_tog, "overlap": round((e_alone + d_alone - max(e_tog, d_tog)) /
                                                                 min(e_alone, d_alone), 3),
                      "img_s_together": round(R * a.ne / (max(e_tog, d_tog) / 1e3) * 0 + imgs / 2 / (max(e_tog, d_tog) / 1e3), 1)}),
          flush=True)
for e in engs:
    e.close()
