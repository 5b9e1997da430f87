"""Per-op HIP-event times of one --batch-image (default 64) 384x384 encode (the engine's timed() names),
fused vs unfused attention / MLP variants side by side.

    python tools/op_times.py [--encodes 3] [--filter s3.,s4.] [--lib LIB]
"""
import argparse
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (shared HIP runtime)

ap = argparse.ArgumentParser()
ap.add_argument("--encodes", type=int, default=3)
ap.add_argument("--filter", default="")
ap.add_argument("--variants", default="production,unfused_attn")
ap.add_argument("--lib", default=None, help="libmathocr.so to load (an A/B build from tools/build_variant.sh)")
ap.add_argument("--batch", type=int, default=64)
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
if a.lib:
    pkg.engine.load_library(a.lib, ab_build=True)
imgs = pkg.synth.make_images(a.batch, 384, 384)
w = pkg.synth.make_weights(1234, "init")
res = {}
for vname in a.variants.split(","):
    var = () if vname == "production" else tuple(vname.split("+"))
    eng = pkg.Engine(img_hw=(384, 384), max_batch=a.batch, precision="bf16x3", variant=var)
    eng.load_weights(w)
    eng.set_images(imgs)
    eng.encode()  # warm
    eng.set_timing(True)
    for _ in range(a.encodes):
        eng.encode()
    res[vname] = eng.timing()
    eng.close()
names = sorted({n for r in res.values() for n in r})
flt = [f for f in a.filter.split(",") if f]
print(f"{'op':28s}" + "".join(f"{v:>22s}" for v in res))
tot = {v: 0.0 for v in res}
for n in names:
    if flt and not any(n.startswith(f) for f in flt):
        continue
    row = f"{n:28s}"
    for v, r in res.items():
        if n in r:
            us = r[n]["total_ms"] * 1000 / a.encodes
            tot[v] += us
            row += f"{us:14.1f} us ({r[n]['launches'] // a.encodes:3d})"
        else:
            row += " " * 22
    print(row)
print(f"{'total':28s}" + "".join(f"{tot[v]:14.1f} us      " for v in res))
