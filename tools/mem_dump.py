"""Dump one encode's memory (bf16x3, 384², synthetic weights / images) to an .npy file, for
bitwise comparisons of two library builds (tools/sessions/*: --lib A vs --lib B).

    python tools/mem_dump.py OUT.npy [--lib LIB] [--variant unfused_attn] [--batch 4] [--decode 24]
"""
import argparse
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--lib", default=None)
ap.add_argument("--variant", default="")
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--decode", type=int, default=0, help="also decode this many greedy steps and save the logits")
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
if a.lib:
    pkg.engine.load_library(a.lib, ab_build=True)
var = tuple(v for v in a.variant.split(",") if v)
eng = pkg.Engine(img_hw=(384, 384), max_batch=a.batch, precision="bf16x3", variant=var)
eng.load_weights(pkg.synth.make_weights(1234, "init"))
eng.encode(pkg.synth.make_images(a.batch, 384, 384))
np.save(a.out, eng.memory())
if a.decode:
    r = eng.decode(max_steps=a.decode, stop="none", want_logits=True)
    np.save(a.out.replace(".npy", "_logits.npy"), r.logits)
    np.save(a.out.replace(".npy", "_ids.npy"), r.ids)
eng.close()
print("saved", a.out)
