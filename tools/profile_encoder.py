"""Run the encoder (and optionally a short decode) of one 64-image 384x384 batch, for
rocprofv3 PMC passes that must stay small (counter collection serialises dispatches).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- python tools/profile_encoder.py
"""
import argparse
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (shared HIP runtime)

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="bf16x3")
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--encodes", type=int, default=1)
ap.add_argument("--decode-steps", type=int, default=0)
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
eng = pkg.Engine(img_hw=(384, 384), max_batch=a.batch, precision=a.precision)
eng.load_weights(pkg.synth.make_weights(1234, "init"))
eng.set_images(pkg.synth.make_images(a.batch, 384, 384))
for _ in range(a.encodes):
    eng.encode()
if a.decode_steps:
    eng.decode(max_steps=a.decode_steps, stop="none")
eng.close()
print("done")
