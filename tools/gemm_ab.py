"""Per-kernel-class encoder timings (HIP events) of one engine, for A/B runs of GEMM
variants selected by environment (MOCR_GEMM_RING=0|2|3):

    MOCR_GEMM_RING=2 python tools/gemm_ab.py --precision bf16x3
"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (shared HIP runtime)

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="bf16x3")
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--encodes", type=int, default=5)
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
eng = pkg.Engine(img_hw=(384, 384), max_batch=a.batch, precision=a.precision)
eng.load_weights(pkg.synth.make_weights(1234, "init"))
eng.set_images(pkg.synth.make_images(a.batch, 384, 384))
eng.encode()
eng.set_timing(True)
for _ in range(a.encodes):
    eng.encode()
st = eng.timing()
eng.close()
tot = sum(v["total_ms"] for v in st.values()) / a.encodes
rows = {k: (v["total_ms"] / v["launches"] * 1e3, v["flops"] / v["total_ms"] * 1e-9 if v["total_ms"] else 0)
        for k, v in sorted(st.items())}
print(json.dumps({"ring": os.environ.get("MOCR_GEMM_RING", "default"), "precision": a.precision,
                  "encoder_ms": tot, "us_tflops": rows}))
