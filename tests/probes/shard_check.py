"""Debug aid: the sharded-test fixture (g96x320_b4_eos) decoded at B=4 and as two B=2
shards in one process, compared with the fixture ids; prints the first mismatch per row.
    python tests/probes/shard_check.py [--lib path/libmathocr.so]
"""
import argparse
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--precision", default="bf16x3")
a = ap.parse_args()
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
if a.lib:
    pkg.engine.load_library(a.lib, ab_build=True)
from tests.conftest import load_golden  # noqa: E402
from oracle.gen_golden import apply_eos_boost  # noqa: E402

g = load_golden("g96x320_b4_eos")
m = g["meta"]
ref = g["ids"]
steps = ref.shape[1] - 1
w = apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"])
imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])


def run(lo, hi):
    eng = pkg.Engine(img_hw=(m["H"], m["W"]), max_batch=hi - lo, precision=a.precision, device=0)
    eng.load_weights(w)
    eng.encode(imgs[lo:hi])
    r = eng.decode(max_steps=steps, stop="none").ids
    eng.close()
    return r


def report(tag, out):
    for i in range(out.shape[0]):
        bad = np.nonzero(out[i] != ref[i])[0]
        print(f"{tag} row {i}: " + ("ok" if not len(bad) else f"first mismatch col {bad[0]} ({len(bad)} cols)"), flush=True)


report("B4", run(0, 4))
report("2xB2", np.concatenate([run(0, 2), run(2, 4)]))
report("4xB1", np.concatenate([run(i, i + 1) for i in range(4)]))
