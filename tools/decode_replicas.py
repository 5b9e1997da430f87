"""R engine replicas decoding concurrently (no encoder): for rocprofv3 kernel traces of
decode-kernel durations and in-stream gaps at R = 1 vs R = 3 (tools/trace_gaps.py)."""
import importlib
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 1
pkg = importlib.import_module("handwritten-math-ocr-api_amd")
w = pkg.synth.make_weights(1234, "init")
engs = []
for r in range(R):
    e = pkg.Engine(img_hw=(384, 384), max_batch=64, precision="bf16x3", device=0)
    e.load_weights(w)
    e.set_images(pkg.synth.make_images(64, 384, 384, seed0=1000 + 64 * r))
    e.encode()
    e.decode(max_steps=128, stop="none")
    engs.append(e)
th = [threading.Thread(target=lambda e=e: [e.decode(max_steps=128, stop="none") for _ in range(2)]) for e in engs]
[t.start() for t in th]
[t.join() for t in th]
print("done")
