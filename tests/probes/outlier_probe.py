"""CPU precision probe (test infrastructure, imports the oracle): how the narrow K/V
storage of the bench path (fp24 self- and cross-attention K/V, or int16 cross-attention
K/V with one scale per (row, column) over the memory's keys) moves the teacher-forced
logits on a badly conditioned encoder memory.

Two kinds of outliers, config-2 shape (384x384, bench weights, 8 images, 128 steps):
  * channels: rows of encoder.projection.weight scaled 30-100x (the g384_b8_outlier
    fixture's weights, oracle/gen_golden.py OUTLIER_ROWS);
  * tokens: 2 of the 144 memory tokens of every image scaled 10-300x (a memory the
    weights cannot produce here, fed to the decoder directly), so each K/V column has
    two keys far above the rest -- the case where a per-column int16 scale loses the
    most bits on the other keys.

    python tests/probes/outlier_probe.py > profiles/r04/outlier_probe.log
"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import model_ref  # noqa: E402
from oracle.gen_golden import OUTLIER_ROWS, apply_proj_outliers  # noqa: E402

pkg = importlib.import_module("handwritten-math-ocr-api_amd")
_orig = F._in_projection_packed
MODE = {"dt": None}


def fp24(x):
    bits = x.contiguous().view(torch.int32)
    return ((bits + 0x80) & ~0xFF).view(torch.float32)


def i16_chan(x):
    s = x.abs().amax(dim=0, keepdim=True).clamp_min(1e-30) / 32767.0
    return torch.round(x / s) * s


def patched(q, k, v, w, b=None):
    qq, kk, vv = _orig(q, k, v, w, b)
    if MODE["dt"] == "fp24":
        kk, vv = fp24(kk), fp24(vv)
    elif MODE["dt"] == "i16":  # int16 cross-attention K/V, fp24 self-attention cache
        kk, vv = (i16_chan(kk), i16_chan(vv)) if q is not k else (fp24(kk), fp24(vv))
    return qq, kk, vv


F._in_projection_packed = patched


def probe(label, model, mem):
    MODE["dt"] = None
    ys, _ = model_ref.greedy_decode(model, memory=mem, max_steps=128, stop="none")
    ref = model_ref.teacher_forced_logits(model, mem, ys)
    marg = model_ref.top2_margins(ref)
    out = [f"{label}: memory max|x| {float(mem.abs().max()):.1f}, min top-2 margin {float(marg.min()):.1e}"]
    for dt in ("fp24", "i16"):
        MODE["dt"] = dt
        o = model_ref.teacher_forced_logits(model, mem, ys)
        flips = int((o.argmax(-1) != ref.argmax(-1)).sum())
        out.append(f"{dt} max|d logits| {(o - ref).abs().max().item():.2e} argmax flips {flips}")
    print(" | ".join(out), flush=True)


torch.set_num_threads(min(16, os.cpu_count() or 1))
imgs = torch.from_numpy(pkg.synth.make_images(8, 384, 384, seed0=1000))
w = pkg.synth.make_weights(1234, "init")
model = model_ref.build_model(w)
mem0 = model_ref.encode(model, imgs)
probe("bench weights", model, mem0)
wo = apply_proj_outliers(pkg.synth.make_weights(1234, "init"), OUTLIER_ROWS)
mo = model_ref.build_model(wo)
probe(f"channel outliers {OUTLIER_ROWS}", mo, model_ref.encode(mo, imgs))
for scale in (10, 30, 100, 300):
    mem = mem0.clone()
    mem[:, [5, 77], :] *= scale
    probe(f"token outliers: tokens 5, 77 x{scale}", model, mem)
