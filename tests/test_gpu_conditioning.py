"""GPU: the narrow K/V storage of the bench path on inputs it could get wrong.

* A badly conditioned encoder memory: the config-2 shape (384x384,
  greedy 128 steps, bench weights) with four memory channels scaled 30-100x
  (``encoder.projection.weight`` rows, ``oracle/gen_golden.py`` OUTLIER_ROWS), fixture
  pinned by the reference's own ``src/inference.py`` glue.  The int16 cross-attention K/V
  keeps one scale per (layer, row, column) over the 144 keys, so large columns are where
  it would lose bits.  Token ids exact, teacher-forced logits within 1e-3, on the
  production path (quantised in the crosskv GEMM's epilogue), on a beam-capable engine
  (quantised by ``quant_kv_i16_kernel``) and on the fp24 / fp32 K/V variants.
* Non-finite values: a NaN in the memory must reach the engine's
  non-finite-logits error on every K/V format, not decode into a finite wrong formula.
"""
import json

import numpy as np
import pytest

from conftest import check_logit_windows
from oracle.gen_golden import apply_proj_outliers

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3


def outlier_engine(pkg, g, variant=(), max_beam=0):
    m = g["meta"]
    eng = pkg.Engine(img_hw=(m["H"], m["W"]), max_batch=m["B"], precision="bf16x3", variant=variant,
                     max_beam=max_beam)
    eng.load_weights(apply_proj_outliers(pkg.synth.make_weights(m["seed"], m["variant"]), m["proj_outliers"]))
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], seed0=m["img_seed"]))
    return eng


@pytest.mark.parametrize("variant,max_beam", [((), 0), ((), 2), (("cross_kv_f24",), 0), (("self_kv_f24",), 0),
                                              (("kv_f32",), 0)],
                         ids=["int16-epilogue", "int16-pass", "fp24", "self-fp24", "fp32"])
def test_outlier_memory_kv_formats(pkg, golden, variant, max_beam):
    g = golden("g384_b8_outlier")
    m = g["meta"]
    assert m["proj_outliers"] and m["glue_checked"]
    eng = outlier_engine(pkg, g, variant, max_beam)
    mem = eng.memory()
    assert np.abs(g["memory"]).max() > 100.0  # the outlier channels are there
    rel = float(np.abs(mem - g["memory"]).max() / np.abs(g["memory"]).max())
    assert rel < 1e-4, rel
    res = eng.decode(max_steps=m["steps"], stop="batch")
    margins = g["margins"]
    tie = 1e-4
    for r in range(g["ids"].shape[0]):
        near = np.flatnonzero(margins[r] < tie)
        end = g["ids"].shape[1] if near.size == 0 else int(near[0]) + 1
        np.testing.assert_array_equal(res.ids[r, :end], g["ids"][r, :end], err_msg=f"row {r}")
    tf = eng.decode(max_steps=m["steps"], stop="none", forced=g["ids"], want_logits=True)
    r, n = g["logits"].shape[:2]
    err = float(np.abs(tf.logits[:r, :n] - g["logits"]).max())
    ok = margins >= tie
    np.testing.assert_array_equal(tf.logits.argmax(-1)[ok], g["ids"][:, 1:][ok])
    print("PARITY_RECORD", json.dumps({"fixture": "g384_b8_outlier", "kv": list(variant) or ["int16"],
                                       "max_beam": max_beam, "memory_rel_err": rel, "logits_max_abs_err": err,
                                       "rows_equal": int(sum(np.array_equal(res.ids[i], g["ids"][i])
                                                             for i in range(g["ids"].shape[0])))}))
    assert err < LOGIT_TOL, err
    check_logit_windows(tf.logits, g, label=f"g384_b8_outlier {'+'.join(variant) or 'int16'} beam{max_beam}")
    eng.close()


@pytest.mark.parametrize("variant,max_beam", [((), 0), ((), 2), (("cross_kv_f24",), 0), (("self_kv_f24",), 0),
                                              (("kv_f32",), 0)],
                         ids=["int16-epilogue", "int16-pass", "fp24", "self-fp24", "fp32"])
def test_nan_memory_is_reported(pkg, variant, max_beam):
    """One NaN in a memory channel's projection weight makes every cross-attention K/V
    column NaN; the decode must fail with the non-finite-logits error."""
    w = pkg.synth.make_weights(1234, "init")
    pw = w["encoder.projection.weight"].copy()
    pw[5, 17] = np.nan
    w["encoder.projection.weight"] = pw
    eng = pkg.Engine(img_hw=(384, 384), max_batch=2, precision="bf16x3", variant=variant, max_beam=max_beam)
    eng.load_weights(w)
    eng.encode(pkg.synth.make_images(2, 384, 384, seed0=1000))
    assert np.isnan(eng.memory()[:, :, 5]).all()
    with pytest.raises(pkg.MocrError, match="non-finite"):
        eng.decode(max_steps=8, stop="none")
    eng.close()


@pytest.mark.parametrize("variant", [(), ("self_kv_f24",)], ids=["self-int16", "self-fp24"])
def test_nan_self_attention_is_reported(pkg, variant):
    """A NaN in one key row of layer 0's self-attention projection makes that head's new keys
    NaN at every step; on the int16 cache (one scale per key over its 32 values) the scale
    carries the NaN, so the decode fails with the non-finite-logits error as on fp24."""
    w = pkg.synth.make_weights(1234, "init")
    k = "decoder.decoder.layers.0.self_attn.in_proj_weight"
    iw = w[k].copy()
    iw[256 + 40, 3] = np.nan  # a row of W_k (rows 256..511), head 1
    w[k] = iw
    eng = pkg.Engine(img_hw=(384, 384), max_batch=2, precision="bf16x3", variant=variant)
    eng.load_weights(w)
    eng.encode(pkg.synth.make_images(2, 384, 384, seed0=1000))
    with pytest.raises(pkg.MocrError, match="non-finite"):
        eng.decode(max_steps=8, stop="none")
    eng.close()


def test_engine_after_nan_poisoned_engine(pkg):
    """The int16 self-attention cache's value scales of keys not yet written are read by the
    key loop (masked by a zero weight): they are zeroed at allocation and masked in the
    kernel, so an engine allocated where a NaN-poisoned engine's cache was freed decodes as a
    fresh one."""
    w = pkg.synth.make_weights(1234, "init")
    imgs = pkg.synth.make_images(2, 384, 384, seed0=1000)

    def run(weights):
        eng = pkg.Engine(img_hw=(384, 384), max_batch=2, precision="bf16x3")
        eng.load_weights(weights)
        eng.encode(imgs)
        try:
            return eng.decode(max_steps=24, stop="none").ids
        finally:
            eng.close()

    clean = run(w)
    bad = dict(w)
    k = "decoder.decoder.layers.0.self_attn.in_proj_weight"
    iw = w[k].copy()
    iw[512:768, :] = np.nan  # W_v: every value (and value scale) of the cache is NaN
    bad[k] = iw
    with pytest.raises(pkg.MocrError, match="non-finite"):
        run(bad)
    np.testing.assert_array_equal(run(w), clean)
