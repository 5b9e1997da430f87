"""GPU: the ResNet18 + Transformer-encoder variant (BASELINE config 5,
src/model_res18trans.py) through the C-ABI, against the fixtures the reference's own
glue produced (oracle/gen_golden.py make_res18_fixture) and the CPU oracle.

Tolerances: token ids exact; memory max|Δ| <= 1e-3 * max(1, max|ref|) (the convs run
bf16x3: split-operand bf16 MFMA, ~1e-5 relative per layer); logits under teacher
forcing <= 1e-3.
"""
import numpy as np
import pytest
import torch

from oracle import model_ref, res18_ref
from oracle.gen_golden import apply_eos_boost

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))


def engine_for(pkg, m, precision="fp32", max_batch=None):
    w = apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"], arch="res18trans"), m["eos_boost"])
    eng = pkg.Engine(img_hw=(m["H"], m["W"]), max_batch=max_batch or m["B"], precision=precision, arch="res18trans")
    eng.load_weights(w)
    eng.set_encoder_pos(pkg.synth.make_pos_table(m["pos_seed"], eng.memory_tokens))
    return eng, w


@pytest.mark.parametrize("name", ["r384_b8_pert", "r96x320_b4_eos"])
def test_res18_matches_reference_fixture(pkg, golden, name):
    g = golden(name)
    m = g["meta"]
    eng, w = engine_for(pkg, m)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    mem = eng.memory()
    assert rel_err(mem, g["memory"]) <= 1e-3
    res = eng.decode(max_steps=m["steps"], stop="batch")
    eng.close()
    assert res.n_steps == m["n_steps"]
    np.testing.assert_array_equal(res.ids, g["ids"])


def test_res18_teacher_forced_logits(pkg, golden):
    g = golden("r384_b8_pert")
    m = g["meta"]
    eng, w = engine_for(pkg, m)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    n = g["logits"].shape[1]
    res = eng.decode(max_steps=n, stop="none", forced=g["ids"][:, :n + 1], want_logits=True)
    eng.close()
    assert np.abs(res.logits[:, :, :] - g["logits"]).max() <= 1e-3


def test_res18_batch_dependence_matches_oracle(pkg):
    """The encoder attends across the batch (src/model_res18trans.py:61-62): an image's
    memory depends on its batch, and the engine follows the oracle for each batch."""
    w = pkg.synth.make_weights(3, "perturbed", arch="res18trans")
    imgs = pkg.synth.make_images(5, 96, 320, seed0=1000)
    model = res18_ref.build_model(w)
    eng = pkg.Engine(img_hw=(96, 320), max_batch=5, precision="fp32", arch="res18trans")
    eng.load_weights(w)
    pos = pkg.synth.make_pos_table(1, eng.memory_tokens)
    eng.set_encoder_pos(pos)
    mems = []
    for B in (5, 2):
        eng.encode(imgs[:B])
        mems.append(eng.memory())
        with torch.no_grad():
            ref = model.encoder(torch.from_numpy(imgs[:B]), torch.from_numpy(pos)).numpy()
        assert rel_err(mems[-1], ref) <= 1e-3
    eng.close()
    assert np.abs(mems[0][:2] - mems[1]).max() > 1e-3


@pytest.mark.parametrize("precision", ["bf16x3", "bf16"])
def test_res18_precisions(pkg, golden, precision):
    g = golden("r384_b8_pert")
    m = g["meta"]
    eng, w = engine_for(pkg, m, precision=precision)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    mem = eng.memory()
    res = eng.decode(max_steps=m["steps"], stop="batch")
    eng.close()
    if precision == "bf16x3":
        assert rel_err(mem, g["memory"]) <= 1e-3
        np.testing.assert_array_equal(res.ids, g["ids"])
    else:  # single-pass bf16 convs: not token-exact, still close
        assert rel_err(mem, g["memory"]) <= 5e-2


def test_res18_requires_pos_table(pkg):
    eng = pkg.Engine(img_hw=(96, 320), max_batch=1, precision="fp32", arch="res18trans")
    eng.load_weights(pkg.synth.make_weights(3, "init", arch="res18trans"))
    with pytest.raises(pkg.engine.MocrError, match="mocr_set_encoder_pos"):
        eng.encode(pkg.synth.make_images(1, 96, 320))
    eng.close()
