"""CPU: the oracle restatement against the golden fixtures (generated from the
reference's own glue by oracle/gen_golden.py) and against HF Swin."""
import numpy as np
import pytest
import torch

from oracle import model_ref, swin_ref
from oracle.gen_golden import apply_eos_boost


def _model(pkg, meta):
    w = apply_eos_boost(pkg.synth.make_weights(meta["seed"], meta["variant"]), meta["eos_boost"])
    return model_ref.build_model(w)


def test_param_count(pkg):
    m = model_ref.build_model(pkg.synth.make_weights(3, "init"))
    assert model_ref.count_params(m) == 37_450_293  # README.md:89 "37.45M", V = 5075


def test_oracle_reproduces_golden_384(pkg, golden):
    g = golden("g384_b1_init")
    m = g["meta"]
    model = _model(pkg, m)
    imgs = torch.from_numpy(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    mem = model_ref.encode(model, imgs)
    np.testing.assert_allclose(mem.numpy(), g["memory"], rtol=0, atol=1e-5)
    ys, logits = model_ref.greedy_decode(model, memory=mem, max_steps=m["steps"], stop=m["stop"],
                                         record_logits=True)
    np.testing.assert_array_equal(ys.numpy(), g["ids"])
    np.testing.assert_allclose(torch.stack(logits, 1)[:, :g["logits"].shape[1]].numpy(), g["logits"], atol=1e-5)


def test_oracle_reproduces_golden_96x320_batch_stop(pkg, golden):
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    model = _model(pkg, m)
    imgs = torch.from_numpy(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    mem = model_ref.encode(model, imgs)
    np.testing.assert_allclose(mem.numpy(), g["memory"], atol=1e-5)
    ys, logits = model_ref.greedy_decode(model, memory=mem, max_steps=m["steps"], stop="batch", record_logits=True)
    np.testing.assert_array_equal(ys.numpy(), g["ids"])
    # the late teacher-forced windows (steps 40-47 and the last 8 before the global stop)
    logits = torch.stack(logits, 1).numpy()
    assert g["win_steps"].tolist() == list(range(40, 48)) + list(range(ys.shape[1] - 9, ys.shape[1] - 1))
    np.testing.assert_allclose(logits[:, g["win_steps"]], g["win_logits"], atol=1e-5)


def test_detokenize_matches_reference_strings(pkg, golden):
    g = golden("g96x320_b4_eos")
    _, idx2char = pkg.synth.synthetic_vocab()
    assert [pkg.utils.detokenize(r, idx2char) for r in g["ids"]] == g["meta"]["strings"]


def test_serving_oracle_matches_fixture(pkg, golden):
    for name in ("serve96x320_eos", "serve96x320_empty"):
        g = golden(name)
        m = g["meta"]
        model = _model(pkg, m)
        img = torch.from_numpy(pkg.synth.make_images(1, m["H"], m["W"], m["img_seed"], m["img_kind"]))
        toks, lp_sum, conf = model_ref.serving_predict(model, img)
        assert toks == g["tokens"].tolist()
        assert abs(conf - m["confidence"]) <= 1e-6 * max(1.0, abs(m["confidence"]))
        _, idx2char = pkg.synth.synthetic_vocab()
        if toks:
            f = pkg.utils.clean_latex_output(pkg.utils.tokens_to_latex(toks, idx2char))
        else:
            f = pkg.im2latex.EMPTY_MESSAGE
        assert f == m["formula"]


def test_oracle_swin_matches_hf_384(pkg):
    pytest.importorskip("transformers")
    from oracle import hf_crosscheck
    w = pkg.synth.make_weights(17, "perturbed")
    err, scale = hf_crosscheck.crosscheck(w, pkg.synth.make_images(1, 384, 384, 77))
    assert err < 1e-5 * max(1.0, scale), (err, scale)


def _device_region(y, P, s):
    """Python copy of csrc/common.h shift_region (the engine's mask region id)."""
    if s == 0:
        return 2
    return int(y >= P - 7) + int(y >= P - s)


@pytest.mark.parametrize("pH,pW,sh,sw", [(98, 98, 3, 3), (28, 84, 3, 3), (7, 21, 0, 3), (7, 14, 0, 3),
                                          (14, 42, 3, 3), (49, 49, 3, 3), (21, 7, 3, 0)])
def test_shift_mask_regions(pH, pW, sh, sw):
    """torchvision builds the shift mask with python slices; with a zero shift on one
    axis the (-0, None) slice covers the whole axis.  The engine's arithmetic form must
    give the same region map (up to relabelling) on the padded map."""
    ref = swin_ref.shift_region_ids(pH, pW, sh, sw).numpy()
    dev = np.array([[3 * _device_region(y, pH, sh) + _device_region(x, pW, sw) for x in range(pW)]
                    for y in range(pH)])
    # same partition: equal ids <-> equal ids
    a = ref.reshape(-1)
    b = dev.reshape(-1)
    assert np.array_equal(a[:, None] == a[None, :], b[:, None] == b[None, :])



def test_oracle_resnet18_matches_hf(pkg):
    """oracle/res18_ref.py's torchvision-resnet18 restatement (BasicBlock, eval BN, 1-channel
    stem) against HF transformers ResNetModel with the same weights (torchvision itself is
    not installed): the two are independent implementations of the same network."""
    from oracle import hf_crosscheck
    w = pkg.synth.make_weights(1234, "init", arch="res18trans")
    err, scale = hf_crosscheck.crosscheck_resnet18(w, pkg.synth.make_images(2, 384, 384, 77))
    assert err < 1e-4 * max(1.0, scale), (err, scale)

@pytest.mark.parametrize("name", ["r384_b8_pert", "r96x320_b4_eos"])
def test_res18_oracle_reproduces_golden(pkg, golden, name):
    """ResNet18-trans (BASELINE config 5): the restatement reproduces the fixtures the
    reference's own src/model_res18trans.py + src/inference.py produced."""
    from oracle import res18_ref
    g = golden(name)
    m = g["meta"]
    w = apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"], arch="res18trans"), m["eos_boost"])
    model = res18_ref.build_model(w)
    imgs = torch.from_numpy(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    pos = torch.from_numpy(pkg.synth.make_pos_table(m["pos_seed"], g["memory"].shape[1]))
    with torch.no_grad():
        mem = model.encoder(imgs, pos)
    np.testing.assert_allclose(mem.numpy(), g["memory"], rtol=0, atol=1e-5)
    ys, logits = model_ref.greedy_decode(model, memory=mem, max_steps=m["steps"], stop=m["stop"], record_logits=True)
    np.testing.assert_array_equal(ys.numpy(), g["ids"])
    np.testing.assert_allclose(torch.stack(logits, 1)[:, :g["logits"].shape[1]].numpy(), g["logits"], atol=1e-5)


def test_res18_encoder_attends_across_the_batch(pkg):
    """Quirk of src/model_res18trans.py:61-62 (batch_first=True on a [w, B, d] tensor):
    an image's memory depends on the other images of its batch."""
    from oracle import res18_ref
    model = res18_ref.build_model(pkg.synth.make_weights(3, "perturbed", arch="res18trans"))
    imgs = torch.from_numpy(pkg.synth.make_images(3, 96, 320, seed0=1000))
    pos = torch.from_numpy(pkg.synth.make_pos_table(1, 10))
    with torch.no_grad():
        full = model.encoder(imgs, pos)
        alone = model.encoder(imgs[:1], pos)
    assert not torch.allclose(full[:1], alone, atol=1e-3)
