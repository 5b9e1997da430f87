"""GPU parity: libmathocr.so (through its C-ABI) vs the CPU oracle and the golden fixtures.

Tolerances (north_star: token ids bit-exact, logits within 1e-3):
* token ids: exact;
* logits under teacher forcing: max |Δ| <= 1e-3 (fp32 engine: observed ~1e-5);
* encoder maps / memory: max |Δ| <= 1e-3 * max(1, max|ref|).
"""
import numpy as np
import pytest
import torch

from conftest import check_logit_windows
from oracle import model_ref
from oracle.gen_golden import apply_eos_boost

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3


def rel_err(a, b):
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))


def make_engine(pkg, meta, max_batch=None, precision="fp32", variant=()):
    eng = pkg.Engine(img_hw=(meta["H"], meta["W"]), max_batch=max_batch or meta.get("B", 1), precision=precision,
                     variant=variant)
    w = apply_eos_boost(pkg.synth.make_weights(meta["seed"], meta["variant"]), meta["eos_boost"])
    eng.load_weights(w)
    return eng, w


@pytest.fixture(scope="module")
def g384(pkg, golden):
    g = golden("g384_b2_pert")
    m = g["meta"]
    eng, w = make_engine(pkg, m)
    imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])
    yield g, eng, w, imgs
    eng.close()


def test_encoder_stages_match_oracle(pkg, g384):
    g, eng, w, imgs = g384
    model = model_ref.build_model(w)
    _, stages = model_ref.encode(model, torch.from_numpy(imgs), stages=True)
    eng.set_images(imgs)
    for k, ref in enumerate(stages):
        got = eng.encode_until(k, tuple(ref.shape))
        e = rel_err(got, ref.numpy())
        assert e < 1e-4, f"features[{k}] rel err {e}"


@pytest.mark.parametrize("variant", [(), ("unfused_attn",), ("unfused_attn", "unfused_mlp"), ("s4_fused_attn",),
                                     ("window_rows",), ("unfused_attn", "window_rows"), ("s3_large_batch",),
                                     ("s3_large_batch", "unfused_mlp"), ("s3_large_batch", "unfused_ln_gemm"), ("s3_large_batch", "unfused_s3_tail"),
                                     ("unfused_ln_gemm",)])
def test_bf16x3_encoder_stages_match_oracle(pkg, golden, variant):
    """bf16x3 encoder stage by stage: the fused stage-1/2 attention half (wattn.hip) and
    MLP half (mlp.hip), the stage-3 no-proj kernel, the stage-4 two-half kernel (off in
    production), merge 1 in mlp.hip's lngemm384_kernel, stage 3's >= 128-image path (norm1
    + qkv in lngemm384_kernel,
    the window attention, mlp.hip's C = 384 fused MLP) and the unfused kernels they replace (MOCR_VARIANT_* flags), all within 1e-4 of
    the fp32 oracle.  384x384: the stage-1 map is 96x96, padded to 98
    (zero tokens) and rolled by 3 on odd blocks."""
    g = golden("g384_b2_pert")
    m = g["meta"]
    eng, w = make_engine(pkg, m, precision="bf16x3", variant=variant)
    imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])
    _, stages = model_ref.encode(model_ref.build_model(w), torch.from_numpy(imgs), stages=True)
    eng.set_images(imgs)
    for k, ref in enumerate(stages):
        got = eng.encode_until(k, tuple(ref.shape))
        e = rel_err(got, ref.numpy())
        assert e < 1e-4, f"features[{k}] rel err {e}"
    eng.close()


@pytest.mark.parametrize("case,base", [("g384_b2_pert", ()), ("g384_b2_pert", ("unfused_attn",)),
                                       ("g96x320_b4_eos", ("unfused_attn",))])
def test_pixel_rows_bitwise_window_rows(pkg, golden, case, base):
    """The unfused window attention over the image's tokens (production: stage 4; with
    unfused_attn: every stage) against the same sequence over the partitioned window rows
    (MOCR_VARIANT_WINDOW_ROWS): the padded tokens' k / v taken from the qkv bias must give
    the same bits as the qkv GEMM of their zero LayerNorm rows, so the encoder memory is
    bitwise equal (96x320: padding on both axes at every stage, shifted windows)."""
    g = golden(case)
    m = g["meta"]
    imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])
    mem = []
    for variant in (base, base + ("window_rows",)):
        eng, _ = make_engine(pkg, m, precision="bf16x3", variant=variant)
        eng.encode(imgs)
        mem.append(eng.memory())
        eng.close()
    assert np.array_equal(mem[0].view(np.uint32), mem[1].view(np.uint32))


def test_memory_matches_golden(pkg, g384):
    g, eng, w, imgs = g384
    eng.encode(imgs)
    mem = eng.memory()
    assert rel_err(mem, g["memory"]) < 1e-4


def test_greedy_ids_match_golden_384(pkg, g384):
    g, eng, w, imgs = g384
    eng.encode(imgs)
    res = eng.decode(max_steps=g["meta"]["steps"], stop="batch")
    assert res.n_steps == g["ids"].shape[1] - 1
    np.testing.assert_array_equal(res.ids, g["ids"])


def test_teacher_forced_logits_384(pkg, g384):
    g, eng, w, imgs = g384
    eng.encode(imgs)
    S = g["ids"].shape[1] - 1
    res = eng.decode(max_steps=S, stop="none", forced=g["ids"], want_logits=True, want_logp=True)
    n = g["logits"].shape[1]
    err = float(np.abs(res.logits[:, :n] - g["logits"]).max())
    assert err < LOGIT_TOL, err
    # argmax under teacher forcing reproduces the greedy ids
    np.testing.assert_array_equal(res.ids[:, 1:], g["ids"][:, 1:])


@pytest.mark.parametrize("variant", [(), ("logits_f32",), ("kv_f32",), ("cross_kv_f24",), ("self_kv_f24",)])
@pytest.mark.parametrize("name", ["g384_b2_pert", "g96x320_b4_eos"])
def test_teacher_forced_logits_bf16x3(pkg, golden, name, variant):
    """The bench precision (bf16x3 encoder GEMMs, attention, fold GEMMs and logits of the
    decode step, int16 cross K/V with per-column scales, the int16 self-attention cache
    with per-key scales; MOCR_VARIANT_LOGITS_F32: fp32 logits; MOCR_VARIANT_KV_F32: fp32
    K/V; CROSS_KV_F24 / SELF_KV_F24: fp24): teacher-forced logits within the north star's
    1e-3, ids token-exact."""
    g = golden(name)
    m = g["meta"]
    eng, _ = make_engine(pkg, m, precision="bf16x3", variant=variant)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    S = g["ids"].shape[1] - 1
    res = eng.decode(max_steps=S, stop="none", forced=g["ids"], want_logits=True)
    eng.close()
    n = g["logits"].shape[1]
    err = float(np.abs(res.logits[:, :n] - g["logits"]).max())
    print(f"{name} bf16x3 teacher-forced logits max|d| = {err:.2e}")
    assert err < LOGIT_TOL, err
    if "win_steps" in g:  # the late windows, up to the last steps before the global stop
        check_logit_windows(res.logits, g, label=f"{name} bf16x3 {'+'.join(variant) or 'production'}")
    margins = g["margins"]
    ok = margins >= 1e-4  # near-ties a different fp32 summation order may flip
    assert np.array_equal(res.ids[:, 1:][ok], g["ids"][:, 1:][ok])


@pytest.mark.parametrize("variant", [("dec_unfolded",), ("dec_narrow",)])
def test_decode_variant_matches_golden(pkg, golden, variant):
    """MOCR_VARIANT_DEC_UNFOLDED (the 8-kernel greedy step, LayerNorms applied by their
    consumers) and MOCR_VARIANT_DEC_NARROW (the folded step on decfold.hip's 16x16-tile
    GEMMs and decoder.hip's logits kernel instead of decwide.hip's wide tiles) give the
    fixture's ids and teacher-forced logits, as the production step does."""
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    eng, _ = make_engine(pkg, m, variant=variant)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    res = eng.decode(max_steps=m["steps"], stop="batch")
    np.testing.assert_array_equal(res.ids, g["ids"])
    S = g["ids"].shape[1] - 1
    tf = eng.decode(max_steps=S, stop="none", forced=g["ids"], want_logits=True)
    n = g["logits"].shape[1]
    assert float(np.abs(tf.logits[:, :n] - g["logits"]).max()) < LOGIT_TOL
    eng.close()


def test_decode_is_deterministic(pkg, g384):
    g, eng, w, imgs = g384
    eng.encode(imgs)
    a = eng.decode(max_steps=32, stop="none", want_logits=True)
    b = eng.decode(max_steps=32, stop="none", want_logits=True)
    np.testing.assert_array_equal(a.ids, b.ids)
    np.testing.assert_array_equal(a.logits, b.logits)


def test_init_weights_384(pkg, golden):
    g = golden("g384_b1_init")
    m = g["meta"]
    eng, _ = make_engine(pkg, m)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    assert rel_err(eng.memory(), g["memory"]) < 1e-4
    res = eng.decode(max_steps=m["steps"], stop="batch")
    np.testing.assert_array_equal(res.ids, g["ids"])
    eng.close()


def test_96x320_batch_global_stop(pkg, golden):
    """Padded maps, shift disabled on one axis (stages 3-4), EOS reached at different
    steps per row: rows keep generating until the whole batch has finished."""
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    eng, _ = make_engine(pkg, m)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    assert rel_err(eng.memory(), g["memory"]) < 1e-4
    res = eng.decode(max_steps=m["steps"], stop="batch")
    assert res.n_steps == g["ids"].shape[1] - 1
    np.testing.assert_array_equal(res.ids, g["ids"])
    eng.close()


def test_sub_batches_match_golden_prefix(pkg, golden):
    """40 images with the batch-global stop (EOS at different steps per row).
    Rows 0-3 are the golden fixture's images: their ids agree with the fixture up to
    the fixture's stop step (later steps depend only on earlier ones)."""
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    eng, _ = make_engine(pkg, dict(m, B=40))
    eng.encode(pkg.synth.make_images(40, m["H"], m["W"], m["img_seed"], m["img_kind"]))
    res = eng.decode(max_steps=m["steps"], stop="batch")
    n_ref = g["ids"].shape[1]
    np.testing.assert_array_equal(res.ids[:4, :n_ref], g["ids"])
    # batch-global stop: every row has produced EOS by the last step, and some row's
    # first EOS is exactly the last step
    first_eos = [int(np.argmax(r[1:] == 2)) + 1 if (r[1:] == 2).any() else None for r in res.ids]
    if res.n_steps < m["steps"]:
        assert all(f is not None for f in first_eos)
        assert max(first_eos) == res.n_steps
    # fixed-length decode of the same batch gives the same prefix
    full = eng.decode(max_steps=m["steps"], stop="none")
    np.testing.assert_array_equal(full.ids[:, :res.n_steps + 1], res.ids)
    eng.close()


def test_batch_invariance_384(pkg, g384):
    """A row's tokens do not depend on the rest of the batch: row 1 of the B=2 fixture
    decoded alone (B=1) gives the same ids."""
    g, _, w, imgs = g384
    eng = pkg.Engine(img_hw=(384, 384), max_batch=1)
    eng.load_weights(w)
    eng.encode(imgs[1:2])
    res = eng.decode(max_steps=g["meta"]["steps"], stop="none")
    np.testing.assert_array_equal(res.ids[0], g["ids"][1])
    eng.close()


def test_long_chain_rows_bitwise(pkg, g384):
    """A 520-row chain (above 480 rows every fold GEMM takes decwide.hip's 32 x 32 tiles
    with the vectorised epilogue, and the FFN keeps two k steps in flight) gives rows 0-1
    bitwise the logits of the 2-row chain (16-row tiles, one column per thread): the
    LayerNorm slice statistics sum the same pairs with the same rounding in both epilogue
    shapes.  Both encodes run stage 3 on its large-batch kernels, so the
    memory is bitwise equal too."""
    g, _, w, imgs = g384
    S = 24
    big = np.concatenate([imgs, pkg.synth.make_images(518, 384, 384, seed0=5000)], 0)
    out, mem = {}, {}
    for rows, x in ((520, big), (2, imgs)):
        eng = pkg.Engine(img_hw=(384, 384), max_batch=rows, precision="bf16x3", variant=("s3_large_batch",))
        eng.load_weights(w)
        eng.encode(x)
        mem[rows] = eng.memory()[:2]
        r = eng.decode(max_steps=S, stop="none", want_logits=True)
        out[rows] = (r.ids[:2].copy(), r.logits[:2].copy())
        eng.close()
    np.testing.assert_array_equal(mem[520], mem[2])
    np.testing.assert_array_equal(out[520][0], out[2][0])
    np.testing.assert_array_equal(out[520][1], out[2][1])


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_wide_chain_rows_bitwise(pkg, g384, precision):
    """A 100-row decode chain (decwide.hip: 32-row fold-GEMM tiles, 64-column logits tiles,
    a partial last row tile) gives rows 0-1 bitwise the logits and ids of the 2-row chain
    (16-row tiles, 32-column logits tiles): every output element sums the same k in the
    same order whatever the tile shape, so rows do not depend on the chain they decode in.
    Rows 0-1 are the B=2 fixture's images; their ids match the fixture.  (Below 128 images
    the encoder takes the same kernels at both batch sizes, so the memory is bitwise equal
    too.)"""
    g, _, w, imgs = g384
    S = 24
    others = pkg.synth.make_images(98, 384, 384, seed0=5000)
    big = np.concatenate([imgs, others], 0)
    out, mem = {}, {}
    for rows, x in ((100, big), (2, imgs)):
        eng = pkg.Engine(img_hw=(384, 384), max_batch=rows, precision=precision)
        eng.load_weights(w)
        eng.encode(x)
        mem[rows] = eng.memory()[:2]
        out[rows] = eng.decode(max_steps=S, stop="none", want_logits=True)
        eng.close()
    np.testing.assert_array_equal(out[100].ids[:2], out[2].ids)
    np.testing.assert_array_equal(out[2].ids, g["ids"][:, :S + 1])
    np.testing.assert_array_equal(mem[100], mem[2])
    np.testing.assert_array_equal(out[100].logits[:2], out[2].logits)


@pytest.mark.parametrize("precision,tol,variant", [("bf16x3", 1e-4, ()), ("bf16", 3e-2, ()),
                                                   ("bf16", 3e-2, ("s3_large_batch",))])
def test_bf16_encoder_modes(pkg, golden, precision, tol, variant):
    """bf16 MFMA encoder GEMMs: bf16x3 (split hi/lo operands) keeps fp32-level memory
    error and the golden token ids; plain bf16 is checked for its looser error only."""
    g = golden("g384_b2_pert")
    m = g["meta"]
    eng, _ = make_engine(pkg, m, precision=precision, variant=variant)
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    assert rel_err(eng.memory(), g["memory"]) < tol
    res = eng.decode(max_steps=m["steps"], stop="none", forced=g["ids"], want_logits=True)
    lerr = float(np.abs(res.logits[:, :g["logits"].shape[1]] - g["logits"]).max())
    if precision == "bf16x3":
        assert lerr < LOGIT_TOL, lerr
        greedy = eng.decode(max_steps=m["steps"], stop="batch")
        np.testing.assert_array_equal(greedy.ids, g["ids"])
    else:
        assert lerr < 0.05, lerr
    eng.close()


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_serving_predict_matches_reference(pkg, golden, precision):
    """im2latex.predict on the engine == the reference app/src/im2latex.py output
    (formula string and confidence) for the EOS and the empty-output fixtures; the
    batched predict gives the same per-image results."""
    vocab, idx2char = pkg.synth.synthetic_vocab()
    eng = pkg.Engine(img_hw=(96, 320), max_batch=4, precision=precision)
    imgs, expected = [], []
    for name in ("serve96x320_eos", "serve96x320_empty"):
        m = golden(name)["meta"]
        eng.load_weights(apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"]))
        img = pkg.synth.make_images(1, m["H"], m["W"], m["img_seed"], m["img_kind"])
        formula, conf = pkg.im2latex.predict(eng, img, vocab, idx2char)
        assert formula == m["formula"]
        assert conf == pytest.approx(m["confidence"], rel=1e-4, abs=1e-7)
        imgs.append(img)
        expected.append((formula, conf))
    # batched: both images under the EOS fixture's weights, vs single-image calls
    m = golden("serve96x320_eos")["meta"]
    eng.load_weights(apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"]))
    batch = np.concatenate(imgs + imgs[:1], 0)
    got = pkg.im2latex.predict_batch(eng, batch, vocab, idx2char)
    single = [pkg.im2latex.predict(eng, batch[i:i + 1], vocab, idx2char) for i in range(batch.shape[0])]
    assert [g[0] for g in got] == [s[0] for s in single]
    np.testing.assert_allclose([g[1] for g in got], [s[1] for s in single], rtol=1e-6)
    assert got[0][0] == expected[0][0]
    eng.close()


def test_inference_predict_strings(pkg, golden):
    """src/inference.py predict(): strings of the 96x320 batch fixture."""
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    vocab, idx2char = pkg.synth.synthetic_vocab()
    eng, _ = make_engine(pkg, dict(m, B=3))  # max_batch 3 < 4 images: chunked decode
    imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])
    assert pkg.inference.predict(imgs, eng, vocab, idx2char, "cuda") == m["strings"]
    eng.close()


def test_predict_script_batch1(pkg, golden):
    """src/predict.py predict(): one image at a time, stop at its own EOS, tokens
    output_seq[1:-1] (sos and EOS dropped) -- each row of the 96x320 fixture."""
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    vocab, idx2char = pkg.synth.synthetic_vocab()
    eng, _ = make_engine(pkg, dict(m, B=1))
    imgs = pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"])
    for r in range(m["B"]):
        row = g["ids"][r]
        e = int(np.flatnonzero(row[1:] == pkg.synth.EOS_ID)[0]) + 1  # column of the first EOS
        expected = [idx2char[int(i)] for i in row[1:e]]
        assert pkg.predict.predict(imgs[r:r + 1], eng, vocab, idx2char) == expected
    eng.close()


def test_cu_mask_and_priority_exclude_each_other(pkg):
    """HIP makes an engine stream with a CU mask or a priority, not both: the
    second setting fails instead of silently dropping the first; clearing one allows the
    other, and the engine still decodes correctly on the rebuilt stream."""
    g = pkg.synth
    eng = pkg.Engine(img_hw=(96, 320), max_batch=1, precision="fp32")
    eng.set_cu_mask(range(128))
    with pytest.raises(pkg.MocrError, match="CU mask"):
        eng.set_stream_priority(1)
    # the normal priority on a masked stream keeps the mask: still refused
    eng.set_stream_priority(0)
    with pytest.raises(pkg.MocrError, match="CU mask"):
        eng.set_stream_priority(1)
    eng.set_cu_mask(None)
    eng.set_stream_priority(1)
    with pytest.raises(pkg.MocrError, match="priority"):
        eng.set_cu_mask(range(64))
    # clearing a mask the stream does not have keeps its priority: a mask is still refused
    eng.set_cu_mask(None)
    with pytest.raises(pkg.MocrError, match="priority"):
        eng.set_cu_mask(range(64))
    eng.set_stream_priority(0)
    eng.set_cu_mask(range(64))
    eng.load_weights(g.make_weights(5, "perturbed"))
    eng.encode(g.make_images(1, 96, 320, 1000, "ink"))
    a = eng.decode(max_steps=4, stop="none").ids
    eng.set_cu_mask(None)
    b = eng.decode(max_steps=4, stop="none").ids
    np.testing.assert_array_equal(a, b)
    eng.close()
