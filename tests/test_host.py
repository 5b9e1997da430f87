"""CPU: host-side logic around the engine (weights, tokenizer, pre-processing, serving
result assembly, batching) — no GPU calls."""
import numpy as np
import pytest


def test_pack_state_dict_aliases(pkg):
    w = pkg.synth.make_weights(2, "perturbed", vocab=300)
    blob = pkg.weights.pack_state_dict(w)
    assert blob.dtype == np.float32 and blob.size == sum(v.size for v in w.values())
    # a training checkpoint stores the encoder under encoder.swin.features.* as well
    alias = {("encoder.swin." + k[len("encoder."):] if k.startswith("encoder.features.") else k): v
             for k, v in w.items()}
    alias["decoder.tgt_mask"] = np.zeros((150, 150), np.float32)
    alias["encoder.swin.norm.weight"] = np.ones(768, np.float32)
    np.testing.assert_array_equal(pkg.weights.pack_state_dict(alias), blob)
    bad = dict(w)
    bad["decoder.fc_out.bias"] = bad["decoder.fc_out.bias"][:-1]
    with pytest.raises(ValueError):
        pkg.weights.pack_state_dict(bad, vocab=300)
    missing = dict(w)
    del missing["encoder.projection.weight"]
    with pytest.raises(KeyError):
        pkg.weights.pack_state_dict(missing)


def test_checkpoint_roundtrip(pkg, tmp_path):
    import torch
    w = pkg.synth.make_weights(4, "init", vocab=200)
    path = tmp_path / "best_model.pth"
    torch.save({"epoch": 3, "model_state_dict": {k: torch.from_numpy(v) for k, v in w.items()}}, path)
    sd = pkg.weights.load_checkpoint(str(path))
    np.testing.assert_array_equal(pkg.weights.pack_state_dict(sd), pkg.weights.pack_state_dict(w))


def test_synthetic_weights_deterministic(pkg):
    a = pkg.synth.make_weights(9, "init", vocab=100)
    b = pkg.synth.make_weights(9, "init", vocab=100)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    t = pkg.synth.make_weights(9, "init", tied=True, vocab=100)
    np.testing.assert_array_equal(t["decoder.decoder.layers.0.linear1.weight"],
                                  t["decoder.decoder.layers.7.linear1.weight"])


@pytest.mark.parametrize("formula,tokens", [
    (r"\frac{x^2}{2}", ["\\frac", "{", "x", "^", "2", "}", "{", "2", "}"]),
    (r"a_{12}+\alpha", ["a", "_", "{", "12", "}", "+", "\\alpha"]),
    (r"\sum _ { i = 0 } ^ { n }", ["\\sum", "_", "{", "i", "=", "0", "}", "^", "{", "n", "}"]),
    ("xy 3.5", ["xy", "3", ".", "5"]),
])
def test_tokenize_latex(pkg, formula, tokens):
    assert pkg.utils.tokenize_latex(formula) == tokens


@pytest.mark.parametrize("raw,clean", [
    (r"\begin {matrix} a \end {matrix}", r"\begin{matrix} a \end{matrix}"),
    (r"x { abc } y", r"x {abc} y"),
    (r"a \ \ b", r"a \\ b"),
    (r"\frac { x } { 2 }", r"\frac {x} { 2 }"),
])
def test_clean_latex_output(pkg, raw, clean):
    assert pkg.utils.clean_latex_output(raw) == clean


def test_tokens_to_latex_drops_specials(pkg):
    vocab, idx2char = pkg.synth.synthetic_vocab(50)
    ids = [vocab["<sos>"], vocab["x"], vocab["<pad>"], vocab["+"], vocab["y"], vocab["<eos>"], 10_000]
    assert pkg.utils.tokens_to_latex(ids, idx2char) == "x + y"
    assert pkg.utils.detokenize([1, vocab["x"], 0, vocab["y"], 2, vocab["z"]], idx2char) == "x y"


def test_load_vocab(pkg, tmp_path):
    import json
    vocab, idx2char = pkg.synth.synthetic_vocab(20)
    p = tmp_path / "vocab.json"
    p.write_text(json.dumps({"vocab": vocab, "idx2char": {str(k): v for k, v in idx2char.items()}}))
    v2, i2 = pkg.utils.load_vocab(str(p))
    assert v2 == vocab and i2 == idx2char


def test_preprocess_image(pkg):
    from PIL import Image
    rng = np.random.default_rng(0)
    rgb = Image.fromarray(rng.integers(0, 256, size=(150, 500, 3), dtype=np.uint8), "RGB")
    x = pkg.preprocess.preprocess_image(rgb)
    assert x.shape == (1, 1, 96, 320) and x.dtype == np.float32
    assert x.min() >= -1.0 and x.max() <= 1.0
    ref = np.asarray(rgb.convert("L").resize((320, 96), Image.BILINEAR), np.float32) / 255.0
    np.testing.assert_allclose(x[0, 0], (ref - 0.5) / 0.5, atol=1e-6)


def test_serving_row_result_semantics(pkg):
    """app/src/im2latex.py:33-55: the EOS step's log-prob is summed, the token count
    excludes it; an immediate EOS gives the fixed message and 0.0."""
    vocab, idx2char = pkg.synth.synthetic_vocab(50)
    x, y = vocab["x"], vocab["y"]
    ids = np.array([1, x, y, 2, x], np.int32)
    logp = np.array([-0.5, -1.0, -0.25, -3.0], np.float32)
    f, conf = pkg.im2latex._row_result(ids, logp, 4, 2, idx2char)
    assert f == "x y"
    assert conf == pytest.approx(float(np.exp(np.float32((-0.5 - 1.0 - 0.25) / 2))))
    f, conf = pkg.im2latex._row_result(np.array([1, 2, 2], np.int32), np.array([-0.1, -0.1], np.float32), 2, 2,
                                       idx2char)
    assert f == pkg.im2latex.EMPTY_MESSAGE and conf == 0.0
    # no EOS within max steps: every step counts
    f, conf = pkg.im2latex._row_result(np.array([1, x, x], np.int32), np.array([-1.0, -1.0], np.float32), 2, 2,
                                       idx2char)
    assert f == "x x" and conf == pytest.approx(float(np.exp(np.float32(-1.0))))


class _FakeEngine:
    """CPU stand-in for Engine.greedy used to test the host batching logic only."""
    max_batch = 3
    pad = 0

    def __init__(self, rows):
        self.rows = rows
        self.calls = []

    def greedy(self, images, max_steps, stop):
        from types import SimpleNamespace
        self.calls.append(images.shape[0])
        ids = np.array([self.rows[int(im[0, 0, 0])] for im in images], np.int32)
        return SimpleNamespace(ids=ids)


def test_inference_predict_chunks_batches(pkg):
    vocab, idx2char = pkg.synth.synthetic_vocab(50)
    x, y = vocab["x"], vocab["y"]
    rows = [[1, x, 2, 0], [1, y, y, 2], [1, 2, 0, 0], [1, x, y, 2], [1, y, 2, 0]]
    eng = _FakeEngine(rows)
    images = np.zeros((5, 1, 4, 4), np.float32)
    images[:, 0, 0, 0] = np.arange(5)
    out = pkg.inference.predict(images, eng, vocab, idx2char, "cpu")
    assert eng.calls == [3, 2]
    assert out == ["x", "y y", "", "x y", "y"]


def test_shard_bounds(pkg):
    for n, world in ((512, 8), (10, 3), (3, 4)):
        spans = [pkg.parallel.shard_bounds(n, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_replica_pool_imap_order_and_errors(pkg):
    import threading
    import time

    class E:
        def __init__(self, i):
            self.i = i

    pool = pkg.pipeline.ReplicaPool(engines=[E(0), E(1), E(2)])
    seen = set()

    def fn(eng, k):
        seen.add(threading.get_ident())
        time.sleep(0.01 * ((k * 7) % 3))
        return k * 10, eng.i

    out = list(pool.imap(fn, range(12)))
    assert [o[0] for o in out] == [k * 10 for k in range(12)]
    assert len({o[1] for o in out}) > 1  # work spread over replicas

    def bad(eng, k):
        if k == 4:
            raise RuntimeError("boom")
        return k

    got = []
    with pytest.raises(RuntimeError):
        for v in pool.imap(bad, range(8)):
            got.append(v)
    assert got == [0, 1, 2, 3]


def test_global_stop_over_shards(pkg):
    """SURVEY §8(e) option 2 on gathered ids: the batch stops after the step at which the
    last row produced its first EOS; a row that never does keeps the full width."""
    import numpy as np
    eos = pkg.synth.EOS_ID
    ids = np.full((3, 9), 7, np.int32)
    ids[:, 0] = pkg.synth.SOS_ID
    ids[0, 3] = eos  # step 2
    ids[1, 6] = eos  # step 5 (the global stop)
    ids[2, 2] = eos  # step 1, then post-EOS tokens
    ids[2, 4] = eos
    out, n = pkg.parallel.global_stop(ids, eos)
    assert n == 6 and out.shape == (3, 7)
    np.testing.assert_array_equal(out, ids[:, :7])
    ids[1, 6] = 7  # row 1 never finishes: no stop
    out, n = pkg.parallel.global_stop(ids, eos)
    assert n == 8 and out.shape == (3, 9)


def test_decode_into_tensor_checks(pkg):
    """``Engine.decode_into`` hands a raw device pointer to
    ``mocr_decode_device``, which writes batch x (max_steps + 1) int32 through it; the
    tensor's shape, dtype, layout and device are checked before the call."""
    import torch

    class FakeCuda:  # the attributes check_ids_tensor reads, as a CUDA tensor has them
        def __init__(self, shape, dtype=torch.int32, contiguous=True, index=0):
            self.shape, self.dtype, self.is_cuda = shape, dtype, True
            self._c, self.device = contiguous, torch.device("cuda", index)

        def is_contiguous(self):
            return self._c

    check = pkg.engine.check_ids_tensor
    check(FakeCuda((4, 9)), 4, 8, 0)  # accepted
    bad = [
        (torch.zeros(4, 9, dtype=torch.int32), 4, 8, 0),   # host tensor
        (FakeCuda((4, 9), dtype=torch.int64), 4, 8, 0),    # dtype
        (FakeCuda((4, 8)), 4, 8, 0),                       # too narrow: the C side writes 9 columns
        (FakeCuda((3, 9)), 4, 8, 0),                       # fewer rows than the encoded batch
        (FakeCuda((4, 9), contiguous=False), 4, 8, 0),     # strided
        (FakeCuda((4, 9), index=1), 4, 8, 0),              # another device
        (FakeCuda((0, 9)), 0, 8, 0),                       # nothing encoded
    ]
    for args in bad:
        with pytest.raises(ValueError):
            check(*args)
