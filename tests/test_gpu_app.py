"""GPU: the FastAPI surface on the real engine — /predict and the batched /predict/batch
return what im2latex.predict returns for each image on its own."""
import base64
import importlib
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
pytest.importorskip("fastapi")


def _png(seed):
    from PIL import Image
    rng = np.random.default_rng(seed)
    im = Image.fromarray(rng.integers(0, 256, size=(64, 256), dtype=np.uint8), "L")
    buf = io.BytesIO()
    im.save(buf, format="PNG")
    return buf.getvalue()


def test_app_on_engine(pkg):
    from fastapi.testclient import TestClient
    from oracle.gen_golden import apply_eos_boost
    appmod = importlib.import_module("handwritten-math-ocr-api_amd.app.main")
    vocab, idx2char = pkg.synth.synthetic_vocab()
    eng = pkg.Engine(img_hw=(96, 320), max_batch=10, precision="bf16x3")
    eng.load_weights(apply_eos_boost(pkg.synth.make_weights(21, "perturbed"), 1.72))
    client = TestClient(appmod.create_app(appmod.State(eng, vocab, idx2char)))
    pngs = [_png(i) for i in range(4)]
    single = []
    for p in pngs:
        from PIL import Image
        single.append(pkg.im2latex.predict(eng, pkg.preprocess.preprocess_image(Image.open(io.BytesIO(p))), vocab,
                                           idx2char))
    r = client.post("/predict", files={"file": ("a.png", pngs[0], "image/png")})
    assert r.status_code == 200, r.text
    assert r.json()["formula"] == single[0][0]
    r = client.post("/predict/batch", json={"images": [base64.b64encode(p).decode() for p in pngs]})
    body = r.json()
    assert body["successful_predictions"] == 4
    assert [x["formula"] for x in body["results"]] == [s[0] for s in single]
    np.testing.assert_allclose([x["confidence"] for x in body["results"]], [s[1] for s in single], rtol=1e-6)
    eng.close()


def test_load_model_checkpoint_file(pkg, golden, tmp_path):
    """f2 on the GPU: a training checkpoint file ({'model_state_dict': ...} with the
    encoder.swin.features.* aliases and the buffers the reference's state_dict holds,
    src/utils.py:61-71) through im2latex.load_model (weights-only torch.load) decodes the
    96x320 fixture batch to the reference's ids, batch-global stop included."""
    import torch
    from oracle.gen_golden import apply_eos_boost
    g = golden("g96x320_b4_eos")
    m = g["meta"]
    w = apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"])
    sd = {}
    for k, v in w.items():
        sd[k] = torch.from_numpy(v)
        if k.startswith("encoder.features."):  # the alias the reference's state_dict carries too
            sd["encoder.swin." + k[len("encoder."):]] = torch.from_numpy(v)
    sd["decoder.tgt_mask"] = torch.triu(torch.full((150, 150), float("-inf")), diagonal=1)
    path = tmp_path / "best_model.pth"
    torch.save({"epoch": 7, "model_state_dict": sd}, path)
    vocab, _ = pkg.synth.synthetic_vocab()
    eng = pkg.im2latex.load_model(str(path), vocab, "cuda:0", max_batch=m["B"], precision="fp32")
    eng.encode(pkg.synth.make_images(m["B"], m["H"], m["W"], m["img_seed"], m["img_kind"]))
    res = eng.decode(max_steps=m["steps"], stop="batch")
    eng.close()
    np.testing.assert_array_equal(res.ids, g["ids"])


def test_predict_microbatch_on_engine(pkg, golden):
    """VERDICT r05 item 7 on the GPU: 8 concurrent /predict requests are decoded as ONE
    engine call, and each returns what im2latex.predict returns for its image alone;
    then 8 copies of the serving fixture's image through the micro-batcher return the
    reference's own formula and confidence (``serve96x320_eos``, made by the reference's
    ``app/src/im2latex.py``)."""
    import threading
    from fastapi.testclient import TestClient
    from PIL import Image
    from oracle.gen_golden import apply_eos_boost
    appmod = importlib.import_module("handwritten-math-ocr-api_amd.app.main")
    vocab, idx2char = pkg.synth.synthetic_vocab()
    m = golden("serve96x320_eos")["meta"]
    eng = pkg.Engine(img_hw=(96, 320), max_batch=8, precision="bf16x3")
    eng.load_weights(apply_eos_boost(pkg.synth.make_weights(m["seed"], m["variant"]), m["eos_boost"]))
    pngs = [_png(i) for i in range(8)]
    single = [pkg.im2latex.predict(eng, pkg.preprocess.preprocess_image(Image.open(io.BytesIO(p))), vocab, idx2char)
              for p in pngs]
    st = appmod.State(eng, vocab, idx2char, batch_window_ms=5000, max_batch=8)
    client = TestClient(appmod.create_app(st))
    out = [None] * 8

    def one(i):
        out[i] = client.post("/predict", files={"file": (f"{i}.png", pngs[i], "image/png")})

    th = [threading.Thread(target=one, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert all(r is not None and r.status_code == 200 for r in out), [r and r.text for r in out]
    assert [r.json()["formula"] for r in out] == [s[0] for s in single]
    np.testing.assert_allclose([r.json()["confidence"] for r in out], [s[1] for s in single], rtol=1e-6)
    assert st.batcher.batch_sizes == [8]
    # the fixture image, 8 requests at once, straight into the batcher
    img = pkg.synth.make_images(1, m["H"], m["W"], m["img_seed"], m["img_kind"])
    futs = [st.batcher.submit(img) for _ in range(8)]
    res = [f.result(120) for f in futs]
    assert st.batcher.batch_sizes == [8, 8]
    for formula, conf in res:
        assert formula == m["formula"]
        assert conf == pytest.approx(m["confidence"], rel=1e-4, abs=1e-7)
    st.close()
    eng.close()
