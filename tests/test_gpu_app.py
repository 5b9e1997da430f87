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
