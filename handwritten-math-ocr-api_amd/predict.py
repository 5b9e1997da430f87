"""Batch-1 greedy prediction with the reference script's interface (``src/predict.py``).

``predict(image_tensor, model, vocab, idx2token, max_len=150)`` mirrors
``src/predict.py:49-67`` with an ``Engine`` in place of the module: encoder once, greedy
argmax appended until EOS or ``max_len`` steps, then ``output_seq[1:-1]`` mapped through
``idx2token`` -- so sos and the last token are dropped (the EOS when one was produced,
otherwise the ``max_len``-th token, as the reference does).  On one image the engine's
batch-global stop is exactly the script's per-sequence ``break``.
``preprocess_image(path)`` is ``src/predict.py:36-46`` (RGB, grayscale, resize to
``config.img_h x img_w``, [-1, 1]).
"""
from __future__ import annotations

import numpy as np

from .config import config
from .preprocess import preprocess_image as _preprocess


def preprocess_image(image_path: str) -> np.ndarray:
    from PIL import Image
    return _preprocess(Image.open(image_path).convert("RGB"))


def predict(image_tensor, model, vocab, idx2token, max_len: int = 150):
    """Tokens (strings) of one image [1, 1, H, W]."""
    if hasattr(image_tensor, "detach"):
        image_tensor = image_tensor.detach().cpu().numpy()
    img = np.ascontiguousarray(image_tensor, dtype=np.float32)
    if img.ndim != 4 or img.shape[0] != 1:
        raise ValueError("predict takes one image [1, 1, H, W]")
    if model.sos != vocab[config.sos_token] or model.eos != vocab[config.eos_token]:
        raise ValueError("engine sos/eos ids differ from the vocabulary's")
    res = model.greedy(img, max_steps=max_len, stop="batch")
    output_seq = res.ids[0, :res.n_steps + 1].tolist()
    return [idx2token[idx] for idx in output_seq[1:-1]]
