"""Batched greedy inference with the reference's call signature (``src/inference.py:7-42``).

``predict(images, model, vocab, idx2char, device, beam_size=3)`` takes an ``Engine`` in
place of the PyTorch model and returns one string per image.  Semantics follow the
reference: encoder once, greedy argmax for up to ``config.max_seq_len`` steps, stop once
every row has produced EOS (rows keep generating until then), detokenise by skipping
sos/pad and stopping at the first eos.  ``beam_size`` is accepted and unused, as in the
reference.  Batches larger than the engine's ``max_batch`` are decoded in chunks; a
row's string depends only on its tokens up to its first EOS, which do not depend on
the other rows, so chunking does not change any output.
"""
from __future__ import annotations

import numpy as np

from .config import config
from .utils import detokenize


def _as_numpy(images):
    if hasattr(images, "detach"):
        images = images.detach().cpu().numpy()
    return np.ascontiguousarray(images, dtype=np.float32)


def greedy_ids(model, images, max_steps: int = config.max_seq_len, stop: str = "batch"):
    """Token ids [B, n+1] (column 0 = sos) for any batch size, decoded in engine-sized chunks."""
    images = _as_numpy(images)
    out = []
    for i in range(0, images.shape[0], model.max_batch):
        res = model.greedy(images[i:i + model.max_batch], max_steps=max_steps, stop=stop)
        out.append(res.ids)
    width = max(o.shape[1] for o in out)
    pad = [np.pad(o, ((0, 0), (0, width - o.shape[1])), constant_values=model.pad) for o in out]
    return np.concatenate(pad, axis=0)


def predict(images, model, vocab, idx2char, device=None, beam_size=3, max_steps: int = config.max_seq_len):
    ids = greedy_ids(model, images, max_steps=max_steps, stop="batch")
    return [detokenize(row, idx2char) for row in ids]
