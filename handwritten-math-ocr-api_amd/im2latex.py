"""Serving inference with the reference's call signatures (``app/src/im2latex.py``).

* ``load_model(model_path, vocab, device)`` -> an ``Engine`` holding the checkpoint's
  weights.  The reference unpickles a whole module with ``torch.load(weights_only=False)``
  (:7-13); here only state-dict checkpoints are read, with the safe loader
  (``weights.load_checkpoint``).
* ``predict(model, image_tensor, vocab, idx2char, device)`` -> ``(formula, confidence)``
  (:15-55): greedy decode of one image; per step the log of the softmax probability of
  the chosen token plus 1e-10 is summed, the EOS step included; tokens stop before EOS;
  confidence = exp(sum / number of tokens) in float32; an empty result returns the
  fixed message and 0.0; the token string goes through ``tokens_to_latex`` and
  ``clean_latex_output``.
* ``predict_batch(model, images, ...)``: the same per image, but all images decoded as
  one batch on the GPU (the reference's ``/predict/batch`` loops image by image,
  ``app/src/main.py:546-570``).  Each row's result uses only its steps up to its own
  first EOS, so it equals the single-image result.
"""
from __future__ import annotations

import numpy as np

from .config import config
from .utils import clean_latex_output, tokens_to_latex

EMPTY_MESSAGE = r"\text{Unable to detect a formula from the image. Please verify the model.}"


def load_model(model_path: str, vocab=None, device=None, max_batch: int = config.max_batch_images,
               precision: str = "bf16x3"):
    from .engine import Engine
    from .weights import load_checkpoint

    sd = load_checkpoint(model_path)
    n_vocab = len(vocab) if vocab is not None else None
    eng = Engine(img_hw=(config.img_h, config.img_w), vocab=n_vocab or int(sd["decoder.fc_out.weight"].shape[0]),
                 max_batch=max_batch, precision=precision, device=_device_index(device))
    eng.load_weights(sd)
    return eng


def _device_index(device) -> int:
    if device is None or device in ("cuda", "cpu"):
        return 0
    if isinstance(device, int):
        return device
    s = str(device)
    return int(s.split(":")[1]) if ":" in s else 0


def _row_result(ids_row, logp_row, n_steps, eos, idx2char):
    toks, lp_sum = [], 0.0
    for t in range(n_steps):
        tok = int(ids_row[t + 1])
        lp_sum += float(logp_row[t])
        if tok == eos:
            break
        toks.append(tok)
    if not toks:
        return EMPTY_MESSAGE, 0.0
    avg = lp_sum / len(toks)
    confidence = float(np.exp(np.float32(avg)))
    return clean_latex_output(tokens_to_latex(toks, idx2char)), confidence


def predict_batch(model, images, vocab, idx2char, device=None, max_steps: int = config.max_seq_len):
    if hasattr(images, "detach"):
        images = images.detach().cpu().numpy()
    images = np.ascontiguousarray(images, dtype=np.float32)
    eos = vocab.get(config.eos_token, model.eos) if vocab else model.eos
    results = []
    for i in range(0, images.shape[0], model.max_batch):
        model.encode(images[i:i + model.max_batch])
        res = model.decode(max_steps=max_steps, stop="batch", want_logp=True)
        for b in range(res.ids.shape[0]):
            results.append(_row_result(res.ids[b], res.logp[b], res.n_steps, eos, idx2char))
    return results


def predict(model, image_tensor, vocab, idx2char, device=None):
    return predict_batch(model, image_tensor, vocab, idx2char, device)[0]
