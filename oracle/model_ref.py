"""ORACLE (test infrastructure only): fp32 CPU restatement of the reference model and its greedy decodes.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this.  It is the checker, never the thing shipped or measured.

* ``EncoderSwin`` / ``DecoderTransformer`` / ``FormulaRecognitionModel`` follow
  ``src/model_swin.py:13-101`` (the serving copy ``app/src/model_swin.py`` differs
  only in the captions slice, :100).  The decoder uses ``torch.nn.TransformerDecoder``
  directly — the same third-party code the reference calls.
* ``greedy_decode`` follows ``src/inference.py:13-27``: encoder once, full-prefix
  re-decode every step (no KV cache), argmax of the last position, batch-global stop.
* ``serving_predict`` follows ``app/src/im2latex.py:15-55`` (batch 1, softmax,
  ``log(p + 1e-10)`` summed including the EOS step, confidence
  ``exp(sum / n_tokens_excluding_eos)``).
* ``detokenize`` follows ``src/inference.py:29-40``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
from torch.nn import TransformerDecoder, TransformerDecoderLayer

from .swin_ref import swin_t

D_MODEL, N_HEADS, D_FF, N_LAYERS, MAX_POS = 256, 8, 512, 8, 150


class EncoderSwin(nn.Module):
    """``src/model_swin.py:13-46``."""

    def __init__(self, d_model=D_MODEL):
        super().__init__()
        self.swin = swin_t()
        orig = self.swin.features[0][0]
        new = nn.Conv2d(1, orig.out_channels, kernel_size=orig.kernel_size, stride=orig.stride,
                        padding=orig.padding, bias=orig.bias is not None)
        with torch.no_grad():
            new.weight.copy_(torch.mean(orig.weight, dim=1, keepdim=True))
            new.bias.copy_(orig.bias)
        self.swin.features[0][0] = new
        self.features = self.swin.features
        self.projection = nn.Linear(768, d_model)

    def forward(self, x):
        x = self.features(x)
        b, h, w, c = x.shape
        return self.projection(x.view(b, h * w, c))


class DecoderTransformer(nn.Module):
    """``src/model_swin.py:49-88``."""

    def __init__(self, vocab, d_model=D_MODEL, nhead=N_HEADS, d_ff=D_FF, n_layers=N_LAYERS,
                 max_pos=MAX_POS):
        super().__init__()
        self.embedding = nn.Embedding(vocab, d_model)
        self.pos_encoder = nn.Embedding(max_pos, d_model)
        layer = TransformerDecoderLayer(d_model=d_model, nhead=nhead, dim_feedforward=d_ff, dropout=0.2)
        self.decoder = TransformerDecoder(layer, num_layers=n_layers)
        self.fc_out = nn.Linear(d_model, vocab)
        self.register_buffer("tgt_mask", torch.triu(torch.ones(max_pos, max_pos) * float("-inf"), diagonal=1))

    def forward(self, encoder_out, tgt):
        e = self.embedding(tgt)
        pos = torch.arange(0, tgt.size(1)).unsqueeze(0).to(tgt.device)
        e = e + self.pos_encoder(pos)
        out = self.decoder(e.permute(1, 0, 2), encoder_out.permute(1, 0, 2),
                           tgt_mask=self.tgt_mask[:tgt.size(1), :tgt.size(1)])
        return self.fc_out(out.permute(1, 0, 2))


class FormulaRecognitionModel(nn.Module):
    """``src/model_swin.py:91-101``."""

    def __init__(self, vocab, n_layers=N_LAYERS, max_pos=MAX_POS):
        super().__init__()
        self.encoder = EncoderSwin()
        self.decoder = DecoderTransformer(vocab, n_layers=n_layers, max_pos=max_pos)

    def forward(self, images, captions):
        return self.decoder(self.encoder(images), captions[:, :-1])


def build_model(weights: dict, vocab: int | None = None, n_layers: int = N_LAYERS) -> FormulaRecognitionModel:
    """Construct the oracle model and load ``synth.make_weights`` output (names of the
    ``encoder.features.*`` alias; the ``encoder.swin.features.*`` alias is the same
    Parameter objects, so loading one fills both)."""
    vocab = vocab or weights["decoder.fc_out.weight"].shape[0]
    max_pos = weights["decoder.pos_encoder.weight"].shape[0]
    m = FormulaRecognitionModel(vocab, n_layers=n_layers, max_pos=max_pos)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in weights.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    unexpected = [k for k in unexpected]
    assert not unexpected, unexpected
    # Whatever is missing must be an alias, an index buffer, the mask, or unused swin.norm/head.
    for k in missing:
        assert (k.startswith("encoder.swin.") or k.endswith("relative_position_index")
                or k == "decoder.tgt_mask"), k
    m.eval()
    return m


@torch.no_grad()
def encode(model, images: torch.Tensor, stages: bool = False):
    """Encoder output [B, M, 256]; with ``stages`` also the NHWC output of every features[i]."""
    if not stages:
        return model.encoder(images)
    outs = []
    x = images
    for f in model.encoder.features:
        x = f(x)
        outs.append(x)
    b, h, w, c = x.shape
    return model.encoder.projection(x.view(b, h * w, c)), outs


@torch.no_grad()
def greedy_decode(model, images=None, memory=None, max_steps: int = 150, sos=1, eos=2,
                  stop: str = "batch", record_logits: bool = False):
    """``src/inference.py:13-27``: returns (ys [B, n+1] int64, list of last-position logits).

    ``stop="batch"`` breaks once every row has produced EOS (the reference);
    ``stop="none"`` runs exactly ``max_steps`` steps.
    """
    if memory is None:
        memory = model.encoder(images)
    B = memory.shape[0]
    ys = torch.full((B, 1), sos, dtype=torch.long)
    finished = torch.zeros(B, dtype=torch.bool)
    logits = []
    for _ in range(max_steps):
        out = model.decoder(memory, ys)
        last = out[:, -1, :]
        if record_logits:
            logits.append(last.clone())
        nxt = last.argmax(dim=-1, keepdim=True)
        ys = torch.cat([ys, nxt], dim=1)
        finished |= nxt.squeeze(1) == eos
        if stop == "batch" and finished.all():
            break
    return ys, logits


@torch.no_grad()
def beam_search(model, images=None, memory=None, beam: int = 4, max_steps: int = 256, sos=1, eos=2, pad=0,
                stop: str = "batch"):
    """Beam search as this build specifies it.  The reference accepts
    ``beam_size`` (``src/inference.py:7``, ``src/config.py:50``) but never uses it, so no
    reference implementation exists: parity is unpinned by the reference, and this
    restatement is the specification ``mocr_decode_beam`` is tested against.

    - Per image, K = ``beam`` hypotheses, kept in rank order.  Score = sum over steps of
      log_softmax(last-position logits) of the chosen token (fp32), no length penalty.
    - Step 0 starts from one live hypothesis [sos] at score 0; the other K-1 start at -inf
      (so the first step does not pick K copies of the same token).
    - Every step, a live hypothesis k offers V candidates, score_k + logp_k[v], flat index
      k*V + v.  A finished hypothesis (it has emitted EOS) is retained: it offers exactly
      one candidate, itself extended by ``pad`` at unchanged score, flat index k*V.
    - The K best candidates of an image (higher score first, then lower flat index)
      become the new beam, in that order.
    - ``stop="batch"`` ends after the step at which every hypothesis of every image is
      finished; ``stop="none"`` runs exactly ``max_steps`` steps.

    Decoder rows are full-prefix recomputes exactly as ``greedy_decode`` (the reference
    loop, ``src/inference.py:13-27``).  Returns (seqs [B, K, n+1] int64, scores [B, K]
    float32, n_steps); seqs[:, 0] is the best hypothesis.
    """
    if memory is None:
        memory = model.encoder(images)
    B, K = memory.shape[0], beam
    mem = memory.repeat_interleave(K, dim=0)  # decoder row r = b*K + k reads image b
    seqs = torch.full((B * K, 1), sos, dtype=torch.long)
    scores = torch.full((B, K), float("-inf"))
    scores[:, 0] = 0.0
    fin = torch.zeros(B * K, dtype=torch.bool)
    n = 0
    for _ in range(max_steps):
        out = model.decoder(mem, seqs)
        logp = torch.log_softmax(out[:, -1, :], dim=-1)
        V = logp.shape[1]
        cand = scores.reshape(B * K, 1) + logp
        cand[fin] = float("-inf")
        cand[fin, 0] = scores.reshape(-1)[fin]
        cand = cand.reshape(B, K * V)
        order = torch.sort(-cand, dim=1, stable=True).indices[:, :K]  # ties: lower flat index
        new_scores = cand.gather(1, order)
        parent = (torch.arange(B).unsqueeze(1) * K + order // V).reshape(-1)
        tok = (order % V).reshape(-1)
        pfin = fin[parent]
        tok = torch.where(pfin, torch.full_like(tok, pad), tok)
        seqs = torch.cat([seqs[parent], tok.unsqueeze(1)], dim=1)
        fin = pfin | (tok == eos)
        scores = new_scores
        n += 1
        if stop == "batch" and bool(fin.all()):
            break
    return seqs.reshape(B, K, -1), scores, n


@torch.no_grad()
def teacher_forced_logits(model, memory, ys):
    """Last-position logits of every step when the decoder is fed ``ys[:, :t+1]``
    (one full-prefix pass; row t of the result is step t's logits)."""
    return model.decoder(memory, ys[:, :-1])


@torch.no_grad()
def serving_predict(model, image, max_steps=150, sos=1, eos=2):
    """``app/src/im2latex.py:15-55`` token loop: returns (tokens, log_probs_sum, confidence).

    The serving copy re-runs the whole model per step (:27); that is mathematically
    the same as encoding once, which is what is done here.
    """
    memory = model.encoder(image)
    target = torch.tensor([[sos]], dtype=torch.long)
    toks, lp_sum = [], 0.0
    for _ in range(max_steps):
        out = model.decoder(memory, target)
        logits = out[:, -1, :]
        probs = torch.softmax(logits, dim=-1)
        nxt = torch.argmax(probs, dim=-1)
        lp = torch.log(probs + 1e-10)[0, nxt.item()].item()
        lp_sum += lp
        if nxt.item() == eos:
            break
        toks.append(nxt.item())
        target = torch.cat([target, nxt.unsqueeze(-1)], dim=-1)
    if not toks:
        return toks, lp_sum, 0.0
    conf = torch.exp(torch.tensor(lp_sum / len(toks))).item()
    return toks, lp_sum, conf


def detokenize(seq, idx2char, sos="<sos>", eos="<eos>", pad="<pad>"):
    """``src/inference.py:29-40``."""
    toks = []
    for idx in seq:
        t = idx2char[int(idx)]
        if t in (sos, pad):
            continue
        if t == eos:
            break
        toks.append(t)
    return " ".join(toks)


def top2_margins(logits: torch.Tensor) -> np.ndarray:
    v = torch.topk(logits, 2, dim=-1).values
    return (v[..., 0] - v[..., 1]).numpy()


def count_params(model) -> int:
    return sum(p.numel() for p in model.parameters())


