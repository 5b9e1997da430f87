"""Seeded synthetic weights and images for the Swin-T + 8-layer decoder hot path.

There are no checkpoints and no network, so both the engine and the CPU oracle
regenerate the same 37 M parameters from a seed.  Every tensor
is drawn with numpy ``PCG64`` in a fixed order, using the initialisation the
reference model gets at construction time:

* torchvision Swin ``Linear``: trunc-normal(σ=0.02, a=-2, b=2), bias 0
  (torchvision ``SwinTransformer.__init__`` init loop; the 1-channel stem and the
  projection are replaced in ``src/model_swin.py:19-37``);
* relative-position tables: trunc-normal(σ=0.02);
* LayerNorm: weight 1, bias 0;
* stem ``Conv2d(1,96,4,4)``: kaiming-uniform(a=√5) drawn for 3 input channels and
  averaged over them (``src/model_swin.py:29-32``); bias U(±1/√48);
* ``projection`` / ``linear1`` / ``linear2`` / ``fc_out`` / ``out_proj``:
  torch ``Linear`` default (kaiming-uniform a=√5 → U(±1/√fan_in), bias U(±1/√fan_in));
  MHA ``out_proj.bias`` and ``in_proj_bias`` are 0, ``in_proj_weight`` xavier-uniform
  (``torch/nn/modules/activation.py`` ``_reset_parameters``);
* ``Embedding``: N(0, 1).

``variant="init"`` reproduces those distributions.  ``variant="perturbed"`` also
gives every bias and LayerNorm affine parameter a non-trivial value, so that a
kernel that drops a bias (e.g. the padded-window keys, whose k/v equal the qkv
bias) cannot pass parity by accident.  ``tied=True`` makes the 8 decoder layers
identical, as ``nn.TransformerDecoder``'s deep-copied clones are at
construction (``torch/nn/modules/transformer.py`` ``_get_clones``).

Key names follow the reference ``FormulaRecognitionModel.state_dict()`` with the
``encoder.features.*`` alias.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

# Reference model constants (src/config.py:17-47, app/src/config.py:22-54).
D_MODEL = 256
N_HEADS = 8
D_FF = 512
N_LAYERS = 8
MAX_POS = 150
VOCAB = 5075
PAD_ID, SOS_ID, EOS_ID, UNK_ID = 0, 1, 2, 3

# torchvision swin_t (Appendix A).
EMBED_DIM = 96
DEPTHS = (2, 2, 6, 2)
HEADS = (3, 6, 12, 24)
WINDOW = 7
ENC_DIM = 768


def _trunc_normal(rng, shape, std=0.02, a=-2.0, b=2.0):
    x = rng.standard_normal(size=shape) * std
    bad = (x < a) | (x > b)
    while bad.any():
        x[bad] = rng.standard_normal(size=int(bad.sum())) * std
        bad = (x < a) | (x > b)
    return x


def _uniform(rng, shape, bound):
    return rng.uniform(-bound, bound, size=shape)


def decoder_specs(vocab: int, max_pos: int, n_layers: int, d_model: int = D_MODEL, d_ff: int = D_FF,
                  stack: str = "decoder.decoder.layers"):
    """The decoder's tensors (shared by both encoder variants; only the layer-stack
    name differs: ``decoder.decoder`` in src/model_swin.py:64, ``decoder.transformer_decoder``
    in src/model_res18trans.py:79)."""
    specs = []
    add = specs.append
    add(("decoder.embedding.weight", (vocab, d_model), "emb", 0))
    add(("decoder.pos_encoder.weight", (max_pos, d_model), "emb", 0))
    for l in range(n_layers):
        p = f"{stack}.{l}."
        for att in ("self_attn", "multihead_attn"):
            add((p + att + ".in_proj_weight", (3 * d_model, d_model), "xavier", 0))
            add((p + att + ".in_proj_bias", (3 * d_model,), "zero_b", 0))
            add((p + att + ".out_proj.weight", (d_model, d_model), "lin_w", d_model))
            add((p + att + ".out_proj.bias", (d_model,), "zero_b", 0))
        add((p + "linear1.weight", (d_ff, d_model), "lin_w", d_model))
        add((p + "linear1.bias", (d_ff,), "lin_b", d_model))
        add((p + "linear2.weight", (d_model, d_ff), "lin_w", d_ff))
        add((p + "linear2.bias", (d_model,), "lin_b", d_ff))
        for n in (1, 2, 3):
            add((p + f"norm{n}.weight", (d_model,), "ln_w", 0))
            add((p + f"norm{n}.bias", (d_model,), "ln_b", 0))
    add(("decoder.fc_out.weight", (vocab, d_model), "lin_w", d_model))
    add(("decoder.fc_out.bias", (vocab,), "lin_b", d_model))
    return specs


def param_specs(vocab: int = VOCAB, max_pos: int = MAX_POS, n_layers: int = N_LAYERS,
                d_model: int = D_MODEL, d_ff: int = D_FF):
    """Ordered (name, shape, init-kind, fan_in) for every tensor the hot path uses.

    The order is the engine's weight-blob order (include/mathocr.h).
    """
    specs = []
    add = specs.append
    add(("encoder.features.0.0.weight", (EMBED_DIM, 1, 4, 4), "stem_w", 48))
    add(("encoder.features.0.0.bias", (EMBED_DIM,), "stem_b", 48))
    add(("encoder.features.0.2.weight", (EMBED_DIM,), "ln_w", 0))
    add(("encoder.features.0.2.bias", (EMBED_DIM,), "ln_b", 0))
    dim = EMBED_DIM
    for s in range(4):
        fi = 1 + 2 * s
        h = HEADS[s]
        for j in range(DEPTHS[s]):
            p = f"encoder.features.{fi}.{j}."
            add((p + "norm1.weight", (dim,), "ln_w", 0))
            add((p + "norm1.bias", (dim,), "ln_b", 0))
            add((p + "attn.qkv.weight", (3 * dim, dim), "swin_w", 0))
            add((p + "attn.qkv.bias", (3 * dim,), "swin_b", 0))
            add((p + "attn.proj.weight", (dim, dim), "swin_w", 0))
            add((p + "attn.proj.bias", (dim,), "swin_b", 0))
            add((p + "attn.relative_position_bias_table", ((2 * WINDOW - 1) ** 2, h), "swin_table", 0))
            add((p + "norm2.weight", (dim,), "ln_w", 0))
            add((p + "norm2.bias", (dim,), "ln_b", 0))
            add((p + "mlp.0.weight", (4 * dim, dim), "swin_w", 0))
            add((p + "mlp.0.bias", (4 * dim,), "swin_b", 0))
            add((p + "mlp.3.weight", (dim, 4 * dim), "swin_w", 0))
            add((p + "mlp.3.bias", (dim,), "swin_b", 0))
        if s < 3:
            p = f"encoder.features.{fi + 1}."
            add((p + "norm.weight", (4 * dim,), "ln_w", 0))
            add((p + "norm.bias", (4 * dim,), "ln_b", 0))
            add((p + "reduction.weight", (2 * dim, 4 * dim), "swin_w", 0))
            dim *= 2
    add(("encoder.projection.weight", (d_model, ENC_DIM), "lin_w", ENC_DIM))
    add(("encoder.projection.bias", (d_model,), "lin_b", ENC_DIM))
    specs += decoder_specs(vocab, max_pos, n_layers, d_model, d_ff)
    return specs


def make_weights(seed: int = 1234, variant: str = "init", tied: bool = False,
                 vocab: int = VOCAB, max_pos: int = MAX_POS, n_layers: int = N_LAYERS, arch: str = "swin"):
    """Return an OrderedDict name -> float32 ndarray (blob order)."""
    if variant not in ("init", "perturbed"):
        raise ValueError(f"unknown variant {variant!r}")
    pert = variant == "perturbed"
    rng = np.random.Generator(np.random.PCG64(seed))
    out = OrderedDict()
    first_layer = {}
    if arch == "swin":
        specs = param_specs(vocab, max_pos, n_layers)
    elif arch == "res18trans":
        specs = param_specs_res18(vocab, max_pos)
    else:
        raise ValueError(f"unknown arch {arch!r}")
    for name, shape, kind, fan_in in specs:
        if tied and name.startswith("decoder.decoder.layers.") and not name.startswith("decoder.decoder.layers.0."):
            suffix = name.split(".", 4)[4]
            out[name] = first_layer[suffix].copy()
            continue
        if kind == "stem_w":
            # kaiming_uniform(a=sqrt(5)) on the RGB kernel [96,3,4,4]: bound = 1/sqrt(fan_in=48)
            w3 = _uniform(rng, (shape[0], 3) + shape[2:], 1.0 / math.sqrt(48))
            a = w3.mean(axis=1, keepdims=True)
        elif kind == "stem_b":
            a = _uniform(rng, shape, 1.0 / math.sqrt(fan_in))
        elif kind == "ln_w":
            a = np.ones(shape) + (0.1 * rng.standard_normal(shape) if pert else 0.0)
        elif kind == "ln_b":
            a = 0.05 * rng.standard_normal(shape) if pert else np.zeros(shape)
        elif kind in ("swin_w", "swin_table"):
            a = _trunc_normal(rng, shape, 0.02)
        elif kind == "swin_b":
            a = 0.02 * rng.standard_normal(shape) if pert else np.zeros(shape)
        elif kind == "lin_w":
            a = _uniform(rng, shape, 1.0 / math.sqrt(fan_in))
        elif kind == "lin_b":
            a = _uniform(rng, shape, 1.0 / math.sqrt(fan_in))
        elif kind == "xavier":
            fan_out, fin = shape
            a = _uniform(rng, shape, math.sqrt(6.0 / (fin + fan_out)))
        elif kind == "zero_b":
            a = _uniform(rng, shape, 0.05) if pert else np.zeros(shape)
        elif kind == "emb":
            a = rng.standard_normal(shape)
        elif kind == "res_conv":
            # torchvision ResNet: kaiming_normal_(mode="fan_out", nonlinearity="relu")
            a = rng.standard_normal(shape) * math.sqrt(2.0 / (shape[0] * shape[2] * shape[3]))
        elif kind == "res_conv1":
            # the 3-channel conv1 [64,3,7,7] averaged over RGB (src/model_res18trans.py:28-30)
            w3 = rng.standard_normal((shape[0], 3) + shape[2:]) * math.sqrt(2.0 / (shape[0] * 49))
            a = w3.mean(axis=1, keepdims=True)
        elif kind == "bn_w":
            a = np.ones(shape) + (0.1 * rng.standard_normal(shape) if pert else 0.0)
        elif kind == "bn_b":
            a = 0.05 * rng.standard_normal(shape) if pert else np.zeros(shape)
        elif kind == "bn_mean":
            a = 0.1 * rng.standard_normal(shape) if pert else np.zeros(shape)
        elif kind == "bn_var":
            a = rng.uniform(0.5, 1.5, size=shape) if pert else np.ones(shape)
        else:  # pragma: no cover
            raise AssertionError(kind)
        a = np.ascontiguousarray(a, dtype=np.float32)
        out[name] = a
        if tied and name.startswith("decoder.decoder.layers.0."):
            first_layer[name.split(".", 4)[4]] = a
    return out


def make_images(batch: int, height: int = 384, width: int = 384, seed0: int = 1000,
                kind: str = "uniform"):
    """[B,1,H,W] float32 images; image i is drawn from PCG64(seed0 + i).

    ``uniform``: U(-1, 1).  ``ink``: white (+1) background with
    dark (-1) random strokes, closer to a normalised handwriting scan.
    """
    imgs = np.empty((batch, 1, height, width), dtype=np.float32)
    for i in range(batch):
        rng = np.random.Generator(np.random.PCG64(seed0 + i))
        if kind == "uniform":
            imgs[i, 0] = rng.uniform(-1.0, 1.0, size=(height, width)).astype(np.float32)
        elif kind == "ink":
            im = np.ones((height, width), dtype=np.float32)
            for _ in range(12):
                y, x = rng.uniform(0, height), rng.uniform(0, width)
                dy, dx = rng.normal(0, 1, 2)
                n = int(rng.integers(20, 120))
                for _ in range(n):
                    y = min(max(y + dy + rng.normal(0, 0.5), 0), height - 1)
                    x = min(max(x + dx + rng.normal(0, 0.5), 0), width - 1)
                    im[int(y), int(x)] = -1.0
                    if int(y) + 1 < height:
                        im[int(y) + 1, int(x)] = -1.0
            imgs[i, 0] = im
        else:
            raise ValueError(kind)
    return imgs


def synthetic_vocab(vocab: int = VOCAB):
    """vocab (str->id) and idx2char (id->str) in the reference's vocab.json shape.

    Special tokens first (``src/utils.py:111``: pad/sos/eos/unk = 0/1/2/3), then
    distinct printable pseudo-LaTeX tokens.
    """
    toks = ["<pad>", "<sos>", "<eos>", "<unk>"]
    base = ["\\frac", "\\sqrt", "\\alpha", "\\beta", "\\sum", "\\int", "{", "}", "_", "^",
            "x", "y", "z", "+", "-", "=", "(", ")", "\\begin", "\\end", "matrix", "\\\\", "&"]
    toks += base
    i = 0
    while len(toks) < vocab:
        toks.append(f"\\tok{i}")
        i += 1
    toks = toks[:vocab]
    v = {t: k for k, t in enumerate(toks)}
    return v, {k: t for t, k in v.items()}


# ResNet18 + Transformer-encoder variant (src/model_res18trans.py:13-64, BASELINE config 5).
RES_CH = (64, 128, 256, 512)
RES_ENC_LAYERS = 8   # src/config.py:28
RES_DEC_LAYERS = 8   # src/config.py:29


def param_specs_res18(vocab: int = VOCAB, max_pos: int = MAX_POS, n_enc: int = RES_ENC_LAYERS,
                      n_dec: int = RES_DEC_LAYERS, d_model: int = D_MODEL, d_ff: int = D_FF):
    """Blob order of the ResNet18-trans model: ``encoder.features`` = torchvision
    resnet18 children [conv1, bn1, relu, maxpool, layer1..4] (indices 0..7), the
    projection, the 8 post-norm ``TransformerEncoderLayer`` (batch_first), then the
    decoder.  BatchNorm running statistics are part of the blob (eval BN)."""
    specs = []
    add = specs.append

    def bn(p, c):
        add((p + ".weight", (c,), "bn_w", 0))
        add((p + ".bias", (c,), "bn_b", 0))
        add((p + ".running_mean", (c,), "bn_mean", 0))
        add((p + ".running_var", (c,), "bn_var", 0))

    add(("encoder.features.0.weight", (64, 1, 7, 7), "res_conv1", 0))
    bn("encoder.features.1", 64)
    cin = 64
    for li, c in enumerate(RES_CH):
        for blk in range(2):
            p = f"encoder.features.{4 + li}.{blk}."
            stride = 2 if (li > 0 and blk == 0) else 1
            add((p + "conv1.weight", (c, cin if blk == 0 else c, 3, 3), "res_conv", 0))
            bn(p + "bn1", c)
            add((p + "conv2.weight", (c, c, 3, 3), "res_conv", 0))
            bn(p + "bn2", c)
            if blk == 0 and (stride != 1 or cin != c):
                add((p + "downsample.0.weight", (c, cin, 1, 1), "res_conv", 0))
                bn(p + "downsample.1", c)
        cin = c
    add(("encoder.projection.weight", (d_model, 512), "lin_w", 512))
    add(("encoder.projection.bias", (d_model,), "lin_b", 512))
    for l in range(n_enc):
        p = f"encoder.transformer_encoder.layers.{l}."
        add((p + "self_attn.in_proj_weight", (3 * d_model, d_model), "xavier", 0))
        add((p + "self_attn.in_proj_bias", (3 * d_model,), "zero_b", 0))
        add((p + "self_attn.out_proj.weight", (d_model, d_model), "lin_w", d_model))
        add((p + "self_attn.out_proj.bias", (d_model,), "zero_b", 0))
        add((p + "linear1.weight", (d_ff, d_model), "lin_w", d_model))
        add((p + "linear1.bias", (d_ff,), "lin_b", d_model))
        add((p + "linear2.weight", (d_model, d_ff), "lin_w", d_ff))
        add((p + "linear2.bias", (d_model,), "lin_b", d_ff))
        for n in (1, 2):
            add((p + f"norm{n}.weight", (d_model,), "ln_w", 0))
            add((p + f"norm{n}.bias", (d_model,), "ln_b", 0))
    specs += decoder_specs(vocab, max_pos, n_dec, d_model, d_ff, stack="decoder.transformer_decoder.layers")
    return specs


def make_pos_table(seed: int, tokens: int = 12, d_model: int = D_MODEL):
    """The per-forward positional table of the ResNet18-trans encoder
    (src/model_res18trans.py:57-59 draws ``nn.Embedding(tokens, d_model)``, i.e. N(0,1),
    from torch's global RNG inside every forward).  The engine takes it as an input;
    this is the table torch draws right after ``torch.manual_seed(seed)``."""
    import torch
    g = torch.Generator().manual_seed(seed)
    return torch.randn(tokens, d_model, generator=g).numpy().astype(np.float32)
