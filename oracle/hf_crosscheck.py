"""ORACLE (test infrastructure only): pin ``swin_ref`` against an independent Swin.

torchvision is not installed, so the Swin restatement is checked against
HuggingFace ``transformers`` ``SwinModel`` (``transformers/models/swin/modeling_swin.py``),
which implements the same v1 Swin and matches torchvision semantics whenever every
stage map is larger than the 7×7 window (true at 384×384; HF clamps the window
instead of padding below that, ``modeling_swin.py:576-582``).  The final
``layernorm`` is bypassed because the reference skips ``swin.norm``
(``src/model_swin.py:39-46``).  HF scales q·kᵀ after the matmul and torchvision
before it, so agreement is to fp32 rounding, not bitwise.
"""
from __future__ import annotations

import numpy as np
import torch

from .swin_ref import SwinT


def hf_swin_from_weights(weights: dict, image_hw=(384, 384)):
    from transformers import SwinConfig, SwinModel

    cfg = SwinConfig(image_size=list(image_hw), patch_size=4, num_channels=1, embed_dim=96,
                     depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=7, mlp_ratio=4.0,
                     qkv_bias=True, hidden_act="gelu", layer_norm_eps=1e-5, drop_path_rate=0.0,
                     hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                     use_absolute_embeddings=False)
    m = SwinModel(cfg, add_pooling_layer=False)
    m.layernorm = torch.nn.Identity()
    t = lambda k: torch.from_numpy(np.asarray(weights[k]))  # noqa: E731
    sd = {
        "embeddings.patch_embeddings.projection.weight": t("encoder.features.0.0.weight"),
        "embeddings.patch_embeddings.projection.bias": t("encoder.features.0.0.bias"),
        "embeddings.norm.weight": t("encoder.features.0.2.weight"),
        "embeddings.norm.bias": t("encoder.features.0.2.bias"),
    }
    dim = 96
    for s, depth in enumerate((2, 2, 6, 2)):
        for j in range(depth):
            src = f"encoder.features.{1 + 2 * s}.{j}."
            dst = f"encoder.layers.{s}.blocks.{j}."
            qw, kw, vw = t(src + "attn.qkv.weight").split(dim, 0)
            qb, kb, vb = t(src + "attn.qkv.bias").split(dim, 0)
            sd.update({
                dst + "layernorm_before.weight": t(src + "norm1.weight"),
                dst + "layernorm_before.bias": t(src + "norm1.bias"),
                dst + "attention.q_proj.weight": qw, dst + "attention.q_proj.bias": qb,
                dst + "attention.k_proj.weight": kw, dst + "attention.k_proj.bias": kb,
                dst + "attention.v_proj.weight": vw, dst + "attention.v_proj.bias": vb,
                dst + "attention.o_proj.weight": t(src + "attn.proj.weight"),
                dst + "attention.o_proj.bias": t(src + "attn.proj.bias"),
                dst + "attention.relative_position_bias.relative_position_bias_table":
                    t(src + "attn.relative_position_bias_table"),
                dst + "layernorm_after.weight": t(src + "norm2.weight"),
                dst + "layernorm_after.bias": t(src + "norm2.bias"),
                dst + "mlp.fc1.weight": t(src + "mlp.0.weight"), dst + "mlp.fc1.bias": t(src + "mlp.0.bias"),
                dst + "mlp.fc2.weight": t(src + "mlp.3.weight"), dst + "mlp.fc2.bias": t(src + "mlp.3.bias"),
            })
        if s < 3:
            src = f"encoder.features.{2 + 2 * s}."
            dst = f"encoder.layers.{s}.downsample."
            sd.update({dst + "norm.weight": t(src + "norm.weight"), dst + "norm.bias": t(src + "norm.bias"),
                       dst + "reduction.weight": t(src + "reduction.weight")})
            dim *= 2
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("relative_position_index" in k or k.startswith("layernorm") for k in missing), missing
    return m.eval()


def restated_swin_from_weights(weights: dict) -> SwinT:
    m = SwinT(in_chans=1)
    sd = {k[len("encoder."):]: torch.from_numpy(np.asarray(v)) for k, v in weights.items()
          if k.startswith("encoder.features.")}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    return m.eval()


@torch.no_grad()
def crosscheck(weights: dict, images: np.ndarray):
    """Return (max |Δ|, max |ref|) between the restated features and HF's."""
    x = torch.from_numpy(images)
    ours = restated_swin_from_weights(weights).features(x)
    b, h, w, c = ours.shape
    theirs = hf_swin_from_weights(weights, images.shape[-2:])(x).last_hidden_state
    return float((ours.view(b, h * w, c) - theirs).abs().max()), float(theirs.abs().max())


# ------------------------------------------------------------------ ResNet18 (BASELINE config 5)
def hf_resnet18_from_weights(weights: dict):
    """HF ``ResNetModel`` (``transformers/models/resnet/modeling_resnet.py``: BasicLayer,
    shortcut conv1x1 + BN where the shape changes, no downsampling in stage 1) configured as
    torchvision ``resnet18`` with a 1-channel stem, loaded with the same weights as
    ``res18_ref``'s ``encoder.features.*`` (torchvision names)."""
    from transformers import ResNetConfig, ResNetModel

    cfg = ResNetConfig(num_channels=1, embedding_size=64, hidden_sizes=[64, 128, 256, 512], depths=[2, 2, 2, 2],
                       layer_type="basic", hidden_act="relu", downsample_in_first_stage=False)
    m = ResNetModel(cfg)
    t = lambda k: torch.from_numpy(np.asarray(weights[k]))  # noqa: E731

    def conv_bn(dst, conv, bn):
        return {dst + "convolution.weight": t(conv + ".weight"), dst + "normalization.weight": t(bn + ".weight"),
                dst + "normalization.bias": t(bn + ".bias"), dst + "normalization.running_mean": t(bn + ".running_mean"),
                dst + "normalization.running_var": t(bn + ".running_var")}

    f = "encoder.features."
    sd = conv_bn("embedder.embedder.", f + "0", f + "1")  # features = conv1, bn1, relu, maxpool, layer1..4
    for s in range(4):
        for j in range(2):
            src = f"{f}{4 + s}.{j}."
            dst = f"encoder.stages.{s}.layers.{j}."
            sd.update(conv_bn(dst + "layer.0.", src + "conv1", src + "bn1"))
            sd.update(conv_bn(dst + "layer.1.", src + "conv2", src + "bn2"))
            if src + "downsample.0.weight" in weights:
                sd.update(conv_bn(dst + "shortcut.", src + "downsample.0", src + "downsample.1"))
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith("num_batches_tracked") for k in missing), missing
    return m.eval()


@torch.no_grad()
def crosscheck_resnet18(weights: dict, images: np.ndarray):
    """Return (max |Δ|, max |ref|) between ``res18_ref``'s backbone map [B, 512, h, w] (the
    restated torchvision resnet18 without avgpool / fc, src/model_res18trans.py:16-32) and
    HF's ``last_hidden_state``."""
    from . import res18_ref
    x = torch.from_numpy(images)
    ours = res18_ref.build_model(weights).encoder.features(x)
    theirs = hf_resnet18_from_weights(weights)(x).last_hidden_state
    assert ours.shape == theirs.shape, (ours.shape, theirs.shape)
    return float((ours - theirs).abs().max()), float(theirs.abs().max())
