"""ORACLE (test infrastructure only): CPU fp32 restatement of torchvision ``swin_t().features``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package.  The product path (``handwritten-math-ocr-api_amd``) never
does.

The reference calls ``torchvision.models.swin_t(weights=Swin_T_Weights.DEFAULT)``
(``src/model_swin.py:17``) and keeps only ``.features`` (``:35,40``).  torchvision
0.21/0.22 (pinned in ``requirements.txt:2`` / ``app/requirements.txt:3``) is not
installed in this image, so this file restates its published algorithm
 with the same module tree and ``state_dict`` key names:

* ``features[0]`` = Conv2d(3→96, k4, s4) → Permute(NCHW→NHWC) → LayerNorm(96)
* ``features[1,3,5,7]`` = stages of (2, 2, 6, 2) ``SwinTransformerBlock`` (v1),
  heads (3, 6, 12, 24), window 7, shift 3 on odd blocks
* ``features[2,4,6]`` = ``PatchMerging``
* eval mode: stochastic depth and dropout are identity.

Parity of this restatement is pinned against HF ``SwinModel`` at 384×384
(``oracle/hf_crosscheck.py``).  The 96×320 padded/shift-disabled corner cases are
not covered by any installed implementation ("parity unpinned" for those, see
DESIGN.md §4) and follow torchvision's ``shifted_window_attention`` exactly.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

WINDOW = 7


class Permute(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.dims = dims

    def forward(self, x):
        return torch.permute(x, self.dims)


def relative_position_index(window: int = WINDOW) -> torch.Tensor:
    """torchvision ``ShiftedWindowAttention.define_relative_position_index``."""
    coords = torch.stack(torch.meshgrid(torch.arange(window), torch.arange(window), indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += window - 1
    rel[:, :, 1] += window - 1
    rel[:, :, 0] *= 2 * window - 1
    return rel.sum(-1).flatten()


def shift_region_ids(pad_h: int, pad_w: int, sh: int, sw: int, window: int = WINDOW) -> torch.Tensor:
    """The ``attn_mask`` region map of torchvision's ``shifted_window_attention``.

    Built with the same nine slice assignments, including the python-slice
    behaviour for a zero shift on one axis (``(-0, None)`` covers the whole axis,
    so the last assignment along that axis wins).
    """
    m = torch.zeros((pad_h, pad_w))
    h_slices = ((0, -window), (-window, -sh), (-sh, None))
    w_slices = ((0, -window), (-window, -sw), (-sw, None))
    count = 0
    for h in h_slices:
        for w in w_slices:
            m[h[0]:h[1], w[0]:w[1]] = count
            count += 1
    return m


def shifted_window_attention(x, qkv_weight, proj_weight, rel_bias, num_heads, shift,
                             qkv_bias, proj_bias, window: int = WINDOW):
    """torchvision ``shifted_window_attention`` (v1, eval mode)."""
    B, H, W, C = x.shape
    pad_r = (window - W % window) % window
    pad_b = (window - H % window) % window
    x = F.pad(x, (0, 0, 0, pad_r, 0, pad_b))
    _, pH, pW, _ = x.shape
    sh, sw = shift, shift
    if window >= pH:
        sh = 0
    if window >= pW:
        sw = 0
    if sh + sw > 0:
        x = torch.roll(x, shifts=(-sh, -sw), dims=(1, 2))
    nW = (pH // window) * (pW // window)
    x = x.view(B, pH // window, window, pW // window, window, C)
    x = x.permute(0, 1, 3, 2, 4, 5).reshape(B * nW, window * window, C)
    qkv = F.linear(x, qkv_weight, qkv_bias)
    qkv = qkv.reshape(x.size(0), x.size(1), 3, num_heads, C // num_heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * (C // num_heads) ** -0.5
    attn = q.matmul(k.transpose(-2, -1))
    attn = attn + rel_bias
    if sh + sw > 0:
        m = shift_region_ids(pH, pW, sh, sw, window)
        m = m.view(pH // window, window, pW // window, window).permute(0, 2, 1, 3).reshape(nW, window * window)
        m = m.unsqueeze(1) - m.unsqueeze(2)
        m = m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)
        attn = attn.view(x.size(0) // nW, nW, num_heads, x.size(1), x.size(1))
        attn = attn + m.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, num_heads, x.size(1), x.size(1))
    attn = F.softmax(attn, dim=-1)
    x = attn.matmul(v).transpose(1, 2).reshape(x.size(0), x.size(1), C)
    x = F.linear(x, proj_weight, proj_bias)
    x = x.view(B, pH // window, pW // window, window, window, C)
    x = x.permute(0, 1, 3, 2, 4, 5).reshape(B, pH, pW, C)
    if sh + sw > 0:
        x = torch.roll(x, shifts=(sh, sw), dims=(1, 2))
    return x[:, :H, :W, :].contiguous()


class ShiftedWindowAttention(nn.Module):
    def __init__(self, dim, window, shift, num_heads):
        super().__init__()
        self.window = window
        self.shift = shift
        self.num_heads = num_heads
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * window - 1) ** 2, num_heads))
        self.register_buffer("relative_position_index", relative_position_index(window))

    def rel_bias(self):
        n = self.window * self.window
        b = self.relative_position_bias_table[self.relative_position_index].view(n, n, -1)
        return b.permute(2, 0, 1).contiguous().unsqueeze(0)

    def forward(self, x):
        return shifted_window_attention(x, self.qkv.weight, self.proj.weight, self.rel_bias(),
                                        self.num_heads, self.shift, self.qkv.bias, self.proj.bias,
                                        self.window)


class MLP(nn.Sequential):
    """torchvision.ops.MLP(dim, [4dim, dim], GELU, dropout): indices 0 and 3 are the Linears."""

    def __init__(self, dim, hidden):
        super().__init__(nn.Linear(dim, hidden), nn.GELU(), nn.Dropout(0.0), nn.Linear(hidden, dim),
                         nn.Dropout(0.0))


class SwinTransformerBlock(nn.Module):
    def __init__(self, dim, num_heads, shift):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-5)
        self.attn = ShiftedWindowAttention(dim, WINDOW, shift, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-5)
        self.mlp = MLP(dim, 4 * dim)

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        x = x + self.mlp(self.norm2(x))
        return x


def patch_merging_pad(x):
    H, W, _ = x.shape[-3:]
    x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2))
    x0 = x[..., 0::2, 0::2, :]
    x1 = x[..., 1::2, 0::2, :]
    x2 = x[..., 0::2, 1::2, :]
    x3 = x[..., 1::2, 1::2, :]
    return torch.cat([x0, x1, x2, x3], -1)


class PatchMerging(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(4 * dim, eps=1e-5)

    def forward(self, x):
        return self.reduction(self.norm(patch_merging_pad(x)))


class SwinT(nn.Module):
    """``torchvision.models.swin_t`` module tree (features + unused norm/head)."""

    def __init__(self, in_chans=3, embed_dim=96, depths=(2, 2, 6, 2), heads=(3, 6, 12, 24),
                 num_classes=1000):
        super().__init__()
        layers = [nn.Sequential(nn.Conv2d(in_chans, embed_dim, kernel_size=4, stride=4),
                                Permute([0, 2, 3, 1]), nn.LayerNorm(embed_dim, eps=1e-5))]
        dim = embed_dim
        for s, depth in enumerate(depths):
            layers.append(nn.Sequential(*[SwinTransformerBlock(dim, heads[s], 0 if j % 2 == 0 else WINDOW // 2)
                                          for j in range(depth)]))
            if s < len(depths) - 1:
                layers.append(PatchMerging(dim))
                dim *= 2
        self.features = nn.Sequential(*layers)
        self.norm = nn.LayerNorm(dim, eps=1e-5)
        self.permute = Permute([0, 3, 1, 2])
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.flatten = nn.Flatten(1)
        self.head = nn.Linear(dim, num_classes)

    def forward(self, x):
        x = self.norm(self.features(x))
        return self.head(self.flatten(self.avgpool(self.permute(x))))


def swin_t(weights=None, progress=True, **kwargs):
    """Signature-compatible stand-in for ``torchvision.models.swin_t`` (random init only)."""
    if weights is not None:
        raise RuntimeError("pretrained weights are not available offline")
    return SwinT(**kwargs)
