"""ORACLE (test infrastructure only): CPU restatement of the ResNet18 + Transformer-encoder
model (``src/model_res18trans.py:13-106``, BASELINE config 5) and of torchvision
``resnet18`` (torchvision 0.21/0.22 ``models/resnet.py``: BasicBlock, eval BatchNorm),
which is not installed here.

``resnet18()`` keeps torchvision's module names (conv1, bn1, relu, maxpool, layer1..4,
avgpool, fc) so the reference's own glue (``list(resnet.children())[:-2]``) builds the
same ``encoder.features.*`` tree from it.  ``EncoderCNN.forward`` takes the positional
table that the reference draws inside every forward (``nn.Embedding(12, 256)``,
src/model_res18trans.py:57-59) as an explicit input; ``oracle/gen_golden.py`` pins this
restatement against the reference glue with the global RNG seeded so that both see
the same table.
"""
from __future__ import annotations

import torch
import torch.nn as nn

D_MODEL, N_HEADS, D_FF = 256, 8, 512
N_ENC, N_DEC, MAX_POS = 8, 8, 150


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class ResNet18(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(64, 2)
        self.layer2 = self._make_layer(128, 2, 2)
        self.layer3 = self._make_layer(256, 2, 2)
        self.layer4 = self._make_layer(512, 2, 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)

    def _make_layer(self, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, down)]
        self.inplanes = planes
        layers += [BasicBlock(planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(weights=None, **kw):
    return ResNet18(**kw)


class EncoderCNN(nn.Module):
    """src/model_res18trans.py:13-64 with the per-forward positional table as input."""

    def __init__(self):
        super().__init__()
        r = resnet18()
        r.conv1 = nn.Conv2d(1, 64, 7, 2, 3, bias=False)
        self.features = nn.Sequential(*list(r.children())[:-2])
        self.adaptive_pool = nn.AdaptiveAvgPool2d((1, None))
        self.projection = nn.Linear(512, D_MODEL)
        layer = nn.TransformerEncoderLayer(D_MODEL, N_HEADS, D_FF, 0.2, batch_first=True)
        self.transformer_encoder = nn.TransformerEncoder(layer, N_ENC)

    def forward(self, x, pos_table, stages=False):
        f = self.features(x)                                   # [B, 512, h, w]
        x = self.projection(self.adaptive_pool(f).permute(0, 3, 2, 1)).squeeze(2)  # [B, w, 256]
        x = x + pos_table[: x.size(1)].unsqueeze(0)
        # (w, B, d) with batch_first=True: attention runs across the images (:61-62)
        x = self.transformer_encoder(x.permute(1, 0, 2)).permute(1, 0, 2)
        return (x, f) if stages else x


class DecoderTransformer(nn.Module):
    """src/model_res18trans.py:67-98."""

    def __init__(self, vocab, max_pos=MAX_POS):
        super().__init__()
        self.embedding = nn.Embedding(vocab, D_MODEL)
        self.pos_encoder = nn.Embedding(max_pos, D_MODEL)
        layer = nn.TransformerDecoderLayer(D_MODEL, N_HEADS, D_FF, 0.2)
        self.transformer_decoder = nn.TransformerDecoder(layer, N_DEC)
        self.fc_out = nn.Linear(D_MODEL, vocab)
        self.register_buffer("tgt_mask", torch.triu(torch.ones(max_pos, max_pos) * float("-inf"), diagonal=1))

    def forward(self, encoder_out, tgt):
        e = self.embedding(tgt) + self.pos_encoder(torch.arange(tgt.size(1)).unsqueeze(0))
        out = self.transformer_decoder(e.permute(1, 0, 2), encoder_out.permute(1, 0, 2),
                                       tgt_mask=self.tgt_mask[: tgt.size(1), : tgt.size(1)])
        return self.fc_out(out.permute(1, 0, 2))


class Res18TransModel(nn.Module):
    def __init__(self, vocab, max_pos=MAX_POS):
        super().__init__()
        self.encoder = EncoderCNN()
        self.decoder = DecoderTransformer(vocab, max_pos)


def build_model(weights: dict) -> Res18TransModel:
    vocab = weights["decoder.fc_out.weight"].shape[0]
    max_pos = weights["decoder.pos_encoder.weight"].shape[0]
    m = Res18TransModel(vocab, max_pos)
    sd = {k: torch.from_numpy(v) for k, v in weights.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith("num_batches_tracked") or k == "decoder.tgt_mask" for k in missing), missing
    return m.eval()
