"""Weight blob packing and checkpoint loading.

The engine takes one flat float32 blob in ``synth.param_specs`` order.  A reference
training checkpoint (``src/utils.py:61-71``: ``{'model_state_dict': ...}``) stores every
encoder tensor twice — under ``encoder.swin.features.*`` and its alias
``encoder.features.*`` (``src/model_swin.py:35``) — plus the unused
``encoder.swin.norm`` / ``encoder.swin.head`` and the ``decoder.tgt_mask`` buffer.
``pack_state_dict`` accepts either alias, ignores the unused entries and checks
every shape.  Checkpoints are read with ``torch.load(weights_only=True)`` only: the
serving ``model.pth`` is a pickled module (``app/src/im2latex.py:11``) and is refused
rather than unpickled.
"""
from __future__ import annotations

import numpy as np

from . import synth


def _to_numpy(v):
    if hasattr(v, "detach"):
        v = v.detach().cpu().float().numpy()
    return np.asarray(v, dtype=np.float32)


def detect_arch(sd) -> str:
    """``res18trans`` for a src/model_res18trans.py state dict, else ``swin``."""
    return "res18trans" if any(k.startswith("encoder.transformer_encoder.") for k in sd) else "swin"


def pack_state_dict(sd, vocab=None, max_pos=None, n_layers=synth.N_LAYERS, arch=None) -> np.ndarray:
    if vocab is None:
        vocab = int(_to_numpy(sd["decoder.fc_out.weight"]).shape[0])
    if max_pos is None:
        max_pos = int(_to_numpy(sd["decoder.pos_encoder.weight"]).shape[0])
    arch = arch or detect_arch(sd)
    specs = synth.param_specs(vocab, max_pos, n_layers) if arch == "swin" else synth.param_specs_res18(vocab, max_pos)
    parts = []
    for name, shape, _, _ in specs:
        key = name
        if key not in sd and name.startswith("encoder.features."):
            key = "encoder.swin." + name[len("encoder."):]
        if key not in sd:
            raise KeyError(f"state dict has no {name!r}")
        a = _to_numpy(sd[key])
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(a.shape)} != expected {tuple(shape)}")
        parts.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts), dtype=np.float32)


def load_checkpoint(path: str):
    """Return the state dict of a reference checkpoint file (safe loader only)."""
    import torch
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict) and "model_state_dict" in obj:
        obj = obj["model_state_dict"]
    if not isinstance(obj, dict):
        raise ValueError(f"{path}: not a state dict / training checkpoint")
    return obj
