"""Image pre-processing of the serving path (``app/src/preprocess.py:6-17``).

The reference composes torchvision ``Grayscale(1) -> Resize((96, 320)) -> ToTensor ->
Normalize([0.5], [0.5])`` on a PIL image.  For PIL inputs torchvision delegates each
step to PIL / plain arithmetic: ``Grayscale`` is ``img.convert("L")``, ``Resize`` is
``img.resize((w, h), Image.BILINEAR)``, ``ToTensor`` divides the uint8 pixels by 255
and ``Normalize`` computes ``(x - 0.5) / 0.5``.  The same steps are done here without
torchvision, returning a float32 ``[1, 1, H, W]`` array in [-1, 1].
"""
from __future__ import annotations

import numpy as np

from .config import config


def preprocess_image(image, height: int = config.img_h, width: int = config.img_w) -> np.ndarray:
    from PIL import Image

    gray = image.convert("L")
    gray = gray.resize((width, height), Image.BILINEAR)
    x = np.asarray(gray, dtype=np.uint8).astype(np.float32) / np.float32(255.0)
    x = (x - np.float32(0.5)) / np.float32(0.5)
    return x[None, None, :, :].astype(np.float32)
