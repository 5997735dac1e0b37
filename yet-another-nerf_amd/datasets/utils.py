"""Image loading and resizing shared by the loaders."""
from __future__ import annotations

from pathlib import Path
from typing import Union

import numpy as np
import torch


def load_image(path: Union[str, Path]) -> np.ndarray:
    """RGB float32 in [0, 1], HxWx3 (reference dataset/utils.py:8-11). PIL's convert("RGB") drops an alpha channel
    without compositing it over a background, as the reference does (Blender PNGs are RGBA)."""
    from PIL import Image
    with Image.open(path) as im:
        arr = np.array(im.convert("RGB"))
    return arr.astype(np.float32) / 255.0


def resize_linear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """Bilinear resize with half-pixel centres and no anti-aliasing: the sampling of cv2.resize(INTER_LINEAR) used
    by the reference for `scale_down` (blender_dataset.py:69), computed with torch (cv2 is not a dependency here).
    Parity with cv2 itself is unpinned (no cv2 in this environment); the shape convention is the caller's."""
    t = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)[None]
    out = torch.nn.functional.interpolate(t, size=(out_h, out_w), mode="bilinear", align_corners=False,
                                          antialias=False)
    return out[0].permute(1, 2, 0).contiguous().numpy()
