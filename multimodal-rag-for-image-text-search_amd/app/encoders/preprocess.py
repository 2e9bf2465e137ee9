"""Host image preprocessing: decode -> RGB -> resize (shortest edge 224, bicubic) ->
centre crop 224 -> u8 HWC. Everything after (rescale, mean/std normalise, layout) is
fused into the GPU patch-embed kernel.

Restates CLIPImageProcessor's PIL path (the processor the reference loads for
openai/clip-vit-base-patch32, app/ml/embeddings.py:39-43, 84-85):
``get_resize_output_image_size(default_to_square=False)`` — new_short = 224,
new_long = int(224 * long / short) — then ``PIL.Image.resize((w, h), BICUBIC)`` on the
uint8 image, then ``center_crop`` with top = (h - 224) // 2, left = (w - 224) // 2.
Checked against transformers' CLIPImageProcessor in tests/test_compat_cpu.py.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import List, Sequence, Union

import numpy as np
from PIL import Image

SIZE = 224


def to_u8_224(img: Image.Image, size: int = SIZE) -> np.ndarray:
    if img.mode != "RGB":
        img = img.convert("RGB")
    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    nw, nh = (new_short, new_long) if w <= h else (new_long, new_short)
    if (nw, nh) != (w, h):
        img = img.resize((nw, nh), resample=Image.BICUBIC)
    a = np.asarray(img, dtype=np.uint8)
    top, left = (nh - size) // 2, (nw - size) // 2
    if top >= 0 and left >= 0:
        return np.ascontiguousarray(a[top:top + size, left:left + size])
    # smaller than the crop: zero-pad around the centre (transformers pads the same way)
    out = np.zeros((size, size, 3), dtype=np.uint8)
    t0, l0 = max(0, -top), max(0, -left)
    sh, sw = min(nh, size), min(nw, size)
    out[t0:t0 + sh, l0:l0 + sw] = a[max(0, top):max(0, top) + sh, max(0, left):max(0, left) + sw]
    return out


def load_batch(items: Sequence[Union[str, Path, Image.Image]], workers: int = 8) -> np.ndarray:
    """Decode + resize + crop a batch in a thread pool (PIL releases the GIL)."""

    def one(x):
        if isinstance(x, Image.Image):
            return to_u8_224(x)
        with Image.open(x) as im:
            return to_u8_224(im.convert("RGB"))

    if len(items) == 0:
        return np.empty((0, SIZE, SIZE, 3), dtype=np.uint8)
    with ThreadPoolExecutor(max_workers=max(1, min(workers, len(items)))) as ex:
        return np.stack(list(ex.map(one, items)))
