"""oracle/imgprep.py (restatement of Pillow's fixed-point bicubic resampler + the
CLIPImageProcessor shortest-edge resize and centre crop) is pinned against PIL itself —
the library the reference's processor calls (app/ml/embeddings.py:84-85)."""
from __future__ import annotations

import numpy as np
import pytest
from PIL import Image

from app.encoders.preprocess import to_u8_224
from oracle.imgprep import coeffs, resize_crop

SIZES = [(640, 480), (480, 640), (224, 224), (225, 224), (224, 225), (100, 150), (1000, 223), (223, 1000),
         (333, 777), (1280, 720), (50, 60), (17, 400), (2000, 1999)]


def _image(w, h, seed):
    rng = np.random.default_rng(seed)
    if seed % 2:
        return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    # smooth content (gradients + a little noise): the regime of real photos
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)), ((x + y) * 127 // max(w + h, 1))], -1)
    return np.clip(base + rng.integers(-8, 9, base.shape), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("wh", SIZES)
def test_oracle_matches_pil(wh):
    w, h = wh
    for seed in (w + h, w + h + 1):
        a = _image(w, h, seed)
        np.testing.assert_array_equal(resize_crop(a), to_u8_224(Image.fromarray(a)))


def test_taps_sum_to_one_fixed_point():
    for n_in, n_out in [(640, 298), (480, 224), (100, 224), (1999, 224)]:
        _, counts, taps = coeffs(n_in, n_out, 0, n_out)
        for c, t in zip(counts, taps):
            assert len(t) == c and abs(sum(t) - (1 << 22)) <= c  # rounding of each tap
