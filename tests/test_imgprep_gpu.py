"""K0 (csrc/imgprep.hip) on the GPU is byte-identical to the reference's preprocessing:
PIL bicubic shortest-edge resize + centre crop (app/encoders/preprocess.py:to_u8_224, the
restatement of CLIPImageProcessor pinned in test_compat_cpu.py), on one mixed-size batch:
downscale, upscale, unchanged width or height, identity, extreme aspect ratios, a 12 MP
photo size."""
from __future__ import annotations

import numpy as np
import pytest
from PIL import Image

from app.encoders.preprocess import to_u8_224

pytestmark = pytest.mark.gpu

SIZES = [(640, 480), (480, 640), (224, 224), (225, 224), (224, 225), (224, 900), (100, 150), (1000, 223),
         (223, 1000), (333, 777), (1920, 1080), (50, 60), (17, 400), (4000, 3000)]


def _img(w, h, seed):
    rng = np.random.default_rng(seed)
    if seed % 2:
        return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)), ((x + y) * 127 // max(w + h, 1))], -1)
    return np.clip(base + rng.integers(-8, 9, base.shape), 0, 255).astype(np.uint8)


def test_resize_crop_device_bit_exact(cuda):
    from app.encoders.preprocess import resize_crop_device

    imgs = [_img(w, h, i) for i, (w, h) in enumerate(SIZES)]
    got = resize_crop_device(imgs).cpu().numpy()
    for i, a in enumerate(imgs):
        np.testing.assert_array_equal(got[i], to_u8_224(Image.fromarray(a)), err_msg=str(SIZES[i]))


def test_load_batch_device_files(cuda, tmp_path):
    """Decode (host) + resize/crop (GPU) from files, incl. grayscale and RGBA sources."""
    from app.encoders.preprocess import load_batch, load_batch_device

    paths = []
    for i, (w, h, mode) in enumerate([(300, 200, "RGB"), (200, 300, "L"), (512, 512, "RGBA"), (224, 224, "RGB")]):
        a = _img(w, h, 100 + i)
        im = Image.fromarray(a).convert(mode)
        p = tmp_path / f"im{i}.png"
        im.save(p)
        paths.append(p)
    np.testing.assert_array_equal(load_batch_device(paths).cpu().numpy(), load_batch(paths))
    assert load_batch_device([]).shape == (0, 224, 224, 3)
