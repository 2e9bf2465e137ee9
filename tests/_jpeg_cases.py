"""Synthetic JPEG files for the K13 tests (generated with Pillow, the reference's decoder): photo-
like content (a smooth field + upsampled coarse noise + fine noise) and white noise, every
quality / subsampling / size class the decoder distinguishes, optimised Huffman tables, restart
intervals, grayscale; plus files K13 must refuse (progressive, CMYK, 4:4:0-like, tiny chroma)."""
from __future__ import annotations

import io

import numpy as np
from PIL import Image


def photo(h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    coarse = rng.integers(0, 256, (h // 16 + 1, w // 16 + 1, 3), dtype=np.uint8)
    img = np.asarray(Image.fromarray(coarse).resize((w, h), Image.BILINEAR), dtype=np.int16)
    return np.clip(img + rng.integers(-4, 5, (h, w, 3)), 0, 255).astype(np.uint8)


def jpeg_bytes(a: np.ndarray, **kw) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, "JPEG", **kw)
    return buf.getvalue()


def supported_cases():
    """(name, bytes) K13 decodes: Pillow's output is the expected RGB array."""
    out = []
    sizes = [(480, 640), (768, 1024), (9, 17), (65, 33), (57, 101), (224, 224), (3, 7), (201, 300), (5, 5)]
    for i, (h, w) in enumerate(sizes):
        a = photo(h, w, 10 + i)
        n = np.random.default_rng(40 + i).integers(0, 256, (h, w, 3), dtype=np.uint8)
        for q in (50, 90, 100):
            for sub in (0, 1, 2):
                out.append((f"photo{h}x{w}_q{q}_s{sub}", jpeg_bytes(a, quality=q, subsampling=sub)))
        out.append((f"noise{h}x{w}_q90_s2", jpeg_bytes(n, quality=90, subsampling=2)))
        out.append((f"gray{h}x{w}_q85", jpeg_bytes(a[..., 0], quality=85)))
    a = photo(480, 640, 3)
    out.append(("optimized_huffman", jpeg_bytes(a, quality=85, optimize=True)))
    out.append(("restart_blocks3", jpeg_bytes(a, quality=85, restart_marker_blocks=3)))
    out.append(("restart_rows1", jpeg_bytes(a, quality=85, restart_marker_rows=1)))
    out.append(("q1", jpeg_bytes(a, quality=1)))
    return out


def unsupported_cases():
    a = photo(96, 128, 5)
    return [("progressive", jpeg_bytes(a, quality=85, progressive=True)),
            ("cmyk", _cmyk(a)),
            ("tiny_chroma_w3", jpeg_bytes(photo(5, 3, 6), quality=90, subsampling=2))]


def _cmyk(a: np.ndarray) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(a).convert("CMYK").save(buf, "JPEG", quality=85)
    return buf.getvalue()


def damaged_cases():
    """(name, bytes) of damaged files: cut inside the entropy-coded data and closed with EOI (libjpeg
    finishes the MCU in progress with zero bits and leaves the rest zero), cut with nothing after
    (Pillow raises "image file is truncated"), an RST0 / RST7 spliced in (in a restart-interval
    file: out of order, libjpeg resynchronises), for plain and restart-interval files."""
    out = []
    for seed, (h, w, sub, kw) in enumerate([(480, 640, 2, {}), (301, 223, 0, {}), (480, 640, 1, {"restart_marker_rows": 1}),
                                            (200, 300, 2, {"restart_marker_blocks": 3})]):
        b = jpeg_bytes(photo(h, w, 50 + seed), quality=90, subsampling=sub, **kw)
        for frac in (0.1, 0.5, 0.95, 0.999):
            cut = int(len(b) * frac)
            out.append((f"f{seed}_cut{frac}_eoi", b[:cut] + b"\xff\xd9"))
            out.append((f"f{seed}_cut{frac}", b[:cut]))
            out.append((f"f{seed}_rst0_at{frac}", b[:cut] + b"\xff\xd0" + b[cut:]))
            out.append((f"f{seed}_rst7_at{frac}", b[:cut] + b"\xff\xd7" + b[cut:]))
    return out


def pillow_rgb(b: bytes) -> np.ndarray:
    with Image.open(io.BytesIO(b)) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)
