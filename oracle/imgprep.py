"""CPU restatement of the reference's image resize (TEST INFRASTRUCTURE ONLY).

The reference preprocesses images with CLIPImageProcessor (app/ml/embeddings.py:84-85),
whose PIL backend resizes the shortest edge to 224 with ``Image.resize(..., BICUBIC)`` and
centre-crops 224 (restated in app/encoders/preprocess.py:to_u8_224, pinned against
transformers in tests/test_compat_cpu.py). The arithmetic lives in Pillow's
``libImaging/Resample.c`` (third-party, Pillow 12.2.0 installed here, unpinned by the
reference): restated here and pinned against PIL itself in tests/test_imgprep_cpu.py.

Algorithm (8-bit path):
  * ``precompute_coeffs``: scale = (double)(in1 - in0) / outSize, filterscale = max(scale, 1),
    support = 2 * filterscale (bicubic, a = -0.5); per output position xx:
    center = in0 + (xx + 0.5) * scale, xmin = max((int)(center - support + 0.5), 0),
    xmax = min((int)(center + support + 0.5), inSize) - xmin,
    w[x] = bicubic((x + xmin - center + 0.5) / filterscale), normalised by their sum;
  * ``normalize_coeffs_8bpc``: int32 k = (int)(w * 2^22 +- 0.5) (round half away from 0);
  * horizontal pass (only if the width changes) then vertical pass (only if the height
    changes), each ``clip8((2^21 + sum u8 * k) >> 22)`` back to u8.
Only the rows / columns of the centre crop are computed — each output pixel depends on
its own coefficients only, so this equals a full resize followed by the crop.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def coeffs(in_size: int, out_size: int, o0: int, count: int) -> Tuple[List[int], List[int], List[List[int]]]:
    """(xmin, xcount, int32 taps) for output positions o0 .. o0+count-1 (Resample.c
    precompute_coeffs + normalize_coeffs_8bpc)."""
    scale = float(np.float32(in_size) - np.float32(0.0)) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    xmins, xcounts, taps = [], [], []
    for xx in range(o0, o0 + count):
        center = 0.0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        k = []
        for x in range(xmax):
            w = _bicubic((x + xmin - center + 0.5) * ss)
            k.append(w)
            ww += w
        if ww != 0.0:
            k = [v / ww for v in k]
        kk = [int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS)) for v in k]
        xmins.append(xmin)
        xcounts.append(xmax)
        taps.append(kk)
    return xmins, xcounts, taps


def _pass(src: np.ndarray, xmins, xcounts, taps, axis: int) -> np.ndarray:
    """One 8-bit resample pass along `axis` (1 = columns, 0 = rows) of an HxWx3 u8 array."""
    s = src.astype(np.int64)
    outs = []
    for xmin, n, kk in zip(xmins, xcounts, taps):
        acc = np.full((s.shape[1 - axis], 3), 1 << (PRECISION_BITS - 1), dtype=np.int64)
        for j in range(n):
            line = s[:, xmin + j, :] if axis == 1 else s[xmin + j, :, :]
            acc = acc + line * kk[j]
        acc = acc.astype(np.int32)  # C int arithmetic (no overflow occurs for 8-bit inputs)
        outs.append(np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8))
    return np.stack(outs, axis=axis)


def resize_crop(img: np.ndarray, size: int = 224) -> np.ndarray:
    """u8 HxWx3 -> u8 size x size x 3, equal to app.encoders.preprocess.to_u8_224."""
    h, w = img.shape[:2]
    short, long_ = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long_ / short)
    nw, nh = (new_short, new_long) if w <= h else (new_long, new_short)
    top, left = (nh - size) // 2, (nw - size) // 2
    out = img
    # the row window the cropped output rows need (whole crop if the height is unchanged)
    if nh != h:
        ymins, ycounts, ytaps = coeffs(h, nh, top, size)
        y0 = min(ymins)
        y1 = max(a + b for a, b in zip(ymins, ycounts))
    else:
        y0, y1 = top, top + size
    rows = out[y0:y1]
    if nw != w:
        xmins, xcounts, xtaps = coeffs(w, nw, left, size)
        rows = _pass(rows, xmins, xcounts, xtaps, axis=1)
    else:
        rows = rows[:, left:left + size]
    if nh != h:
        rows = _pass(rows, [m - y0 for m in ymins], ycounts, ytaps, axis=0)
    return np.ascontiguousarray(rows)


__all__ = ["coeffs", "resize_crop", "PRECISION_BITS"]
