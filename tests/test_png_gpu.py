"""K14 (csrc/png.hip): PNG scanline reconstruction + convert("RGB") on the GPU after the host
inflate, against Pillow (the reference's decoder, app/ml/embeddings.py:82-89) byte for byte, and
the preprocessing path built on it (load_batch_device) against the all-host path."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from _png_cases import bad_idat_crc_case, filtered_png, pillow_rgb, supported_cases, unsupported_cases

pytestmark = pytest.mark.gpu


def _inflate(b: bytes):
    from app import _native

    lib = _native.load()
    w, h, nraw, bpp = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int64(0), ctypes.c_int32(0)
    assert lib.mrag_png_probe(b, len(b), ctypes.byref(w), ctypes.byref(h), ctypes.byref(nraw)) == 1
    raw = np.empty(nraw.value, np.uint8)
    assert lib.mrag_png_inflate(b, len(b), raw.ctypes.data, nraw.value, ctypes.byref(bpp)) == 1
    return raw, (w.value, h.value, bpp.value)


def _unfilter_batch(cases, cuda):
    import torch

    from app import _native

    inf = [_inflate(b) for _, b in cases]
    dims = np.array([d for _, d in inf], dtype=np.int32)
    sizes = dims[:, 0].astype(np.int64) * dims[:, 1] * 3
    offs = np.zeros(len(cases), dtype=np.int64)
    offs[1:] = np.cumsum(sizes)[:-1]
    out = torch.full((int(sizes.sum()),), 7, dtype=torch.uint8, device=cuda)
    raws = (ctypes.c_void_p * len(cases))(*[r.ctypes.data for r, _ in inf])
    _native.call("mrag_png_unfilter", ctypes.cast(raws, ctypes.c_void_p), dims.ctypes.data, len(cases),
                 out.data_ptr(), offs.ctypes.data, 0, torch.cuda.current_stream(cuda).cuda_stream)
    host = out.cpu().numpy()
    return [host[o:o + s].reshape(int(d[1]), int(d[0]), 3) for o, s, d in zip(offs, sizes, dims)]


def test_unfilter_matches_pillow(cuda):
    cases = supported_cases()
    for (name, b), g in zip(cases, _unfilter_batch(cases, cuda)):  # one launch, every image
        np.testing.assert_array_equal(g, pillow_rgb(b), err_msg=name)
    for i in range(0, len(cases), 9):  # small batches: the scratch buffers are reused and regrown
        for (name, b), g in zip(cases[i:i + 9], _unfilter_batch(cases[i:i + 9], cuda)):
            np.testing.assert_array_equal(g, pillow_rgb(b), err_msg=name)


def test_unfilter_widest_and_tallest(cuda):
    """The LDS carry row at its limit (8192 pixels wide, several 64-row bands) and a one-pixel-wide
    image 700 rows tall (eleven bands, one active column)."""
    rng = np.random.default_rng(5)
    wide = filtered_png(rng.integers(0, 256, (130, 8192, 4), dtype=np.uint8), 6)
    tall = filtered_png(rng.integers(0, 256, (700, 1, 3), dtype=np.uint8), 2)
    for (name, b), g in zip([("wide", wide), ("tall", tall)], _unfilter_batch([("wide", wide), ("tall", tall)], cuda)):
        np.testing.assert_array_equal(g, pillow_rgb(b), err_msg=name)
    from app import _native

    too_wide = filtered_png(rng.integers(0, 256, (2, 8193, 1), dtype=np.uint8), 0)
    w, h, n = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int64(0)
    assert _native.load().mrag_png_probe(too_wide, len(too_wide), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n)) == 0


def test_load_batch_device_png_mix_equals_host(cuda, tmp_path):
    """PNGs K14 takes (RGB, RGBA, L, LA) and ones it leaves to Pillow (palette, 16-bit, bilevel) with
    JPEGs in one batch: the 224x224 u8 inputs equal the all-host path's, with and without
    MRAG_HOST_DECODE."""
    from PIL import Image

    from _jpeg_cases import photo
    from app.encoders.preprocess import load_batch, load_batch_device

    items = []
    sup = [c for c in supported_cases() if c[0].startswith(("photo480x640", "noise201x300", "filters300x201"))]
    left = [c for c in unsupported_cases() if c[0] != "bad_crc"]  # Pillow refuses that one itself
    sup.append(("bad_idat_crc", bad_idat_crc_case()))  # Pillow skips IDAT CRCs: K14 takes it
    for i, (name, b) in enumerate(sup + left):
        p = tmp_path / f"{i}_{name}.png"
        p.write_bytes(b)
        items.append(str(p))
    for i in range(3):
        p = tmp_path / f"j{i}.jpg"
        Image.fromarray(photo(300 + 40 * i, 400, 50 + i)).save(p, quality=90)
        items.append(str(p))
    ref = load_batch(items)
    np.testing.assert_array_equal(load_batch_device(items).cpu().numpy(), ref)
    os.environ["MRAG_HOST_DECODE"] = "1"
    try:
        np.testing.assert_array_equal(load_batch_device(items).cpu().numpy(), ref)
    finally:
        del os.environ["MRAG_HOST_DECODE"]


def test_native_files_equal_per_file_path(cuda, tmp_path):
    """The group host half in one library call (NativePrepared: mrag_files_prepare, then
    mrag_files_decode) gives the per-file path's device pixels byte for byte over JPEGs, PNGs K14
    takes and files both leave to Pillow; a missing file raises FileNotFoundError in both."""
    import torch

    from _jpeg_cases import photo
    from PIL import Image

    from app.encoders import preprocess as pp

    items = []
    sup = [c for c in supported_cases() if c[0].startswith(("photo480x640", "noise201x300", "filters300x201"))]
    left = [c for c in unsupported_cases() if c[0] != "bad_crc"]
    for i, (name, b) in enumerate(sup + left):
        p = tmp_path / f"{i}_{name}.png"
        p.write_bytes(b)
        items.append(str(p))
    for i in range(3):
        p = tmp_path / f"j{i}.jpg"
        Image.fromarray(photo(300 + 40 * i, 400, 50 + i)).save(p, quality=90, progressive=(i == 2))
        items.append(str(p))

    def dev_pixels(flag):
        pp._NATIVE_FILES = flag
        try:
            prep = pp.prepare_batch(items)
            assert isinstance(prep, pp.NativePrepared) == flag
            d = pp.upload_decode(prep, device=0)
            torch.cuda.synchronize()
            return [d.pix[int(o):int(o) + int(h * w * 3)].cpu().numpy().reshape(h, w, 3)
                    for o, (h, w) in zip(d.offsets, d.dims)]
        finally:
            pp._NATIVE_FILES = True

    nat, per = dev_pixels(True), dev_pixels(False)
    for p, a, b in zip(items, nat, per):
        np.testing.assert_array_equal(a, b, err_msg=p)
    assert pp.NativePrepared(items).kind.tolist().count(0) == len(left) + 1  # + the progressive JPEG
    for flag in (True, False):
        pp._NATIVE_FILES = flag
        try:
            with pytest.raises(FileNotFoundError):
                pp.load_batch_device(items[:2] + [str(tmp_path / "missing.png")])
        finally:
            pp._NATIVE_FILES = True
