"""The ingest host half in one library call (csrc/files.hip: mrag_files_prepare / info / bytes /
free) on the CPU: each file's kind and size agree with the per-file probes _prepare_one uses
(mrag_jpeg_probe, mrag_png_probe), the bytes are the file's, unreadable files are marked, and
NativePrepared decodes the files the GPU decoders leave with Pillow. No GPU (mrag_files_decode,
the device half, is covered by the -m gpu tests)."""
from __future__ import annotations

import ctypes
import io
import os

import numpy as np
import pytest

import _jpeg_cases as J
import _png_cases as P


def _files(tmp_path):
    items = []
    cases = ([(f"j_{n}", ".jpg", b) for n, b in J.supported_cases()[:4]]
             + [(f"ju_{n}", ".jpg", b) for n, b in J.unsupported_cases()]
             + [(f"p_{n}", ".png", b) for n, b in P.supported_cases()[:6]]
             + [(f"pu_{n}", ".png", b) for n, b in P.unsupported_cases() if n != "bad_crc"]
             + [("trunc", ".png", P.truncated_stream_case())])
    for i, (name, ext, b) in enumerate(cases):
        p = tmp_path / f"{i}_{name}{ext}"
        p.write_bytes(b)
        items.append((str(p), b))
    return items


def _probe(lib, b):
    """The per-file classification of preprocess._prepare_one: 1 JPEG, 2 PNG, 0 other."""
    w, h, n = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int64(0)
    if b[:2] == b"\xff\xd8":
        return (1, w.value, h.value) if lib.mrag_jpeg_probe(b, len(b), ctypes.byref(w), ctypes.byref(h)) == 1 \
            else (0, 0, 0)
    if lib.mrag_png_probe(b, len(b), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n)) == 1:
        raw, bpp = np.empty(n.value, np.uint8), ctypes.c_int32(0)
        if lib.mrag_png_inflate(b, len(b), raw.ctypes.data, n.value, ctypes.byref(bpp)) == 1:
            return 2, w.value, h.value
    return 0, 0, 0


@pytest.mark.parametrize("device_decode", [1, 0])
def test_prepare_matches_per_file_probes(tmp_path, device_decode):
    from app import _native

    lib = _native.load()
    items = _files(tmp_path)
    paths = [p for p, _ in items] + [str(tmp_path / "missing.jpg")]
    n = len(paths)
    names = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    h = ctypes.c_void_p()
    _native.call("mrag_files_prepare", ctypes.cast(names, ctypes.c_void_p), n, 4, device_decode, -1, ctypes.byref(h))
    try:
        kind, w, hh = (np.zeros(n, np.int32) for _ in range(3))
        _native.call("mrag_files_info", h, kind.ctypes.data, w.ctypes.data, hh.ctypes.data)
        assert kind[-1] == -1
        for i, (p, b) in enumerate(items):
            want = _probe(lib, b) if device_decode else (0, 0, 0)
            assert (kind[i], w[i], hh[i]) == want, p
            ptr, size = ctypes.c_void_p(), ctypes.c_int64()
            _native.call("mrag_files_bytes", h, i, ctypes.byref(ptr), ctypes.byref(size))
            assert ctypes.string_at(ptr.value, size.value) == b, p
        if device_decode:
            assert set(kind[:-1].tolist()) == {0, 1, 2}
    finally:
        lib.mrag_files_free(h)


def test_prepare_bad_arguments():
    from app import _native

    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.mrag_files_prepare(None, 3, 1, 1, -1, ctypes.byref(h)) != 0
    assert lib.mrag_files_prepare(None, 0, 1, 1, -1, None) != 0
    assert lib.mrag_files_prepare(None, 0, 1, 1, -1, ctypes.byref(h)) == 0  # an empty group
    ptr, size = ctypes.c_void_p(), ctypes.c_int64()
    assert lib.mrag_files_bytes(h, 0, ctypes.byref(ptr), ctypes.byref(size)) != 0  # index out of range
    lib.mrag_files_free(h)


def test_native_prepared_host_files(tmp_path):
    """NativePrepared: files the GPU decoders leave get Pillow's RGB array and its size; a missing
    file raises the reference's FileNotFoundError (Image.open(path) in embed_images_batch)."""
    from app.encoders.preprocess import NativePrepared

    items = _files(tmp_path)
    prep = NativePrepared([p for p, _ in items])
    assert len(prep) == len(items)
    assert prep.host
    for i, (p, b) in enumerate(items):
        if i in prep.host:
            assert prep.kind[i] == 0
            ref = J.pillow_rgb(b)
            np.testing.assert_array_equal(prep.host[i], ref, err_msg=p)
            assert tuple(prep.dims[i]) == ref.shape[:2]
        else:
            assert prep.kind[i] in (1, 2)
            assert tuple(prep.dims[i]) == J.pillow_rgb(b).shape[:2], p
    del prep
    with pytest.raises(FileNotFoundError):
        NativePrepared([items[0][0], str(tmp_path / "missing.jpg")])


def _kinds(tmp_path, blobs, max_pixels):
    from app import _native

    lib = _native.load()
    paths = []
    for i, b in enumerate(blobs):
        ext = "jpg" if b[:2] == b"\xff\xd8" else "png"
        p = tmp_path / f"lim{i}.{ext}"
        p.write_bytes(b)
        paths.append(os.fsencode(str(p)))
    names = (ctypes.c_char_p * len(paths))(*paths)
    h = ctypes.c_void_p()
    _native.call("mrag_files_prepare", ctypes.cast(names, ctypes.c_void_p), len(paths), 2, 1, max_pixels,
                 ctypes.byref(h))
    try:
        kind, w, hh = (np.zeros(len(paths), np.int32) for _ in range(3))
        _native.call("mrag_files_info", h, kind.ctypes.data, w.ctypes.data, hh.ctypes.data)
        return kind.tolist()
    finally:
        lib.mrag_files_free(h)


def _sof_resized(b: bytes, h: int, w: int) -> bytes:
    """A JPEG whose frame header claims h x w (the entropy-coded data unchanged): the header a
    decompression bomb carries."""
    i = 2
    while i + 4 <= len(b):
        marker, seglen = b[i + 1], int.from_bytes(b[i + 2:i + 4], "big")
        if marker == 0xC0:
            return b[:i + 5] + h.to_bytes(2, "big") + w.to_bytes(2, "big") + b[i + 9:]
        i += 2 + seglen
    raise AssertionError("no SOF0")


def test_prepare_pixel_limit(tmp_path):
    """files above Pillow's decompression-bomb limit (max(1,w)*max(1,h) > MAX_IMAGE_PIXELS)
    are kind 0, so Pillow warns / raises DecompressionBombError for them as in the reference; at or
    below the limit, and with no limit (-1), the GPU decoders take them."""
    from PIL import Image

    jpg = J.jpeg_bytes(J.photo(48, 64, 1), quality=90)
    png = P.supported_cases()[0][1]
    with Image.open(io.BytesIO(png)) as im:
        pw, ph = im.size
    assert _kinds(tmp_path, [jpg, png], -1) == [1, 2]
    assert _kinds(tmp_path, [jpg, png], max(48 * 64, pw * ph)) == [1, 2]
    assert _kinds(tmp_path, [jpg, png], min(48 * 64, pw * ph) - 1) == [0, 0]
    assert _kinds(tmp_path, [jpg, png], 0) == [0, 0]
    bomb = _sof_resized(jpg, 20000, 20000)  # 4e8 px > 2 x Pillow's default limit
    assert _kinds(tmp_path, [bomb], -1) == [1]
    assert _kinds(tmp_path, [bomb], Image.MAX_IMAGE_PIXELS) == [0]


def test_native_prepared_raises_pillows_bomb_error(tmp_path, monkeypatch):
    """The drop-in passes Image.MAX_IMAGE_PIXELS at call time: a file above twice the limit raises
    Pillow's DecompressionBombError (reference: Image.open(path) in embed_images_batch), one above
    the limit decodes with Pillow's DecompressionBombWarning."""
    import warnings

    from PIL import Image

    from app.encoders.preprocess import NativePrepared

    p = tmp_path / "a.jpg"
    b = J.jpeg_bytes(J.photo(48, 64, 2), quality=90)
    p.write_bytes(b)
    monkeypatch.setattr(Image, "MAX_IMAGE_PIXELS", 48 * 64 // 3)
    with pytest.raises(Image.DecompressionBombError):
        NativePrepared([str(p)])
    monkeypatch.setattr(Image, "MAX_IMAGE_PIXELS", 48 * 64 - 1)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        prep = NativePrepared([str(p)])
    assert prep.kind[0] == 0 and any(issubclass(c.category, Image.DecompressionBombWarning) for c in caught)
    np.testing.assert_array_equal(prep.host[0], J.pillow_rgb(b))
    monkeypatch.setattr(Image, "MAX_IMAGE_PIXELS", None)
    assert NativePrepared([str(p)]).kind[0] == 1
