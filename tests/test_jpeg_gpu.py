"""K13 (csrc/jpeg.hip): baseline JPEG decode on the GPU against Pillow (the reference's decoder,
app/ml/embeddings.py:82-89) byte for byte, and the preprocessing path built on it
(load_batch_device: K13 for the JPEGs it takes, Pillow on host threads for the rest, K0 resize)
against the all-host path."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from _jpeg_cases import damaged_cases, overlong_run_cases, photo, pillow_rgb, supported_cases, unsupported_cases

pytestmark = pytest.mark.gpu


def _decode_batch(cases, cuda):
    import torch

    from app import _native

    dims = [pillow_rgb(b).shape for _, b in cases]
    sizes = np.array([h * w * 3 for h, w, _ in dims], dtype=np.int64)
    offs = np.zeros(len(cases), dtype=np.int64)
    offs[1:] = np.cumsum(sizes)[:-1]
    out = torch.full((int(sizes.sum()),), 7, dtype=torch.uint8, device=cuda)
    files = (ctypes.c_char_p * len(cases))(*[b for _, b in cases])
    fsz = np.array([len(b) for _, b in cases], dtype=np.int64)
    _native.call("mrag_jpeg_decode", ctypes.cast(files, ctypes.c_void_p), fsz.ctypes.data, len(cases), out.data_ptr(),
                 offs.ctypes.data, 0, torch.cuda.current_stream(cuda).cuda_stream)
    host = out.cpu().numpy()
    return [host[o:o + s].reshape(d) for o, s, d in zip(offs, sizes, dims)]


def test_decode_matches_pillow(cuda):
    cases = supported_cases() + overlong_run_cases()  # + AC runs past 63
    got = _decode_batch(cases, cuda)  # one batch: every segment of every file in one launch
    for (name, b), g in zip(cases, got):
        np.testing.assert_array_equal(g, pillow_rgb(b), err_msg=name)
    for i in range(0, len(cases), 7):  # small batches: the scratch buffers are reused and regrown
        for (name, b), g in zip(cases[i:i + 7], _decode_batch(cases[i:i + 7], cuda)):
            np.testing.assert_array_equal(g, pillow_rgb(b), err_msg=name)


def test_decode_refuses_unsupported(cuda):
    from app import _native

    with pytest.raises(_native.NativeError):
        _decode_batch(unsupported_cases()[:1], cuda)


def test_load_batch_device_mixed_equals_host(cuda, tmp_path):
    """JPEGs (K13), a progressive JPEG, a PNG, a grayscale JPEG and an in-memory PIL image in one
    batch: the device path's 224x224 u8 inputs equal the all-host path's byte for byte, with and
    without MRAG_HOST_DECODE."""
    from PIL import Image

    from app.encoders.preprocess import load_batch, load_batch_device

    items = []
    for i, (h, w) in enumerate([(480, 640), (600, 800), (768, 1024), (640, 480), (301, 223)]):
        a = photo(h, w, 100 + i)
        p = tmp_path / f"a{i}.jpg"
        Image.fromarray(a).save(p, quality=90)
        items.append(str(p))
    a = photo(300, 400, 7)
    Image.fromarray(a).save(tmp_path / "prog.jpg", quality=80, progressive=True)
    Image.fromarray(a).save(tmp_path / "img.png")
    Image.fromarray(a[..., 1]).save(tmp_path / "gray.jpg", quality=80)
    items += [str(tmp_path / "prog.jpg"), str(tmp_path / "img.png"), str(tmp_path / "gray.jpg"), Image.fromarray(a)]
    ref = load_batch(items)
    np.testing.assert_array_equal(load_batch_device(items).cpu().numpy(), ref)
    os.environ["MRAG_HOST_DECODE"] = "1"
    try:
        np.testing.assert_array_equal(load_batch_device(items).cpu().numpy(), ref)
    finally:
        del os.environ["MRAG_HOST_DECODE"]


def test_embed_images_batch_groups_equal_host_decode(cuda, tmp_path):
    """embed_images_batch over 600 files (JPEG for K13 + PNG for K14; decode groups of 256, the
    last partial): the embeddings equal those of the all-host decode (MRAG_HOST_DECODE=1) bit for
    bit, since the 224x224 inputs are byte-identical."""
    from PIL import Image

    from app.ml import embeddings as emb

    paths = []
    for i in range(600):
        h, w = [(120, 160), (150, 200), (97, 131)][i % 3]
        a = photo(h, w, 1000 + i)
        p = tmp_path / (f"f{i}.png" if i % 5 == 4 else f"f{i}.jpg")
        Image.fromarray(a).save(p, **({} if i % 5 == 4 else {"quality": 85}))
        paths.append(str(p))
    gpu = emb.embed_images_batch(paths)
    os.environ["MRAG_HOST_DECODE"] = "1"
    try:
        host = emb.embed_images_batch(paths)
    finally:
        del os.environ["MRAG_HOST_DECODE"]
    np.testing.assert_array_equal(gpu, host)


def test_damaged_files_as_pillow(cuda, tmp_path):
    """Damaged JPEGs through load_batch_device: the ones Pillow decodes give the all-host path's
    bytes (K13 for those it takes, Pillow for the rest); one Pillow refuses raises, as it does in
    the reference's embed_images_batch."""
    from app.encoders.preprocess import load_batch, load_batch_device

    ok, refused = [], []
    for i, (name, b) in enumerate(damaged_cases()):
        p = tmp_path / f"{i}_{name}.jpg"
        p.write_bytes(b)
        try:
            pillow_rgb(b)
            ok.append(str(p))
        except OSError:
            refused.append(str(p))
    np.testing.assert_array_equal(load_batch_device(ok).cpu().numpy(), load_batch(ok))
    assert refused
    with pytest.raises(OSError):
        load_batch_device(ok[:3] + refused[:1])


def test_embed_images_batch_group_host_half_equals_per_file(cuda, tmp_path):
    """embed_images_batch with the host half as one library call per group (preprocess._NATIVE_FILES
    True: processor.decode -> NativePrepared) equals the per-file host half (_prepare_one on the
    decode pool) bit for bit."""
    from PIL import Image

    from app.encoders import preprocess as pp
    from app.ml import embeddings as emb

    paths = []
    for i in range(300):
        a = photo(110 + i % 7, 150, 3000 + i)
        p = tmp_path / (f"g{i}.png" if i % 4 == 3 else f"g{i}.jpg")
        Image.fromarray(a).save(p, **({} if i % 4 == 3 else {"quality": 85}))
        paths.append(str(p))
    keep = pp._NATIVE_FILES
    try:
        pp._NATIVE_FILES = False
        per_file = emb.embed_images_batch(paths)
        pp._NATIVE_FILES = True
        group = emb.embed_images_batch(paths)
    finally:
        pp._NATIVE_FILES = keep
    np.testing.assert_array_equal(group, per_file)
