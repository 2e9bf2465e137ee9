"""Image preprocessing: decode -> RGB -> resize (shortest edge 224, bicubic) -> centre
crop 224 -> u8 HWC. Everything after (rescale, mean/std normalise, layout) is fused into
the GPU patch-embed kernel.

Two implementations with identical bytes: ``load_batch_device`` (the default for the
native encoders) decodes baseline JPEGs on the GPU (``mrag_jpeg_decode``, K13 in csrc/jpeg.hip —
libjpeg-turbo's decode as Pillow runs it, restated), 8-bit grey / RGB(A) PNGs by a zlib inflate on
host threads and the scanline reconstruction on the GPU (``mrag_png_unfilter``, K14 in
csrc/png.hip), every other file on host threads with Pillow, and runs the resize + crop on the
GPU (``mrag_image_resize_crop``, K0 in csrc/imgprep.hip — Pillow's fixed-point resampler
restated); ``load_batch`` does all of it with PIL on the host. ``MRAG_HOST_DECODE=1`` decodes
every file on the host (A/B timing).

Restates CLIPImageProcessor's PIL path (the processor the reference loads for
openai/clip-vit-base-patch32, app/ml/embeddings.py:39-43, 84-85):
``get_resize_output_image_size(default_to_square=False)`` — new_short = 224,
new_long = int(224 * long / short) — then ``PIL.Image.resize((w, h), BICUBIC)`` on the
uint8 image, then ``center_crop`` with top = (h - 224) // 2, left = (w - 224) // 2.
Checked against transformers' CLIPImageProcessor in tests/test_compat_cpu.py.
"""
from __future__ import annotations

import ctypes
import io
import os
import threading
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import List, Sequence, Union

import numpy as np
from PIL import Image

SIZE = 224


def decode_workers() -> int:
    """Host threads for image decode: the cores this process may use (affinity mask, capped by a
    cgroup CPU quota when one is set — a GPU box lists the whole node's cores), at most 32. PIL
    releases the GIL inside its decoders, so decode throughput grows with them (the ingest path
    is decode-bound: DESIGN.md §6)."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except Exception:
        pass
    return max(1, min(32, n))


_POOL = None
_POOL_LOCK = threading.Lock()


def _pool() -> ThreadPoolExecutor:
    """One process-wide decode pool (created on first use, reused by every batch)."""
    global _POOL
    with _POOL_LOCK:
        if _POOL is None:
            _POOL = ThreadPoolExecutor(max_workers=decode_workers(), thread_name_prefix="mrag-decode")
        return _POOL


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


def decode_rgb(x: Union[str, Path, Image.Image]) -> np.ndarray:
    """Decode only: u8 HxWx3 RGB (the part of preprocessing that stays on the host)."""
    if isinstance(x, Image.Image):
        return np.asarray(x if x.mode == "RGB" else x.convert("RGB"), dtype=np.uint8)
    with Image.open(x) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


def resize_crop_device(arrays: Sequence[np.ndarray], device: int = 0, size: int = SIZE):
    """u8 HxWx3 host arrays -> u8 [n, size, size, 3] CUDA tensor, resized + centre-cropped
    on the GPU (bit-identical to ``to_u8_224``)."""
    import ctypes

    import torch

    from app import _native

    n = len(arrays)
    dev = torch.device("cuda", device)
    out = torch.empty((n, size, size, 3), dtype=torch.uint8, device=dev)
    if n == 0:
        return out
    arrays = [np.ascontiguousarray(a, dtype=np.uint8) for a in arrays]
    for a in arrays:
        if a.ndim != 3 or a.shape[2] != 3:
            raise ValueError(f"expected HxWx3 u8 images, got shape {a.shape}")
    sizes = np.array([a.size for a in arrays], dtype=np.int64)
    offsets = np.zeros(n, dtype=np.int64)
    offsets[1:] = np.cumsum(sizes)[:-1]
    host = torch.empty(int(sizes.sum()), dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for a, o, sz in zip(arrays, offsets, sizes):
        hv[o:o + sz] = a.reshape(-1)
    pix = host.to(dev, non_blocking=True)
    widths = np.array([a.shape[1] for a in arrays], dtype=np.int32)
    heights = np.array([a.shape[0] for a in arrays], dtype=np.int32)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _native.call("mrag_image_resize_crop", pix.data_ptr(),
                     offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                     widths.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                     heights.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n, size, out.data_ptr(), stream)
    return out


def decode_batch(items: Sequence[Union[str, Path, Image.Image]]) -> List[np.ndarray]:
    """Host decode of a batch on the process-wide pool: u8 HxWx3 RGB arrays, in order."""
    if len(items) == 0:
        return []
    return list(_pool().map(decode_rgb, items))


_PNG_SIG = b"\x89PNG\r\n\x1a\n"


def max_pixels() -> int:
    """Pillow's decompression-bomb limit as read at call time (``Image.MAX_IMAGE_PIXELS``; -1 for
    None = no limit). A file above it is left to Pillow, which warns (or raises
    DecompressionBombError above twice the limit) exactly as the reference's Image.open does."""
    m = Image.MAX_IMAGE_PIXELS
    return -1 if m is None else int(m)


def _over_limit(w: int, h: int) -> bool:
    m = max_pixels()
    return m >= 0 and max(1, w) * max(1, h) > m


def _prepare_one(x):
    """The host half for one item: a JPEG K13 decodes -> ("jpeg", file bytes, (h, w), 0), None; a
    PNG K14 reconstructs -> ("png", inflated scanlines, (h, w), bytes per pixel), None; anything
    else (a PIL image, a palette or 16-bit PNG, a progressive JPEG ...) -> None, its u8 HxWx3 RGB
    decoded here with Pillow."""
    if isinstance(x, Image.Image):
        return None, decode_rgb(x)
    with open(x, "rb") as f:
        b = f.read()
    if os.environ.get("MRAG_HOST_DECODE") != "1":
        from app import _native

        w, h = ctypes.c_int32(0), ctypes.c_int32(0)
        if b[:2] == b"\xff\xd8":
            if (_native.load().mrag_jpeg_probe(b, len(b), ctypes.byref(w), ctypes.byref(h)) == 1
                    and not _over_limit(w.value, h.value)):
                return ("jpeg", b, (h.value, w.value), 0), None
        elif b[:8] == _PNG_SIG:
            lib, nraw = _native.load(), ctypes.c_int64(0)
            if (lib.mrag_png_probe(b, len(b), ctypes.byref(w), ctypes.byref(h), ctypes.byref(nraw)) == 1
                    and not _over_limit(w.value, h.value)):
                raw = np.empty(nraw.value, dtype=np.uint8)
                bpp = ctypes.c_int32(0)
                if lib.mrag_png_inflate(b, len(b), raw.ctypes.data, nraw.value, ctypes.byref(bpp)) == 1:
                    return ("png", raw, (h.value, w.value), bpp.value), None
    with Image.open(io.BytesIO(b)) as im:
        return None, np.asarray(im.convert("RGB"), dtype=np.uint8)


class NativePrepared:
    """A group's host half done by the library (``mrag_files_prepare``: file reads, probes and the
    PNGs' inflate on its own threads, no interpreter lock between files): the handle owning the
    bytes K13 / K14 decode from, each file's kind and size, and Pillow arrays for the files the GPU
    decoders do not take (kind 0). Unreadable files raise here, as Image.open would."""

    def __init__(self, paths: Sequence[Union[str, Path]]):
        from app import _native

        lib = _native.load()
        n = len(paths)
        names = (ctypes.c_char_p * n)(*[os.fsencode(os.fspath(p)) for p in paths])
        h = ctypes.c_void_p()
        dev = 0 if os.environ.get("MRAG_HOST_DECODE") == "1" else 1
        _native.call("mrag_files_prepare", ctypes.cast(names, ctypes.c_void_p), n, decode_workers(), dev,
                     max_pixels(), ctypes.byref(h))
        self._lib, self.handle = lib, h
        kind, w, hh = (np.zeros(n, np.int32) for _ in range(3))
        _native.call("mrag_files_info", h, kind.ctypes.data, w.ctypes.data, hh.ctypes.data)
        self.kind = kind
        self.dims = np.stack([hh, w], axis=1).astype(np.int64)
        self.host: dict = {}
        left = [int(i) for i in np.nonzero(kind <= 0)[0]]

        def host_decode(i: int) -> np.ndarray:
            if kind[i] < 0:  # the reference's error for this path (or, if it reads now, its decode)
                with open(paths[i], "rb") as f:
                    b = f.read()
            else:
                ptr, size = ctypes.c_void_p(), ctypes.c_int64()
                _native.call("mrag_files_bytes", h, i, ctypes.byref(ptr), ctypes.byref(size))
                b = ctypes.string_at(ptr.value, size.value) if size.value else b""
            with Image.open(io.BytesIO(b)) as im:
                return np.asarray(im.convert("RGB"), dtype=np.uint8)

        # Pillow's decoders release the interpreter lock: the files the GPU decoders leave (progressive
        # JPEGs, palette PNGs, WebP ...) decode on the process-wide pool; map keeps their order and
        # raises the first failing file's exception, as the per-file loop would
        decoded = list(_pool().map(host_decode, left)) if len(left) > 1 else [host_decode(i) for i in left]
        for i, a in zip(left, decoded):
            self.host[i] = a
            self.dims[i] = a.shape[:2]

    def __len__(self):
        return len(self.kind)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self._lib.mrag_files_free(h)
            self.handle = None


_NATIVE_FILES = True  # path lists through mrag_files_prepare (False: _prepare_one per file on the pool)


def prepare_batch(items: Sequence[Union[str, Path, Image.Image]]) -> list:
    """The host half of ``load_batch_device``: for a list of file paths one library call
    (``NativePrepared``); otherwise per item on the process-wide pool — file bytes of the JPEGs the
    GPU decodes, inflated scanlines of the PNGs it reconstructs, Pillow arrays of everything else
    (embed_images_batch runs it for the next batch while the GPU works on the current one)."""
    if len(items) == 0:
        return []
    if _NATIVE_FILES and all(isinstance(x, (str, Path)) for x in items):
        return NativePrepared(list(items))
    return list(_pool().map(_prepare_one, items))


class DeviceImages:
    """Decoded RGB images of a group in one device buffer: image i is dims[i] = (h, w) at byte
    offsets[i] of ``pix`` (u8 HxWx3) — what K0 resizes from."""

    def __init__(self, pix, offsets: np.ndarray, dims: np.ndarray):
        self.pix, self.offsets, self.dims = pix, offsets, dims

    def __len__(self):
        return len(self.offsets)


def upload_decode(prepared: list, device: int = 0) -> DeviceImages:
    """The device half's decode into one pixel buffer: the host-decoded images (one pinned copy),
    then K13's JPEGs and K14's PNGs, each kind in one launch, on the calling thread's current
    stream; the pixels are complete when it returns (any stream may read them)."""
    import torch

    from app import _native

    n = len(prepared)
    dev = torch.device("cuda", device)
    if isinstance(prepared, NativePrepared):
        dims = prepared.dims
        sizes = dims[:, 0] * dims[:, 1] * 3
        host = sorted(prepared.host)
        gpu = [i for i in range(n) if prepared.kind[i] > 0]
        offsets = np.zeros(n, dtype=np.int64)  # host-decoded images first (one copy), then K13's / K14's
        pos = 0
        for i in host + gpu:
            offsets[i] = pos
            pos += int(sizes[i])
        pix = torch.empty(max(pos, 1), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            if host:
                nh = int(sum(int(sizes[i]) for i in host))
                staging = torch.empty(nh, dtype=torch.uint8, pin_memory=True)
                sv = staging.numpy()
                for i in host:
                    sv[offsets[i]:offsets[i] + sizes[i]] = prepared.host[i].reshape(-1)
                pix[:nh].copy_(staging, non_blocking=True)
            if gpu:
                _native.call("mrag_files_decode", prepared.handle, pix.data_ptr(), offsets.ctypes.data, device, stream)
            else:
                torch.cuda.current_stream(dev).synchronize()  # a lone copy is complete on return too
        return DeviceImages(pix, offsets, dims)
    for j, a in prepared:
        if a is not None and (a.ndim != 3 or a.shape[2] != 3):
            raise ValueError(f"expected HxWx3 u8 images, got shape {a.shape}")
    dims = np.array([j[2] if j is not None else a.shape[:2] for j, a in prepared], dtype=np.int64).reshape(n, 2)
    sizes = dims[:, 0] * dims[:, 1] * 3
    host = [i for i in range(n) if prepared[i][1] is not None]
    jpeg = [i for i in range(n) if prepared[i][0] is not None and prepared[i][0][0] == "jpeg"]
    png = [i for i in range(n) if prepared[i][0] is not None and prepared[i][0][0] == "png"]
    offsets = np.zeros(n, dtype=np.int64)  # host-decoded images first (one contiguous copy), then K13's, K14's
    pos = 0
    for i in host + jpeg + png:
        offsets[i] = pos
        pos += int(sizes[i])
    pix = torch.empty(max(pos, 1), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        if host:
            nh = int(sum(int(sizes[i]) for i in host))
            staging = torch.empty(nh, dtype=torch.uint8, pin_memory=True)
            sv = staging.numpy()
            for i in host:
                sv[offsets[i]:offsets[i] + sizes[i]] = np.ascontiguousarray(prepared[i][1], dtype=np.uint8).reshape(-1)
            pix[:nh].copy_(staging, non_blocking=True)
        if jpeg:
            files = (ctypes.c_char_p * len(jpeg))(*[prepared[i][0][1] for i in jpeg])
            fsz = np.array([len(prepared[i][0][1]) for i in jpeg], dtype=np.int64)
            offs = np.ascontiguousarray(offsets[jpeg])
            _native.call("mrag_jpeg_decode", ctypes.cast(files, ctypes.c_void_p), fsz.ctypes.data, len(jpeg),
                         pix.data_ptr(), offs.ctypes.data, device, stream)
        if png:
            raws = (ctypes.c_void_p * len(png))(*[prepared[i][0][1].ctypes.data for i in png])
            pdims = np.array([[prepared[i][0][2][1], prepared[i][0][2][0], prepared[i][0][3]] for i in png],
                             dtype=np.int32)
            offs = np.ascontiguousarray(offsets[png])
            _native.call("mrag_png_unfilter", ctypes.cast(raws, ctypes.c_void_p), pdims.ctypes.data, len(png),
                         pix.data_ptr(), offs.ctypes.data, device, stream)
        if host and not (jpeg or png):  # K13 / K14 return complete; a lone copy must be too
            torch.cuda.current_stream(dev).synchronize()
    return DeviceImages(pix, offsets, dims)


def resize_images(imgs: DeviceImages, start: int = 0, count: int = -1, device: int = 0, size: int = SIZE):
    """K0 resize + centre crop of images [start, start + count) of a decoded group -> u8
    [count, size, size, 3] CUDA tensor."""
    import torch

    from app import _native

    stop = len(imgs) if count < 0 else min(len(imgs), start + count)
    n = max(0, stop - start)
    dev = torch.device("cuda", device)
    out = torch.empty((n, size, size, 3), dtype=torch.uint8, device=dev)
    if n == 0:
        return out
    offsets = np.ascontiguousarray(imgs.offsets[start:stop], dtype=np.int64)
    widths = np.ascontiguousarray(imgs.dims[start:stop, 1], dtype=np.int32)
    heights = np.ascontiguousarray(imgs.dims[start:stop, 0], dtype=np.int32)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _native.call("mrag_image_resize_crop", imgs.pix.data_ptr(),
                     offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                     widths.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                     heights.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n, size, out.data_ptr(), stream)
    return out


def upload_resize(prepared: list, device: int = 0, size: int = SIZE):
    """The whole device half: decode (K13, K14, host copies), then K0 -> u8 [n, size, size, 3]."""
    return resize_images(upload_decode(prepared, device=device), device=device, size=size)


def load_batch_device(items: Sequence[Union[str, Path, Image.Image]], device: int = 0):
    """Decode (baseline JPEG on the GPU, PNG reconstruction on the GPU after a host inflate, the rest
    on the host thread pool), resize + crop on the GPU: u8 [n, 224, 224, 3] CUDA tensor."""
    return upload_resize(prepare_batch(items), device=device)
