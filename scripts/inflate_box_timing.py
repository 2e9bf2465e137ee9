#!/usr/bin/env python3
"""The PNG host half on this machine: per-PNG times of the library's probe + inflate
(mrag_png_probe / mrag_png_inflate) against Python's zlib on the same IDAT streams, and
prepare_batch over the bench's ingest files (one thread and the decode pool)."""
import ctypes, json, os, shutil, struct, sys, tempfile, time, zlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from app import _native  # noqa: E402
from app.encoders.preprocess import _prepare_one, prepare_batch  # noqa: E402

lib = _native.load()
d = tempfile.mkdtemp()
try:
    paths = bench._write_images(d, 512)
    pngs = [p for p in paths if p.endswith(".png")]
    files = [open(p, "rb").read() for p in pngs]
    res = {"pngs": len(files), "cpus": os.cpu_count()}
    w, h, n, bpp = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
    outs = []
    for b in files:
        assert lib.mrag_png_probe(b, len(b), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n)) == 1
        outs.append(np.empty(n.value, np.uint8))
    for rep in range(2):
        t = time.perf_counter()
        for b, o in zip(files, outs):
            assert lib.mrag_png_inflate(b, len(b), o.ctypes.data, o.size, ctypes.byref(bpp)) == 1
        res["library_inflate_ms"] = round((time.perf_counter() - t) / len(files) * 1e3, 3)
    t = time.perf_counter()
    for b in files:
        lib.mrag_png_probe(b, len(b), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n))
    res["probe_ms"] = round((time.perf_counter() - t) / len(files) * 1e3, 3)
    streams = []
    for b in files:
        i, z = 8, b""
        while i < len(b):
            ln, = struct.unpack(">I", b[i:i + 4])
            if b[i + 4:i + 8] == b"IDAT":
                z += b[i + 8:i + 8 + ln]
            i += 12 + ln
        streams.append(z)
    t = time.perf_counter()
    for z in streams:
        zlib.decompress(z)
    res["python_zlib_ms"] = round((time.perf_counter() - t) / len(files) * 1e3, 3)
    for rep in range(2):
        t = time.perf_counter()
        for p in paths[:128]:
            _prepare_one(p)
        res["prepare_one_thread_ms_per_file"] = round((time.perf_counter() - t) / 128 * 1e3, 3)
        t = time.perf_counter()
        prepare_batch(paths)
        res["prepare_batch_pool_img_s"] = round(len(paths) / (time.perf_counter() - t), 1)
    print(json.dumps(res), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
