#!/usr/bin/env python3
"""The library host half (NativePrepared over groups of 256 of the bench's ingest files) alone and
embed_images_batch whole, at 8 / 16 / 24 / 32 host threads in mrag_files_prepare, interleaved
twice: img/s of each, and the device decode (K13 + K14) alone for scale."""
import json, os, shutil, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from app.encoders import preprocess as pp  # noqa: E402
from app.ml import embeddings as emb  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
d = tempfile.mkdtemp(prefix="mrag_native_thr_")
base = pp.decode_workers
try:
    paths = bench._write_images(d, n)
    emb.embed_images_batch(paths[:256])
    ref = emb.embed_images_batch(paths)
    torch.cuda.synchronize()
    groups = [paths[i:i + 256] for i in range(0, n, 256)]
    prepared = [pp.NativePrepared(g) for g in groups]
    t0 = time.perf_counter()
    for _ in range(3):
        imgs = [pp.upload_decode(p) for p in prepared]
    torch.cuda.synchronize()
    print(json.dumps({"stage": "k13_k14_device", "images_per_s": round(3 * n / (time.perf_counter() - t0), 1),
                      "default_threads": base()}), flush=True)
    del imgs, prepared
    for rnd in range(2):
        for th in (8, 16, 24, 32):
            pp.decode_workers = lambda th=th: th
            t0 = time.perf_counter()
            for g in groups:
                pp.NativePrepared(g)
            t_prep = time.perf_counter() - t0
            t0 = time.perf_counter()
            out = emb.embed_images_batch(paths)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            print(json.dumps({"round": rnd, "threads": th, "host_half_images_per_s": round(n / t_prep, 1),
                              "ingest_images_per_s": round(n / t, 1), "equal_rows": bool(np.array_equal(out, ref))}),
                  flush=True)
finally:
    pp.decode_workers = base
    shutil.rmtree(d, ignore_errors=True)
