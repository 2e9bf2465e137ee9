#!/usr/bin/env python3
"""embed_images_batch over the bench's ingest files, three host halves interleaved three times:
per file on the decode pool two groups ahead (embeddings._PREP_PER_FILE), one prepare_batch per
group through the library (preprocess._NATIVE_FILES: mrag_files_prepare, no interpreter lock
between files), and one prepare_batch per group on the pool. img/s and host CPU s per call."""
import json, os, shutil, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from app.encoders import preprocess as pp  # noqa: E402
from app.ml import embeddings as emb  # noqa: E402

MODES = {"per_file": (True, True), "native_group": (False, True), "pool_group": (False, False)}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
d = tempfile.mkdtemp(prefix="mrag_native_ab_")
try:
    paths = bench._write_images(d, n)
    emb.embed_images_batch(paths[:256])
    ref = emb.embed_images_batch(paths)
    torch.cuda.synchronize()
    for rnd in range(3):
        for mode, (per_file, native) in MODES.items():
            emb._PREP_PER_FILE, pp._NATIVE_FILES = per_file, native
            c0, t0 = os.times(), time.perf_counter()
            out = emb.embed_images_batch(paths)
            torch.cuda.synchronize()
            t, c1 = time.perf_counter() - t0, os.times()
            print(json.dumps({"round": rnd, "mode": mode, "images_per_s": round(n / t, 1),
                              "cpu_s": round(c1.user - c0.user + c1.system - c0.system, 2),
                              "equal_rows": bool(np.array_equal(out, ref))}), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
