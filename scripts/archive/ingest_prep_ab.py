#!/usr/bin/env python3
"""embed_images_batch over the bench's ingest files with the host half submitted per file (two
groups ahead, embeddings._PREP_PER_FILE = True) vs one prepare_batch per group (False),
interleaved three times: img/s and host CPU s per call."""
import json, os, shutil, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from app.ml import embeddings as emb  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
d = tempfile.mkdtemp(prefix="mrag_prep_ab_")
try:
    paths = bench._write_images(d, n)
    emb.embed_images_batch(paths[:256])
    ref = emb.embed_images_batch(paths)
    torch.cuda.synchronize()
    for rnd in range(3):
        for per_file in (True, False):
            emb._PREP_PER_FILE = per_file
            c0, t0 = os.times(), time.perf_counter()
            out = emb.embed_images_batch(paths)
            torch.cuda.synchronize()
            t, c1 = time.perf_counter() - t0, os.times()
            print(json.dumps({"round": rnd, "per_file": per_file, "images_per_s": round(n / t, 1),
                              "cpu_s": round(c1.user - c0.user + c1.system - c0.system, 2),
                              "equal_rows": bool(np.array_equal(out, ref))}), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
