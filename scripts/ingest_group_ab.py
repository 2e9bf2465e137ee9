#!/usr/bin/env python3
"""embed_images_batch over the bench's ingest files (bench._write_images) with 1, 2 and 4 encoder
batches per K13 decode group, interleaved twice; img/s and host CPU seconds per call."""
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from app.ml import embeddings as emb  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
d = tempfile.mkdtemp(prefix="mrag_ingest_ab_")
try:
    paths = bench._write_images(d, n)
    emb.embed_images_batch(paths[:256])
    torch.cuda.synchronize()
    for rnd in range(2):
        for g in (4, 2, 1):
            emb._DECODE_GROUP_BATCHES = g
            c0 = os.times()
            t0 = time.perf_counter()
            emb.embed_images_batch(paths)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            c1 = os.times()
            print(json.dumps({"round": rnd, "group_batches": g, "images_per_s": round(n / t, 1),
                              "wall_s": round(t, 3), "cpu_s": round((c1.user - c0.user) + (c1.system - c0.system), 2)}),
                  flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
