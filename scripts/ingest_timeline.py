#!/usr/bin/env python3
"""Where embed_images_batch's time went with its two-stage loop (host prepare of batch i + 1 on a
worker while the calling thread decodes, resizes and encodes batch i; the loop before the decode
moved to its own thread): the bench's ingest files, the calling thread's time split into waiting
for the prepared batch, K13 / K14 decode, K0 resize and the ViT (each synchronous)."""
import json
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from app.ml import embeddings as emb  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
d = tempfile.mkdtemp(prefix="mrag_ingest_tl_")
try:
    paths = bench._write_images(d, n)
    emb.embed_images_batch(paths[:256])
    model, proc = emb._ensure_clip(), emb._ensure_processor()
    for rnd in range(3):
        torch.cuda.synchronize()
        t = {"wait_prepared": 0.0, "decode_k13_k14": 0.0, "resize_k0": 0.0, "vit": 0.0}
        t0 = time.perf_counter()
        starts = list(range(0, n, 256))
        with ThreadPoolExecutor(max_workers=1) as ahead:
            nxt = ahead.submit(proc.decode, paths[0:256])
            for i, s in enumerate(starts):
                a = time.perf_counter()
                prepared = nxt.result()
                b = time.perf_counter()
                if i + 1 < len(starts):
                    nxt = ahead.submit(proc.decode, paths[starts[i + 1]:starts[i + 1] + 256])
                imgs = proc.decode_device(prepared)
                c = time.perf_counter()
                inputs = proc.from_device(imgs, 0, 256)
                torch.cuda.synchronize()
                e = time.perf_counter()
                emb._to_numpy(model.get_image_features(**emb._kwargs(inputs)))
                f = time.perf_counter()
                t["wait_prepared"] += b - a
                t["decode_k13_k14"] += c - b
                t["resize_k0"] += e - c
                t["vit"] += f - e
        wall = time.perf_counter() - t0
        print(json.dumps({"round": rnd, "images_per_s": round(n / wall, 1), "wall_ms": round(wall * 1e3, 1),
                          **{k: round(v * 1e3, 1) for k, v in t.items()}}), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
