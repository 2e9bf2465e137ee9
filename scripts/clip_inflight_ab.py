#!/usr/bin/env python3
"""CLIP ViT-B/32 batch-256 img/s with 2, 3, 4 and 5 batches in flight (bench_clip_images), one
JSON line per setting, interleaved rounds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

from app.encoders import bench_clip_images  # noqa: E402

for rnd in range(2):
    for k in (2, 3, 4, 5):
        r = bench_clip_images(steps=30, warmup=3, inflight=k)
        print(json.dumps({"round": rnd, "inflight": k, "images_per_s": r["value"]}), flush=True)
