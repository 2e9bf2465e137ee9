"""CLIP ViT-B/32 image-tower bench on one GPU (config 2), for profiling runs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
from app.encoders import bench_clip_images  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
inflight = int(sys.argv[2]) if len(sys.argv) > 2 else 2
print(json.dumps(bench_clip_images(steps=steps, warmup=2, inflight=inflight)))
