#!/usr/bin/env python3
"""The bench's call-pattern leg alone (one query per search over 1M x 512, bench.call_pattern_leg):
prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from app.vector_store import FlatIndex  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn((bench.ROWS_PER_GPU, bench.DIM), generator=g, device=dev)
x = x / x.norm(dim=1, keepdim=True)
ix = FlatIndex(bench.DIM)
ix.add(x)
del x
q = torch.randn((bench.NQ, bench.DIM), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
out = bench.call_pattern_leg(ix, q, reps=int(os.environ.get("REPS", "200")))
print(json.dumps(out), flush=True)
