#!/usr/bin/env python3
"""One small token batch repeated (for a kernel trace): tower (minilm | clip_text), B, T, reps.
Host pointers (the graph-replay path), synthetic weights."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import numpy as np  # noqa: E402

from app.encoders import CLIP_TEXT_B32, MINILM_L6, GpuEncoder  # noqa: E402

tower, b, t, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
cfg = MINILM_L6 if tower == "minilm" else CLIP_TEXT_B32
enc = GpuEncoder(cfg)
rng = np.random.default_rng(1)
ids = rng.integers(1000, 30000, (b, t)).astype(np.int32)
mask = np.ones_like(ids)
for _ in range(reps):
    enc.embed_tokens(ids, mask)
print("done", tower, b, t, reps)
