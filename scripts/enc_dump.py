"""Dump CLIP image (B=256), CLIP-text and MiniLM (1000 x 16 tokens) embeddings to an .npz, for
bit-identity A/B checks between kernel variants selected by env: python scripts/enc_dump.py out.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
os.environ.setdefault("MRAG_SYNTHETIC_WEIGHTS", "1")
from app.encoders import CLIP_TEXT_B32, CLIP_VISION_B32, MINILM_L6, GpuEncoder  # noqa: E402

rng = np.random.default_rng(3)
imgs = rng.integers(0, 256, (256, 224, 224, 3), dtype=np.uint8)
ids = rng.integers(1000, 30000, (1000, 16)).astype(np.int32)
ids[:, 0], ids[:, -1] = 101, 102
cids = rng.integers(1, 49405, (1000, 16)).astype(np.int32)
cids[:, 0], cids[:, -1] = 49406, 49407
mask = np.ones_like(ids)
out = {
    "clip_image": GpuEncoder(CLIP_VISION_B32).embed_images(imgs),
    "minilm": GpuEncoder(MINILM_L6).embed_tokens(ids, mask),
    "clip_text": GpuEncoder(CLIP_TEXT_B32).embed_tokens(cids, mask),
}
np.savez(sys.argv[1], **out)
print({k: v.shape for k, v in out.items()})
