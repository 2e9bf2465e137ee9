"""Position / batch independence of the encoders at reduced depth: a sequence alone vs inside a
padded batch and two copies of one sequence at different row offsets, per number of layers
(which layer first breaks it), and the same batch twice (determinism). Written to localise the
round-4 LayerNorm-fold experiment's ulp-level position dependence (notes/gemm_experiments.md)."""
import dataclasses
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT, os.path.join(ROOT, "tests")]
from app.encoders import CLIP_TEXT_B32, CLIP_VISION_B32, MINILM_L6, GpuEncoder  # noqa: E402


def text_case(cfg, L, lens, normalize=False):
    c = dataclasses.replace(cfg, layers=L)
    T = max(lens)
    rng = np.random.default_rng(17)
    ids = np.zeros((len(lens), T), np.int32)
    mask = np.zeros((len(lens), T), np.int32)
    for i, n in enumerate(lens):
        if cfg.kind == 3:
            ids[i, :n] = rng.integers(1000, 30000, n)
            ids[i, 0], ids[i, n - 1] = 101, 102
        else:
            ids[i, :n] = rng.integers(1, 49405, n)
            ids[i, 0], ids[i, n - 1] = 49406, 49407
            ids[i, n:] = 49407
        mask[i, :n] = 1
    enc = GpuEncoder(c)
    b1 = enc.embed_tokens(ids, mask, normalize=normalize)
    b2 = enc.embed_tokens(ids, mask, normalize=normalize)
    out = {"tower": cfg.kind, "layers": L, "lens": lens, "deterministic": bool(np.array_equal(b1, b2))}
    for i, n in enumerate(lens):
        a = enc.embed_tokens(ids[i:i + 1, :n], mask[i:i + 1, :n], normalize=normalize)
        out[f"seq{i}_maxdiff"] = float(np.abs(a[0] - b1[i]).max())
    # the same sequence at row offsets 0 and T (two copies)
    two = enc.embed_tokens(np.concatenate([ids[1:2], ids[1:2]]), np.concatenate([mask[1:2], mask[1:2]]),
                           normalize=normalize)
    out["copy_rows_maxdiff"] = float(np.abs(two[0] - two[1]).max())
    print(json.dumps(out), flush=True)


def image_case(L):
    c = dataclasses.replace(CLIP_VISION_B32, layers=L)
    g = np.load(os.path.join(ROOT, "tests", "golden", "golden_clip_image.npz"))
    imgs = np.concatenate([g["images_u8"]] * 4)
    n0 = len(g["images_u8"])
    enc = GpuEncoder(c)
    b = enc.embed_images(imgs[:n0], normalize=False)
    s = enc.embed_images(imgs[:2 * n0], normalize=False)
    print(json.dumps({"tower": 1, "layers": L, "n0": n0, "first": float(np.abs(s[:n0] - b).max()),
                      "second": float(np.abs(s[n0:2 * n0] - b).max())}), flush=True)


for L in (1, 2, 3):
    text_case(CLIP_TEXT_B32, L, [3, 16, 40])
for L in (1, 2):
    text_case(MINILM_L6, L, [3, 16, 40, 130])
for L in (1, 2, 3):
    image_case(L)
