#!/usr/bin/env python3
"""Small token batches (the reference's one query per retrieve call): per-call wall time of
mrag_encoder_embed_tokens with host pointers (hipGraph replay for <= 2048 tokens) against device
pointers (direct launches; torch tensors in and out, synchronised), MiniLM and CLIP text, synthetic
weights. One JSON line per (tower, B, T)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from app.encoders import CLIP_TEXT_B32, MINILM_L6, GpuEncoder  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
rng = np.random.default_rng(5)
for name, cfg, lo, hi, bos, eos in (("minilm", MINILM_L6, 1000, 30000, 101, 102),
                                    ("clip_text", CLIP_TEXT_B32, 1, 49405, 49406, 49407)):
    enc = GpuEncoder(cfg)
    for b, t in ((1, 12), (1, 32), (4, 16), (16, 32), (32, 64)):
        ids = rng.integers(lo, hi, (b, t)).astype(np.int32)
        ids[:, 0], ids[:, -1] = bos, eos
        mask = np.ones_like(ids)
        res = {"tower": name, "B": b, "T": t}
        for mode in ("host_graph", "device_direct"):
            if mode == "host_graph":
                def call():
                    return enc.embed_tokens(ids, mask)
            else:
                di, dm = torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev)

                def call():
                    out = enc.embed_tokens(di, dm)
                    return out.cpu().numpy()  # the caller's read-back (synchronises)
            for _ in range(20):
                call()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                call()
            torch.cuda.synchronize()
            res[mode + "_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
        print(json.dumps(res), flush=True)
