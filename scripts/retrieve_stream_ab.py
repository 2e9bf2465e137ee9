#!/usr/bin/env python3
"""The per-query retrieve leg (bench.retrieve_pattern_leg) with the CLIP-text query encode's
stream varied, arms interleaved: "pool" = a side stream from torch's pool (the round-5
form), "prio" = a high-priority side stream, "same" = the worker thread encodes on its current
stream (host overlap only; the form shipped since session 34).
GPU_MAX_HW_QUEUES comes from the environment (bench's import sets 8 unless it is set)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from app.cache import clear_all_caches  # noqa: E402
from app.ml import retrieve as rmod  # noqa: E402
from app.vector_store import FlatIndex  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn((bench.ROWS_PER_GPU, bench.DIM), generator=g, device=dev)
x = x / x.norm(dim=1, keepdim=True)
ix = FlatIndex(bench.DIM)
ix.add(x)
del x
own = rmod._image_query_in_worker
pool_s = torch.cuda.Stream(device=dev)
prio_s = torch.cuda.Stream(device=dev, priority=-1)
side = {}


def on_side_stream(query, d):
    with torch.cuda.device(d), torch.cuda.stream(side[0]):
        return rmod.embed_query_for_images(query)


ARMS = ("pool", "prio", "same")
for r in range(-1, rounds):  # round -1: every arm once, not reported (first-use costs)
    for arm in ARMS[r % 3:] + ARMS[:r % 3] if r >= 0 else ARMS:
        if arm in ("pool", "prio"):
            side[0] = pool_s if arm == "pool" else prio_s
            rmod._image_query_in_worker = on_side_stream
        else:
            rmod._image_query_in_worker = own
        clear_all_caches()
        out = bench.retrieve_pattern_leg(ix, reps=100)
        if r < 0:
            continue
        print(json.dumps({"queues": os.environ.get("GPU_MAX_HW_QUEUES"), "arm": arm, "round": r,
                          "retrieve_text_ms": out["retrieve_text_ms"], "retrieve_images_ms": out["retrieve_images_ms"],
                          "query_pair_ms": out["query_pair_ms"]}), flush=True)
rmod._image_query_in_worker = own
