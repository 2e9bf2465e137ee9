#!/usr/bin/env python3
"""The bench's per-query retrieve leg (bench.retrieve_pattern_leg: retrieve_text then
retrieve_images per distinct query over 1M x 384 + 1M x 512 tables) in two arms, interleaved:
"text_first" = this package's retrieve_text (its search and chunk lookup run while the CLIP-text
encode finishes), "embeddings_first" = the reference's order (both query vectors, then the search:
app.ml.retrieve._get_embeddings rebound, which retrieve_text honours as a seam)."""
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
own = rmod._get_embeddings
for r in range(rounds):
    for arm in ("embeddings_first", "text_first"):
        rmod._get_embeddings = (lambda q: own(q)) if arm == "embeddings_first" else own
        clear_all_caches()  # the leg's query strings repeat from call to call
        out = bench.retrieve_pattern_leg(ix, reps=100)
        print(json.dumps({"arm": arm, "round": r, "retrieve_text_ms": out["retrieve_text_ms"],
                          "retrieve_images_ms": out["retrieve_images_ms"], "query_pair_ms": out["query_pair_ms"],
                          "hits": out["hits"]}), flush=True)
rmod._get_embeddings = own
