#!/usr/bin/env python3
"""K7 main-scan time vs k on the config-5 shard shapes (512k x 384 and 512k x 512, Q = 1000):
how much the group-test fires (more rows pass a lower k-th threshold) cost as k grows.
python scripts/knn_k_sweep.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

from app.vector_store import FlatIndex  # noqa: E402

dev = torch.device("cuda", 0)
for dim in (384, 512):
    g = torch.Generator(device=dev).manual_seed(2000 + dim)
    x = torch.randn((1 << 19, dim), generator=g, device=dev)
    ix = FlatIndex(dim)
    ix.add(x)
    del x
    q = torch.randn((1000, dim), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    for k in [int(v) for v in os.environ.get("KS", "1,6,10,12,16,32,50,64").split(",")]:
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            for _ in range(3):
                ix.search(q, k)
            s.synchronize()
            ix.profile(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                ix.search(q, k)
            e1.record(s)
            s.synchronize()
            ms, n = ix.profile(0)
            unc, _ = ix.last_stats()
        print(json.dumps({"dim": dim, "rows": 1 << 19, "k": k, "scan_ms": round(ms / n, 4),
                          "search_ms": round(e0.elapsed_time(e1) / 10, 4), "uncertified": unc}), flush=True)
