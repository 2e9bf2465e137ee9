#!/usr/bin/env python3
"""K7 A/B on the bench's config-3 shard (1M x 512, seed 1000; 1000 queries, seed 1): average
main-scan launch (HIP events in the library) over `steps` one-at-a-time searches, the whole-search
time, a digest of the results (to check variants against each other), and the one-query search
time. Variants are chosen by environment (read once per process), so run one process per arm."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

from app.vector_store import FlatIndex  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn((1 << 20, 512), generator=g, device=dev)
x = x / x.norm(dim=1, keepdim=True)
ix = FlatIndex(512)
ix.add(x)
del x
q = torch.randn((1000, 512), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
s = torch.cuda.Stream(device=dev)
with torch.cuda.stream(s):
    for _ in range(5):
        ix.search(q, 10)
    s.synchronize()
    ix.profile(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        sc, r = ix.search(q, 10)
    s.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ms, n = ix.profile(0)
    digest = hashlib.sha256(r.cpu().numpy().tobytes() + sc.cpu().numpy().tobytes()).hexdigest()[:16]
    unc, _ = ix.last_stats()
    q1 = q[:1].contiguous()
    for _ in range(20):
        ix.search(q1, 10)
    s.synchronize()
    ix.profile(1)
    t0 = time.perf_counter()
    for _ in range(200):
        ix.search(q1, 10)
    s.synchronize()
    dt1 = (time.perf_counter() - t0) / 200
    ms1, n1 = ix.profile(0)
print(json.dumps({"env": {k: os.path.basename(v) for k, v in os.environ.items() if k.startswith("MRAG_")}, "scan_ms": round(ms / n, 4),
                  "search_ms": round(dt * 1e3, 4), "tflops": round(2 * 1000 * (1 << 20) * 512 / (ms / n) / 1e9, 1),
                  "digest": digest, "uncertified": unc, "q1_search_ms": round(dt1 * 1e3, 4),
                  "q1_scan_ms": round(ms1 / n1, 4)}), flush=True)
