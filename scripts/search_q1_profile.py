#!/usr/bin/env python3
"""Where a one-query drop-in search spends its time (the reference's per-query pattern):
LanceDBStore.search_text over a 1M x 384 table (one user) vs FlatIndex.search on the same host
query, then cProfile of the store call (tottime, top 25)."""
import cProfile
import os
import pstats
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
os.environ["MRAG_STORE_PERSIST"] = "0"

import numpy as np  # noqa: E402
import torch  # noqa: E402

from app.storage.lancedb_store import LanceDBStore  # noqa: E402
from app.vector_store import FlatIndex  # noqa: E402

N, D, K, REPS = 1 << 20, 384, 50, 300
dev = torch.device("cuda", 0)
x = torch.randn((N, D), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
ix = FlatIndex(D)
ix.add(x)
del x
store = LanceDBStore(tempfile.mkdtemp(prefix="mrag_q1prof_"))
t = store._text_table
t.index, t.dim = ix, D
t.chunk_ids = [f"t{i % 65536}" for i in range(N)]
t.metas = ['{"page_no": 1}'] * N
t.labels = {"u0": 0}
q = np.random.default_rng(2).standard_normal(D).astype(np.float32)
ql = q.tolist()


def timed(f, n=REPS):
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


print("flatindex_search_host_q1_ms", round(timed(lambda: ix.search(q[None, :], K, label=0)), 4))
print("store_search_text_ms", round(timed(lambda: store.search_text("u0", ql, K)), 4))
pr = cProfile.Profile()
pr.enable()
for _ in range(REPS):
    store.search_text("u0", ql, K)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
