"""K7 v5 isolation: top-1 mismatches against the oracle per (dim, n, data) with the row's
position in its 48-row tile, so a staging/masking fault shows up as a row-position pattern."""
import os
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
sys.path.insert(0, "multimodal-rag-for-image-text-search_amd")
from _data import clustered_corpus, unit_rows  # noqa: E402
from oracle.knn import flat_cosine_topk  # noqa: E402

import torch  # noqa: E402,F401
from app.vector_store import FlatIndex  # noqa: E402

for d, n, kind in [(128, 270_000, "clus"), (256, 270_000, "clus"), (512, 270_000, "clus"), (128, 30_000, "clus")]:
    x = unit_rows(n, d, 3) if kind == "rand" else clustered_corpus(n, d, 11, n_clusters=64, spread=0.05, dup_frac=0.05)
    q = np.random.default_rng(5).standard_normal((1000, d)).astype(np.float32)
    ix = FlatIndex(d)
    ix.add(x)
    s, r = ix.search(q, 1)
    stats = ix.last_stats()
    os_, or_ = flat_cosine_topk(x, np.zeros(n), q, 1)
    bad = np.nonzero(r[:, 0] != or_[:, 0])[0]
    msg = f"d={d} n={n} {kind}: bad={len(bad)} stats={stats}"
    if len(bad):
        tr = or_[bad, 0]
        msg += f" true%48 hist={np.bincount(tr % 48, minlength=48).tolist()} got%48={np.bincount(r[bad, 0] % 48, minlength=48).tolist()}"
        msg += f" true tiles mod 8={np.bincount((tr // 48) % 8, minlength=8).tolist()}"
        xn = x / np.maximum(np.linalg.norm(x, axis=1, keepdims=True), 1e-12)
        qn = q / np.linalg.norm(q, axis=1, keepdims=True)
        for b in bad[:12]:
            g, t = r[b, 0], or_[b, 0]
            msg += (f"\n  q{b}: got {g} (gpu {s[b,0]:.5f} exact {float(xn[g] @ qn[b]):.5f}) true {t} ({os_[b,0]:.5f})"
                    f" diff {int(g) - int(t)} dup={bool(np.array_equal(x[g], x[t]))}")
    print(msg, flush=True)
