"""Deterministic synthetic inputs shared by tests, golden generator and bench.

Everything is a pure function of (seed, shape) through numpy's PCG64, so the GPU box
regenerates exactly the corpora the golden fixtures were computed on (each fixture
also stores a sha256 of its inputs to prove it).
"""
from __future__ import annotations

import hashlib

import numpy as np


def unit_rows(n: int, d: int, seed) -> np.ndarray:
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, d), dtype=np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x


def clustered_corpus(n: int, d: int, seed, n_clusters: int = 16, spread: float = 0.02,
                     dup_frac: float = 0.05) -> np.ndarray:
    """Rows = cluster centre + small noise, plus exact duplicate rows (ties) and a
    few zero rows — the shapes real CLIP/MiniLM corpora have (near-duplicate frames,
    re-ingested chunks)."""
    rng = np.random.default_rng(seed)
    centres = rng.standard_normal((n_clusters, d)).astype(np.float32)
    assign = rng.integers(0, n_clusters, size=n)
    x = centres[assign] + spread * rng.standard_normal((n, d)).astype(np.float32)
    ndup = int(n * dup_frac)
    if ndup:
        src = rng.integers(0, n, size=ndup)
        dst = rng.integers(0, n, size=ndup)
        x[dst] = x[src]
    x[rng.integers(0, n, size=max(1, n // 1000))] = 0.0
    return x.astype(np.float32)


def labels_for(n: int, n_users: int, seed) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.integers(0, n_users, size=n).astype(np.int32)


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
