"""The reference's two normalisers, restated (test oracle only).

* ``app/ml/embeddings.py:46-49``: rows / np.linalg.norm(axis=1), zero norms -> 1.
* ``app/storage/lancedb_store.py:63-69``: one vector, f32, / np.linalg.norm; returned
  unchanged when the norm is <= 0.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def embeddings_normalize(x: np.ndarray) -> np.ndarray:
    norms = np.linalg.norm(x, axis=1, keepdims=True)
    norms[norms == 0] = 1.0
    return x / norms


def store_normalize(vector: Sequence[float]) -> List[float]:
    arr = np.asarray(vector, dtype=np.float32)
    norm = np.linalg.norm(arr)
    if norm <= 0:
        return arr.tolist()
    return (arr / norm).tolist()
