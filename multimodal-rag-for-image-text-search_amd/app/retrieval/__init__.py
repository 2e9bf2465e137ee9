"""Batched retrieval on the GPU engine (the reference's empty ``app/retrieval``).

The reference answers one query per call (``retrieve_text`` / ``retrieve_images``,
app/ml/retrieve.py:41-100), each a separate scan. These entry points take many
queries at once: one encoder batch per tower and ONE flat-index launch per modality
for the whole batch, then the same per-query post-processing and the reference's
z-score fusion (rerank off). Results for query i equal ``retrieve_text(user, q_i)`` /
``retrieve_images`` / ``retrieve`` without the cache.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from app.settings import settings


def _store():
    from app.ml import retrieve as r

    return r._LANCEDB_STORE, r._METADATA_STORE


def search_batch(modality: str, user_id: str, query_vecs: np.ndarray, top_k: int) -> List[List[Dict[str, Any]]]:
    """Raw hits ({chunk_id, score, meta}) for every row of ``query_vecs``, one GPU launch."""
    store, _ = _store()
    table = store._text_table if modality == "text" else store._image_table
    q = np.asarray(query_vecs, dtype=np.float32)
    if q.ndim == 1:
        q = q[None, :]
    norms = np.linalg.norm(q, axis=1, keepdims=True)
    q = np.where(norms > 0, q / np.where(norms > 0, norms, 1), q).astype(np.float32)
    with table.lock:
        table._load()  # replay a persisted table on first use in this process
        label = table.labels.get(user_id)
        if table.index is None or label is None:
            return [[] for _ in range(len(q))]
        s, r = table.index.search(q, max(int(top_k), 1), label=label)
        out = []
        for i in range(len(q)):
            rows = [{"chunk_id": table.chunk_ids[row], "_distance": np.float32(1.0) - np.float32(sc),
                     "meta": table.metas[row]} for sc, row in zip(s[i], r[i]) if row >= 0]
            out.append(store._format_results(rows))
        return out


def retrieve_batch(user_id: str, queries: Sequence[str], top_k_text: Optional[int] = None,
                   top_k_image: Optional[int] = None) -> List[List[Dict[str, Any]]]:
    """Fused text+image results per query (rerank off), batched end to end."""
    from app.ml import retrieve as r
    from app.ml.embeddings import _ensure_clip, _ensure_processor, _normalize, _to_numpy

    tk = top_k_text or settings.retrieval.index_topk_text
    ik = top_k_image or settings.retrieval.index_topk_image
    qs = list(queries)
    if not qs:
        return []
    text_vecs = r.embed_text_batch(qs)
    proc, model = _ensure_processor(), _ensure_clip()
    img_vecs = _normalize(_to_numpy(model.get_text_features(**proc(text=qs))))
    blank = np.array([not q.strip() for q in qs])
    img_vecs[blank] = 0.0
    th = search_batch("text", user_id, text_vecs, tk)
    ih = search_batch("image", user_id, img_vecs, ik)
    _, meta = _store()
    out = []
    for i in range(len(qs)):
        texts, images = [], []
        for e in th[i]:
            c = meta.get_chunk(e["chunk_id"])
            if c and c.text:
                texts.append({"chunk_id": c.id, "modality": "text", "score": float(e["score"]),
                              "metadata": r._prepare_metadata(c), "text": c.text})
        for e in ih[i]:
            c = meta.get_chunk(e["chunk_id"])
            if c:
                images.append({"chunk_id": c.id, "modality": "image", "score": float(e["score"]),
                               "metadata": r._prepare_metadata(c), "text": None})
        out.append(r._fuse_results(texts, images))
    return out


__all__ = ["search_batch", "retrieve_batch"]
