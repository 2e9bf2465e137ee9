"""Batched retrieval on the GPU engine (the reference's empty ``app/retrieval``).

The reference answers one query per call (``retrieve_text`` / ``retrieve_images``,
app/ml/retrieve.py:41-100), each a separate scan. These entry points take many
queries at once: one encoder batch per tower, ONE flat-index launch per modality for the
whole batch, ONE cross-encoder batch for every query's rerank pairs (when rerank is on and
a reranker loads, as ``retrieve``), then the same per-query post-processing and the
reference's z-score fusion. Results for query i equal ``retrieve_text(user, q_i)`` /
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
        table._sync()  # replay what any process committed since the last call
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


_BRANCH_POOL = None


def _branch_pool():
    """One worker thread for the image branch of ``retrieve_batch`` (created on first use)."""
    global _BRANCH_POOL
    if _BRANCH_POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _BRANCH_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mrag-image-branch")
    return _BRANCH_POOL


def retrieve_batch(user_id: str, queries: Sequence[str], top_k_text: Optional[int] = None,
                   top_k_image: Optional[int] = None, rerank: Optional[bool] = None) -> List[List[Dict[str, Any]]]:
    """Fused text+image results per query, batched end to end = ``retrieve(user_id, q)``
    (app/ml/retrieve.py:103-117) for every q. ``rerank`` defaults to RERANK_ENABLED; the
    cross-encoder is ``retrieve._get_cross_encoder()`` (False -> no rerank, as retrieve).

    The image branch (CLIP text tower -> image search) runs in a worker thread beside the text
    branch (MiniLM -> text search): each native call returns to its own thread only, so the two
    branches' GPU work overlaps (the config-5 bench leg measures the same arrangement)."""
    from app.ml import retrieve as r
    from app.ml.embeddings import _ensure_clip, _ensure_processor, _normalize, _to_numpy

    tk = top_k_text or settings.retrieval.index_topk_text
    ik = top_k_image or settings.retrieval.index_topk_image
    qs = list(queries)
    if not qs:
        return []

    def image_branch():
        proc, model = _ensure_processor(), _ensure_clip()
        img_vecs = _normalize(_to_numpy(model.get_text_features(**proc(text=qs))))
        blank = np.array([not q.strip() for q in qs])
        img_vecs[blank] = 0.0
        return search_batch("image", user_id, img_vecs, ik)

    fut = _branch_pool().submit(image_branch)
    try:
        text_vecs = r.embed_text_batch(qs)
        th = search_batch("text", user_id, text_vecs, tk)
    except BaseException as text_err:
        # the text branch's error is the one raised; wait for the image branch first (it shares
        # the GPU and the store) and chain its error, if any, instead of replacing this one
        img_err = fut.exception()
        if img_err is not None and text_err.__cause__ is None:
            raise text_err from img_err
        raise
    ih = fut.result()  # re-raises the image branch's error
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
        out.append((texts, images))
    use_rr = settings.retrieval.use_rerank if rerank is None else bool(rerank)
    ce = r._get_cross_encoder() if use_rr else None
    if ce:
        pairs, spans = [], []
        for i, (texts, _) in enumerate(out):
            p = r._rerank_pairs(qs[i], texts) if texts else []
            spans.append((len(pairs), len(p)))
            pairs.extend(p)
        scores = np.asarray(ce.predict(pairs, batch_size=256)).reshape(-1) if pairs else np.empty(0)
        out = [(r._apply_rerank(texts, scores[a:a + n]) if n else texts, images)
               for (texts, images), (a, n) in zip(out, spans)]
    return [r._fuse_results(texts, images) for texts, images in out]


def _z_rows(scores64: np.ndarray, valid: np.ndarray) -> np.ndarray:
    """``_z_scores`` (app/ml/retrieve.py:185-194) of every row's valid prefix: float32 mean
    and std of the list (numpy's own reductions, rows of equal length grouped so each group
    is one contiguous 2-D reduction = the per-list 1-D one), then (v - mean) / std in f64
    on the f64 score; a zero std gives zeros."""
    q, k = scores64.shape
    z = np.zeros((q, k), dtype=np.float64)
    counts = valid.sum(axis=1)
    for n in np.unique(counts):
        if n == 0:
            continue
        rows = np.nonzero(counts == n)[0]
        v = scores64[rows, :n]
        arr = v.astype(np.float32)
        mean = arr.mean(axis=1).astype(np.float64)[:, None]
        std = arr.std(axis=1).astype(np.float64)[:, None]
        with np.errstate(divide="ignore", invalid="ignore"):
            zz = np.where(std == 0, 0.0, (v - mean) / np.where(std == 0, 1.0, std))
        z[rows, :n] = zz
    return z


def fuse_scores(text_scores, image_scores, final_n: Optional[int] = None):
    """Vectorised ``_fuse_results`` with rerank off (app/ml/retrieve.py:158-182) for a batch
    of queries, on the raw per-query hit scores the flat index returns.

    ``text_scores`` f32 [Q, kt], ``image_scores`` f32 [Q, ki] in hit order (score desc),
    ``-inf`` marking missing hits (fewer matches than k). Each hit's score is first taken
    through the drop-in store's path (``1 - f32(1 - s)``, the f64 value a caller sees).
    Returns (``pick`` int64 [Q, final_n]: index into the concatenated text+image hit list,
    -1 past the end; ``combined`` f64 [Q, final_n]), ordered as the reference's stable
    descending sort of text items then image items."""
    n_final = int(final_n or settings.retrieval.final_n)
    ts = np.asarray(text_scores, dtype=np.float32)
    im = np.asarray(image_scores, dtype=np.float32)
    if ts.ndim != 2 or im.ndim != 2 or ts.shape[0] != im.shape[0]:
        raise ValueError("expected [Q, kt] and [Q, ki] score arrays")
    one = np.float32(1.0)

    def caller_scores(s):
        valid = np.isfinite(s)
        s64 = 1.0 - (one - np.where(valid, s, np.float32(0))).astype(np.float64)
        return s64, valid

    t64, tv = caller_scores(ts)
    i64, iv = caller_scores(im)
    comb = np.concatenate([_z_rows(t64, tv), _z_rows(i64, iv)], axis=1)
    valid = np.concatenate([tv, iv], axis=1)
    key = np.where(valid, -comb, np.inf)  # stable ascending on -score == stable descending sort
    order = np.argsort(key, axis=1, kind="stable")[:, :n_final]
    pick = np.where(np.take_along_axis(valid, order, axis=1), order, -1).astype(np.int64)
    combined = np.where(pick >= 0, np.take_along_axis(comb, order, axis=1), np.nan)
    if pick.shape[1] < n_final:  # fewer slots than final_n: pad ([Q, final_n] like K12)
        pad = n_final - pick.shape[1]
        pick = np.pad(pick, ((0, 0), (0, pad)), constant_values=-1)
        combined = np.pad(combined, ((0, 0), (0, pad)), constant_values=np.nan)
    return pick, combined


def fuse_scores_gpu(text_scores, image_scores, final_n: Optional[int] = None):
    """``fuse_scores`` on the GPU (K12, ``mrag_fuse_scores``): torch CUDA f32 ``[Q, kt]`` /
    ``[Q, ki]`` hit scores (as ``FlatIndex.search`` returns them) -> (``pick`` int64 CUDA
    ``[Q, final_n]``, ``combined`` f64 CUDA ``[Q, final_n]``), bit-identical to ``fuse_scores``
    and asynchronous on torch's current stream."""
    import torch

    from app import _native

    n_final = int(final_n or settings.retrieval.final_n)
    ts = text_scores.detach().to(torch.float32).contiguous()
    im = image_scores.detach().to(torch.float32).contiguous()
    if ts.ndim != 2 or im.ndim != 2 or ts.shape[0] != im.shape[0] or ts.device != im.device:
        raise ValueError("expected [Q, kt] and [Q, ki] CUDA score tensors on one device")
    q = ts.shape[0]
    pick = torch.empty((q, n_final), dtype=torch.int64, device=ts.device)
    comb = torch.empty((q, n_final), dtype=torch.float64, device=ts.device)
    stream = torch.cuda.current_stream(ts.device).cuda_stream
    _native.call("mrag_fuse_scores", ts.data_ptr(), ts.shape[1], im.data_ptr(), im.shape[1], q, n_final,
                 pick.data_ptr(), comb.data_ptr(), stream)
    return pick, comb


__all__ = ["search_batch", "retrieve_batch", "fuse_scores", "fuse_scores_gpu"]
