"""Drop-in for the reference's ``app/ml/retrieve.py``.

``retrieve_text`` / ``retrieve_images`` (:41-100): cache -> query embeddings (both
towers, :120-129) -> GPU flat search -> chunk lookup of the hits (one SQLite statement for all
of them when the store has ``get_chunks``) -> result dicts in score order. ``retrieve`` (:103-117): optional cross-encoder rerank + z-score fusion
(:132-195). Module globals ``_LANCEDB_STORE``, ``_METADATA_STORE``,
``embed_text_batch``, ``embed_query_for_images``, ``_get_cross_encoder``,
``get_index_version`` are looked up at call time (test seams, tests/test_retrieve.py).

The cross-encoder (ms-marco-MiniLM-L-6) runs on the GPU (``CrossEncoderModel``,
MRAG_ENC_BERT_PAIR) when RERANKER_MODEL is a local checkpoint directory or cached hub
snapshot (or MRAG_SYNTHETIC_RERANKER=1: synthetic weights, benchmarks / tests); an
unresolvable name offline returns False exactly as the reference does when the load
fails (:29-38), and rerank is skipped. For many queries at once use
``app.retrieval`` (batched GPU search).
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from app.cache import get_query_embeddings, get_retrieval_results, set_query_embeddings, set_retrieval_results
from app.ml.embeddings import embed_query_for_images, embed_text_batch
from app.ml.index_build import get_index_version
from app.settings import settings
from app.storage.lancedb_store import LanceDBStore
from app.storage.schema import Chunk, MetadataStore

_CROSS_ENCODER = None
_LANCEDB_STORE = LanceDBStore(settings.paths.lancedb_dir)
_METADATA_STORE = MetadataStore(os.path.join(settings.paths.lancedb_dir, "metadata.sqlite3"))


def _normalize_query(query: str) -> str:
    return " ".join(query.strip().lower().split())


def _get_cross_encoder():
    global _CROSS_ENCODER
    if _CROSS_ENCODER is None:
        try:
            from sentence_transformers import CrossEncoder

            _CROSS_ENCODER = CrossEncoder(settings.models.reranker)
        except Exception:
            _CROSS_ENCODER = _gpu_cross_encoder()
    return _CROSS_ENCODER


def _gpu_cross_encoder():
    """The GPU cross-encoder when its weights exist locally (RERANKER_MODEL = a checkpoint
    directory or cached hub snapshot) or synthetic reranker weights are requested
    (MRAG_SYNTHETIC_RERANKER=1, benchmarks / tests); otherwise False — the reference's
    outcome when the hub model cannot load. The reranker has its own opt-in because the
    reference's offline behaviour here is "no rerank", not an error."""
    from app.encoders.weights import resolve_model_dir

    name = settings.models.reranker
    synthetic = os.environ.get("MRAG_SYNTHETIC_RERANKER") == "1"
    if resolve_model_dir(name) is None and not synthetic:
        return False
    try:
        from app.encoders.models import CrossEncoderModel

        return CrossEncoderModel(name, synthetic=synthetic)
    except Exception:
        return False


def _prepare_metadata(chunk: Chunk) -> Dict[str, Any]:
    meta = dict(chunk.meta or {})
    meta.setdefault("doc_id", chunk.document_id)
    meta.setdefault("modality", chunk.modality)
    meta.setdefault("page_no", chunk.page_no)
    meta.setdefault("start_ts", chunk.start_ts)
    meta.setdefault("end_ts", chunk.end_ts)
    meta.setdefault("file_path", chunk.file_path)
    return meta


_QUERY_POOL = None  # one worker thread: the CLIP-text query encode beside the MiniLM one


def _image_query_in_worker(query: str, dev: int) -> np.ndarray:
    """The CLIP-text query encode on the worker thread with that thread's default stream current,
    so the encoder runs it on its handle's own stream (made with the handle; a NULL stream
    argument, include/mrag.h). A B = 1 encode is a chain of launch-bound kernels: what overlaps
    with the caller's MiniLM encode and search is mostly the host side. Run inside a side stream
    from torch's pool instead (the round-5 form) it measured slower and erratic: query pair
    1.76-1.97 ms with 3.7 / 4.5 ms outliers against 1.59-1.72 ms this way
    (`profiles/r6s33_r6s34_retrieve_stream_ab.jsonl`), the pool stream presumably sharing a HIP
    hardware queue (4 per process on the GPU pool's boxes) with a stream the other encode used."""
    import torch

    with torch.cuda.device(dev):
        return embed_query_for_images(query)


def _get_embeddings(query: str) -> Tuple[np.ndarray, np.ndarray]:
    """Both query vectors (reference :120-129: MiniLM, then CLIP text). On a GPU the two B = 1
    encodes are independent chains of small launch-bound kernels, so the CLIP-text one runs in a
    worker thread while this thread runs MiniLM (their host sides overlap; the vectors are the
    same, and an exception from either propagates)."""
    text_vec, finish = _text_embedding_first(query)
    return text_vec, finish()


def _text_embedding_first(query: str):
    """``_get_embeddings`` in two halves: the MiniLM vector now, and ``finish()`` -> the CLIP-text
    vector, which also fills the query-embedding cache exactly as ``_get_embeddings`` does.
    retrieve_text runs its search and chunk lookup between the two (they need only the MiniLM
    vector), while the CLIP-text encode is still running in the worker thread."""
    global _QUERY_POOL
    cached = get_query_embeddings(query)
    if cached:
        return cached[0], (lambda: cached[1])
    import torch

    fut = None
    if torch.cuda.is_available():
        if _QUERY_POOL is None:
            from concurrent.futures import ThreadPoolExecutor

            _QUERY_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mrag-query")
        fut = _QUERY_POOL.submit(_image_query_in_worker, query, torch.cuda.current_device())
    try:
        text_vec = embed_text_batch([query])
    except BaseException:
        if fut is not None:
            fut.exception()  # let the image branch finish; the text error is the one raised
        raise

    early = embed_query_for_images(query) if fut is None else None  # no worker: the reference's order

    def finish() -> np.ndarray:
        image_vec = fut.result() if fut is not None else early
        set_query_embeddings(query, text_vec[0] if text_vec.size else np.zeros(384, dtype=np.float32), image_vec)
        return image_vec

    return (text_vec[0] if text_vec.size else np.zeros(384, dtype=np.float32)), finish


_GET_EMBEDDINGS = _get_embeddings  # this module's own; a rebound global is honoured by retrieve_text


def _chunks_for(hits: List[Dict[str, Any]]) -> List[Optional[Chunk]]:
    """The chunk of every hit, in hit order (reference: one ``get_chunk`` per hit, :55-56 / :88):
    one batched lookup when the store offers ``get_chunks`` (the drop-in's SQLite store), else
    per hit (a store without it, e.g. the tests' stand-ins)."""
    store = _METADATA_STORE
    many = getattr(store, "get_chunks", None)
    if many is None or len(hits) < 2:
        return [store.get_chunk(h["chunk_id"]) for h in hits]
    found = many([h["chunk_id"] for h in hits])
    return [found.get(h["chunk_id"]) for h in hits]


def retrieve_text(user_id: str, query: str, top_k: Optional[int] = None) -> List[Dict[str, Any]]:
    top_k = top_k or settings.retrieval.index_topk_text
    version = get_index_version(user_id)
    cached = get_retrieval_results(user_id, f"text::{query}", version)
    if cached is not None:
        return cached
    # the search and the hits' chunks run while the CLIP-text query encode (needed only by
    # retrieve_images) finishes in the worker thread; both vectors are in the cache before this
    # returns or raises, as after the reference's _get_embeddings (an error of the CLIP-text
    # encode is the one raised, as there: it would have stopped the reference before the search)
    if _get_embeddings is _GET_EMBEDDINGS:
        text_vec, finish = _text_embedding_first(query)
    else:  # a substituted _get_embeddings (a test seam) is called as the reference calls it
        text_vec, _ = _get_embeddings(query)
        finish = lambda: None  # noqa: E731
    try:
        if text_vec.size == 0:
            hits, chunks = [], []
        else:
            hits = _LANCEDB_STORE.search_text(user_id, text_vec.tolist(), top_k)
            chunks = _chunks_for(hits)
    except BaseException:
        finish()
        raise
    finish()
    if text_vec.size == 0:
        return []
    results: List[Dict[str, Any]] = []
    for entry, chunk in zip(hits, chunks):
        if not chunk or not chunk.text:
            continue
        results.append({"chunk_id": chunk.id, "modality": "text", "score": float(entry["score"]),
                        "metadata": _prepare_metadata(chunk), "text": chunk.text})
    set_retrieval_results(user_id, f"text::{query}", version, results)
    return results


def retrieve_images(user_id: str, query: str, top_k: Optional[int] = None) -> List[Dict[str, Any]]:
    top_k = top_k or settings.retrieval.index_topk_image
    version = get_index_version(user_id)
    cached = get_retrieval_results(user_id, f"image::{query}", version)
    if cached is not None:
        return cached
    _, image_vec = _get_embeddings(query)
    if image_vec.size == 0:
        return []
    results: List[Dict[str, Any]] = []
    hits = _LANCEDB_STORE.search_image(user_id, image_vec.tolist(), top_k)
    for entry, chunk in zip(hits, _chunks_for(hits)):
        if not chunk:
            continue
        results.append({"chunk_id": chunk.id, "modality": "image", "score": float(entry["score"]),
                        "metadata": _prepare_metadata(chunk), "text": None})
    set_retrieval_results(user_id, f"image::{query}", version, results)
    return results


def retrieve(user_id: str, query: str) -> List[Dict[str, Any]]:
    version = get_index_version(user_id)
    normalized = _normalize_query(query)
    cached = get_retrieval_results(user_id, normalized, version)
    if cached is not None:
        return cached
    text_results = retrieve_text(user_id, query)
    image_results = retrieve_images(user_id, query)
    fused = _fuse_results(_rerank_text(query, text_results), image_results)
    set_retrieval_results(user_id, normalized, version, fused)
    return fused


def _rerank_pairs(query: str, results: List[Dict[str, Any]]) -> List[Tuple[str, str]]:
    """The (query, passage) pairs ``_rerank_text`` scores (reference :142-150)."""
    top = results[: settings.retrieval.rerank_topk]
    return [(query, item["text"]) for item in top if item.get("text")]


def _apply_rerank(results: List[Dict[str, Any]], scores) -> List[Dict[str, Any]]:
    """Reference :151-155 on precomputed cross-encoder scores (zip with the top items)."""
    top = results[: settings.retrieval.rerank_topk]
    for item, score in zip(top, scores):
        item["rerank_score"] = float(score)
    reranked = top + results[len(top):]
    reranked.sort(key=lambda item: item.get("rerank_score", item["score"]), reverse=True)
    return reranked


def _rerank_text(query: str, results: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    if not results or not settings.retrieval.use_rerank:
        return results
    cross_encoder = _get_cross_encoder()
    if not cross_encoder:
        return results
    pairs = _rerank_pairs(query, results)
    if not pairs:
        return results
    return _apply_rerank(results, cross_encoder.predict(pairs))


def _z_scores(values: Sequence[Optional[float]]) -> List[float]:
    numeric = [v for v in values if v is not None]
    if not numeric:
        return []
    arr = np.array(numeric, dtype=np.float32)
    mean, std = float(arr.mean()), float(arr.std())
    if std == 0:
        return [0.0 for _ in values]
    return [float((v - mean) / std) if v is not None else 0.0 for v in values]


def _fuse_results(text_results: List[Dict[str, Any]], image_results: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    text_cos_z = _z_scores([it["score"] for it in text_results])
    rr = [it.get("rerank_score") for it in text_results if "rerank_score" in it]
    text_rr_z = _z_scores(rr) if rr else []
    image_cos_z = _z_scores([it["score"] for it in image_results])
    items: List[Dict[str, Any]] = []
    for idx, item in enumerate(text_results):
        z = ([text_cos_z[idx]] if text_cos_z else []) + ([text_rr_z[idx]] if text_rr_z and idx < len(text_rr_z) else [])
        items.append({**item, "combined_score": float(np.mean(z)) if z else item["score"]})
    for idx, item in enumerate(image_results):
        items.append({**item, "combined_score": float(image_cos_z[idx] if image_cos_z else item["score"])})
    items.sort(key=lambda e: e["combined_score"], reverse=True)
    return items[: settings.retrieval.final_n]


__all__ = ["retrieve_text", "retrieve_images", "retrieve"]
