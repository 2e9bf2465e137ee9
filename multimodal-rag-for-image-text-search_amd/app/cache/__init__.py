"""In-process TTL caches around the retrieval path (call-site compatible).

Same API and keying as the reference's ``app/cache/__init__.py`` (:17-111): query
embeddings keyed by the normalised query text (300 s), retrieval results keyed by
(user, normalised query, index version) (120 s), chat responses (60 s). Memoisation
only — no arithmetic of the hot path lives here.
"""
from __future__ import annotations

import functools
import time
from typing import Any, Callable, Dict, Optional, Tuple

import numpy as np

EMBED_TTL_SEC = 300
RETRIEVAL_TTL_SEC = 120
CHAT_TTL_SEC = 60

_EMBED_CACHE: Dict[str, Tuple[float, Tuple[np.ndarray, np.ndarray]]] = {}
_RETRIEVAL_CACHE: Dict[Tuple[str, str, int], Tuple[float, Any]] = {}
_CHAT_CACHE: Dict[tuple, Tuple[float, Any]] = {}


def _normalize_query(query: str) -> str:
    return " ".join(query.strip().lower().split())


def _live(entry, now: float) -> bool:
    return entry is not None and entry[0] >= now


def clear_all_caches() -> None:
    for c in (_EMBED_CACHE, _RETRIEVAL_CACHE, _CHAT_CACHE):
        c.clear()


def get_query_embeddings(query: str) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    key = _normalize_query(query)
    entry = _EMBED_CACHE.get(key)
    if not entry:
        return None
    if not _live(entry, time.time()):
        _EMBED_CACHE.pop(key, None)
        return None
    return entry[1]


def set_query_embeddings(query: str, text_vec: np.ndarray, image_vec: np.ndarray, ttl: int = EMBED_TTL_SEC) -> None:
    _EMBED_CACHE[_normalize_query(query)] = (time.time() + ttl, (text_vec, image_vec))


def get_retrieval_results(user_id: str, query: str, index_version: int) -> Optional[Any]:
    key = (user_id, _normalize_query(query), index_version)
    entry = _RETRIEVAL_CACHE.get(key)
    if not entry:
        return None
    if not _live(entry, time.time()):
        _RETRIEVAL_CACHE.pop(key, None)
        return None
    return entry[1]


def set_retrieval_results(user_id: str, query: str, index_version: int, results: Any,
                          ttl: int = RETRIEVAL_TTL_SEC) -> None:
    _RETRIEVAL_CACHE[(user_id, _normalize_query(query), index_version)] = (time.time() + ttl, results)


def chat_cache(ttl: int = CHAT_TTL_SEC) -> Callable:
    """Cache ``func(user_id, query, ...)`` by (user, normalised query, index version, kwargs)."""

    def decorator(func: Callable) -> Callable:
        @functools.wraps(func)
        def wrapper(user_id: str, query: str, *args, **kwargs):
            from app.ml.index_build import get_index_version

            key = (user_id, _normalize_query(query), get_index_version(user_id),
                   tuple(sorted(kwargs.items())) if kwargs else ())
            entry = _CHAT_CACHE.get(key)
            if entry and _live(entry, time.time()):
                return entry[1]
            result = func(user_id, query, *args, **kwargs)
            _CHAT_CACHE[key] = (time.time() + ttl, result)
            return result

        return wrapper

    return decorator


__all__ = ["get_query_embeddings", "set_query_embeddings", "get_retrieval_results", "set_retrieval_results",
           "chat_cache", "clear_all_caches"]
