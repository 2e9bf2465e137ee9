"""Hot-path settings, read from the same environment variables as the reference.

Mirrors the subset of ``app/settings.py`` (reference :171-252, defaults config.py:6-115)
that the embed/index/retrieve path reads: model identifiers (MODEL_TEXT, MODEL_CLIP,
RERANKER_MODEL), LANCEDB_DIR, and the retrieval knobs (RERANK_ENABLED, INDEX_TOPK_TEXT,
INDEX_TOPK_IMG, RERANK_TOPK, FINAL_N, CONFIDENCE_TAU). Everything else in the reference's
settings (Gemini, uploads, YouTube, API keys, ...) belongs to out-of-scope subsystems.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Mapping, Optional


def _env(env: Optional[Mapping[str, str]], key: str, default: str) -> str:
    if env is not None and key in env:
        return env[key]
    return os.getenv(key, default)


def _int(env, key, default: int) -> int:
    raw = _env(env, key, str(default))
    try:
        return int(raw)
    except (TypeError, ValueError):
        raise ValueError(f"Environment variable {key} must be an integer, got '{raw}'.")


def _float(env, key, default: float) -> float:
    raw = _env(env, key, str(default))
    try:
        return float(raw)
    except (TypeError, ValueError):
        raise ValueError(f"Environment variable {key} must be a float, got '{raw}'.")


def _bool(env, key, default: bool) -> bool:
    return str(_env(env, key, str(default))).strip().lower() in {"1", "true", "yes", "on"}


@dataclass(frozen=True)
class ModelSettings:
    text: str
    clip: str
    reranker: str


@dataclass(frozen=True)
class PathSettings:
    lancedb_dir: str


@dataclass(frozen=True)
class RetrievalSettings:
    use_rerank: bool
    index_topk_text: int
    index_topk_image: int
    rerank_topk: int
    final_n: int
    confidence_tau: float


@dataclass(frozen=True)
class AppSettings:
    models: ModelSettings
    paths: PathSettings
    retrieval: RetrievalSettings


def load_settings(env: Optional[Mapping[str, str]] = None) -> AppSettings:
    return AppSettings(
        models=ModelSettings(
            text=_env(env, "MODEL_TEXT", "sentence-transformers/all-MiniLM-L6-v2"),
            clip=_env(env, "MODEL_CLIP", "openai/clip-vit-base-patch32"),
            reranker=_env(env, "RERANKER_MODEL", "cross-encoder/ms-marco-MiniLM-L-6-v2"),
        ),
        paths=PathSettings(lancedb_dir=_env(env, "LANCEDB_DIR", "output/lance_db")),
        retrieval=RetrievalSettings(
            use_rerank=_bool(env, "RERANK_ENABLED", True),
            index_topk_text=_int(env, "INDEX_TOPK_TEXT", 50),
            index_topk_image=_int(env, "INDEX_TOPK_IMG", 12),
            rerank_topk=_int(env, "RERANK_TOPK", 8),
            final_n=_int(env, "FINAL_N", 4),
            confidence_tau=_float(env, "CONFIDENCE_TAU", 0.25),
        ),
    )


settings = load_settings()
