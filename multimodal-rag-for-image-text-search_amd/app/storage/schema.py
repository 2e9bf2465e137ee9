"""Chunk metadata catalog used by retrieval (minimal SQLite store).

Out of the hot path (per-hit payload lookup), kept so that
``app.ml.retrieve`` has the same collaborators as the reference
(``app/storage/schema.py``: ``Chunk`` :33-55, ``MetadataStore.get_chunk`` :203-214).
The connection is opened lazily (the reference connects at import time, which fails
when LANCEDB_DIR does not exist yet).
"""
from __future__ import annotations

import json
import os
import sqlite3
import threading
from datetime import datetime
from typing import Any, Dict, Iterable, List, Optional

from pydantic import BaseModel, Field, field_validator


class Document(BaseModel):
    id: str
    user_id: str
    source_type: str
    source_uri: str
    title: Optional[str] = None
    status: str = "pending"


class Chunk(BaseModel):
    id: str
    document_id: str
    modality: str
    text: Optional[str] = None
    page_no: Optional[int] = None
    start_ts: Optional[float] = None
    end_ts: Optional[float] = None
    file_path: Optional[str] = None
    meta: Dict[str, Any] = Field(default_factory=dict)

    @field_validator("modality")
    @classmethod
    def _modality(cls, v: str) -> str:
        if v not in {"text", "image"}:
            raise ValueError(f"modality must be 'text' or 'image', got {v!r}")
        return v


_COLS = ("id", "document_id", "modality", "text", "page_no", "start_ts", "end_ts", "file_path", "meta")


class MetadataStore:
    def __init__(self, db_path: str) -> None:
        self._db_path = db_path
        self._conn: Optional[sqlite3.Connection] = None
        self._lock = threading.Lock()

    def _c(self) -> sqlite3.Connection:
        if self._conn is None:
            d = os.path.dirname(os.path.abspath(self._db_path))
            os.makedirs(d, exist_ok=True)
            self._conn = sqlite3.connect(self._db_path, check_same_thread=False)
            self._conn.row_factory = sqlite3.Row
            self._conn.execute(
                "CREATE TABLE IF NOT EXISTS documents (id TEXT PRIMARY KEY, user_id TEXT, source_type TEXT,"
                " source_uri TEXT, title TEXT, status TEXT, updated_at TEXT)")
            self._conn.execute(
                "CREATE TABLE IF NOT EXISTS chunks (id TEXT PRIMARY KEY, document_id TEXT, modality TEXT, text TEXT,"
                " page_no INTEGER, start_ts REAL, end_ts REAL, file_path TEXT, meta TEXT, updated_at TEXT)")
        return self._conn

    def close(self) -> None:
        if self._conn is not None:
            self._conn.close()
            self._conn = None

    def upsert_document(self, document: Document) -> Document:
        with self._lock:
            c = self._c()
            c.execute("INSERT OR REPLACE INTO documents VALUES (?,?,?,?,?,?,?)",
                      (document.id, document.user_id, document.source_type, document.source_uri, document.title,
                       document.status, datetime.utcnow().isoformat()))
            c.commit()
        return document

    def upsert_chunks(self, chunks: Iterable[Chunk]) -> None:
        with self._lock:
            c = self._c()
            now = datetime.utcnow().isoformat()
            for ch in chunks:
                c.execute("INSERT OR REPLACE INTO chunks VALUES (?,?,?,?,?,?,?,?,?,?)",
                          (ch.id, ch.document_id, ch.modality, ch.text, ch.page_no, ch.start_ts, ch.end_ts,
                           ch.file_path, json.dumps(ch.meta or {}), now))
            c.commit()

    def get_chunk(self, chunk_id: str) -> Optional[Chunk]:
        with self._lock:
            row = self._c().execute("SELECT * FROM chunks WHERE id = ?", (chunk_id,)).fetchone()
        if not row:
            return None
        data = {k: row[k] for k in _COLS}
        data["meta"] = json.loads(data.get("meta") or "{}")
        return Chunk(**data)

    def get_chunks(self, chunk_ids: List[str]) -> Dict[str, Chunk]:
        """``get_chunk`` for many ids in one statement per 500 ids (one retrieval's hits): id ->
        Chunk for the ids present, the same objects ``get_chunk`` builds."""
        rows = []
        with self._lock:
            c = self._c()
            for i in range(0, len(chunk_ids), 500):
                part = chunk_ids[i:i + 500]
                rows += c.execute(f"SELECT * FROM chunks WHERE id IN ({','.join('?' * len(part))})", part).fetchall()
        out = {}
        for row in rows:
            data = {k: row[k] for k in _COLS}
            data["meta"] = json.loads(data.get("meta") or "{}")
            out[data["id"]] = Chunk(**data)
        return out

    def list_chunks(self, document_id: str) -> List[Chunk]:
        with self._lock:
            rows = self._c().execute("SELECT * FROM chunks WHERE document_id = ?", (document_id,)).fetchall()
        out = []
        for row in rows:
            data = {k: row[k] for k in _COLS}
            data["meta"] = json.loads(data.get("meta") or "{}")
            out.append(Chunk(**data))
        return out
