"""Drop-in for the reference's ``app/storage/lancedb_store.py`` backed by the GPU index.

Same names and signatures: ``VectorRow`` (:12-21), ``LanceDBStore(db_path)`` (:24)
with ``upsert_text_vectors`` / ``upsert_image_vectors`` (:87-101), ``search_text`` /
``search_image`` (:103-123) and the static helpers ``_normalize`` (:63-69),
``_prepare_rows`` (:71-85), ``_format_results`` (:125-139), ``_where_clause`` (:141-144).

What changes underneath: the two Lance tables (text_collection / image_collection)
become ``app.vector_store.FlatIndex`` objects resident in HBM; the ``user_id`` filter
becomes an int32 row label (prefilter); a per-row delete becomes a tombstone label.
Every ``LanceDBStore`` opened on the same directory shares the same tables (the
reference's two handles on one directory could miss each other's writes).
Tables persist under ``<db_path>/mrag_tables/<table>/`` (``app.storage.corpus_files``:
fp32 row segments + Parquet payloads + tombstones, atomic manifest) and are replayed into
the GPU index with the same row ids. Processes sharing the directory (the reference's
worker indexing while the API searches) see each other's commits: every search and upsert
first replays what was committed since, and upserts serialise on a file lock.
Semantics pinned in DESIGN.md §3: exact flat cosine (no IVF_PQ — the reference's
index build is attempted on an empty table and swallowed, :51-60), prefilter, order
(score desc, row asc), ``limit(max(top_k, 1))``, ``score = 1 - f32(1 - cos)``.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np

from app.storage.corpus_files import CorpusFiles


@dataclass
class VectorRow:
    """Payload used when writing vectors (same fields as the reference)."""

    chunk_id: str
    user_id: str
    document_id: str
    modality: str
    embedding: Sequence[float]
    meta: Dict[str, Any]


class _Table:
    """One collection: GPU rows + host-side row payloads (+ their files, if persistent).

    With files, the in-memory table is a replay of the committed segments and tombstones in
    manifest order (so row ids agree across processes); ``_sync`` replays what other
    processes committed since the last call, at the start of every search and upsert."""

    def __init__(self, name: str, device: int = 0, directory: Optional[str] = None):
        self.name = name
        self.device = device
        self.files = None
        if directory is not None:
            from app.storage.corpus_files import CorpusFiles

            self.files = CorpusFiles(directory)
        self.index = None  # FlatIndex, created on the first write (dim unknown before)
        self.dim: Optional[int] = None
        self.chunk_ids: List[str] = []
        self.metas: List[str] = []
        self.doc_ids: List[str] = []
        self.by_chunk: Dict[str, List[int]] = {}
        self.labels: Dict[str, int] = {}
        self.lock = threading.RLock()
        self._seen_segments = 0    # committed segments replayed into this process
        self._seen_tombstones = 0  # committed tombstones applied

    def _ensure_index(self, dim: int):
        if self.index is None:
            from app.vector_store import FlatIndex

            self.index = FlatIndex(dim, device=self.device)
            self.dim = dim
        elif dim != self.dim:
            raise ValueError(f"{self.name}: embedding dim {dim} != table dim {self.dim}")

    def _append_rows(self, vectors: np.ndarray, user_ids, chunk_ids, metas, doc_ids) -> None:
        labs = np.asarray([self.labels.setdefault(u, len(self.labels)) for u in user_ids], dtype=np.int32)
        first = self.index.add(np.asarray(vectors), labs)
        self.chunk_ids.extend(chunk_ids)
        self.metas.extend(metas)
        self.doc_ids.extend(doc_ids)
        by_chunk = self.by_chunk
        for row, cid in enumerate(chunk_ids, first):
            rows = by_chunk.get(cid)
            if rows is None:
                by_chunk[cid] = [row]
            else:
                rows.append(row)

    def _kill_rows(self, dead) -> None:
        dead = [int(r) for r in dead]
        if not dead:
            return
        self.index.delete(dead)
        for r in dead:
            rows = self.by_chunk.get(self.chunk_ids[r])
            if rows and r in rows:
                rows.remove(r)
                if not rows:
                    del self.by_chunk[self.chunk_ids[r]]

    def _sync(self) -> None:
        """Replay the segments + tombstones committed (by any process) since the last sync."""
        if self.files is None:
            return
        self.files.refresh()
        m = self.files.manifest
        if len(m["segments"]) > self._seen_segments:
            self._ensure_index(self.files.dim)
            for seg in self.files.segments(self._seen_segments):
                c = seg.rows
                self._append_rows(seg.vectors, c["user_id"], c["chunk_id"], c["meta"], c["document_id"])
                self._seen_segments += 1
        if m["tombstones"] > self._seen_tombstones:
            self._kill_rows(self.files.tombstones(self._seen_tombstones))
            self._seen_tombstones = m["tombstones"]

    _load = _sync  # name used by app.retrieval

    def upsert(self, payloads: List[Dict[str, Any]], vectors: Optional[np.ndarray] = None,
               staged: Optional[str] = None) -> None:
        """Per-row delete of the payloads' chunk ids, then one append. ``vectors`` (f32 [n, dim]):
        the payloads' embeddings already stacked (the array path of LanceDBStore._upsert);
        ``staged``: their Parquet from CorpusFiles.stage_rows (removed if the append fails)."""
        try:
            self._upsert(payloads, vectors, staged)
        finally:
            CorpusFiles.discard_staged(staged)  # renamed into place by a successful append

    def _upsert(self, payloads, vectors, staged) -> None:
        if not payloads:
            return
        with self.lock:
            if vectors is not None:
                emb = np.ascontiguousarray(vectors, dtype=np.float32)
            else:
                emb = np.asarray([p["embedding"] for p in payloads], dtype=np.float32)
            if emb.ndim != 2:
                raise ValueError("all embeddings in one upsert must have the same length")
            with (self.files.write_lock() if self.files is not None else contextlib.nullcontext()):
                self._sync()  # under the writer lock: every committed row is visible here
                self._ensure_index(emb.shape[1])
                # per-row delete of any existing row with the same chunk_id (lancedb_store.py:91-92)
                dead = []
                for p in payloads:
                    dead.extend(self.by_chunk.get(p["chunk_id"], []))
                if self.files is not None:  # durable first: a failed write leaves the table as it was
                    self.files.append(emb, payloads, dead, staged)
                    self._seen_segments += 1
                    self._seen_tombstones += len(dead)
                self._kill_rows(dead)
                self._append_rows(emb, [p["user_id"] for p in payloads], [p["chunk_id"] for p in payloads],
                                  [p["meta"] for p in payloads], [p["document_id"] for p in payloads])

    def search(self, user_id: str, vector: List[float], k: int) -> List[Dict[str, Any]]:
        with self.lock:
            self._sync()
            label = self.labels.get(user_id)
            if self.index is None or label is None:
                return []
            q = np.asarray(vector, dtype=np.float32)[None, :]
            if q.shape[1] != self.dim:
                raise ValueError(f"{self.name}: query dim {q.shape[1]} != table dim {self.dim}")
            s, r = self.index.search(q, k, label=label)
            rows = []
            for score, row in zip(s[0], r[0]):
                if row < 0:
                    break
                rows.append({
                    "chunk_id": self.chunk_ids[row],
                    "_distance": np.float32(1.0) - np.float32(score),  # lance: f32 cosine distance
                    "meta": self.metas[row],
                })
            return rows


_REGISTRY: Dict[str, Dict[str, _Table]] = {}
_REG_LOCK = threading.Lock()


def _tables_for(db_path: str) -> Dict[str, _Table]:
    key = os.path.abspath(db_path)
    with _REG_LOCK:
        if key not in _REGISTRY:
            dev = int(os.environ.get("MRAG_DEVICE", "0"))
            persist = os.environ.get("MRAG_STORE_PERSIST", "1") != "0"
            _REGISTRY[key] = {n: _Table(n, dev, os.path.join(key, "mrag_tables", n) if persist else None)
                              for n in ("text_collection", "image_collection")}
        return _REGISTRY[key]


class LanceDBStore:
    """Two collections (text / image) with exact cosine search on the GPU."""

    def __init__(self, db_path: str) -> None:
        self._db_path = db_path
        tables = _tables_for(db_path)
        self._text_table = tables["text_collection"]
        self._image_table = tables["image_collection"]

    @staticmethod
    def _normalize(vector: Sequence[float]) -> List[float]:
        arr = np.asarray(vector, dtype=np.float32)
        norm = np.linalg.norm(arr)
        if norm <= 0:
            return arr.tolist()
        return (arr / norm).tolist()

    @staticmethod
    def _prepare_rows(rows: Iterable[VectorRow]) -> List[Dict[str, Any]]:
        return [
            {
                "chunk_id": row.chunk_id,
                "user_id": row.user_id,
                "document_id": row.document_id,
                "modality": row.modality,
                "embedding": LanceDBStore._normalize(row.embedding),
                "meta": json.dumps(row.meta or {}),
            }
            for row in rows
        ]

    @staticmethod
    def _normalize_rows(vectors: np.ndarray) -> np.ndarray:
        """``_normalize`` of every row of an f32 [n, dim] array at once, bit for bit: np.linalg.norm
        of a 1-D f32 vector is sqrt(x.dot(x)) — the same BLAS dot per row (its summation order is
        BLAS's, so it is not batched) and an f32 sqrt of the result — then one f32 division of each
        row by its norm; rows of norm <= 0 stay as they are."""
        arr = np.asarray(vectors, dtype=np.float32)
        norms = np.sqrt(np.array([x.dot(x) for x in arr], dtype=np.float32)).reshape(-1, 1)
        out = arr / np.where(norms <= 0, np.float32(1), norms)
        return np.where(norms <= 0, arr, out)

    @staticmethod
    def _prepare_rows_array(rows: List[VectorRow], vectors: Optional[np.ndarray] = None):
        """``_prepare_rows`` for rows whose embeddings are numpy rows (what index_text_nodes /
        index_image_nodes hand this store): the same payload dicts and vector bytes with the
        vectors kept as one f32 array — no per-row list round trip (tolist, then asarray).
        ``vectors``: ``_normalize_rows`` of the rows' embeddings when the caller already made it."""
        if vectors is None:
            vectors = LanceDBStore._normalize_rows(np.stack([np.asarray(r.embedding, dtype=np.float32) for r in rows]))
        payloads = [LanceDBStore._payload(row.chunk_id, row.user_id, row.document_id, row.modality, row.meta)
                    for row in rows]
        for p, v in zip(payloads, vectors):
            p["embedding"] = v
        return payloads, vectors

    @staticmethod
    def _payload(chunk_id: str, user_id: str, document_id: str, modality: str, meta) -> Dict[str, Any]:
        """One row's ``_prepare_rows`` dict without its embedding (set by the caller)."""
        return {
            "chunk_id": chunk_id,
            "user_id": user_id,
            "document_id": document_id,
            "modality": modality,
            "embedding": None,
            "meta": json.dumps(meta or {}),
        }

    def _upsert(self, table: "_Table", rows: Iterable[VectorRow]) -> None:
        rows = list(rows)
        if rows and all(isinstance(r.embedding, np.ndarray) and r.embedding.ndim == 1 for r in rows) \
                and len({r.embedding.shape[0] for r in rows}) == 1:
            payloads, vectors = self._prepare_rows_array(rows)
            table.upsert(payloads, vectors)
        else:
            table.upsert(self._prepare_rows(rows))

    def _stage_image_payloads(self, payloads: List[Dict[str, Any]]) -> Optional[str]:
        """The image table's Parquet of ``payloads`` written ahead of their upsert (None for an
        in-memory table)."""
        files = self._image_table.files
        return files.stage_rows(payloads) if files is not None and payloads else None

    def _upsert_image_payloads(self, payloads: List[Dict[str, Any]], vectors: np.ndarray,
                               staged: Optional[str] = None) -> None:
        """``upsert_image_vectors(rows)`` from the rows' ``_payload`` dicts and ``vectors`` =
        ``_normalize_rows`` of their embeddings (index_image_nodes makes both, and the staged
        Parquet, while the images embed)."""
        if payloads:
            for p, v in zip(payloads, vectors):
                p["embedding"] = v
            self._image_table.upsert(payloads, vectors, staged)
        else:
            CorpusFiles.discard_staged(staged)

    def upsert_text_vectors(self, rows: Iterable[VectorRow]) -> None:
        self._upsert(self._text_table, rows)

    def upsert_image_vectors(self, rows: Iterable[VectorRow]) -> None:
        self._upsert(self._image_table, rows)

    def search_text(self, user_id: str, query_vec: Sequence[float], top_k: int) -> List[Dict[str, Any]]:
        return self._format_results(self._text_table.search(user_id, self._normalize(query_vec), max(top_k, 1)))

    def search_image(self, user_id: str, query_vec: Sequence[float], top_k: int) -> List[Dict[str, Any]]:
        return self._format_results(self._image_table.search(user_id, self._normalize(query_vec), max(top_k, 1)))

    @staticmethod
    def _format_results(rows: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        out = [
            {
                "chunk_id": row.get("chunk_id"),
                "score": 1.0 - float(row.get("_distance", 0.0)),
                "meta": json.loads(row.get("meta") or "{}"),
            }
            for row in rows
        ]
        out.sort(key=lambda item: item["score"], reverse=True)
        return out

    @staticmethod
    def _where_clause(column: str, value: str) -> str:
        safe = str(value).replace("'", "''")
        return f"{column} == '{safe}'"


__all__ = ["VectorRow", "LanceDBStore"]
