"""Drop-in for the reference's ``app/ml/index_build.py``.

``index_text_nodes`` (:46-103): documents -> sentence-split nodes -> metadata-prefixed
texts -> ``embed_text_batch`` -> ``VectorRow``s -> ``upsert_text_vectors`` -> version
bump. ``index_image_nodes`` (:106-155): drop nodes whose file is missing ->
``embed_images_batch`` -> ``upsert_image_vectors`` -> version bump.
``get_index_version`` keys the retrieval cache. Module globals ``_LANCEDB_STORE``,
``_VERSION_FILE``, ``embed_text_batch``, ``embed_images_batch`` are looked up at call
time, so tests can monkeypatch them as the reference's tests do. The version file is
written atomically under a process lock (the reference's read-modify-write races).
"""
from __future__ import annotations

import json
import os
import sys
import threading
from pathlib import Path
from typing import Dict, List, Sequence

import numpy as np

from app.ml.embeddings import embed_images_batch, embed_images_batches, embed_query_for_images, embed_text_batch
from app.ml.splitter import Document, SentenceSplitter
from app.settings import settings
from app.storage.corpus_files import CorpusFiles
from app.storage.lancedb_store import LanceDBStore, VectorRow

_SPLITTER = SentenceSplitter(chunk_size=512, chunk_overlap=64)
_LANCEDB_STORE = LanceDBStore(settings.paths.lancedb_dir)
_VERSION_FILE = Path(settings.paths.lancedb_dir) / "index_versions.json"
_VERSION_LOCK = threading.Lock()
_EMBED_IMAGES_NATIVE = embed_images_batch  # this package's (takes str paths); tests may rebind the global


def _load_versions() -> Dict[str, int]:
    if not _VERSION_FILE.exists():
        return {}
    try:
        return json.loads(_VERSION_FILE.read_text())
    except Exception:
        return {}


def _save_versions(versions: Dict[str, int]) -> None:
    _VERSION_FILE.parent.mkdir(parents=True, exist_ok=True)
    tmp = _VERSION_FILE.with_suffix(".tmp")
    tmp.write_text(json.dumps(versions))
    os.replace(tmp, _VERSION_FILE)


def _bump_version(user_id: str) -> int:
    with _VERSION_LOCK:
        versions = _load_versions()
        versions[user_id] = versions.get(user_id, 0) + 1
        _save_versions(versions)
        return versions[user_id]


def get_index_version(user_id: str) -> int:
    return _load_versions().get(user_id, 0)


def _array_rows() -> bool:
    """True when ``_LANCEDB_STORE`` is this package's store, which takes the embeddings as numpy
    rows and prepares them as one array (LanceDBStore._prepare_rows_array: the same vector bytes
    as the per-row lists). Any other store (a test's stand-in) gets the reference's
    ``embedding.tolist()`` lists (reference app/ml/index_build.py:90,151)."""
    return isinstance(_LANCEDB_STORE, LanceDBStore)


def _row_embedding(embedding, array_rows: bool):
    if array_rows and isinstance(embedding, np.ndarray):
        return embedding
    return embedding.tolist()


def index_text_nodes(user_id: str, nodes: Sequence[Dict[str, object]]) -> List[Dict[str, object]]:
    """Chunk and index text nodes ({id, text, metadata})."""
    documents: List[Document] = []
    for node in nodes:
        text = str(node.get("text") or "").strip()
        if not text:
            continue
        documents.append(Document(text=text, metadata=dict(node.get("metadata", {})), doc_id=str(node.get("id"))))
    if not documents:
        return []
    parsed_nodes = _SPLITTER.get_nodes_from_documents(documents)
    texts = [n.get_content(metadata_mode="all") for n in parsed_nodes]
    if not texts:
        return []
    embeddings = embed_text_batch(texts)
    array_rows = _array_rows()
    rows: List[VectorRow] = []
    stored: List[Dict[str, object]] = []
    for parsed, embedding in zip(parsed_nodes, embeddings):
        meta = dict(parsed.metadata)
        meta.update({"doc_id": parsed.ref_doc_id or parsed.node_id, "user_id": user_id, "modality": "text",
                     "source": meta.get("source")})
        rows.append(VectorRow(chunk_id=parsed.node_id, user_id=user_id, document_id=meta["doc_id"], modality="text",
                              embedding=_row_embedding(embedding, array_rows), meta=meta))
        stored.append({"chunk_id": parsed.node_id, "metadata": meta, "text": parsed.get_content(metadata_mode="none")})
    if rows:
        _LANCEDB_STORE.upsert_text_vectors(rows)
        _bump_version(user_id)
    return stored


def _paths_exist(strs: List[str]) -> List[bool]:
    """``Path(s).exists()`` for every s (reference app/ml/index_build.py:114-118), the stats in one
    library call on host threads (``mrag_paths_exist``): missing -> False, an error Path.exists does
    not ignore -> Path.exists itself raises it; a path Path cannot encode (a NUL byte) -> False."""
    import ctypes

    from app import _native
    from app.encoders.preprocess import decode_workers

    n = len(strs)
    try:  # os.fsencode of every path at once (what it does on POSIX)
        enc = [s.encode(_FS_ENCODING, "surrogateescape") for s in strs]
        bad = [i for i, b in enumerate(enc) if b"\0" in b]
    except UnicodeError:
        enc, bad = [], []
        for i, s in enumerate(strs):
            try:
                enc.append(os.fsencode(s))
                if b"\0" in enc[-1]:
                    bad.append(i)
            except UnicodeError:
                enc.append(b"")
                bad.append(i)
    for i in bad:  # Path.exists: ValueError -> False
        enc[i] = b""
    out = np.zeros(n, np.int32)
    if n:
        names = (ctypes.c_char_p * n)(*enc)
        _native.call("mrag_paths_exist", ctypes.cast(names, ctypes.c_void_p), n, min(8, decode_workers()),
                     out.ctypes.data)
    out[bad] = 0
    res = (out > 0).tolist()
    for i in np.flatnonzero(out < 0).tolist():
        res[i] = Path(strs[i]).exists()  # raises what the reference's check raises
    return res


_FS_ENCODING = sys.getfilesystemencoding()


def index_image_nodes(user_id: str, nodes: Sequence[Dict[str, object]]) -> List[Dict[str, object]]:
    """Index image nodes ({id, metadata{file_path, ...}}) with CLIP embeddings.

    The reference's per-node loop (:110-126) as three steps with the same result: the metadata
    copies and file paths, the existence filter as one library call (_paths_exist), then the
    embed. With this package's embed and store (>= 256 files) the rows' metadata, the store's
    payload dicts and their Parquet are made while the embed pipeline waits for its next decoded
    batch, and each embedded batch is normalised for the store there too (embed_images_batches);
    otherwise the reference's order (a substituted embed_images_batch gets Path objects)."""
    metas = [dict(node.get("metadata", {})) for node in nodes]
    strs = [str(m.get("file_path", "")) for m in metas]
    sel = [i for i, e in enumerate(_paths_exist(strs)) if e]
    if not sel:
        return []
    embed = embed_images_batch
    native = embed is _EMBED_IMAGES_NATIVE
    paths = [strs[i] for i in sel] if native else [Path(strs[i]) for i in sel]

    def build_rows(idx: List[int]) -> List[VectorRow]:
        out = []
        for i in idx:
            metadata = metas[i]
            chunk_id = str(nodes[i].get("id"))
            metadata.update({"doc_id": metadata.get("doc_id", chunk_id), "user_id": user_id, "modality": "image",
                             "source": metadata.get("source")})
            out.append(VectorRow(chunk_id=chunk_id, user_id=user_id, document_id=metadata["doc_id"], modality="image",
                                 embedding=[], meta=metadata))
        return out

    array_rows = _array_rows()
    if native and array_rows and len(sel) >= 256:
        # while this thread would wait for the pipeline's next decoded batch: the store's
        # normalisation of the batches already embedded, then the rows and the store's payload
        # dicts in chunks; one upsert at the end as the reference's (same rows, same bytes)
        out, payloads, pending, staged = [], [], [], []
        embeddings = vectors = None

        def chunks():
            for c0 in range(0, len(sel), 128):
                for i in sel[c0:c0 + 128]:
                    metadata = metas[i]
                    chunk_id = str(nodes[i].get("id"))
                    metadata.update({"doc_id": metadata.get("doc_id", chunk_id), "user_id": user_id,
                                     "modality": "image", "source": metadata.get("source")})
                    payloads.append(LanceDBStore._payload(chunk_id, user_id, metadata["doc_id"], "image", metadata))
                    out.append({"chunk_id": chunk_id, "metadata": metadata})
                yield
            staged.append(_LANCEDB_STORE._stage_image_payloads(payloads))  # the Parquet, ahead of the upsert
            yield

        work = chunks()

        def idle() -> bool:
            if pending:
                o, m = pending.pop()
                vectors[o:o + m] = LanceDBStore._normalize_rows(embeddings[o:o + m])
                return True
            return next(work, False) is None

        try:
            o = 0
            for e in embed_images_batches(paths, idle=idle):
                if embeddings is None:
                    embeddings = np.empty((len(paths), e.shape[1]), np.float32)
                    vectors = np.empty_like(embeddings)
                embeddings[o:o + len(e)] = e
                pending.append((o, len(e)))
                o += len(e)
            while idle():  # what the waits left
                pass
        except BaseException:
            CorpusFiles.discard_staged(staged[0] if staged else None)
            raise
        _LANCEDB_STORE._upsert_image_payloads(payloads, vectors, staged[0])
        _bump_version(user_id)
        return out
    rows = build_rows(sel)
    embeddings = embed(paths)
    for row, embedding in zip(rows, embeddings):
        row.embedding = _row_embedding(embedding, array_rows)
    _LANCEDB_STORE.upsert_image_vectors(rows)
    _bump_version(user_id)
    return [{"chunk_id": row.chunk_id, "metadata": row.meta} for row in rows]


__all__ = ["index_text_nodes", "index_image_nodes", "embed_query_for_images", "get_index_version"]
