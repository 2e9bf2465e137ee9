"""On-disk corpus format: the persistence half of the Lance tables the reference keeps in
``LANCEDB_DIR`` (app/storage/lancedb_store.py:33-44 schema, :87-101 upsert = per-row
``delete(chunk_id == ...)`` then ``add``). SURVEY.md §8f row 2.

One directory per table (``<db>/mrag_tables/<table>/``), append-only:

* ``seg_<k>.f32``      — the segment's rows, fp32 ``[n][dim]`` little-endian, exactly the
                         (re-normalised) vectors the reference would write to Lance;
* ``seg_<k>.parquet``  — the row payloads: chunk_id, user_id, document_id, modality, meta
                         (JSON text), one Arrow row per vector row, same order;
* ``tombstones.i64``   — int64 global row ids deleted by later upserts (append-only);
* ``manifest.json``    — ``{"dim", "segments": [{"name", "rows"}], "tombstones": n}``,
                         replaced atomically (write + fsync + ``os.replace``) after the
                         segment / tombstone bytes are durable, so a crash leaves either
                         the old or the new table, never a torn one.

Global row ids are the concatenation order of the segments, i.e. the GPU index's row ids,
so a reopened table returns the same rows in the same tie order (score desc, row asc).
Readers replay only the segments and tombstones the manifest lists.

Several processes share one directory (the reference's Celery worker indexes while the API
process searches, app/tasks.py:108,165 and api/routes.py:276, both on LANCEDB_DIR): writers
serialise on an exclusive ``fcntl`` lock of ``<dir>/.lock`` and re-read the manifest under
it before appending, so segment names and tombstone offsets never collide; readers need no
lock (the manifest is replaced atomically and lists only durable, immutable bytes) and pick
up other processes' commits with ``refresh()`` (a stat of the manifest per call).
"""
from __future__ import annotations

import contextlib
import fcntl
import json
import os
from dataclasses import dataclass
from typing import Any, Dict, Iterator, List, Optional, Sequence

import numpy as np

COLUMNS = ("chunk_id", "user_id", "document_id", "modality", "meta")


def _fsync_write(path: str, data) -> None:
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


@dataclass
class Segment:
    vectors: np.ndarray          # f32 [n, dim] (memory-mapped)
    rows: Dict[str, List[Any]]   # column -> values


class CorpusFiles:
    """Append-only segment files of one table."""

    def __init__(self, directory: str):
        self.dir = directory
        self.manifest_path = os.path.join(directory, "manifest.json")
        self.manifest: Dict[str, Any] = {"dim": None, "segments": [], "tombstones": 0}
        self._stamp = None
        self._stages_checked = False
        self.refresh()

    def refresh(self) -> bool:
        """Re-read the manifest if another process committed since the last read (True if so)."""
        try:
            st = os.stat(self.manifest_path)
        except FileNotFoundError:
            return False
        stamp = (st.st_ino, st.st_mtime_ns, st.st_size)
        if stamp == self._stamp:
            return False
        with open(self.manifest_path) as f:
            self.manifest = json.load(f)
        self._stamp = stamp
        return True

    @contextlib.contextmanager
    def write_lock(self):
        """Exclusive inter-process writer lock; the manifest is fresh inside it."""
        os.makedirs(self.dir, exist_ok=True)
        fd = os.open(os.path.join(self.dir, ".lock"), os.O_RDWR | os.O_CREAT, 0o644)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX)
            self.refresh()
            if not self._stages_checked:  # once per process and table: a listdir of the segments
                self._stages_checked = True
                self._drop_stale_stages()
            yield self
        finally:
            fcntl.flock(fd, fcntl.LOCK_UN)
            os.close(fd)

    STALE_STAGE_S = 24 * 3600  # a staged Parquet this old belonged to a writer that died

    def _drop_stale_stages(self) -> None:
        """Remove ``stage_rows`` files a crashed writer left (never listed by a manifest); a live
        writer's staged file is younger than any index call (it is written while that call's
        images embed and renamed at its commit)."""
        import time

        now = time.time()
        with contextlib.suppress(OSError):
            for name in os.listdir(self.dir):
                if name.startswith(".stage_") and name.endswith(".parquet"):
                    path = os.path.join(self.dir, name)
                    with contextlib.suppress(OSError):
                        if now - os.stat(path).st_mtime > self.STALE_STAGE_S:
                            os.unlink(path)

    @property
    def dim(self) -> Optional[int]:
        return self.manifest["dim"]

    @property
    def num_rows(self) -> int:
        return sum(s["rows"] for s in self.manifest["segments"])

    def stage_rows(self, rows: Sequence[Dict[str, Any]]) -> str:
        """The payload Parquet of an upcoming ``append``, written and fsynced ahead of it under a
        unique staging name in the table directory (index_image_nodes writes it while its images
        embed); ``append(..., staged=path)`` renames it into place. Not listed by any manifest
        until then; ``discard_staged`` removes it."""
        import tempfile

        import pyarrow as pa
        import pyarrow.parquet as pq

        os.makedirs(self.dir, exist_ok=True)
        fd, path = tempfile.mkstemp(prefix=".stage_", suffix=".parquet", dir=self.dir)
        os.close(fd)
        try:
            pq.write_table(pa.table({c: [str(r[c]) for r in rows] for c in COLUMNS}), path)
            with open(path, "rb") as f:
                os.fsync(f.fileno())
        except BaseException:
            self.discard_staged(path)
            raise
        return path

    @staticmethod
    def discard_staged(path: Optional[str]) -> None:
        if path:
            with contextlib.suppress(FileNotFoundError):
                os.unlink(path)

    def append(self, vectors: np.ndarray, rows: Sequence[Dict[str, Any]], dead: Sequence[int] = (),
               staged: Optional[str] = None) -> None:
        """Durably append one upsert: its tombstones (row ids it replaces) and its rows. Call
        it inside ``write_lock()`` when other processes may write the same table. ``staged``:
        the rows' Parquet from ``stage_rows`` (moved into place instead of written here)."""
        import pyarrow as pa
        import pyarrow.parquet as pq

        v = np.ascontiguousarray(vectors, dtype="<f4")
        if v.ndim != 2 or v.shape[0] != len(rows):
            raise ValueError("vectors must be [n, dim] with one payload row each")
        if staged is not None and pq.read_metadata(staged).num_rows != v.shape[0]:
            raise ValueError("staged payloads do not match the vectors")
        m = json.loads(json.dumps(self.manifest))  # committed to self.manifest only on success
        if m["dim"] is None:
            m["dim"] = int(v.shape[1])
        elif v.shape[1] != m["dim"]:
            raise ValueError(f"dim {v.shape[1]} != table dim {m['dim']}")
        os.makedirs(self.dir, exist_ok=True)
        if len(dead):
            path = os.path.join(self.dir, "tombstones.i64")
            with open(path, "ab"):
                pass
            with open(path, "r+b") as f:
                f.truncate(m["tombstones"] * 8)  # drop bytes of an uncommitted append
                f.seek(0, os.SEEK_END)
                f.write(np.asarray(dead, dtype="<i8").tobytes())
                f.flush()
                os.fsync(f.fileno())
            m["tombstones"] += len(dead)
        if v.shape[0]:
            name = f"seg_{len(m['segments']):06d}"
            _fsync_write(os.path.join(self.dir, name + ".f32"), v.data)  # the array's bytes, no copy
            if staged is not None:
                tmp = staged
            else:
                table = pa.table({c: [str(r[c]) for r in rows] for c in COLUMNS})
                tmp = os.path.join(self.dir, name + ".parquet.tmp")
                pq.write_table(table, tmp)
                with open(tmp, "rb") as f:
                    os.fsync(f.fileno())
            os.replace(tmp, os.path.join(self.dir, name + ".parquet"))
            m["segments"].append({"name": name, "rows": int(v.shape[0])})
        _fsync_write(self.manifest_path, json.dumps(m).encode())
        self.manifest = m
        st = os.stat(self.manifest_path)
        self._stamp = (st.st_ino, st.st_mtime_ns, st.st_size)

    def segments(self, start: int = 0) -> Iterator[Segment]:
        """The committed segments from index ``start`` on (all by default)."""
        import pyarrow.parquet as pq

        dim = self.manifest["dim"]
        for s in self.manifest["segments"][start:]:
            vec = np.memmap(os.path.join(self.dir, s["name"] + ".f32"), dtype="<f4", mode="r",
                            shape=(s["rows"], dim))
            t = pq.read_table(os.path.join(self.dir, s["name"] + ".parquet")).to_pydict()
            yield Segment(vectors=vec, rows=t)

    def tombstones(self, start: int = 0) -> np.ndarray:
        """Committed tombstones from position ``start`` on (all by default)."""
        n = self.manifest["tombstones"]
        if n <= start:
            return np.empty(0, dtype=np.int64)
        return np.fromfile(os.path.join(self.dir, "tombstones.i64"), dtype="<i8", count=n - start,
                           offset=8 * start).astype(np.int64)


__all__ = ["CorpusFiles", "Segment", "COLUMNS"]
