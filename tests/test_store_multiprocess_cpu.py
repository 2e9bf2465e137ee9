"""Several processes on one LANCEDB_DIR: the reference's Celery worker indexes
(app/tasks.py:108,165) while the API process searches (api/routes.py:276). Writers serialise
on the table's file lock and replay other processes' commits first; readers replay what was
committed since their last call. Checked here on CPU with a numpy stand-in for the GPU index
(``_NumpyIndex``, test-only: the product has no CPU search path) in spawned processes; the GPU
version of the reader/writer check is ``test_compat_gpu.py::test_store_sees_other_process``."""
from __future__ import annotations

import multiprocessing as mp
import os

import numpy as np


class _NumpyIndex:
    """Test double of app.vector_store.FlatIndex: exact oracle search over host arrays."""

    def __init__(self, dim, device=0):
        self.x = np.zeros((0, dim), np.float32)
        self.lab = np.zeros(0, np.int32)

    def add(self, rows, labels=0):
        first = len(self.x)
        rows = np.asarray(rows, np.float32)
        self.x = np.concatenate([self.x, rows])
        self.lab = np.concatenate([self.lab, np.broadcast_to(np.asarray(labels, np.int32), (len(rows),))])
        return first

    def delete(self, rows):
        self.lab[np.asarray(rows, np.int64)] = -2

    def search(self, q, k, label=-1):
        from oracle.knn import flat_cosine_topk

        s, r = flat_cosine_topk(self.x, self.lab, q, k, label_filter=label)
        return s.astype(np.float32), r


def _patch():
    import app.vector_store as vs

    vs.FlatIndex = _NumpyIndex


def _writer(db, who, n_batches, q):
    _patch()
    from app.storage.lancedb_store import LanceDBStore, VectorRow

    store = LanceDBStore(db)
    rng = np.random.default_rng(who)
    for b in range(n_batches):
        rows = [VectorRow(f"{who}-{b}-{i}", f"user{who}", "d", "text", rng.standard_normal(16).tolist(), {"w": who})
                for i in range(5)]
        # a chunk id both writers re-upsert: exactly one live row must remain
        rows.append(VectorRow(f"shared-{b}", "shared", "d", "text", rng.standard_normal(16).tolist(), {"w": who}))
        store.upsert_text_vectors(rows)
    q.put(who)


def _fresh_live_rows(db):
    """(chunk_id -> count of live rows) as a new process would replay them."""
    _patch()
    from app.storage import lancedb_store as ls

    ls._REGISTRY.clear()
    t = ls.LanceDBStore(db)._text_table
    t._sync()
    live = t.index.lab >= 0
    out = {}
    for r in np.nonzero(live)[0]:
        out[t.chunk_ids[r]] = out.get(t.chunk_ids[r], 0) + 1
    return out, t


def test_concurrent_writers_lose_nothing(tmp_path):
    db = str(tmp_path / "db")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_writer, args=(db, w, 12, q)) for w in (1, 2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    live, t = _fresh_live_rows(db)
    files = t.files
    assert len(files.manifest["segments"]) == 24  # no segment overwritten by the other writer
    assert files.num_rows == 24 * 6
    for w in (1, 2):
        for b in range(12):
            for i in range(5):
                assert live.get(f"{w}-{b}-{i}") == 1
    for b in range(12):
        assert live.get(f"shared-{b}") == 1  # re-upserts across processes delete the other's row
    assert len(live) == 2 * 12 * 5 + 12


def test_reader_sees_later_commits(tmp_path):
    _patch()
    from app.storage import lancedb_store as ls

    db = str(tmp_path / "db2")
    ls._REGISTRY.clear()
    store = ls.LanceDBStore(db)
    rng = np.random.default_rng(5)
    store.upsert_text_vectors([ls.VectorRow(f"a{i}", "alice", "d", "text", rng.standard_normal(16).tolist(), {})
                               for i in range(10)])
    v = rng.standard_normal(16)
    assert store.search_text("bob", v.tolist(), 5) == []  # bob unknown to this process yet
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_writer, args=(db, 7, 2, q))  # another process indexes user7 + re-upserts
    p.start()
    p.join(120)
    assert p.exitcode == 0
    hits = store.search_text("user7", v.tolist(), 50)  # same store object, same process
    assert len(hits) == 10 and all(h["meta"] == {"w": 7} for h in hits)
    assert len(store.search_text("alice", v.tolist(), 50)) == 10
    # and a write from this process after the other's commits lands after them
    store.upsert_text_vectors([ls.VectorRow("shared-0", "shared", "d", "text", v.tolist(), {"w": "me"})])
    live, t = _fresh_live_rows(db)
    assert live["shared-0"] == 1
    r = [i for i in range(len(t.chunk_ids)) if t.chunk_ids[i] == "shared-0" and t.index.lab[i] >= 0]
    assert t.metas[r[0]] == '{"w": "me"}'
    ls._REGISTRY.clear()
