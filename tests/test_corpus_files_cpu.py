"""On-disk corpus format: durable append-only segments, tombstones and
an atomic manifest; a reopened table sees exactly the committed rows in the same order."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest


def _rows(ids, user="u1"):
    return [{"chunk_id": c, "user_id": user, "document_id": "d" + c, "modality": "text", "meta": json.dumps({"i": c})}
            for c in ids]


def test_append_reopen_roundtrip(tmp_path):
    from app.storage.corpus_files import CorpusFiles

    d = str(tmp_path / "t")
    f = CorpusFiles(d)
    rng = np.random.default_rng(0)
    v1 = rng.standard_normal((5, 8)).astype(np.float32)
    v2 = rng.standard_normal((3, 8)).astype(np.float32)
    f.append(v1, _rows(["a", "b", "c", "d", "e"]))
    f.append(v2, _rows(["b", "f", "g"], user="u2"), dead=[1])
    g = CorpusFiles(d)  # a new process's view
    assert g.dim == 8 and g.num_rows == 8
    segs = list(g.segments())
    np.testing.assert_array_equal(np.concatenate([np.asarray(s.vectors) for s in segs]), np.concatenate([v1, v2]))
    assert sum((s.rows["chunk_id"] for s in segs), []) == ["a", "b", "c", "d", "e", "b", "f", "g"]
    assert segs[1].rows["user_id"] == ["u2"] * 3
    assert g.tombstones().tolist() == [1]
    with pytest.raises(ValueError):
        g.append(np.zeros((1, 4), np.float32), _rows(["x"]))  # dim mismatch


def test_manifest_is_the_commit_point(tmp_path):
    """Bytes written after the last manifest (a crashed append) are invisible on reopen."""
    from app.storage.corpus_files import CorpusFiles

    d = str(tmp_path / "t")
    f = CorpusFiles(d)
    f.append(np.ones((2, 4), np.float32), _rows(["a", "b"]))
    # simulate a crash mid-append: stray segment + tombstone bytes, manifest untouched
    with open(os.path.join(d, "seg_000001.f32"), "wb") as h:
        h.write(np.zeros((3, 4), np.float32).tobytes())
    with open(os.path.join(d, "tombstones.i64"), "ab") as h:
        h.write(np.asarray([0], "<i8").tobytes())
    g = CorpusFiles(d)
    assert g.num_rows == 2 and g.tombstones().size == 0
    # the next append replaces the stray segment and tombstone bytes
    g.append(np.full((1, 4), 2, np.float32), _rows(["c"]), dead=[1])
    h = CorpusFiles(d)
    assert h.num_rows == 3 and h.tombstones().tolist() == [1]
    assert np.asarray(list(h.segments())[1].vectors).tolist() == [[2.0] * 4]


def test_staged_payloads_commit_like_written_ones(tmp_path):
    """stage_rows (index_image_nodes writes the Parquet while its images embed) then
    append(..., staged=...) gives the same files as a plain append; a staged file that does not
    match its vectors is refused and, through _Table.upsert, removed; nothing stays behind."""
    from app.storage.corpus_files import CorpusFiles

    v = np.arange(12, dtype=np.float32).reshape(3, 4)
    a, b = CorpusFiles(str(tmp_path / "a")), CorpusFiles(str(tmp_path / "b"))
    a.append(v, _rows(["x", "y", "z"]))
    path = b.stage_rows(_rows(["x", "y", "z"]))
    assert os.path.exists(path) and CorpusFiles(str(tmp_path / "b")).num_rows == 0  # not committed yet
    b.append(v, _rows(["x", "y", "z"]), staged=path)
    assert not os.path.exists(path)
    for name in ("seg_000000.parquet", "seg_000000.f32"):
        ra = open(os.path.join(a.dir, name), "rb").read()
        rb = open(os.path.join(b.dir, name), "rb").read()
        assert ra == rb, name
    bad = b.stage_rows(_rows(["p", "q"]))
    with pytest.raises(ValueError):
        b.append(v, _rows(["x", "y", "z"]), staged=bad)
    CorpusFiles.discard_staged(bad)
    assert sorted(f for f in os.listdir(b.dir) if f.startswith(".stage_")) == []
    assert CorpusFiles(b.dir).num_rows == 3


def test_table_upsert_removes_a_refused_staged_file(tmp_path):
    from app.storage.corpus_files import CorpusFiles
    from app.storage.lancedb_store import _Table

    t = _Table("image_collection", 0, str(tmp_path / "img"))
    staged = t.files.stage_rows(_rows(["p"]))

    class Boom(Exception):
        pass

    def boom(*a, **k):
        raise Boom()

    t._sync = boom  # fails under the writer lock, before the append
    with pytest.raises(Boom):
        t.upsert(_rows(["p"]), np.ones((1, 4), np.float32), staged)
    assert not os.path.exists(staged)
    assert CorpusFiles(t.files.dir).num_rows == 0


def test_stale_staged_files_are_dropped_by_the_next_writer(tmp_path):
    """A staged Parquet left by a writer that died (older than STALE_STAGE_S) is removed under
    the next writer lock; a fresh one (a live writer's) stays."""
    import time

    from app.storage.corpus_files import CorpusFiles

    f = CorpusFiles(str(tmp_path / "t"))
    old = f.stage_rows(_rows(["a"]))
    fresh = f.stage_rows(_rows(["b"]))
    past = time.time() - CorpusFiles.STALE_STAGE_S - 60
    os.utime(old, (past, past))
    with f.write_lock():
        pass
    assert not os.path.exists(old) and os.path.exists(fresh)
    f.append(np.ones((1, 4), np.float32), _rows(["b"]), staged=fresh)
    assert CorpusFiles(f.dir).num_rows == 1
