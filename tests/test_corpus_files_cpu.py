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
