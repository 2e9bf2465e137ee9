"""The oracle is pinned before it is trusted (CPU, no GPU):

* model restatements (oracle/models.py) reproduce the fixtures produced by the
  reference's own embed_images_batch / embed_text_batch / _normalize code;
* the kNN restatement (oracle/knn.py) reproduces its fixtures and agrees with an
  independent implementation (scikit-learn brute-force cosine NearestNeighbors);
* the normaliser and fusion restatements reproduce the reference's outputs exactly.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from _data import clustered_corpus, labels_for, sha, unit_rows


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="module")
def clip():
    from oracle.models import clip_model

    return clip_model(0)


def test_clip_image_oracle_matches_reference(clip):
    from oracle.models import clip_image_embeds

    g = _load("golden_clip_image.npz")
    got = clip_image_embeds(clip, g["images_u8"])
    np.testing.assert_allclose(got, g["expected"], atol=2e-6)


def test_clip_text_oracle_matches_reference(clip):
    from oracle.models import clip_text_embeds

    g = _load("golden_clip_text.npz")
    np.testing.assert_allclose(clip_text_embeds(clip, g["ids"], g["mask"]), g["expected"], atol=2e-6)


def test_minilm_oracle_matches_reference():
    from oracle.models import bert_model, minilm_embeds

    g = _load("golden_minilm.npz")
    np.testing.assert_allclose(minilm_embeds(bert_model(0), g["ids"], g["mask"]), g["expected"], atol=2e-6)


def test_normalize_restatements_exact():
    from oracle.normalize import embeddings_normalize, store_normalize

    g = _load("golden_normalize.npz")
    np.testing.assert_array_equal(embeddings_normalize(g["x"].copy()), g["expected"])
    for i in range(3):
        np.testing.assert_array_equal(np.asarray(store_normalize(g[f"vec{i}"]), np.float32), g[f"vec{i}_expected"])


def test_fusion_restatement_exact():
    from oracle.fusion import fuse_results, z_scores

    d = json.load(open(os.path.join(GOLDEN, "golden_fusion.json")))
    for c in d["cases"]:
        assert z_scores([it["score"] for it in c["text"]]) == c["z_text"]
        assert fuse_results([dict(i) for i in c["text"]], [dict(i) for i in c["image"]], d["final_n"]) == c["fused"]


def _knn_inputs(tag, shape):
    n, d, seed, nq, k = (int(v) for v in shape)
    X = unit_rows(n, d, seed) if tag != "c" else clustered_corpus(n, d, seed, dup_frac=0.2)
    return X, labels_for(n, 5, seed + 100), unit_rows(nq, d, seed + 200), k


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_knn_oracle_fixture_and_sklearn(tag):
    from sklearn.neighbors import NearestNeighbors

    from oracle.knn import flat_cosine_topk

    g = _load("golden_knn.npz")
    X, lab, Q, k = _knn_inputs(tag, g[f"{tag}_shape"])
    assert sha(X, lab, Q) == str(g[f"{tag}_sha"])
    s, r = flat_cosine_topk(X, lab, Q, k)
    np.testing.assert_array_equal(r, g[f"{tag}_rows"])
    np.testing.assert_array_equal(s, g[f"{tag}_scores"])
    s3, r3 = flat_cosine_topk(X, lab, Q, k, label_filter=3)
    np.testing.assert_array_equal(r3, g[f"{tag}_rows_f3"])
    # independent implementation: sklearn brute cosine (distance = 1 - cos) in f64
    nn = NearestNeighbors(n_neighbors=k, metric="cosine", algorithm="brute").fit(X.astype(np.float64))
    dist, idx = nn.kneighbors(Q.astype(np.float64))
    np.testing.assert_allclose(1.0 - dist, s, atol=1e-12)
    # rows agree except where sklearn breaks exact ties differently (duplicates in "c")
    diff = idx != r
    if diff.any():
        assert np.all(np.abs((1.0 - dist)[diff] - s[diff]) < 1e-12)


def test_knn_oracle_duplicates_tie_by_row():
    """Exact duplicate rows must score bit-identically and come back in row order (the pinned
    tie rule), wherever they sit in the corpus and across the oracle's scan chunks: a blocked
    BLAS product can round one dot product differently at different column positions (~1e-16,
    observed with 640 queries over 30k clustered rows, round 4), which would order duplicates
    by position."""
    from oracle.knn import duplicate_groups, flat_cosine_topk

    x = clustered_corpus(30000, 512, 11, n_clusters=8, spread=0.01, dup_frac=0.2)
    q = x[np.random.default_rng(5).integers(0, len(x), 640)] + np.float32(0.001)
    gid, reps = duplicate_groups(x)
    assert reps.size > 1000
    for chunk in (131072, 7001):  # one chunk / duplicates split across chunks
        s, r = flat_cosine_topk(x, np.zeros(len(x)), q, 50, chunk=chunk)
        g = gid[r]
        for i in range(len(q)):
            for a in range(49):
                if g[i, a] >= 0 and g[i, a] == g[i, a + 1]:
                    assert s[i, a] == s[i, a + 1] and r[i, a] < r[i, a + 1]
        if chunk == 131072:
            first = (s, r)
    np.testing.assert_array_equal(first[1], r)
    np.testing.assert_allclose(first[0], s, rtol=0, atol=1e-14)  # other rows: ulps by chunking
