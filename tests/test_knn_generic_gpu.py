"""K7g (csrc/knn_generic.hip): the exact search for widths above 512 and k above 256, and the
fallback of the fused scan when an uncertified query has more near-ties than its collect
capacity. The reference takes both without limit (app/storage/lancedb_store.py:33-44 stores
list<float32> of any length; :110,121 pass limit(max(top_k, 1)) through; config.py:46-47 makes
the k user-settable). Bar: bit-exact rows and f32 scores against the f64 oracle, as the fused
path (tests/test_knn_gpu.py)."""
from __future__ import annotations

import numpy as np
import pytest

from _data import clustered_corpus, labels_for, unit_rows
from oracle.knn import flat_cosine_topk
from test_knn_gpu import _check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dim", [640, 768, 1000, 1024, 1536])
def test_wide_dims(cuda, dim):
    """ViT-L/14 / MPNet (768), 1024-d and 1536-d embeddings, ragged 1000: clustered rows with
    duplicates and zero rows, a label prefilter, k from 1 to 100."""
    from app.vector_store import FlatIndex

    n = 20_000
    x = clustered_corpus(n, dim, 40 + dim, n_clusters=32, spread=0.05, dup_frac=0.05)
    lab = labels_for(n, 3, 41)
    rng = np.random.default_rng(42)
    q = np.concatenate([x[rng.integers(0, n, 40)] + 0.01 * rng.standard_normal((40, dim)).astype(np.float32),
                        rng.standard_normal((24, dim)).astype(np.float32)])
    ix = FlatIndex(dim)
    ix.add(x, lab)
    for k, f in ((1, -1), (10, -1), (12, 1), (50, 0), (100, -1)):
        s, r = ix.search(q, k, label=f)
        os_, or_ = flat_cosine_topk(x, lab, q, k, label_filter=f)
        _check(s, r, os_, or_)


def test_wide_dim_768_large_corpus_device(cuda):
    """768-d at 300k rows (several GEMM chunks per pass), device pointers and a row offset."""
    import torch

    from app.vector_store import FlatIndex

    g = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn((300_000, 768), generator=g, device=cuda)
    q = torch.randn((500, 768), generator=g, device=cuda)
    ix = FlatIndex(768)
    ix.add(x)
    s, r, s64 = ix.search(q, 10, row_offset=77, with_f64=True)
    os_, or_ = flat_cosine_topk(x.cpu().numpy(), np.zeros(300_000), q.cpu().numpy(), 10, row_offset=77)
    _check(s.cpu().numpy(), r.cpu().numpy(), os_, or_)
    np.testing.assert_allclose(s64.cpu().numpy(), os_, rtol=0, atol=1e-12)


@pytest.mark.parametrize("dim", [384, 512])
def test_k_above_256(cuda, dim):
    """INDEX_TOPK_TEXT set to 300 / 1000 (the fused path's lists hold at most 256)."""
    from app.vector_store import FlatIndex

    n = 40_000
    x = clustered_corpus(n, dim, 50 + dim, n_clusters=16, spread=0.05, dup_frac=0.1)
    lab = labels_for(n, 4, 51)
    q = unit_rows(37, dim, 52)
    ix = FlatIndex(dim)
    ix.add(x, lab)
    for k, f in ((257, -1), (300, 2), (1000, -1)):
        s, r = ix.search(q, k, label=f)
        os_, or_ = flat_cosine_topk(x, lab, q, k, label_filter=f)
        _check(s, r, os_, or_)


def test_k_above_rows_and_deleted(cuda):
    """k beyond the matching rows: -inf / -1 padding, tombstones excluded, both paths."""
    from app.vector_store import FlatIndex

    for dim in (512, 768):
        x = unit_rows(700, dim, 60)
        lab = labels_for(700, 2, 61)
        q = unit_rows(5, dim, 62)
        ix = FlatIndex(dim)
        ix.add(x, lab)
        ix.delete(list(range(0, 700, 7)))
        lab2 = lab.copy()
        lab2[::7] = -2
        for k, f in ((300, -1), (500, 1), (5, 1)):
            s, r = ix.search(q, k, label=f)
            os_, or_ = flat_cosine_topk(x, lab2, q, k, label_filter=f)
            _check(s, r, os_, or_)


def test_duplicate_run_then_large_batch(cuda):
    """a run of near-identical rows (static video frames) bigger than the fused
    path's per-query collect capacity, then a large batch. The overflowing batch goes to K7g
    (per-query storage sized from its histogram); nothing is retained by the index, so the
    next large batch still fits. Results exact."""
    from app.vector_store import FlatIndex

    dim = 256
    frame = unit_rows(1, dim, 70)
    rng = np.random.default_rng(71)
    x = np.concatenate([np.repeat(frame, 20_000, 0) + 1e-4 * rng.standard_normal((20_000, dim)).astype(np.float32),
                        unit_rows(60_000, dim, 72)])
    ix = FlatIndex(dim)
    ix.add(x)
    q = np.concatenate([frame, unit_rows(6000, dim, 73)])
    s, r = ix.search(q, 10)
    unc, retries = ix.last_stats()
    assert retries == 1, (unc, retries)  # the duplicate run overflowed the fused collect
    sel = np.r_[0, np.arange(1, len(q), 97)]
    os_, or_ = flat_cosine_topk(x, np.zeros(len(x)), q[sel], 10)
    _check(s[sel], r[sel], os_, or_)
    q2 = unit_rows(20_000, dim, 74)
    s2, r2 = ix.search(q2, 10)
    os2, or2 = flat_cosine_topk(x, np.zeros(len(x)), q2[:200], 10)
    _check(s2[:200], r2[:200], os2, or2)


def test_sharded_merge_k300(cuda):
    import torch

    from app.vector_store import FlatIndex, topk_merge

    x = clustered_corpus(9000, 768, 80, dup_frac=0.1)
    q = unit_rows(16, 768, 81)
    k = 300
    lists_s, lists_r = [], []
    for sh in np.array_split(np.arange(len(x)), 3):
        ix = FlatIndex(768)
        ix.add(x[sh])
        s, r, s64 = ix.search(torch.from_numpy(q).to(cuda), k, row_offset=int(sh[0]), with_f64=True)
        lists_s.append(s64)
        lists_r.append(r)
    ms, mr, _ = topk_merge(torch.stack(lists_s), torch.stack(lists_r), k)
    os_, or_ = flat_cosine_topk(x, np.zeros(len(x)), q, k)
    _check(ms.cpu().numpy(), mr.cpu().numpy(), os_, or_)
