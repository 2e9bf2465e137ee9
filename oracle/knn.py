"""Exact flat cosine top-k — CPU restatement of the reference's kNN (test oracle only).

Reference call: ``app/storage/lancedb_store.py:103-123``
    self._text_table.search(vector).where("user_id == '…'").metric("cosine")
        .limit(max(top_k, 1)).to_list()
followed by ``_format_results`` (:125-139): ``score = 1 - _distance`` sorted desc.
The arithmetic lives in lancedb/lance (Rust, unpinned in requirements.txt:11, not
installed here): flat cosine distance ``1 - x.y/(|x||y|)``. This module restates it
exactly in float64 with the semantics pinned in DESIGN.md §3:

* score = q.x / (|q| |x|) on the f32 vectors as given; 0 when a norm is 0;
* ``where user_id == …`` is a prefilter (label == filter; filter -1 = every live
  row; label < 0 = deleted row);
* order (score desc, row asc); at most k rows (fewer if fewer rows match).

Pinned against scikit-learn's brute-force cosine NearestNeighbors in
``tests/test_oracle_pinning.py`` (an independent implementation).
"""
from __future__ import annotations

import numpy as np


def cosine_scores(corpus: np.ndarray, queries: np.ndarray) -> np.ndarray:
    """[nq, n] float64 cosine of every (query, row) pair (0 where a norm is 0)."""
    X = np.asarray(corpus, dtype=np.float32).astype(np.float64)
    Q = np.asarray(queries, dtype=np.float32).astype(np.float64)
    xn = np.sqrt(np.einsum("ij,ij->i", X, X))
    qn = np.sqrt(np.einsum("ij,ij->i", Q, Q))
    dots = Q @ X.T
    den = qn[:, None] * xn[None, :]
    with np.errstate(invalid="ignore", divide="ignore"):
        cos = np.where(den > 0, dots / np.where(den > 0, den, 1.0), 0.0)
    return cos


def duplicate_groups(corpus: np.ndarray, block: int = 16384):
    """Rows with identical f32 contents (exact duplicates: re-ingested chunks, repeated frames).

    Returns (gid, reps): gid[row] = group index or -1 for a row without a duplicate, reps[g] =
    the first row of group g. Found by an exact integer hash of the row bits (int64 wraparound,
    deterministic per row) and confirmed byte for byte.
    """
    X = np.ascontiguousarray(corpus, dtype=np.float32)
    n = X.shape[0]
    gid = np.full(n, -1, dtype=np.int64)
    if n < 2:
        return gid, np.zeros(0, dtype=np.int64)
    coef = np.random.default_rng(12345).integers(1, 2**62, size=X.shape[1], dtype=np.int64) | 1
    h = np.empty(n, dtype=np.int64)
    bits = X.view(np.int32)
    with np.errstate(over="ignore"):
        for b0 in range(0, n, block):
            h[b0:b0 + block] = (bits[b0:b0 + block].astype(np.int64) * coef).sum(axis=1)
    order = np.argsort(h, kind="stable")
    hs = h[order]
    starts = np.nonzero(np.r_[True, hs[1:] != hs[:-1]])[0]
    ends = np.r_[starts[1:], n]
    reps = []
    for a, b in zip(starts, ends):
        if b - a < 2:
            continue
        members = np.sort(order[a:b])
        rest = members
        while rest.size > 1:  # split a hash bucket into byte-identical groups
            same = np.all(X[rest] == X[rest[0]], axis=1) & np.all(bits[rest] == bits[rest[0]], axis=1)
            grp = rest[same]
            if grp.size > 1:
                gid[grp] = len(reps)
                reps.append(int(grp[0]))
            rest = rest[~same]
    return gid, np.asarray(reps, dtype=np.int64)


def flat_cosine_topk(corpus, labels, queries, k: int, label_filter: int = -1, row_offset: int = 0,
                     chunk: int = 131072):
    """Exact top-k. Returns (scores f64 [nq,k], rows int64 [nq,k]); empty slots -inf / -1.

    The corpus is scanned in chunks (bounded memory at 1M+ rows); every chunk keeps
    all rows scoring >= its own k-th score, so ties at the boundary survive to the
    final (score desc, row asc) selection. Identical rows score identically (one BLAS
    product per distinct vector: a blocked product may round the same dot product
    differently at different column positions, ~1e-16, which would order exact
    duplicates by position instead of by row).
    """
    corpus = np.asarray(corpus, dtype=np.float32)
    queries = np.asarray(queries, dtype=np.float32)
    if queries.ndim == 1:
        queries = queries[None, :]
    labels = np.asarray(labels, dtype=np.int64)
    nq = queries.shape[0]
    out_s = np.full((nq, k), -np.inf, dtype=np.float64)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    if corpus.shape[0] == 0 or nq == 0:
        return out_s, out_r
    mask = labels >= 0 if label_filter == -1 else labels == label_filter
    all_rows = np.nonzero(mask)[0]
    if all_rows.size == 0:
        return out_s, out_r
    gid, reps = duplicate_groups(corpus)
    rep_cos = cosine_scores(corpus[reps], queries) if reps.size else None
    cand_s = [[] for _ in range(nq)]
    cand_r = [[] for _ in range(nq)]
    for c0 in range(0, all_rows.size, chunk):
        rows = all_rows[c0:c0 + chunk]
        # Residual limit (distinct rows only): the BLAS product rounds a row's f64 score in an
        # order that can depend on the row's position in the chunk, while the GPU rescoring uses
        # one fixed order; two DISTINCT rows whose exact scores differ by less than ~1e-16 could
        # therefore tie-break differently. Bit-identical rows are handled exactly (below).
        cos = cosine_scores(corpus[rows], queries)
        if rep_cos is not None:
            dup = np.nonzero(gid[rows] >= 0)[0]
            if dup.size:
                cos[:, dup] = rep_cos[:, gid[rows[dup]]]
        kk = min(k, rows.size)
        for i in range(nq):
            s = cos[i]
            if kk < rows.size:
                thr = np.partition(s, rows.size - kk)[rows.size - kk]
                sel = np.nonzero(s >= thr)[0]
            else:
                sel = np.arange(rows.size)
            cand_s[i].append(s[sel])
            cand_r[i].append(rows[sel])
    for i in range(nq):
        s = np.concatenate(cand_s[i])
        r = np.concatenate(cand_r[i])
        order = np.lexsort((r, -s))[:k]
        out_s[i, :order.size] = s[order]
        out_r[i, :order.size] = r[order] + row_offset
    return out_s, out_r


def kth_gap(corpus, labels, queries, k: int, label_filter: int = -1) -> np.ndarray:
    """Per-query gap between the k-th and (k+1)-th exact scores (diagnostic)."""
    s, _ = flat_cosine_topk(corpus, labels, queries, k + 1, label_filter)
    return s[:, k - 1] - s[:, k]
