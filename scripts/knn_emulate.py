"""Host emulation of the fused kNN pipeline's bookkeeping (K7 v3 lane lists -> fold -> K8
certificate -> K7c collect -> K10), vectorised in numpy, on the data of
tests/test_knn_gpu.py::test_collect_pass_many_failing_queries.

The approximate scores are fp16(q^) . fp16(x^) in f32 (numpy order, not the MFMA's, but within
the same EPS bound), so this checks the LOGIC of lists, drop bounds, certificate and collect
threshold — not the hardware. Prints how many queries the emulated pipeline gets wrong and, per
stage, the counts the GPU run should show.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from _data import clustered_corpus  # noqa: E402
from oracle.knn import cosine_scores  # noqa: E402

EPS = 1.05e-3
KL3 = 6


def insert(ls, li, v, r, mask):
    """Insert v (row r) into the descending lists ls/li where mask (strict >, as list_insert)."""
    n = ls.shape[1]
    for j in range(n):
        sw = mask & (v > ls[:, j])
        ts, tr = ls[:, j].copy(), li[:, j].copy()
        ls[:, j] = np.where(sw, v, ts)
        li[:, j] = np.where(sw, r, tr)
        v = np.where(sw, ts, v)
        r = np.where(sw, tr, r)


def main(nq=640, k=50, n=30000, d=512, seed=11, qseed=5):
    x = clustered_corpus(n, d, seed, n_clusters=8, spread=0.01, dup_frac=0.2)
    q = x[np.random.default_rng(qseed).integers(0, len(x), nq)] + 0.001
    xn = np.sqrt((x.astype(np.float64) ** 2).sum(1))
    qn = np.sqrt((q.astype(np.float64) ** 2).sum(1))
    x16 = (x.astype(np.float64) * np.where(xn > 0, 1 / np.where(xn > 0, xn, 1), 0)[:, None]).astype(np.float32).astype(np.float16)
    q16 = (q.astype(np.float64) * (1 / qn)[:, None]).astype(np.float32).astype(np.float16)
    approx = q16.astype(np.float32) @ x16.astype(np.float32).T  # [nq, n]
    exact = cosine_scores(x, q)
    ntiles = (n + 63) // 64
    Qp = (nq + 255) // 256 * 256
    qgroups = Qp // 256
    S = max(1, 256 // qgroups)
    S = min(S, ntiles, 4096 // 8)
    if S >= 8:
        S &= ~7
    M = min(k + 32, S * 8)
    print(f"ntiles {ntiles} Qp {Qp} qgroups {qgroups} S {S} M {M}")
    pad = np.full((nq, ntiles * 64 - n), -np.inf, np.float32)
    ap = np.concatenate([approx, pad], 1)  # padding rows masked to -inf
    # lane lists [S, nq, 4 (g4), 6]
    L = S * nq * 4
    ls = np.full((L, KL3), -np.inf, np.float32)
    li = np.full((L, KL3), -1, np.int64)
    sidx = np.repeat(np.arange(S), nq * 4)
    qidx = np.tile(np.repeat(np.arange(nq), 4), S)
    g4 = np.tile(np.arange(4), S * nq)
    my_tiles = (ntiles - 1 - np.arange(S)) // S + 1
    for it in range(my_tiles.max()):
        tile = sidx + it * S
        live = tile < ntiles
        tile_c = np.where(live, tile, 0)
        for rb in range(4):
            rows = [tile_c * 64 + 16 * rb + 4 * g4 + r for r in range(4)]
            sv = [np.where(live, ap[qidx, rr], -np.inf) for rr in rows]
            gm = np.maximum.reduce(sv)
            fire = gm > ls[:, KL3 - 1]
            for r in range(4):
                insert(ls, li, sv[r].copy(), rows[r].copy(), fire & (sv[r] > ls[:, KL3 - 1]))
    # fold the four lanes of each (split, query)
    ls4 = ls.reshape(S * nq, 4, KL3)
    li4 = li.reshape(S * nq, 4, KL3)
    fs = np.full((S * nq, 8), -np.inf, np.float32)
    fi = np.full((S * nq, 8), -1, np.int64)
    fs[:, :KL3] = ls4[:, 0]
    fi[:, :KL3] = li4[:, 0]
    tau = np.where(li4[:, 0, KL3 - 1] >= 0, ls4[:, 0, KL3 - 1], -np.inf)
    for o in (1, 2, 3):
        for j in range(KL3):
            ps, pi = ls4[:, o, j], li4[:, o, j]
            insert(fs, fi, ps.copy(), pi.copy(), (pi >= 0) & (ps > fs[:, 7]))
        tau = np.where(li4[:, o, KL3 - 1] >= 0, np.maximum(tau, ls4[:, o, KL3 - 1]), tau)
    tau = np.where(fi[:, 7] >= 0, np.maximum(tau, fs[:, 7]), tau)
    fs = fs.reshape(S, nq, 8)
    fi = fi.reshape(S, nq, 8)
    tau = tau.reshape(S, nq)
    # K8
    wrong, unc, collected_max = 0, 0, 0
    ref_order = np.lexsort((np.broadcast_to(np.arange(n), exact.shape), -exact), axis=1)[:, :k]
    for qi in range(nq):
        s = fs[:, qi].reshape(-1)
        r = fi[:, qi].reshape(-1)
        ok = r >= 0
        s, r = s[ok], r[ok]
        order = np.lexsort((r, -s.astype(np.float64)))
        s, r = s[order], r[order]
        valid = len(r)
        t = tau[:, qi].max()
        t = max(t, fs[:, qi, 7][fi[:, qi, 7] >= 0].max(initial=-np.inf))
        Mq = min(M, valid)
        a_next = s[Mq] if valid > Mq else -np.inf
        T = max(t, a_next)
        cand = r[:Mq]
        ex = exact[qi, cand]
        o2 = np.lexsort((cand, -ex))
        ex, cand = ex[o2], cand[o2]
        if t == -np.inf and valid <= Mq:
            cert = True
        else:
            cert = Mq >= k and ex[k - 1] > T + EPS
        if cert:
            got = cand[:k]
        else:
            unc += 1
            thr = np.float32(ex[k - 1] - EPS) if Mq >= k else -np.inf
            if np.float64(thr) > ex[k - 1] - EPS:
                thr = np.nextafter(thr, np.float32(-np.inf))
            col = np.nonzero(approx[qi] >= thr)[0]
            collected_max = max(collected_max, len(col))
            e2 = exact[qi, col]
            got = col[np.lexsort((col, -e2))][:k]
        if not np.array_equal(got, ref_order[qi]):
            wrong += 1
            if wrong <= 5:
                print(f"q {qi} cert {cert} T {T:.6f} ex_k {ex[k-1]:.6f} e_k {exact[qi, ref_order[qi][-1]]:.6f}")
    print(f"emulated: wrong {wrong} / {nq}, uncertified {unc}, max collected {collected_max}")


if __name__ == "__main__":
    main()
