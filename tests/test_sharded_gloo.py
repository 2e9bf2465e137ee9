"""N>1 path on CPU: world_size-2 gloo process group running the product's
ShardedFlatIndex orchestration (row offsets, all-gather layout [world, nq, k], merge)
with a CPU stand-in for each rank's local GPU index and a numpy restatement of the
K11 merge as the checker's merge. The merged result must equal the oracle's exact
top-k over the whole (unsharded) corpus, ties included."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _data import clustered_corpus, unit_rows


class _OracleShard:
    """Local-index stand-in: exact top-k of this rank's rows (oracle)."""

    def __init__(self, rows, labels):
        self.rows, self.labels = rows, labels

    def search(self, q, k, label=-1, row_offset=0, with_f64=False):
        from oracle.knn import flat_cosine_topk

        s, r = flat_cosine_topk(self.rows, self.labels, q.numpy(), k, label_filter=label, row_offset=row_offset)
        return torch.from_numpy(s.astype(np.float32)), torch.from_numpy(r), torch.from_numpy(s)


def _merge_np(s64, rows, k):
    s = s64.numpy().transpose(1, 0, 2).reshape(s64.shape[1], -1)
    r = rows.numpy().transpose(1, 0, 2).reshape(rows.shape[1], -1)
    out_s = np.full((s.shape[0], k), -np.inf)
    out_r = np.full((s.shape[0], k), -1, dtype=np.int64)
    for i in range(s.shape[0]):
        ok = r[i] >= 0
        order = np.lexsort((r[i][ok], -s[i][ok]))[:k]
        out_s[i, :order.size] = s[i][ok][order]
        out_r[i, :order.size] = r[i][ok][order]
    return torch.from_numpy(out_s.astype(np.float32)), torch.from_numpy(out_r), torch.from_numpy(out_s)


def _worker(rank, world, port, X, labels, Q, k, label, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from app.vector_store.sharded import ShardedFlatIndex

        bounds = np.linspace(0, len(X), world + 1).astype(int)
        lo, hi = bounds[rank], bounds[rank + 1]
        idx = ShardedFlatIndex(_OracleShard(X[lo:hi], labels[lo:hi]), row_offset=lo, merge=_merge_np)
        s, r = idx.search(torch.from_numpy(Q), k, label=label)
        ret[rank] = (s.numpy(), r.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("label", [-1, 2])
def test_sharded_equals_unsharded(label):
    from oracle.knn import flat_cosine_topk

    X = clustered_corpus(3001, 96, 4, dup_frac=0.3)  # ties across the shard boundary
    labels = np.random.default_rng(1).integers(0, 4, len(X)).astype(np.int32)
    Q = unit_rows(9, 96, 5)
    k = 10
    ret = mp.Manager().dict()
    mp.spawn(_worker, args=(2, _free_port(), X, labels, Q, k, label, ret), nprocs=2, join=True)
    es, er = flat_cosine_topk(X, labels, Q, k, label_filter=label)
    for rank in range(2):
        s, r = ret[rank]
        np.testing.assert_array_equal(r, er)
        np.testing.assert_allclose(s, es.astype(np.float32), atol=1e-7)
