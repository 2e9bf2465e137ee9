"""N>1 path on CPU: world_size 2 and 4 gloo process groups running the product's
ShardedFlatIndex (row offsets, the all-gather of (f64 score, int64 row) lists into the
[world, nq, k] layout K11 consumes, the merge call) with a CPU stand-in for each rank's
local GPU index (the oracle's exact local top-k — what FlatIndex.search returns, pinned by
tests/test_knn_gpu.py) and ``oracle.merge.topk_merge``, the documented restatement of K11
(knn.hip topk_merge_kernel), as the merge. K11 itself is checked against the same
restatement on the GPU (tests/test_knn_gpu.py::test_k11_matches_restatement). The merged
result must equal the oracle's exact top-k over the whole (unsharded) corpus, ties included."""
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


def _merge_k11(s64, rows, k):
    """K11 on the CPU (oracle.merge.topk_merge) behind the torch signature of
    app.vector_store.topk_merge; asserts the gathered layout is [world, nq, k]."""
    from oracle.merge import topk_merge

    world = dist.get_world_size()
    assert s64.dtype == torch.float64 and rows.dtype == torch.int64
    assert s64.shape[0] == world and s64.shape[2] == k and rows.shape == s64.shape
    out = topk_merge(s64.numpy(), rows.numpy(), k)
    return tuple(torch.from_numpy(a) for a in out)


def _worker(rank, world, port, X, labels, Q, k, label, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from app.vector_store.sharded import ShardedFlatIndex

        bounds = np.linspace(0, len(X), world + 1).astype(int)
        lo, hi = bounds[rank], bounds[rank + 1]
        idx = ShardedFlatIndex(_OracleShard(X[lo:hi], labels[lo:hi]), row_offset=lo, merge=_merge_k11)
        s, r = idx.search(torch.from_numpy(Q), k, label=label)
        ret[rank] = (s.numpy(), r.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,label", [(2, -1), (2, 2), (4, -1)])
def test_sharded_equals_unsharded(world, label):
    from oracle.knn import flat_cosine_topk

    X = clustered_corpus(3001, 96, 4, dup_frac=0.3)  # ties across the shard boundary
    labels = np.random.default_rng(1).integers(0, 4, len(X)).astype(np.int32)
    Q = unit_rows(9, 96, 5)
    k = 10
    ret = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), X, labels, Q, k, label, ret), nprocs=world, join=True)
    es, er = flat_cosine_topk(X, labels, Q, k, label_filter=label)
    for rank in range(world):
        s, r = ret[rank]
        np.testing.assert_array_equal(r, er)
        np.testing.assert_allclose(s, es.astype(np.float32), atol=1e-7)
