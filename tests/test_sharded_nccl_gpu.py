"""The `nccl` (= RCCL) branch of ShardedFlatIndex._gather on hardware (BASELINE config 4):
a world-1 RCCL process group on the box's one GPU — no second process, no exec — so the
all_gather_into_tensor at app/vector_store/sharded.py runs under RCCL exactly as on an 8-GPU
node. The corpus is cut into two shards (two FlatIndex objects, global row offsets 0 and n0);
each shard's local top-k (with the f64 scores the merge orders by) goes through the RCCL
all-gather into the [world, Q, k] layout, the two gathered blocks are stacked as two ranks' lists
would be, and K11 (topk_merge) merges them: rows bit-identical and scores equal to one index over
the whole corpus (ties across the shard boundary included: exact duplicates straddle it)."""
from __future__ import annotations

import os
import socket

import pytest

from _data import unit_rows

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_world1(cuda):
    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        pytest.skip("a process group already exists in this process")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        yield dist.group.WORLD
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dim,k,nq", [(512, 10, 1000), (384, 50, 64)])
def test_rccl_gather_then_k11_equals_single_index(rccl_world1, dim, k, nq):
    import torch

    from app.vector_store import FlatIndex, topk_merge
    from app.vector_store.sharded import ShardedFlatIndex

    n0, n1 = 30011, 26003
    x = unit_rows(n0 + n1, dim, 70 + dim)
    x[n0:n0 + 40] = x[n0 - 40:n0]  # exact duplicates on both sides of the shard boundary
    q = torch.from_numpy(unit_rows(nq, dim, 71 + dim)).cuda()
    q[:8] = torch.from_numpy(x[n0 - 8:n0]).cuda()  # queries that hit the duplicates: ties across shards

    whole = FlatIndex(dim)
    whole.add(x)
    ws, wr, ws64 = whole.search(q, k, with_f64=True)

    gathered_s, gathered_r = [], []
    for lo, hi in ((0, n0), (n0, n0 + n1)):
        local = FlatIndex(dim)
        local.add(x[lo:hi])
        sh = ShardedFlatIndex(local, lo, group=rccl_world1)
        assert sh.world == 1
        s, r, s64 = local.search(q, k, row_offset=lo, with_f64=True)
        g64, gr = sh._gather(s64), sh._gather(r)  # the RCCL all_gather_into_tensor branch
        assert g64.shape == (1, nq, k) and gr.shape == (1, nq, k)
        assert g64.is_cuda and gr.is_cuda
        torch.cuda.synchronize()
        assert torch.equal(g64[0], s64) and torch.equal(gr[0], r)  # world 1: the gather is a copy
        # combine's form: scores and rows packed as 16-byte records, one all-gather, split back
        p64, pr = sh._gather_hits(s64, r)
        torch.cuda.synchronize()
        assert p64.dtype == torch.float64 and pr.dtype == torch.int64
        assert torch.equal(p64, g64) and torch.equal(pr, gr)
        gathered_s.append(g64)
        gathered_r.append(gr)

    ms, mr, m64 = topk_merge(torch.cat(gathered_s), torch.cat(gathered_r), k)
    torch.cuda.synchronize()
    assert torch.equal(mr, wr)
    assert torch.equal(m64, ws64)
    assert torch.equal(ms, ws)
    # the duplicated rows were found on both shards and ordered by row across the boundary
    hit = mr[:8].cpu().numpy()
    assert ((hit >= n0 - 40) & (hit < n0)).any() and ((hit >= n0) & (hit < n0 + 40)).any()
