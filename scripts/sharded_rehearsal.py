#!/usr/bin/env python3
"""The N > 1 kNN path (BASELINE config 4) on whatever GPUs the box has, checked end to end:
    MRAG_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29533 scripts/sharded_rehearsal.py
Rank r builds bench.py's shard r (2^18 rows here, seed 1000 + r, global rows r * 2^18 + i) on
GPU r % device_count, every rank searches the same 1000 queries, ShardedFlatIndex all-gathers
the per-shard (f64 score, row) lists and merges them with K11. Rank 0 then rebuilds all shards
into ONE index and checks the sharded result equals the single-index search bit for bit (rows
and f32 scores), the property app/vector_store/sharded.py promises. With the default backend
(nccl = RCCL) this is the driver's N-GPU configuration in small."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402

ROWS, DIM, NQ, K = 1 << 18, 512, 1000, 10


def shard(r, dev):
    g = torch.Generator(device=dev).manual_seed(1000 + r)
    x = torch.randn((ROWS, DIM), generator=g, device=dev)
    return x / x.norm(dim=1, keepdim=True)


def main():
    world, rank, local = bench._dist_setup()
    dev = torch.device("cuda", local)
    from app.vector_store import FlatIndex
    from app.vector_store.sharded import ShardedFlatIndex

    ix = FlatIndex(DIM, device=local)
    ix.add(shard(rank, dev))
    sh = ShardedFlatIndex(ix, row_offset=rank * ROWS)
    q = torch.randn((NQ, DIM), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    s, r = sh.search(q, K)
    s2, r2 = sh.search(q, K)  # twice: deterministic
    ok = {"world": world, "backend": dist.get_backend() if dist.is_initialized() else None}
    if rank == 0:
        whole = FlatIndex(DIM, device=local)
        for j in range(world):
            whole.add(shard(j, dev))
        ws, wr = whole.search(q, K)
        ok["rows_equal_single_index"] = bool(torch.equal(r.cpu(), wr.cpu()))
        ok["scores_equal_single_index"] = bool(torch.equal(s.cpu(), ws.cpu()))
        ok["repeatable"] = bool(torch.equal(r.cpu(), r2.cpu()) and torch.equal(s.cpu(), s2.cpu()))
        ok["rows_from_every_shard"] = sorted({int(v) // ROWS for v in r.cpu().flatten().tolist()})
        print(json.dumps(ok), flush=True)
        assert ok["rows_equal_single_index"] and ok["scores_equal_single_index"] and ok["repeatable"], ok
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
