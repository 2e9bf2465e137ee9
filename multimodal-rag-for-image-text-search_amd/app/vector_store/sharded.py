"""Row-sharded flat index over one node's GPUs (BASELINE config 4).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI). Rank r owns
the contiguous global rows [row_offset_r, row_offset_r + n_r) in its own
``FlatIndex``. A search is:

  1. local exact top-k on every rank (K7/K8/K10; global row ids via row_offset);
  2. ONE all-gather of the per-shard (f64 score, int64 row) lists packed as 16-byte records,
     [world, nq, k, 2] (1000 x 10 x 16 B = 160 KB per rank: latency-bound, far below the scan
     time; one collective per step, not one per list);
  3. the K11 merge under (score desc, row asc) — identical to a single-index search
     because every shard's list is its exact top-k.

No other collective exists on the data path; queries are replicated (every rank gets
the same batch), results are replicated on every rank.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple


class ShardedFlatIndex:
    def __init__(self, local_index, row_offset: int, group=None,
                 merge: Optional[Callable] = None):
        import torch.distributed as dist

        self.local = local_index
        self.row_offset = int(row_offset)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if merge is None:
            from app.vector_store import topk_merge

            merge = topk_merge
        self._merge = merge
        self._buf = None

    def _gather(self, t):
        import torch
        import torch.distributed as dist

        shape = (self.world,) + tuple(t.shape)
        if dist.get_backend(self.group) == "nccl":
            out = torch.empty(shape, dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
            return out
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.stack(parts)

    def search(self, queries, k: int, label: int = -1) -> Tuple:
        """(scores f32 [nq,k], rows int64 [nq,k]) over the whole sharded corpus."""
        return self.combine(self.search_local(queries, k, label=label), k)

    def search_local(self, queries, k: int, label: int = -1) -> Tuple:
        """Step 1 alone: this shard's exact top-k with global row ids (plus the f64 scores the
        merge orders by when world > 1). Safe to run from several host threads at once, each on
        its own stream (the library gives every search its own workspace)."""
        if self.world == 1:
            return self.local.search(queries, k, label=label, row_offset=self.row_offset)
        return self.local.search(queries, k, label=label, row_offset=self.row_offset, with_f64=True)

    def combine(self, local, k: int) -> Tuple:
        """Steps 2-3 on the calling thread's current stream: all-gather + K11 merge. Every rank
        must combine its searches in the same order (one communicator)."""
        if self.world == 1:
            return local
        import torch

        s, r, s64 = local
        if s64.is_cuda:  # produced on another stream: keep the memory until this one is done
            cur = torch.cuda.current_stream(s64.device)
            for t in (s64, r):
                t.record_stream(cur)
        ms, mr, _ = self._merge(*self._gather_hits(s64, r), k)
        return ms, mr

    def _gather_hits(self, s64, r):
        """Every rank's (f64 scores, int64 rows) lists as [world, nq, k] each, in ONE collective:
        a hit's score (its 8 bytes as int64) and row travel as one 16-byte record, [nq, k, 2],
        split back bit for bit."""
        import torch

        packed = torch.stack((s64.contiguous().view(torch.int64), r.to(torch.int64)), dim=-1)
        g = self._gather(packed)
        return g[..., 0].contiguous().view(torch.float64), g[..., 1].contiguous()


__all__ = ["ShardedFlatIndex"]
