"""BASELINE configs 4 and 5 at FULL size on one MI355X, against the CPU oracle.

* C4 — 8M x 512 row-sharded: eight ``FlatIndex`` shards of 2^20 rows (shard r generated exactly
  as bench.py's rank r: torch seed 1000 + r, unit rows) with global row offsets r * 2^20, each
  searched for the bench's 1000 queries (torch seed 1) with f64 scores, the [8, Q, k] lists
  merged by K11 (``topk_merge``) — the single-GPU form of the RCCL all-gather + merge of
  app/vector_store/sharded.py. Checked (a) bit-exact against the exact f64 oracle over the
  concatenated 8M rows on 64 sampled queries and (b) equal, for all 1000 queries, to ONE
  unsharded index of the same 8M rows (the reference's single table,
  app/storage/lancedb_store.py:103-123).
* C5 — 4M x 384 text + 4M x 512 image corpora on one index each (built from the bench's eight
  per-rank chunks, seeds 2000 + r / 3000 + r), both query towers on the bench's synthetic ids,
  text top-50 / image top-12 and the K12 fusion (app/ml/retrieve.py:103-117,158-195), checked on
  64 sampled queries against the exact oracle and oracle.fusion on the same hits.

The oracle runs shard by shard (its per-shard exact top-k lists merged under the tie rule are the
top-k of the concatenation), so host memory stays at one shard.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.fusion import fuse_results
from oracle.knn import flat_cosine_topk
from oracle.merge import topk_merge as oracle_merge

pytestmark = pytest.mark.gpu

SHARD = 1 << 20
NQ = 1000
SAMPLE = np.arange(0, NQ, NQ // 64)[:64]


def _check(s, r, os_, or_):
    assert np.array_equal(r, or_), np.argwhere(r != or_)[:5]
    v = or_ >= 0
    assert np.all(np.isneginf(s[~v]))
    np.testing.assert_allclose(s[v], os_[v].astype(np.float32), rtol=0, atol=1e-6)


@pytest.mark.timeout(900)
def test_config4_8m_x_512_sharded(cuda):
    import torch

    from app.vector_store import FlatIndex, topk_merge

    k = 10
    gq = torch.Generator(device=cuda).manual_seed(1)
    q = torch.randn((NQ, 512), generator=gq, device=cuda)
    qs = q.cpu().numpy()[SAMPLE]
    s64s, rows, cand_s, cand_r = [], [], [], []
    whole = FlatIndex(512)
    for r in range(8):
        g = torch.Generator(device=cuda).manual_seed(1000 + r)
        x = torch.randn((SHARD, 512), generator=g, device=cuda)
        x = x / x.norm(dim=1, keepdim=True)
        ix = FlatIndex(512)
        ix.add(x)
        whole.add(x)
        _, rr, ss = ix.search(q, k, row_offset=r * SHARD, with_f64=True)
        s64s.append(ss)
        rows.append(rr)
        unc, _ = ix.last_stats()
        assert unc == 0, (r, unc)  # random unit rows certify on the first pass
        ix.close()
        xh = x.cpu().numpy()
        del x
        os_, or_ = flat_cosine_topk(xh, np.zeros(SHARD, np.int32), qs, k, row_offset=r * SHARD)
        cand_s.append(os_)
        cand_r.append(or_)
        del xh
    ms, mr, m64 = topk_merge(torch.stack(s64s), torch.stack(rows), k)
    ms, mr = ms.cpu().numpy(), mr.cpu().numpy()
    assert len(whole) == 8 * SHARD
    # (a) the exact oracle over the concatenated 8M rows, on the sample
    _, oref_r, oref64 = oracle_merge(np.stack(cand_s), np.stack(cand_r), k)
    _check(ms[SAMPLE], mr[SAMPLE], oref64, oref_r)
    # (b) sharded == unsharded for every query
    ws, wr = whole.search(q, k)
    np.testing.assert_array_equal(mr, wr.cpu().numpy())
    np.testing.assert_array_equal(ms, ws.cpu().numpy())


@pytest.mark.timeout(900)
def test_config5_4m_plus_4m_fusion(cuda):
    import torch

    from app.encoders import CLIP_TEXT_B32, MINILM_L6, GpuEncoder
    from app.retrieval import fuse_scores_gpu
    from app.settings import settings
    from app.vector_store import FlatIndex

    chunk, T = 1 << 19, 16
    kt, ki, final_n = settings.retrieval.index_topk_text, settings.retrieval.index_topk_image, settings.retrieval.final_n
    gq = torch.Generator(device=cuda).manual_seed(7)  # bench._fusion_queries
    ids_m = torch.randint(1000, 30000, (NQ, T), generator=gq, device=cuda, dtype=torch.int32)
    ids_m[:, 0], ids_m[:, -1] = 101, 102
    ids_c = torch.randint(1, 49405, (NQ, T), generator=gq, device=cuda, dtype=torch.int32)
    ids_c[:, 0], ids_c[:, -1] = 49406, 49407
    tv = GpuEncoder(MINILM_L6).embed_tokens(ids_m, torch.ones_like(ids_m))
    iv = GpuEncoder(CLIP_TEXT_B32).embed_tokens(ids_c)
    results = []
    for dim, seed, qv, k in ((384, 2000, tv, kt), (512, 3000, iv, ki)):
        ix = FlatIndex(dim)
        qh = qv.cpu().numpy()[SAMPLE]
        cs, cr = [], []
        for r in range(8):
            g = torch.Generator(device=cuda).manual_seed(seed + r)
            x = torch.randn((chunk, dim), generator=g, device=cuda)
            ix.add(x)
            xh = x.cpu().numpy()
            del x
            os_, or_ = flat_cosine_topk(xh, np.zeros(chunk, np.int32), qh, k, row_offset=r * chunk)
            cs.append(os_)
            cr.append(or_)
            del xh
        assert len(ix) == 8 * chunk
        s, rr = ix.search(qv, k)
        _, oref_r, oref64 = oracle_merge(np.stack(cs), np.stack(cr), k)
        _check(s.cpu().numpy()[SAMPLE], rr.cpu().numpy()[SAMPLE], oref64, oref_r)
        results.append((s, rr))
        ix.close()
    (st, rt), (si, ri) = results
    gpick, gcomb = fuse_scores_gpu(st, si, final_n)
    gpick, gcomb = gpick.cpu().numpy(), gcomb.cpu().numpy()
    st, rt, si, ri = (a.cpu().numpy() for a in (st, rt, si, ri))
    one = np.float32(1.0)
    for q in SAMPLE:
        # hits as the drop-in store returns them: score = 1 - f32(1 - s) (lancedb_store.py:125-139)
        th = [{"chunk_id": f"t{row}", "score": float(1.0 - float(one - np.float32(sc)))} for sc, row in zip(st[q], rt[q])]
        ih = [{"chunk_id": f"i{row}", "score": float(1.0 - float(one - np.float32(sc)))} for sc, row in zip(si[q], ri[q])]
        ref = fuse_results(th, ih, final_n)
        hits = th + ih
        mine = [hits[p] for p in gpick[q] if p >= 0]
        assert [h["chunk_id"] for h in mine] == [h["chunk_id"] for h in ref], q
        np.testing.assert_array_equal(gcomb[q][: len(ref)], [h["combined_score"] for h in ref])
