"""BASELINE.json workloads on the HIP path, each against the CPU oracle.

* C1 — MiniLM-L6 encode of 1k synthetic sentences through the drop-in ``embed_text_batch``
  (app/ml/embeddings.py:52-70) + brute-force cosine top-10 over 10k x 384.
* C2 — CLIP ViT-B/32 image tower at batch 256 (random 224 x 224 u8, the bench's shape) +
  cosine top-10 over 100k x 512.
* C5 — the mixed text+image leg at its per-GPU size (512k x 384 text + 512k x 512 image rows):
  both query towers on synthetic ids, text top-50 / image top-12, and the vectorised fusion
  ``app.retrieval.fuse_scores`` against the reference-pinned ``oracle.fusion.fuse_results``
  (= app/ml/retrieve.py:158-195) on the same hits.

Encoder rows: 1 - cos <= 1e-4 (north_star) and |diff| <= ABS_MAX against the fp32 oracle, errors
recorded in the numerics table. kNN: bit-exact rows and f32 scores against the exact oracle on
the very query vectors the GPU produced (so the comparison isolates the search).
"""
from __future__ import annotations

import numpy as np
import pytest

from _data import unit_rows
from conftest import record_numerics
from oracle.knn import flat_cosine_topk
from test_encoders_gpu import ABS_MAX, COS_ERR_MAX

pytestmark = pytest.mark.gpu


def _check_knn(s, r, os_, or_):
    assert np.array_equal(r, or_), np.argwhere(r != or_)[:5]
    v = or_ >= 0
    assert np.all(s[~v] == -np.inf)
    np.testing.assert_allclose(s[v], os_[v].astype(np.float32), rtol=0, atol=1e-6)


def _enc_ok(name, got, exp):
    row = record_numerics(name, got, exp)
    assert row["max_1_minus_cos"] <= COS_ERR_MAX, row
    assert row["max_abs_diff"] <= ABS_MAX, row


def _sentences(n: int, seed: int):
    """n sentences of 6..62 words from a seeded word list -> 8..64 tokens with [CLS]/[SEP]."""
    rng = np.random.default_rng(seed)
    words = ["".join(chr(97 + c) for c in rng.integers(0, 26, rng.integers(3, 9))) for _ in range(2000)]
    return [" ".join(rng.choice(words, int(rng.integers(6, 63)))) for _ in range(n)]


def test_config1_minilm_1k_sentences_top10_over_10k(cuda):
    from app.encoders.tokenize import WordPieceTokenizer
    from app.ml import embeddings
    from app.vector_store import FlatIndex
    from oracle.models import bert_model, minilm_embeds

    sentences = _sentences(1000, 1)
    got = embeddings.embed_text_batch(sentences)  # drop-in API: tokenise -> GPU MiniLM -> _normalize
    assert got.shape == (1000, 384) and got.dtype == np.float32
    ids, mask = WordPieceTokenizer(None, max_len=256)(sentences)  # the ids the model was fed
    lens = mask.sum(1)
    assert lens.min() == 8 and lens.max() == 64
    exp = minilm_embeds(bert_model(0), ids, mask)
    _enc_ok("C1_minilm_1000_sentences", got, exp)

    corpus = unit_rows(10_000, 384, 0)
    ix = FlatIndex(384)
    ix.add(corpus)
    s, r = ix.search(got, 10)
    os_, or_ = flat_cosine_topk(corpus, np.zeros(len(corpus)), got, 10)
    _check_knn(s, r, os_, or_)


def test_config2_clip_batch256_top10_over_100k(cuda):
    import torch

    from app.encoders import CLIP_VISION_B32, GpuEncoder
    from app.vector_store import FlatIndex
    from oracle.models import clip_image_embeds, clip_model

    rng = np.random.default_rng(2)
    imgs = rng.integers(0, 256, (256, 224, 224, 3), dtype=np.uint8)
    enc = GpuEncoder(CLIP_VISION_B32)
    got = enc.embed_images(torch.from_numpy(imgs).to(cuda)).cpu().numpy()  # device-resident batch, as the bench
    exp = clip_image_embeds(clip_model(0), imgs)
    _enc_ok("C2_clip_image_batch256", got, exp)
    # the host-pointer entry on the same batch gives the same rows (batch-invariant path)
    np.testing.assert_array_equal(enc.embed_images(imgs), got)

    corpus = unit_rows(100_000, 512, 0)
    ix = FlatIndex(512)
    ix.add(corpus)
    s, r = ix.search(got, 10)
    os_, or_ = flat_cosine_topk(corpus, np.zeros(len(corpus)), got, 10)
    _check_knn(s, r, os_, or_)


def test_config5_fusion_leg(cuda):
    """The bench's config-5 leg on one GPU (512k + 512k rows), checked on a query sample."""
    import torch

    from app.encoders import CLIP_TEXT_B32, MINILM_L6, GpuEncoder
    from app.retrieval import fuse_scores
    from app.settings import settings
    from app.vector_store import FlatIndex
    from oracle.fusion import fuse_results
    from oracle.models import bert_model, clip_model, clip_text_embeds, minilm_embeds

    n_rows, nq, T = 1 << 19, 1000, 16
    kt, ki, final_n = settings.retrieval.index_topk_text, settings.retrieval.index_topk_image, settings.retrieval.final_n
    corpora, indexes = [], []
    for dim, seed in ((384, 2000), (512, 3000)):
        g = torch.Generator(device=cuda).manual_seed(seed)
        x = torch.randn((n_rows, dim), generator=g, device=cuda)
        ix = FlatIndex(dim)
        ix.add(x)
        corpora.append(x.cpu().numpy())
        indexes.append(ix)
        del x
    gq = torch.Generator(device=cuda).manual_seed(7)
    ids_m = torch.randint(1000, 30000, (nq, T), generator=gq, device=cuda, dtype=torch.int32)
    ids_m[:, 0], ids_m[:, -1] = 101, 102
    ids_c = torch.randint(1, 49405, (nq, T), generator=gq, device=cuda, dtype=torch.int32)
    ids_c[:, 0], ids_c[:, -1] = 49406, 49407
    tv = GpuEncoder(MINILM_L6).embed_tokens(ids_m, torch.ones_like(ids_m))
    iv = GpuEncoder(CLIP_TEXT_B32).embed_tokens(ids_c)
    st, rt = indexes[0].search(tv, kt)
    si, ri = indexes[1].search(iv, ki)
    pick, comb = fuse_scores(st.cpu().numpy(), si.cpu().numpy(), final_n)
    from app.retrieval import fuse_scores_gpu

    gpick, gcomb = fuse_scores_gpu(st, si, final_n)  # K12, what the bench leg runs
    np.testing.assert_array_equal(gpick.cpu().numpy(), pick)
    np.testing.assert_array_equal(gcomb.cpu().numpy(), comb)

    sel = np.arange(0, nq, 4)  # 250 of the 1000 queries against the f64 oracle
    tvh, ivh = tv.cpu().numpy(), iv.cpu().numpy()
    idm, idc = ids_m.cpu().numpy(), ids_c.cpu().numpy()
    _enc_ok("C5_minilm_queries_T16", tvh[sel], minilm_embeds(bert_model(0), idm[sel], np.ones_like(idm[sel])))
    _enc_ok("C5_clip_text_queries_T16", ivh[sel], clip_text_embeds(clip_model(0), idc[sel], np.ones_like(idc[sel])))
    ost, ort = flat_cosine_topk(corpora[0], np.zeros(n_rows), tvh[sel], kt)
    osi, ori = flat_cosine_topk(corpora[1], np.zeros(n_rows), ivh[sel], ki)
    st, rt, si, ri = (a.cpu().numpy() for a in (st, rt, si, ri))
    _check_knn(st[sel], rt[sel], ost, ort)
    _check_knn(si[sel], ri[sel], osi, ori)

    one = np.float32(1.0)
    for j, q in enumerate(sel):
        # hits as the drop-in store returns them: score = 1 - f32(1 - s) (lancedb_store.py:125-139)
        th = [{"chunk_id": f"t{row}", "score": float(1.0 - float(one - np.float32(sc)))} for sc, row in zip(st[q], rt[q])]
        ih = [{"chunk_id": f"i{row}", "score": float(1.0 - float(one - np.float32(sc)))} for sc, row in zip(si[q], ri[q])]
        ref = fuse_results(th, ih, final_n)
        hits = th + ih
        mine = [hits[p] for p in pick[q] if p >= 0]
        assert [h["chunk_id"] for h in mine] == [h["chunk_id"] for h in ref], q
        np.testing.assert_array_equal(comb[q][: len(ref)], [h["combined_score"] for h in ref])
