"""GPU cross-encoder (MRAG_ENC_BERT_PAIR) against the oracle
(transformers BertForSequenceClassification, same synthetic weights): logits on the golden
pairs (L up to 512: the attention kernel's long-sequence path), sentence-transformers'
predict() conventions, and the reference's _rerank_text (app/ml/retrieve.py:132-155) on the
GPU model vs the same function on the oracle model.

Tolerance: fp16 GEMM inputs with f32 accumulation through 6 post-LN layers; logits are
checked to |delta| <= 3e-3 (observed 6.2e-4, profiles/r2_numerics.json; their spread on these
pairs is ~0.6)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import GOLDEN, record_numerics

pytestmark = pytest.mark.gpu

ATOL = 3e-3


@pytest.fixture(scope="module")
def ce(cuda):
    from app.encoders.models import CrossEncoderModel

    return CrossEncoderModel()


def test_logits_golden(ce):
    g = np.load(os.path.join(GOLDEN, "golden_cross_encoder.npz"))
    got = ce.enc.score_pairs(g["ids"], g["types"], g["mask"])
    record_numerics("cross_encoder_logits", got, g["logits"], unit=False,
                    logit_spread=float(np.ptp(g["logits"])))
    np.testing.assert_allclose(got, g["logits"], rtol=0, atol=ATOL)
    # a padded row scores like the same row alone (mask + [CLS] pooling)
    one = ce.enc.score_pairs(g["ids"][2:3, :12], g["types"][2:3, :12], g["mask"][2:3, :12])
    np.testing.assert_allclose(one, got[2:3], rtol=0, atol=2e-3)


def test_predict_conventions(ce):
    g = np.load(os.path.join(GOLDEN, "golden_cross_encoder.npz"))
    pairs = [tuple(s.split("\t")) for s in g["pairs"]]
    scores = ce.predict(pairs, batch_size=4)  # two batches of different padded length
    assert scores.dtype == np.float32 and scores.shape == (len(pairs),)
    # no config.json -> sentence-transformers' default for one label: sigmoid of the logits
    np.testing.assert_allclose(scores, 1 / (1 + np.exp(-g["logits"][:, 0])), rtol=0, atol=ATOL / 4)
    single = ce.predict(pairs[0])
    assert np.ndim(single) == 0 and abs(float(single) - float(scores[0])) < 1e-6


def test_rerank_text_matches_oracle(ce, monkeypatch):
    from app.ml import retrieve
    from oracle import models as om

    class OracleCE:
        def __init__(self, tok):
            self.m, self.tok = om.cross_encoder_model(0), tok

        def predict(self, pairs):
            ids, types, mask = self.tok.pairs(pairs)
            z = om.cross_encoder_logits(self.m, ids, types, mask)[:, 0]
            return (1 / (1 + np.exp(-z.astype(np.float64)))).astype(np.float32)

    rng = np.random.default_rng(3)
    words = [f"w{i}" for i in range(300)]
    results = [{"chunk_id": f"c{i}", "modality": "text", "score": float(0.9 - 0.01 * i), "metadata": {},
                "text": " ".join(rng.choice(words, int(rng.integers(5, 200))))} for i in range(12)]
    assert retrieve.settings.retrieval.use_rerank  # RERANK_ENABLED defaults to true (settings.py)
    monkeypatch.setattr(retrieve, "_CROSS_ENCODER", ce)
    got = retrieve._rerank_text("w1 w2 w3", [dict(r) for r in results])
    monkeypatch.setattr(retrieve, "_CROSS_ENCODER", OracleCE(ce.tokenizer))
    ref = retrieve._rerank_text("w1 w2 w3", [dict(r) for r in results])
    assert len(got) == len(ref) == 12
    k = retrieve.settings.retrieval.rerank_topk
    gs = {r["chunk_id"]: r["rerank_score"] for r in got if "rerank_score" in r}
    rs = {r["chunk_id"]: r["rerank_score"] for r in ref if "rerank_score" in r}
    assert gs.keys() == rs.keys() and len(gs) == k
    np.testing.assert_allclose([gs[c] for c in sorted(gs)], [rs[c] for c in sorted(rs)], rtol=0, atol=ATOL / 4)
    # order agrees wherever the oracle's scores are separated by more than the tolerance
    ref_order = [r["chunk_id"] for r in ref]
    got_order = [r["chunk_id"] for r in got]
    for i in range(len(ref_order) - 1):
        a, b = ref_order[i], ref_order[i + 1]
        if a in rs and b in rs and rs[a] - rs[b] > ATOL / 2:
            assert got_order.index(a) < got_order.index(b)
