"""Cross-encoder rerank, CPU side: the golden fixture is reproducible by
the oracle (transformers BertForSequenceClassification, synthetic weights), and the pair
tokenisation calls the HF tokenizer the way sentence-transformers' CrossEncoder does
(padding, truncation='longest_first', max_length) when a vocabulary is present."""
from __future__ import annotations

import os

import numpy as np

from conftest import GOLDEN


def test_golden_cross_encoder_reproducible():
    from oracle import models as om

    g = np.load(os.path.join(GOLDEN, "golden_cross_encoder.npz"))
    got = om.cross_encoder_logits(om.cross_encoder_model(0), g["ids"], g["types"], g["mask"])
    np.testing.assert_allclose(got, g["logits"], rtol=0, atol=1e-5)
    assert g["ids"].shape[1] == 512  # one pair exercises the 512-token truncation


def test_pair_tokenisation_matches_hf_tokenizer(tmp_path):
    from transformers import BertTokenizerFast

    from app.encoders.tokenize import WordPieceTokenizer

    words = ["alpha", "beta", "gamma", "delta", "eps", "zeta", "eta", "theta", "##s", "x", "y"]
    (tmp_path / "vocab.txt").write_text("\n".join(["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + words) + "\n")
    ours = WordPieceTokenizer(str(tmp_path), max_len=12)
    hf = BertTokenizerFast(str(tmp_path / "vocab.txt"), do_lower_case=True)
    pairs = [("alpha beta", "gamma delta eps zeta eta theta x y alpha beta gamma"),
             ("alpha beta gamma delta eps zeta eta", "x y"), ("Alphas beta", "zeta"), ("x", "y")]
    ids, types, mask = ours.pairs(pairs)
    ref = hf([a for a, _ in pairs], [b for _, b in pairs], padding=True, truncation="longest_first", max_length=12,
             return_tensors="np")
    np.testing.assert_array_equal(ids, ref["input_ids"])
    np.testing.assert_array_equal(types, ref["token_type_ids"])
    np.testing.assert_array_equal(mask, ref["attention_mask"])


def test_single_text_tokenisation_matches_hf_tokenizer(tmp_path):
    """MiniLM's tokeniser with a vocabulary (one text, and a batch through encode_batch) gives the
    HF fast tokenizer's ids and mask with truncation=True at max_length, as sentence-transformers
    calls it (reference app/ml/embeddings.py:62-67)."""
    from transformers import BertTokenizerFast

    from app.encoders.tokenize import WordPieceTokenizer

    words = ["alpha", "beta", "gamma", "delta", "eps", "zeta", "eta", "theta", "##s", "x", "y"]
    (tmp_path / "vocab.txt").write_text("\n".join(["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + words) + "\n")
    ours = WordPieceTokenizer(str(tmp_path), max_len=8)
    hf = BertTokenizerFast(str(tmp_path / "vocab.txt"), do_lower_case=True)
    texts = ["alpha beta", "gamma delta eps zeta eta theta x y alpha beta gamma", "Alphas, beta!", "unknownword x"]
    ids, mask = ours(texts)
    ref = hf(texts, padding=True, truncation=True, max_length=8, return_tensors="np")
    np.testing.assert_array_equal(ids, ref["input_ids"])
    np.testing.assert_array_equal(mask, ref["attention_mask"])
    for t in texts:
        assert ours.encode_one(t) == hf(t, truncation=True, max_length=8)["input_ids"]
