"""The offline stand-in tokeniser (app/encoders/tokenize.py, no local vocabulary): the library's
ASCII path (mrag_hash_tokenize) gives exactly the Python path's ids — _basic_tokens (NFC, lower,
`\\w+|[^\\w\\s]`) + _hash_id (crc32) — for every ASCII character, long words, truncation, empty
texts, and batches mixing non-ASCII texts (which stay on the Python path); the CLIP tokeniser
still raises on texts over 77 positions with their exact length."""
from __future__ import annotations

import numpy as np
import pytest


def _python_ids(tok, texts):
    seqs = [tok.encode_one(t) for t in texts]
    return seqs


def _check(tok, texts):
    ids, mask = tok(texts)
    ref = _python_ids(tok, texts)
    T = max(len(s) for s in ref)
    assert ids.shape == (len(texts), T) and mask.shape == ids.shape
    for i, s in enumerate(ref):
        assert ids[i, :len(s)].tolist() == s, i
        assert mask[i].sum() == len(s) and mask[i, :len(s)].all()


def _random_ascii(rng, n, lo=0, hi=200):
    alphabet = [chr(c) for c in range(128)]
    return ["".join(rng.choice(alphabet, int(rng.integers(lo, hi)))) for _ in range(n)]


def test_wordpiece_hash_native_equals_python():
    from app.encoders.tokenize import WordPieceTokenizer

    rng = np.random.default_rng(0)
    tok = WordPieceTokenizer(max_len=32)
    texts = _random_ascii(rng, 300)
    texts += ["", " ", "\x1c\x1d\x1e\x1f", "A" * 700 + " tail", "Hello, World! foo_bar BAZ 123abc",
              "\t\n\v\f\r x \x00\x7f y", "word " * 100]
    _check(tok, texts)


def test_wordpiece_hash_mixed_non_ascii_batch():
    from app.encoders.tokenize import WordPieceTokenizer

    rng = np.random.default_rng(1)
    tok = WordPieceTokenizer(max_len=256)
    texts = _random_ascii(rng, 40) + ["café au lait", "naïve résumé ÉCOLE", "ﬁne Ⅸ ＡＢＣ", "日本語 テキスト"]
    _check(tok, texts)


def test_clip_hash_native_equals_python_and_raises_on_long():
    from app.encoders.tokenize import ClipTokenizer

    rng = np.random.default_rng(2)
    tok = ClipTokenizer()
    texts = _random_ascii(rng, 64, 0, 60)
    _check(tok, texts)
    long = texts + ["w " * 76]  # 76 tokens + BOS + EOS = 78 > 77
    with pytest.raises(ValueError, match="78"):
        tok(long)
    ok = texts + ["w " * 75]  # exactly 77 positions
    _check(tok, ok)


def test_ascii_batches_take_the_library_path(monkeypatch):
    """With 16+ ASCII texts no text goes through the Python tokeniser (the library did them)."""
    from app.encoders import tokenize as tk

    seen = []
    orig = tk._basic_tokens
    monkeypatch.setattr(tk, "_basic_tokens", lambda t, lower=True: seen.append(t) or orig(t, lower))
    tok = tk.WordPieceTokenizer(max_len=64)
    texts = [f"Sentence number {i}, with punctuation!" for i in range(20)] + ["déjà vu"]
    ids, mask = tok(texts)
    assert seen == ["déjà vu"]
    assert ids[0, :3].tolist() == [tk.WordPieceTokenizer.CLS] + [tk._hash_id(w, 1000, 30522) for w in ["sentence", "number"]]
