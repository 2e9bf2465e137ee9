"""Host tokenisation for the text towers.

The reference tokenises inside sentence-transformers (WordPiece, max_seq_length 256)
and CLIPProcessor (BPE, padding=True, no truncation: >77 tokens raises), both loaded by
hub name — unavailable offline. Two sources, in order:

1. a local model directory (MODEL_TEXT / MODEL_CLIP) with ``vocab.txt`` (WordPiece)
   or ``vocab.json`` + ``merges.txt`` (CLIP BPE): the real tokenisers (``tokenizers``
   / transformers, installed);
2. otherwise a deterministic hashing tokeniser with the same special tokens, lengths
   and padding conventions (BERT-style basic pre-tokenisation; ids hashed into the
   vocabulary). Embeddings then differ from the pretrained model's — only weights
   loaded from a checkpoint make them meaningful — but shapes, masks, truncation and
   throughput are those of the reference. Parity tests feed token ids directly.
"""
from __future__ import annotations

import os
import re
import unicodedata
import zlib
from typing import List, Optional, Sequence, Tuple

import numpy as np

_PUNCT = re.compile(r"\w+|[^\w\s]", re.UNICODE)


def _basic_tokens(text: str, lower: bool = True) -> List[str]:
    t = unicodedata.normalize("NFC", text)
    if lower:
        t = t.lower()
    return _PUNCT.findall(t)


def _hash_id(tok: str, lo: int, hi: int) -> int:
    return lo + zlib.crc32(tok.encode("utf-8")) % (hi - lo)


class _HashIds:
    """_hash_id over a token list with a per-tokeniser memo (a corpus repeats its words: the
    index_text_nodes leg's chunks tokenise ~3x faster); the ids are _hash_id's."""

    def __init__(self, lo: int, hi: int, cap: int = 1 << 20):
        self.lo, self.hi, self.cap = lo, hi, cap
        self.memo: dict = {}

    def __call__(self, toks: List[str]) -> List[int]:
        memo = self.memo
        out = []
        for t in toks:
            i = memo.get(t)
            if i is None:
                i = _hash_id(t, self.lo, self.hi)
                if len(memo) < self.cap:
                    memo[t] = i
            out.append(i)
        return out


_NATIVE_MIN = 16  # texts per call from which the library's ASCII path is used


def _hash_bodies(texts: Sequence[str], ids_of, cap: int) -> Tuple[np.ndarray, np.ndarray]:
    """The hashed token ids of every text, at most ``cap`` per text, as a [n, cap] int32 matrix
    and the per-text counts: ASCII texts through the library (mrag_hash_tokenize: the same tokens
    and crc32 as _basic_tokens + _hash_id, on its own threads) when there are enough of them,
    every other text (and every text without the library) through the Python path ``ids_of``."""
    n = len(texts)
    body = np.zeros((n, cap), dtype=np.int32)
    counts = np.full(n, -1, dtype=np.int32)
    asc = [i for i, t in enumerate(texts) if t.isascii()]
    if len(asc) >= _NATIVE_MIN:
        try:
            import ctypes

            from app import _native
            from app.encoders.preprocess import decode_workers

            bufs = [texts[i].encode("ascii") for i in asc]
            arr = (ctypes.c_char_p * len(bufs))(*bufs)
            lens = np.asarray([len(b) for b in bufs], dtype=np.int64)
            nb = np.zeros((len(asc), cap), dtype=np.int32)
            nc = np.zeros(len(asc), dtype=np.int32)
            _native.call("mrag_hash_tokenize", ctypes.cast(arr, ctypes.c_void_p), lens.ctypes.data, len(asc),
                         ids_of.lo, ids_of.hi, cap, min(8, decode_workers()), nb.ctypes.data, nc.ctypes.data)
            sel = np.asarray(asc)
            body[sel] = nb
            counts[sel] = nc
        except (OSError, ImportError):  # no library here: the Python path below
            pass
    for i in np.flatnonzero(counts < 0).tolist():
        ids = ids_of(_basic_tokens(texts[i]))[:cap]
        body[i, :len(ids)] = ids
        counts[i] = len(ids)
    return body, counts


def _assemble(body: np.ndarray, counts: np.ndarray, first: int, last: int, pad: int) -> Tuple[np.ndarray, np.ndarray]:
    """[first] + body[:count] + [last], padded with ``pad`` to the longest: (ids, mask) int32."""
    n = len(counts)
    T = int(counts.max()) + 2 if n else 2
    col = np.arange(T, dtype=np.int32)[None, :]
    c = counts.astype(np.int32)[:, None]
    ids = np.full((n, T), pad, dtype=np.int32)
    inner = (col >= 1) & (col <= c)
    if T > 2:
        ids[:, 1:T - 1] = np.where(inner[:, 1:T - 1], body[:, :T - 2], pad)
    ids[:, 0] = first
    ids[np.arange(n), counts + 1] = last
    mask = (col < c + 2).astype(np.int32)
    return ids, mask


class WordPieceTokenizer:
    """MiniLM tokeniser: [CLS] ... [SEP], truncation to max_len (ST: 256)."""

    CLS, SEP, PAD = 101, 102, 0

    def __init__(self, model_dir: Optional[str] = None, max_len: int = 256, vocab: int = 30522):
        self.max_len = max_len
        self.vocab = vocab
        self._tok = None
        self._ids = _HashIds(1000, vocab)
        if model_dir and os.path.exists(os.path.join(model_dir, "vocab.txt")):
            from tokenizers import BertWordPieceTokenizer

            self._vocab_path = os.path.join(model_dir, "vocab.txt")
            self._tok = BertWordPieceTokenizer(self._vocab_path, lowercase=True)
            # truncation=True at max_length, [CLS] and the final [SEP] kept (sentence-transformers)
            self._tok.enable_truncation(max_length=max_len)

    def encode_one(self, text: str) -> List[int]:
        if self._tok is not None:
            return self._tok.encode(text).ids  # includes [CLS]/[SEP], truncated to max_len
        body = self._ids(_basic_tokens(text))
        return [self.CLS] + body[: self.max_len - 2] + [self.SEP]

    def __call__(self, texts: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
        if self._tok is None and len(texts) >= _NATIVE_MIN:
            return _assemble(*_hash_bodies(texts, self._ids, self.max_len - 2), self.CLS, self.SEP, self.PAD)
        if self._tok is not None and len(texts) > 1:  # the fast tokeniser's batch form (its own threads)
            seqs = [e.ids for e in self._tok.encode_batch(list(texts))]
        else:
            seqs = [self.encode_one(t) for t in texts]
        T = max(len(s) for s in seqs)
        ids = np.full((len(seqs), T), self.PAD, dtype=np.int32)
        mask = np.zeros((len(seqs), T), dtype=np.int32)
        for i, s in enumerate(seqs):
            ids[i, : len(s)] = s
            mask[i, : len(s)] = 1
        return ids, mask

    def _body(self, text: str) -> List[int]:
        if self._tok is not None:
            return self._tok.encode(text, add_special_tokens=False).ids
        return self._ids(_basic_tokens(text))

    def encode_pair(self, a: str, b: str) -> Tuple[List[int], List[int]]:
        """[CLS] a [SEP] b [SEP] with token types 0 / 1, truncated 'longest_first' (one
        token at a time from the longer side) to max_len — the HF tokenizer's
        truncation=True for pairs, as CrossEncoder.predict calls it."""
        if self._tok is not None:
            if getattr(self, "_pair_tok", None) is None:
                from tokenizers import BertWordPieceTokenizer

                self._pair_tok = BertWordPieceTokenizer(self._vocab_path, lowercase=True)
                self._pair_tok.enable_truncation(max_length=self.max_len, strategy="longest_first")
            enc = self._pair_tok.encode(a, b)
            return list(enc.ids), list(enc.type_ids)
        x, y = self._body(a), self._body(b)
        budget = self.max_len - 3
        while len(x) + len(y) > budget:
            if len(x) > len(y):
                x.pop()
            else:
                y.pop()
        ids = [self.CLS] + x + [self.SEP] + y + [self.SEP]
        types = [0] * (len(x) + 2) + [1] * (len(y) + 1)
        return ids, types

    def pairs(self, pairs: Sequence[Tuple[str, str]]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        enc = [self.encode_pair(a, b) for a, b in pairs]
        T = max(len(i) for i, _ in enc)
        ids = np.full((len(enc), T), self.PAD, dtype=np.int32)
        types = np.zeros((len(enc), T), dtype=np.int32)
        mask = np.zeros((len(enc), T), dtype=np.int32)
        for r, (i, t) in enumerate(enc):
            ids[r, : len(i)] = i
            types[r, : len(t)] = t
            mask[r, : len(i)] = 1
        return ids, types, mask


class ClipTokenizer:
    """CLIP BPE: <|startoftext|> ... <|endoftext|>, padding=True (pad = EOS id), no
    truncation; sequences longer than 77 raise like the reference's model call."""

    BOS, EOS = 49406, 49407

    def __init__(self, model_dir: Optional[str] = None, max_len: int = 77, vocab: int = 49408):
        self.max_len = max_len
        self.vocab = vocab
        self._tok = None
        self._ids = _HashIds(256, self.BOS)
        if model_dir and os.path.exists(os.path.join(model_dir, "vocab.json")) and \
                os.path.exists(os.path.join(model_dir, "merges.txt")):
            from transformers import CLIPTokenizer

            self._tok = CLIPTokenizer(os.path.join(model_dir, "vocab.json"), os.path.join(model_dir, "merges.txt"))

    def encode_one(self, text: str) -> List[int]:
        if self._tok is not None:
            return list(self._tok(text)["input_ids"])
        return [self.BOS] + self._ids(_basic_tokens(text)) + [self.EOS]

    def __call__(self, texts: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
        if self._tok is None and len(texts) >= _NATIVE_MIN:
            body, counts = _hash_bodies(texts, self._ids, self.max_len - 1)
            if int(counts.max()) < self.max_len - 1:  # else a text is too long: its exact length below
                return _assemble(body, counts, self.BOS, self.EOS, self.EOS)
        seqs = [self.encode_one(t) for t in texts]
        T = max(len(s) for s in seqs)
        if T > self.max_len:
            raise ValueError(f"Sequence length {T} exceeds the CLIP text maximum of {self.max_len} positions")
        ids = np.full((len(seqs), T), self.EOS, dtype=np.int32)
        mask = np.zeros((len(seqs), T), dtype=np.int32)
        for i, s in enumerate(seqs):
            ids[i, : len(s)] = s
            mask[i, : len(s)] = 1
        return ids, mask
