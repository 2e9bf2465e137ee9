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
