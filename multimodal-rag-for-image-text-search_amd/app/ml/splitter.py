"""Text-node construction for ``index_text_nodes`` (host side, off the GPU path).

The reference uses llama_index ``SentenceSplitter(chunk_size=512, chunk_overlap=64)``
(app/ml/index_build.py:14,64) and embeds ``node.get_content(metadata_mode="all")``
(:65) — "key: value" metadata lines, a blank line, then the chunk text. llama_index is
not installed; ``SentenceSplitter`` below restates its algorithm.
"""
from __future__ import annotations

import re
import uuid
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

_SENT = re.compile(r"[^.!?\n]+(?:[.!?]+|\n+|$)")


@dataclass
class TextNode:
    text: str
    metadata: Dict[str, Any] = field(default_factory=dict)
    ref_doc_id: Optional[str] = None
    node_id: str = field(default_factory=lambda: str(uuid.uuid4()))

    def get_content(self, metadata_mode: str = "none") -> str:
        if metadata_mode == "all" and self.metadata:
            meta = "\n".join(f"{k}: {v}" for k, v in self.metadata.items())
            return f"{meta}\n\n{self.text}"
        return self.text


@dataclass
class Document:
    text: str
    metadata: Dict[str, Any] = field(default_factory=dict)
    doc_id: Optional[str] = None


# llama_index.core defaults (node_parser/text/sentence.py, node_parser/text/utils.py)
DEFAULT_PARAGRAPH_SEP = "\n\n\n"
CHUNKING_REGEX = "[^,.;。？！]+[,.;。？！]?"
# fallback token counter: the GPT-2/cl100k pre-tokenizer pattern (each match is >= 1 BPE
# token; whole words of common English text are usually exactly one)
_PRETOKEN = re.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?[A-Za-z]+| ?[0-9]{1,3}| ?[^\sA-Za-z0-9]+|\s+(?!\S)|\s+""")
# fallback sentence spans: Punkt's default behaviour on untrained text — a sentence ends at
# [.!?] (plus closing quotes/brackets) followed by whitespace; the whitespace stays with it
_SENT_SPAN = re.compile(r"\S.*?(?:[.!?][\"')\]]*(?=\s|$)|$)", re.S)


def _default_tokenizer():
    try:  # what llama_index uses (get_tokenizer(): tiktoken cl100k_base)
        import tiktoken

        enc = tiktoken.get_encoding("cl100k_base")
        return enc.encode
    except Exception:
        return lambda text: _PRETOKEN.findall(text)


def _default_sentence_split():
    try:  # llama_index split_by_sentence_tokenizer(): nltk PunktSentenceTokenizer spans
        import nltk

        tok = nltk.tokenize.PunktSentenceTokenizer()

        def split(text: str) -> List[str]:
            spans = list(tok.span_tokenize(text))
            return [text[a:(spans[i + 1][0] if i + 1 < len(spans) else len(text))] for i, (a, _) in enumerate(spans)]

        return split
    except Exception:
        def split(text: str) -> List[str]:
            starts = [m.start() for m in _SENT_SPAN.finditer(text)]
            if not starts:
                return [text] if text else []
            starts[0] = 0
            return [text[a:(starts[i + 1] if i + 1 < len(starts) else len(text))] for i, a in enumerate(starts)]

        return split


def _split_keep_sep(sep: str):
    def split(text: str) -> List[str]:
        parts = text.split(sep)
        return [p for p in ([parts[0]] + [sep + q for q in parts[1:]]) if p]

    return split


@dataclass
class _Split:
    text: str
    is_sentence: bool
    token_size: int


class SentenceSplitter:
    """Restatement of llama_index.core SentenceSplitter (chunk_size / chunk_overlap in
    tokens): split by paragraph ("\\n\\n\\n"), then sentences, then the sub-sentence
    regex, then words, then characters, recursively until every piece fits; merge pieces
    greedily into chunks, carrying up to chunk_overlap tokens of the previous chunk's tail
    (a new chunk always takes its first split, so it may exceed the budget by the carried
    overlap); strip and drop empty chunks. Metadata-aware: the chunk budget is chunk_size minus the
    token count of the document's "key: value" metadata block (get_content(all) prepends
    it). Token counts use tiktoken cl100k_base and sentences nltk Punkt when installed —
    neither is here, so the fallbacks above are used and chunk boundaries are unpinned
    (SURVEY §8f row 4)."""

    def __init__(self, chunk_size: int = 1024, chunk_overlap: int = 200, separator: str = " ",
                 paragraph_separator: str = DEFAULT_PARAGRAPH_SEP, secondary_chunking_regex: str = CHUNKING_REGEX,
                 tokenizer=None, chunking_tokenizer_fn=None):
        if chunk_overlap > chunk_size:
            raise ValueError(f"Got a larger chunk overlap ({chunk_overlap}) than chunk size ({chunk_size}), "
                             "should be smaller.")
        self.chunk_size = chunk_size
        self.chunk_overlap = chunk_overlap
        self._tokenizer = tokenizer or _default_tokenizer()
        sent = chunking_tokenizer_fn or _default_sentence_split()
        self._split_fns = [_split_keep_sep(paragraph_separator), sent]
        rx = re.compile(secondary_chunking_regex)
        self._sub_sentence_split_fns = [lambda t: rx.findall(t), _split_keep_sep(separator), lambda t: list(t)]

    def _token_size(self, text: str) -> int:
        return len(self._tokenizer(text))

    def _get_splits_by_fns(self, text: str):
        for fn in self._split_fns:
            splits = fn(text)
            if len(splits) > 1:
                return splits, True
        for fn in self._sub_sentence_split_fns:
            splits = fn(text)
            if len(splits) > 1:
                break
        return splits, False

    def _split(self, text: str, chunk_size: int) -> List[_Split]:
        size = self._token_size(text)
        if size <= chunk_size:
            return [_Split(text, True, size)]
        pieces, is_sentence = self._get_splits_by_fns(text)
        out: List[_Split] = []
        for p in pieces:
            n = self._token_size(p)
            if n <= chunk_size:
                out.append(_Split(p, is_sentence, n))
            else:
                out.extend(self._split(p, chunk_size))
        return out

    def _merge(self, splits: List[_Split], chunk_size: int) -> List[str]:
        chunks: List[str] = []
        cur: List[tuple] = []
        cur_len = 0
        new_chunk = True

        def close_chunk():
            nonlocal cur, cur_len, new_chunk
            chunks.append("".join(t for t, _ in cur))
            last = cur
            cur, cur_len, new_chunk = [], 0, True
            i = len(last) - 1
            while i >= 0 and cur_len + last[i][1] <= self.chunk_overlap:
                cur_len += last[i][1]
                cur.insert(0, last[i])
                i -= 1

        splits = list(splits)
        while splits:
            sp = splits[0]
            if sp.token_size > chunk_size:
                raise ValueError("Single token exceeded chunk size")
            if cur_len + sp.token_size > chunk_size and not new_chunk:
                close_chunk()
            elif sp.is_sentence or cur_len + sp.token_size <= chunk_size or new_chunk:
                cur_len += sp.token_size
                cur.append((sp.text, sp.token_size))
                splits.pop(0)
                new_chunk = False
            else:
                close_chunk()
        if not new_chunk:
            chunks.append("".join(t for t, _ in cur))
        return [c.strip() for c in chunks if c.strip()]

    def split_text_metadata_aware(self, text: str, metadata_str: str) -> List[str]:
        effective = self.chunk_size - self._token_size(metadata_str)
        if effective <= 0:
            raise ValueError(f"Metadata length ({self.chunk_size - effective}) is longer than chunk size "
                             f"({self.chunk_size}). Consider increasing the chunk size or decreasing the size of "
                             "your metadata to avoid this.")
        return self.split_text(text, effective)

    def split_text(self, text: str, chunk_size: Optional[int] = None) -> List[str]:
        if text == "":
            return [text]
        cs = self.chunk_size if chunk_size is None else chunk_size
        return self._merge(self._split(text, cs), cs)

    def get_nodes_from_documents(self, documents: List[Document]) -> List[TextNode]:
        nodes: List[TextNode] = []
        for d in documents:
            meta = "\n".join(f"{k}: {v}" for k, v in d.metadata.items())
            for chunk in self.split_text_metadata_aware(d.text, meta):
                nodes.append(TextNode(text=chunk, metadata=dict(d.metadata), ref_doc_id=d.doc_id))
        return nodes
