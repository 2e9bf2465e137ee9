"""Text-node construction for ``index_text_nodes`` (host side, off the GPU path).

The reference uses llama_index ``SentenceSplitter(chunk_size=512, chunk_overlap=64)``
(app/ml/index_build.py:14,64) and embeds ``node.get_content(metadata_mode="all")``
(:65) — "key: value" metadata lines, a blank line, then the chunk text. llama_index
and its tiktoken vocabulary are not installed; this splitter keeps the contract
(sentence-aware packing into <= chunk_size token chunks with chunk_overlap tokens of
overlap, document metadata inherited by every node, uuid4 node ids) with whitespace
tokens as the token count. SURVEY.md §8f lists an exact restatement as a later row.
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


class SentenceSplitter:
    def __init__(self, chunk_size: int = 512, chunk_overlap: int = 64):
        if chunk_overlap >= chunk_size:
            raise ValueError("chunk_overlap must be smaller than chunk_size")
        self.chunk_size = chunk_size
        self.chunk_overlap = chunk_overlap

    def _pieces(self, text: str) -> List[str]:
        out = []
        for s in _SENT.findall(text):
            s = s.strip()
            if not s:
                continue
            words = s.split()
            while len(words) > self.chunk_size:  # over-long sentence: split on words
                out.append(" ".join(words[: self.chunk_size]))
                words = words[self.chunk_size:]
            if words:
                out.append(" ".join(words))
        return out

    def split_text(self, text: str) -> List[str]:
        pieces = self._pieces(text)
        chunks: List[str] = []
        cur: List[str] = []
        cur_len = 0
        for p in pieces:
            n = len(p.split())
            if cur and cur_len + n > self.chunk_size:
                chunks.append(" ".join(cur))
                keep: List[str] = []
                k_len = 0
                for q in reversed(cur):  # carry up to chunk_overlap tokens of whole sentences
                    qn = len(q.split())
                    if k_len + qn > self.chunk_overlap:
                        break
                    keep.insert(0, q)
                    k_len += qn
                cur, cur_len = keep, k_len
            cur.append(p)
            cur_len += n
        if cur:
            chunks.append(" ".join(cur))
        return chunks

    def get_nodes_from_documents(self, documents: List[Document]) -> List[TextNode]:
        nodes: List[TextNode] = []
        for d in documents:
            for chunk in self.split_text(d.text):
                nodes.append(TextNode(text=chunk, metadata=dict(d.metadata), ref_doc_id=d.doc_id))
        return nodes
