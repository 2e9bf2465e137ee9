"""Compatibility shim for the reference's dead ``app/embedding/embedder.py`` (:15-68).

Nothing in the reference imports ``Embedder`` except a stale test; it is kept as a thin
facade over the same GPU encoders so code written against it still runs. Outputs follow
what the reference's ``SentenceTransformer(...).encode(convert_to_tensor=True)`` returns
(sentence-transformers is not installed here, so this is a restatement, parity unpinned):

* ``embed_text`` -> MiniLM [N,384] float32, unit rows (all-MiniLM-L6-v2's pipeline ends in a
  Normalize module; no extra numpy ``_normalize``);
* ``embed_text_for_images`` -> CLIP text features [N,512] float32, NOT normalised
  (sentence-transformers' CLIPModel module returns ``text_embeds`` = the projection);
* ``embed_images`` -> CLIP image features [N,512] float32, NOT normalised (``image_embeds``);
* empty input -> ``np.empty((0, 0))`` (float64, as the reference); model-name resolution
  and errors as ``app.encoders.models`` (an unresolvable name raises).
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence

import numpy as np

from app.settings import settings


class _LlamaTextEmbedding:
    """Minimal stand-in for the LlamaIndex HuggingFaceEmbedding handle."""

    def __init__(self, embedder: "Embedder"):
        self._e = embedder

    def get_text_embedding(self, text: str) -> List[float]:
        return self._e.embed_text([text])[0].tolist()

    def get_text_embedding_batch(self, texts: Sequence[str], **kw) -> List[List[float]]:
        return self._e.embed_text(list(texts)).tolist()

    def get_query_embedding(self, query: str) -> List[float]:
        return self.get_text_embedding(query)


class Embedder:
    def __init__(self, text_model_name: Optional[str] = None, clip_model_name: Optional[str] = None) -> None:
        from app.encoders.models import ClipModel, ClipProcessor, MiniLMSentenceModel

        self._text_model = MiniLMSentenceModel(text_model_name or settings.models.text)
        self._clip = ClipModel(clip_model_name or settings.models.clip)
        self._proc = ClipProcessor(clip_model_name or settings.models.clip)
        self._llama_text_embed = _LlamaTextEmbedding(self)

    def llama_text_embedder(self):
        return self._llama_text_embed

    def embed_text(self, text_list: Sequence[str]) -> np.ndarray:
        if not text_list:
            return np.empty((0, 0))
        return self._text_model.encode(list(text_list), convert_to_tensor=True).cpu().numpy()

    def embed_text_for_images(self, text_list: Sequence[str]) -> np.ndarray:
        if not text_list:
            return np.empty((0, 0))
        inputs = self._proc(text=list(text_list))
        return self._clip.get_text_features(**inputs).cpu().numpy()

    def embed_images(self, image_paths: Iterable[str]) -> np.ndarray:
        paths = list(image_paths)
        if not paths:
            return np.empty((0, 0))
        return self._clip.get_image_features(**self._proc(images=paths)).cpu().numpy()
