"""``Embedder`` compat shim (reference app/embedding/embedder.py:15-68): shapes,
dtypes and the empty-input convention ``np.empty((0, 0))``, the LlamaIndex handle, and the
model-resolution policy. The model objects are replaced by dummies here (as the reference's
own tests do for its embedding helpers); values through the GPU towers are checked in
``tests/test_embedder_gpu.py``."""
from __future__ import annotations

import numpy as np
import pytest
import torch


class _DummyText:
    def __init__(self, name=None, device=None):
        self.name = name

    def encode(self, sentences, batch_size=32, convert_to_tensor=False, **kw):
        x = torch.arange(len(sentences) * 384, dtype=torch.float32).reshape(len(sentences), 384) + 1
        x = x / x.norm(dim=1, keepdim=True)
        return x if convert_to_tensor else x.numpy()


class _DummyClip:
    def __init__(self, name=None, device=None):
        self.name = name

    def get_text_features(self, input_ids=None, attention_mask=None, **kw):
        return torch.full((len(input_ids), 512), 2.0)

    def get_image_features(self, images_u8=None, **kw):
        return torch.full((len(images_u8), 512), 3.0)


class _DummyProc:
    def __init__(self, name=None):
        self.name = name

    def __call__(self, images=None, text=None, **kw):
        if images is not None:
            return {"images_u8": np.zeros((len(images), 224, 224, 3), np.uint8)}
        return {"input_ids": np.ones((len(text), 5), np.int32), "attention_mask": np.ones((len(text), 5), np.int32)}


@pytest.fixture
def embedder(monkeypatch):
    import app.encoders.models as m

    monkeypatch.setattr(m, "MiniLMSentenceModel", _DummyText)
    monkeypatch.setattr(m, "ClipModel", _DummyClip)
    monkeypatch.setattr(m, "ClipProcessor", _DummyProc)
    from app.embedding.embedder import Embedder

    return Embedder()


def test_empty_inputs_are_0x0(embedder):
    for fn in (embedder.embed_text, embedder.embed_text_for_images, embedder.embed_images):
        out = fn([])
        assert isinstance(out, np.ndarray) and out.shape == (0, 0)


def test_shapes_and_values(embedder):
    t = embedder.embed_text(["a", "b", "c"])
    assert t.shape == (3, 384) and t.dtype == np.float32
    np.testing.assert_allclose(np.linalg.norm(t, axis=1), 1.0, rtol=1e-6)
    ti = embedder.embed_text_for_images(["x", "y"])
    assert ti.shape == (2, 512) and np.all(ti == 2.0)  # raw CLIP text features (no normalise)
    im = embedder.embed_images(["p1.png", "p2.png", "p3.png", "p4.png"])
    assert im.shape == (4, 512) and np.all(im == 3.0)  # raw CLIP image features


def test_default_model_names(embedder):
    from app.settings import settings

    assert embedder._text_model.name == settings.models.text
    assert embedder._clip.name == settings.models.clip


def test_llama_handle(embedder):
    h = embedder.llama_text_embedder()
    v = h.get_text_embedding("hello")
    assert isinstance(v, list) and len(v) == 384
    b = h.get_text_embedding_batch(["a", "b"])
    assert len(b) == 2 and len(b[0]) == 384
    assert h.get_query_embedding("hello") == v


def test_unresolvable_model_raises(monkeypatch, tmp_path):
    monkeypatch.delenv("MRAG_SYNTHETIC_WEIGHTS", raising=False)
    monkeypatch.setenv("HF_HOME", str(tmp_path))
    monkeypatch.setenv("HOME", str(tmp_path))
    for v in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE", "SENTENCE_TRANSFORMERS_HOME"):
        monkeypatch.delenv(v, raising=False)
    from app.embedding.embedder import Embedder

    with pytest.raises(OSError):
        Embedder()
