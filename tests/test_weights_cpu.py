"""Weight loading policy (CPU): the reference loads models by hub name and raises when it
cannot (app/ml/embeddings.py:23-43: SentenceTransformer(...) / CLIPModel.from_pretrained);
the drop-in must not silently substitute synthetic weights. Synthetic weights are an explicit
opt-in (MRAG_SYNTHETIC_WEIGHTS=1); checkpoints load from a directory or a cached hub snapshot,
as safetensors or pytorch_model.bin (torch.load weights_only=True)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from app.encoders.weights import (
    EncoderConfig,
    checkpoint_state_dict,
    encoder_weights,
    param_specs,
    resolve_model_dir,
    synth_state_dict,
)

TINY_BERT = EncoderConfig(kind=3, hidden=8, layers=1, heads=2, intermediate=16, max_positions=8, vocab=12, act=1,
                          ln_eps=1e-12)


@pytest.fixture
def offline(monkeypatch, tmp_path):
    """No synthetic opt-in and an empty Hugging Face cache."""
    monkeypatch.delenv("MRAG_SYNTHETIC_WEIGHTS", raising=False)
    monkeypatch.delenv("MRAG_SYNTHETIC_RERANKER", raising=False)
    for v in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE", "SENTENCE_TRANSFORMERS_HOME"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("HF_HOME", str(tmp_path / "hf"))
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    return tmp_path


def test_hub_name_without_checkpoint_raises(offline, monkeypatch):
    from app.encoders.models import ClipModel, ClipProcessor, MiniLMSentenceModel
    from app.ml import embeddings

    with pytest.raises(OSError, match="MRAG_SYNTHETIC_WEIGHTS"):
        MiniLMSentenceModel("sentence-transformers/all-MiniLM-L6-v2")
    with pytest.raises(OSError):
        ClipModel("openai/clip-vit-base-patch32")
    with pytest.raises(OSError):
        ClipProcessor("openai/clip-vit-base-patch32")
    # through the reference's entry points (lazy singletons, app/ml/embeddings.py:23-43)
    monkeypatch.setattr(embeddings, "_TEXT_MODEL", None)
    monkeypatch.setattr(embeddings, "_CLIP_MODEL", None)
    monkeypatch.setattr(embeddings, "_CLIP_PROCESSOR", None)
    with pytest.raises(OSError):
        embeddings.embed_text_batch(["a sentence"])
    with pytest.raises(OSError):
        embeddings.embed_query_for_images("a photo of a cat")
    # the empty conventions still hold without touching a model (:59-60, :97-98)
    assert embeddings.embed_text_batch([]).shape == (0, 384)
    assert np.array_equal(embeddings.embed_query_for_images("   "), np.zeros(512, np.float32))


def test_encoder_weights_policy(offline, monkeypatch):
    with pytest.raises(OSError):
        encoder_weights(TINY_BERT, "org/some-model")
    assert encoder_weights(TINY_BERT, "org/some-model", synthetic=True) == (None, None)
    monkeypatch.setenv("MRAG_SYNTHETIC_WEIGHTS", "1")
    assert encoder_weights(TINY_BERT, None) == (None, None)


def test_reranker_offline_is_skipped_like_the_reference(offline):
    # the reference swallows the CrossEncoder load failure and skips rerank (retrieve.py:29-38)
    from app.ml import retrieve

    assert retrieve._gpu_cross_encoder() is False


def _write_checkpoint(d, fmt):
    sd = dict(synth_state_dict(TINY_BERT, seed=5))
    os.makedirs(d, exist_ok=True)
    if fmt == "safetensors":
        from safetensors.numpy import save_file

        save_file({k: np.ascontiguousarray(v) for k, v in sd.items()}, os.path.join(d, "model.safetensors"))
    else:
        import torch

        torch.save({k: torch.from_numpy(v.copy()) for k, v in sd.items()}, os.path.join(d, "pytorch_model.bin"))
    return sd


@pytest.mark.parametrize("fmt", ["safetensors", "bin"])
def test_checkpoint_formats(tmp_path, fmt):
    d = str(tmp_path / fmt)
    sd = _write_checkpoint(d, fmt)
    got = checkpoint_state_dict(d, TINY_BERT)
    assert set(got) == {n for n, _, _ in param_specs(TINY_BERT)}
    for k, v in sd.items():
        assert np.array_equal(got[k], v), k


def test_checkpoint_errors(tmp_path):
    empty = tmp_path / "empty"
    empty.mkdir()
    with pytest.raises(FileNotFoundError):
        checkpoint_state_dict(str(empty), TINY_BERT)
    with pytest.raises(FileNotFoundError):
        checkpoint_state_dict(str(tmp_path / "nope"), TINY_BERT)
    partial = tmp_path / "partial"
    sd = dict(synth_state_dict(TINY_BERT))
    sd.pop("encoder.layer.0.output.dense.weight")
    partial.mkdir()
    from safetensors.numpy import save_file

    save_file(sd, str(partial / "model.safetensors"))
    with pytest.raises(ValueError, match="lacks 1 parameters"):
        checkpoint_state_dict(str(partial), TINY_BERT)


def test_hub_cache_snapshot_resolution(offline):
    hub = offline / "hf" / "hub" / "models--org--tiny-bert"
    snap = hub / "snapshots" / "abc123"
    _write_checkpoint(str(snap), "safetensors")
    (hub / "refs").mkdir(parents=True)
    (hub / "refs" / "main").write_text("abc123")
    assert resolve_model_dir("org/tiny-bert") == str(snap)
    sd, d = encoder_weights(TINY_BERT, "org/tiny-bert")
    assert d == str(snap) and sd is not None
    assert resolve_model_dir("org/other") is None
    assert resolve_model_dir(str(snap)) == str(snap)
