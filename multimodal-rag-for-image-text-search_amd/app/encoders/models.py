"""Model objects with the call signatures the reference's embedding helpers use, so the
module-global seams of ``app/ml/embeddings.py`` (``_TEXT_MODEL``, ``_CLIP_MODEL``,
``_CLIP_PROCESSOR``) keep working — the tests monkeypatch them with dummies exactly
as the reference's tests do (tests/test_embeddings.py:14-57).

* ``MiniLMSentenceModel.encode(...)``  ~ SentenceTransformer.encode (all-MiniLM-L6-v2:
  WordPiece -> BERT -> mean pooling -> Normalize), on the GPU encoder.
* ``ClipModel.get_image_features / get_text_features``  ~ CLIPModel's, returning the
  projected features as a CUDA tensor.
* ``ClipProcessor(images=... | text=...)``  ~ CLIPProcessor: host decode/resize/crop to
  u8 224x224 (normalisation is fused on the GPU) and CLIP tokenisation.
"""
from __future__ import annotations

import json
import os
from typing import Optional, Sequence, Tuple

import numpy as np

from app.encoders import CLIP_TEXT_B32, CLIP_VISION_B32, MINILM_L6, GpuEncoder, load_encoder
from app.encoders.preprocess import (load_batch, load_batch_device, prepare_batch, resize_images, upload_decode,
                                      upload_resize)
from app.encoders.tokenize import ClipTokenizer, WordPieceTokenizer
from app.encoders.weights import encoder_weights, resolve_model_dir, synth_state_dict, synthetic_allowed, SYNTHETIC_ENV


def _device_index() -> int:
    return int(os.environ.get("MRAG_DEVICE", "0"))


def _model_dir(name: Optional[str], need: Sequence[Sequence[str]] = (), synthetic: Optional[bool] = None) -> Optional[str]:
    """Local directory of a model name (directory or cached hub snapshot), checked for the
    tokenizer files in ``need`` (any one group complete). None only when synthetic
    weights are explicitly requested; otherwise an unresolvable name raises like the
    reference's hub loaders (app/ml/embeddings.py:23-43)."""
    d = resolve_model_dir(name)
    if d is None:
        if synthetic_allowed() if synthetic is None else synthetic:
            return None
        raise OSError(f"model {name!r} is neither a local checkpoint directory nor in the local Hugging Face "
                      f"cache (no network here); set {SYNTHETIC_ENV}=1 for synthetic weights")
    if need and not any(all(os.path.exists(os.path.join(d, f)) for f in grp) for grp in need):
        raise FileNotFoundError(f"{d} has no tokenizer files (one of {[list(g) for g in need]})")
    return d


_WORDPIECE_FILES = (("vocab.txt",),)
_CLIP_BPE_FILES = (("vocab.json", "merges.txt"),)


class BatchInputs(dict):
    """dict with ``.to(device)`` and attribute access (BatchFeature stand-in)."""

    def to(self, device):
        return self

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


class MiniLMSentenceModel:
    def __init__(self, name: Optional[str] = None, device: Optional[int] = None):
        d = _model_dir(name, _WORDPIECE_FILES)
        self.device = _device_index() if device is None else device
        self._pool = _HandlePool(_handle_maker(MINILM_L6, d, self.device))
        self._pool.first()  # load now, as SentenceTransformer(name) does
        self.tokenizer = WordPieceTokenizer(d, max_len=256)

    @property
    def enc(self):
        return self._pool.first()

    def to(self, device):
        return self

    def encode(self, sentences: Sequence[str], batch_size: int = 32, convert_to_tensor: bool = False,
               device=None, show_progress_bar=None, **kw):
        import torch

        sentences = list(sentences)
        out = torch.empty((len(sentences), MINILM_L6.hidden), dtype=torch.float32, device=f"cuda:{self.device}")
        if not sentences:
            return out if convert_to_tensor else out.cpu().numpy()
        # length-sorted batches like sentence-transformers; rows are independent, so the
        # GPU batch is sized for throughput (>= the caller's batch_size)
        order = np.argsort([-len(s) for s in sentences], kind="stable")
        gb = max(int(batch_size), 256)
        h = self._pool.acquire()  # concurrent callers run on their own handles / streams
        try:
            for s0 in range(0, len(order), gb):
                idx = order[s0:s0 + gb]
                ids, mask = self.tokenizer([sentences[i] for i in idx])
                emb = h.embed_tokens(torch.from_numpy(ids).to(out.device), torch.from_numpy(mask).to(out.device),
                                     normalize=True)
                out[torch.from_numpy(idx).to(out.device)] = emb
            res = out if convert_to_tensor else out.cpu().numpy()
        finally:
            self._pool.release(h)
        return res


def _handle_maker(cfg, model_dir, device):
    """Builder of identical encoder handles for a _HandlePool: the checkpoint (or the synthetic
    state dict) is read once and shared by every handle of the pool; the pool drops it once it
    holds all its handles."""
    import threading

    lock = threading.Lock()
    cache = {}

    def make():
        with lock:
            if "sd" not in cache:
                sd, _ = encoder_weights(cfg, model_dir)
                cache["sd"] = sd if sd is not None else dict(synth_state_dict(cfg, 0))
            sd = cache["sd"]
        return GpuEncoder(cfg, device=device, state_dict=sd)

    def done():
        with lock:
            cache.clear()

    make.done = done
    return make


class _HandlePool:
    """Encoder handles of one model for concurrent callers: a call takes a free handle (a new one,
    up to `limit`, when all are busy; else it waits), so requests from several threads run their
    forwards at once on separate workspaces and streams instead of queueing on one handle's lock
    (three image batches in flight: +23 % throughput, notes/work_in_flight.md). Every handle
    holds the same weights, so a request's result does not depend on the handle it got. A new
    handle is built outside the pool's lock (a slot is reserved first), so releases and other
    acquirers never wait for a weight upload.
    env MRAG_ENCODER_HANDLES (default 3; 1 = one handle, the round-1 behaviour)."""

    def __init__(self, make):
        import threading

        self._make = make
        self._limit = max(1, int(os.environ.get("MRAG_ENCODER_HANDLES", "3")))
        self._all = []
        self._free = []
        self._pending = 0  # slots reserved by handles being built
        self._cv = threading.Condition()

    def _build(self, free_it: bool):
        try:
            h = self._make()
        except BaseException:
            with self._cv:
                self._pending -= 1
                self._cv.notify_all()
            raise
        with self._cv:
            self._pending -= 1
            self._all.append(h)
            if free_it:
                self._free.append(h)
            full = len(self._all) >= self._limit
            self._cv.notify_all()
        if full and hasattr(self._make, "done"):
            self._make.done()  # every handle built: the shared host weights are no longer needed
        return h

    def first(self):
        with self._cv:
            while not self._all and self._pending:
                self._cv.wait()
            if self._all:
                return self._all[0]
            self._pending += 1
        self._build(free_it=True)
        with self._cv:
            return self._all[0]

    def acquire(self):
        with self._cv:
            while not self._free and len(self._all) + self._pending >= self._limit:
                self._cv.wait()
            if self._free:
                return self._free.pop()
            self._pending += 1
        return self._build(free_it=False)

    def release(self, h):
        with self._cv:
            self._free.append(h)
            self._cv.notify_all()


class ClipModel:
    def __init__(self, name: Optional[str] = None, device: Optional[int] = None):
        self.dir = _model_dir(name)  # raises here, as CLIPModel.from_pretrained would
        self.device = _device_index() if device is None else device
        self._vision_pool = _HandlePool(_handle_maker(CLIP_VISION_B32, self.dir, self.device))
        self._text_pool = None

    def to(self, device):
        return self

    def _text_cfg(self):
        cfg = CLIP_TEXT_B32
        if self.dir and os.path.exists(os.path.join(self.dir, "config.json")):
            tc = json.load(open(os.path.join(self.dir, "config.json"))).get("text_config", {})
            eos = tc.get("eos_token_id", cfg.eos_token_id)
            from dataclasses import replace

            cfg = replace(cfg, eos_token_id=-1 if eos == 2 else int(eos))  # legacy configs pool at argmax(ids)
        return cfg

    @property
    def vision(self):
        return self._vision_pool.first()

    def _texts(self):
        if self._text_pool is None:
            self._text_pool = _HandlePool(_handle_maker(self._text_cfg(), self.dir, self.device))
        return self._text_pool

    @property
    def text(self):
        return self._texts().first()

    def get_image_features(self, images_u8=None, pixel_values=None, **kw):
        import torch

        if images_u8 is None:
            raise TypeError("the GPU image tower takes u8 224x224 images (images_u8=), as produced by ClipProcessor")
        x = images_u8 if isinstance(images_u8, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(images_u8))
        x = x.to(f"cuda:{self.device}")
        h = self._vision_pool.acquire()  # a handle reused on another stream waits for its last call
        try:
            return h.embed_images(x, normalize=False)
        finally:
            self._vision_pool.release(h)

    def get_text_features(self, input_ids=None, attention_mask=None, **kw):
        import torch

        ids = input_ids if isinstance(input_ids, torch.Tensor) else torch.from_numpy(np.asarray(input_ids))
        dev = f"cuda:{self.device}"
        m = None
        if attention_mask is not None:
            m = attention_mask if isinstance(attention_mask, torch.Tensor) else torch.from_numpy(np.asarray(attention_mask))
            m = m.to(dev)
        pool = self._texts()
        h = pool.acquire()  # concurrent query encodes run on their own handles / streams
        try:
            return h.embed_tokens(ids.to(dev), m, normalize=False)
        finally:
            pool.release(h)


class ClipProcessor:
    def __init__(self, name: Optional[str] = None):
        self.tokenizer = ClipTokenizer(_model_dir(name, _CLIP_BPE_FILES))

    def to(self, device):
        return self

    def __call__(self, *, images=None, text=None, return_tensors="pt", padding=None, **kw):
        if images is not None:
            if os.environ.get("MRAG_HOST_RESIZE") == "1":  # A/B: PIL resize on the host
                return BatchInputs(images_u8=load_batch(list(images)))
            return BatchInputs(images_u8=load_batch_device(list(images), device=_device_index()))
        if text is not None:
            ids, mask = self.tokenizer(list(text))
            return BatchInputs(input_ids=ids, attention_mask=mask)
        raise ValueError("ClipProcessor needs images= or text=")

    # The two halves of images= for a caller that pipelines batches (embed_images_batch prepares
    # batch i + 1 on the host — file reads, Pillow decode of what K13 does not take — while batch i
    # is decoded, resized and encoded on the GPU).
    @staticmethod
    def decode(images):
        return prepare_batch(list(images))

    @staticmethod
    def from_decoded(prepared):
        return BatchInputs(images_u8=upload_resize(prepared, device=_device_index()))

    # A group of several encoder batches: one K13 launch for the group, then K0 per batch.
    @staticmethod
    def decode_device(prepared):
        return upload_decode(prepared, device=_device_index())

    @staticmethod
    def from_device(imgs, start, count):
        return BatchInputs(images_u8=resize_images(imgs, start, count, device=_device_index()))


class CrossEncoderModel:
    """GPU stand-in for ``sentence_transformers.CrossEncoder`` as the reference uses it
    (``CrossEncoder(settings.models.reranker).predict(pairs)``, app/ml/retrieve.py:29-38,
    148): BertForSequenceClassification (MRAG_ENC_BERT_PAIR: BERT-6L/384 on the MiniLM
    kernels + [CLS] pooler + classifier) on "[CLS] query [SEP] passage [SEP]" pairs.

    ``predict`` restates sentence-transformers' (unpinned, not installed) semantics:
    batches of ``batch_size`` pairs, tokenizer truncation 'longest_first' to
    ``max_length`` (512 = the model's positions), logits -> activation -> for one label
    a float32 vector (a scalar for a single pair). The default activation comes from the
    checkpoint's ``config.json`` key ``sbert_ce_default_activation_function`` (the
    ms-marco cross-encoders set Identity: raw logits) and otherwise is Sigmoid for one
    label / Identity for several — sentence-transformers' rule."""

    def __init__(self, model_name_or_path: Optional[str] = None, max_length: Optional[int] = None,
                 device: Optional[int] = None, seed: int = 0, synthetic: Optional[bool] = None):
        from app.encoders.weights import MSMARCO_MINILM_L6_CE

        d = _model_dir(model_name_or_path, _WORDPIECE_FILES, synthetic)
        self.device = _device_index() if device is None else device
        self.cfg = MSMARCO_MINILM_L6_CE
        self.enc = load_encoder(self.cfg, d, device=self.device, seed=seed, synthetic=d is None)
        self.tokenizer = WordPieceTokenizer(d, max_len=max_length or self.cfg.max_positions)
        self.num_labels = self.cfg.proj_dim
        act = None
        if d and os.path.exists(os.path.join(d, "config.json")):
            with open(os.path.join(d, "config.json")) as f:
                act = json.load(f).get("sbert_ce_default_activation_function")
        if act is not None:
            self.activation = "identity" if act.endswith("Identity") else ("sigmoid" if act.endswith("Sigmoid") else act)
        else:
            self.activation = "sigmoid" if self.num_labels == 1 else "identity"

    def to(self, device):
        return self

    def logits(self, pairs: Sequence[Tuple[str, str]], batch_size: int = 32) -> np.ndarray:
        out = []
        for i in range(0, len(pairs), batch_size):
            ids, types, mask = self.tokenizer.pairs(pairs[i:i + batch_size])
            out.append(self.enc.score_pairs(ids, types, mask))
        return np.concatenate(out) if out else np.empty((0, self.num_labels), dtype=np.float32)

    def predict(self, sentences, batch_size: int = 32, show_progress_bar=None, activation_fct=None,
                apply_softmax: bool = False, convert_to_numpy: bool = True, convert_to_tensor: bool = False, **kw):
        single = len(sentences) > 0 and isinstance(sentences[0], str)
        pairs = [tuple(sentences)] if single else [tuple(p) for p in sentences]
        z = self.logits(pairs, batch_size)
        if activation_fct is not None:
            import torch

            z = activation_fct(torch.from_numpy(z)).numpy()
        elif self.activation == "sigmoid":
            z = (1.0 / (1.0 + np.exp(-z.astype(np.float64)))).astype(np.float32)
        if apply_softmax and z.shape[1] > 1:
            e = np.exp(z - z.max(axis=1, keepdims=True))
            z = e / e.sum(axis=1, keepdims=True)
        scores = z[:, 0] if self.num_labels == 1 else z
        scores = np.asarray(scores, dtype=np.float32)
        if convert_to_tensor:
            import torch

            scores = torch.from_numpy(scores)
        return scores[0] if single else scores
