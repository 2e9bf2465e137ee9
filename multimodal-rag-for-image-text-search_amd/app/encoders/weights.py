"""Encoder configurations and parameter sources.

The reference loads pretrained weights by hub name (``config.py:10-12``:
``openai/clip-vit-base-patch32``, ``sentence-transformers/all-MiniLM-L6-v2``) — not
reachable offline. Parameters therefore come from one of two sources, both keyed by
the Hugging Face state-dict names the C ABI expects:

* a local checkpoint (``model.safetensors`` or ``pytorch_model.bin``) when ``MODEL_CLIP``
  / ``MODEL_TEXT`` names a directory or a hub id cached locally (drop-in for real
  deployments);
* only on explicit request (``MRAG_SYNTHETIC_WEIGHTS=1``) a deterministic synthetic
  generator: a counter-based splitmix64 stream per parameter name, so the GPU box, the
  oracle and the golden fixtures all see bit-identical weights without shipping 600 MB.
  Throughput does not depend on the weight values; parity is defined on identical
  weights (SURVEY.md §7 hard part 2).

Anything else raises, as the reference's loaders do.
"""
from __future__ import annotations

import math
import os
import zlib
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np


@dataclass(frozen=True)
class EncoderConfig:
    kind: int  # 1 CLIP vision, 2 CLIP text, 3 BERT, 4 BERT pair classifier (cross-encoder)
    hidden: int
    layers: int
    heads: int
    intermediate: int
    max_positions: int = 0
    vocab: int = 0
    proj_dim: int = 0
    image_size: int = 0
    patch_size: int = 0
    act: int = 0  # 0 quick_gelu, 1 gelu_erf
    eos_token_id: int = -1
    ln_eps: float = 1e-5


# CLIP ViT-B/32 (transformers CLIPVisionConfig defaults == openai/clip-vit-base-patch32)
CLIP_VISION_B32 = EncoderConfig(kind=1, hidden=768, layers=12, heads=12, intermediate=3072, proj_dim=512,
                                image_size=224, patch_size=32, act=0, ln_eps=1e-5)
# CLIP text tower (CLIPTextConfig defaults; eos 49407 -> first-EOS pooling)
CLIP_TEXT_B32 = EncoderConfig(kind=2, hidden=512, layers=12, heads=8, intermediate=2048, max_positions=77,
                              vocab=49408, proj_dim=512, act=0, eos_token_id=49407, ln_eps=1e-5)
# all-MiniLM-L6-v2 = BertModel(hidden 384, 6 layers, 12 heads, intermediate 1536)
MINILM_L6 = EncoderConfig(kind=3, hidden=384, layers=6, heads=12, intermediate=1536, max_positions=512,
                          vocab=30522, act=1, ln_eps=1e-12)
# cross-encoder/ms-marco-MiniLM-L-6-v2 (the reference's RERANKER_MODEL default) =
# BertForSequenceClassification(MiniLM-L6 dims, num_labels = 1); proj_dim carries num_labels
MSMARCO_MINILM_L6_CE = EncoderConfig(kind=4, hidden=384, layers=6, heads=12, intermediate=1536, max_positions=512,
                                     vocab=30522, proj_dim=1, act=1, ln_eps=1e-12)


def param_specs(cfg: EncoderConfig) -> List[Tuple[str, Tuple[int, ...], str]]:
    """(state-dict name, shape, init kind) of every parameter the forward reads."""
    D, I = cfg.hidden, cfg.intermediate
    out: List[Tuple[str, Tuple[int, ...], str]] = []
    if cfg.kind in (1, 2):
        pre = "vision_model." if cfg.kind == 1 else "text_model."
        if cfg.kind == 1:
            g = cfg.image_size // cfg.patch_size
            out += [
                (pre + "embeddings.class_embedding", (D,), "emb"),
                (pre + "embeddings.patch_embedding.weight", (D, 3, cfg.patch_size, cfg.patch_size), "linear"),
                (pre + "embeddings.position_embedding.weight", (g * g + 1, D), "emb"),
                (pre + "pre_layrnorm.weight", (D,), "ln_w"),
                (pre + "pre_layrnorm.bias", (D,), "ln_b"),
            ]
        else:
            out += [
                (pre + "embeddings.token_embedding.weight", (cfg.vocab, D), "emb"),
                (pre + "embeddings.position_embedding.weight", (cfg.max_positions, D), "emb"),
            ]
        for i in range(cfg.layers):
            l = f"{pre}encoder.layers.{i}."
            for p in ("q_proj", "k_proj", "v_proj", "out_proj"):
                out += [(l + f"self_attn.{p}.weight", (D, D), "linear"), (l + f"self_attn.{p}.bias", (D,), "bias")]
            out += [
                (l + "layer_norm1.weight", (D,), "ln_w"), (l + "layer_norm1.bias", (D,), "ln_b"),
                (l + "layer_norm2.weight", (D,), "ln_w"), (l + "layer_norm2.bias", (D,), "ln_b"),
                (l + "mlp.fc1.weight", (I, D), "linear"), (l + "mlp.fc1.bias", (I,), "bias"),
                (l + "mlp.fc2.weight", (D, I), "linear"), (l + "mlp.fc2.bias", (D,), "bias"),
            ]
        if cfg.kind == 1:
            out += [
                (pre + "post_layernorm.weight", (D,), "ln_w"), (pre + "post_layernorm.bias", (D,), "ln_b"),
                ("visual_projection.weight", (cfg.proj_dim, D), "linear"),
            ]
        else:
            out += [
                (pre + "final_layer_norm.weight", (D,), "ln_w"), (pre + "final_layer_norm.bias", (D,), "ln_b"),
                ("text_projection.weight", (cfg.proj_dim, D), "linear"),
            ]
    else:
        b = "bert." if cfg.kind == 4 else ""  # BertForSequenceClassification wraps BertModel as .bert
        out += [
            (b + "embeddings.word_embeddings.weight", (cfg.vocab, D), "emb"),
            (b + "embeddings.position_embeddings.weight", (cfg.max_positions, D), "emb"),
            (b + "embeddings.token_type_embeddings.weight", (2, D), "emb"),
            (b + "embeddings.LayerNorm.weight", (D,), "ln_w"),
            (b + "embeddings.LayerNorm.bias", (D,), "ln_b"),
        ]
        if cfg.kind == 4:
            out += [
                ("bert.pooler.dense.weight", (D, D), "linear"), ("bert.pooler.dense.bias", (D,), "bias"),
                ("classifier.weight", (cfg.proj_dim, D), "linear"), ("classifier.bias", (cfg.proj_dim,), "bias"),
            ]
        for i in range(cfg.layers):
            l = f"{b}encoder.layer.{i}."
            for p in ("query", "key", "value"):
                out += [(l + f"attention.self.{p}.weight", (D, D), "linear"), (l + f"attention.self.{p}.bias", (D,), "bias")]
            out += [
                (l + "attention.output.dense.weight", (D, D), "linear"), (l + "attention.output.dense.bias", (D,), "bias"),
                (l + "attention.output.LayerNorm.weight", (D,), "ln_w"), (l + "attention.output.LayerNorm.bias", (D,), "ln_b"),
                (l + "intermediate.dense.weight", (I, D), "linear"), (l + "intermediate.dense.bias", (I,), "bias"),
                (l + "output.dense.weight", (D, I), "linear"), (l + "output.dense.bias", (D,), "bias"),
                (l + "output.LayerNorm.weight", (D,), "ln_w"), (l + "output.LayerNorm.bias", (D,), "ln_b"),
            ]
    return out


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform(name: str, n: int, seed: int) -> np.ndarray:
    """n values in [-1, 1) from a counter-based stream keyed by (name, seed)."""
    key = np.uint64((zlib.crc32(name.encode()) << 32) | (zlib.adler32(name.encode()) & 0xFFFFFFFF)) ^ np.uint64(seed)
    ctr = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _splitmix64(ctr * np.uint64(0xD1B54A32D192ED03) + key)
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return (2.0 * u - 1.0).astype(np.float32)


def synth_param(name: str, shape: Tuple[int, ...], kind: str, seed: int = 0) -> np.ndarray:
    n = int(np.prod(shape))
    u = _uniform(name, n, seed)
    if kind == "linear":
        fan_in = int(np.prod(shape[1:]))
        v = u * np.float32(math.sqrt(3.0 / fan_in))
    elif kind == "bias":
        v = u * np.float32(0.02)
    elif kind == "ln_w":
        v = np.float32(1.0) + u * np.float32(0.1)
    elif kind == "ln_b":
        v = u * np.float32(0.05)
    elif kind == "emb":
        v = u * np.float32(0.1)
    else:
        raise ValueError(kind)
    return v.reshape(shape).astype(np.float32)


def synth_state_dict(cfg: EncoderConfig, seed: int = 0) -> Iterator[Tuple[str, np.ndarray]]:
    for name, shape, kind in param_specs(cfg):
        yield name, synth_param(name, shape, kind, seed)


SYNTHETIC_ENV = "MRAG_SYNTHETIC_WEIGHTS"


def synthetic_allowed() -> bool:
    """Synthetic weights are an explicit opt-in (benchmarks, tests): ``MRAG_SYNTHETIC_WEIGHTS=1``."""
    return os.environ.get(SYNTHETIC_ENV) == "1"


def _hub_caches() -> List[str]:
    env = os.environ
    out = [env.get("HF_HUB_CACHE"), env.get("HUGGINGFACE_HUB_CACHE"), env.get("SENTENCE_TRANSFORMERS_HOME")]
    if env.get("HF_HOME"):
        out.append(os.path.join(env["HF_HOME"], "hub"))
    out.append(os.path.join(os.path.expanduser("~"), ".cache", "huggingface", "hub"))
    return [c for c in out if c]


def resolve_model_dir(name: Optional[str]) -> Optional[str]:
    """A local directory for a model name: the name itself when it is a directory, else the
    snapshot of that hub id in the local Hugging Face cache (``models--org--name/snapshots``,
    the revision ``refs/main`` names first). None when neither exists — there is no network."""
    if not name:
        return None
    if os.path.isdir(name):
        return name
    for cache in _hub_caches():
        repo = os.path.join(cache, "models--" + name.replace("/", "--"))
        snaps = os.path.join(repo, "snapshots")
        if not os.path.isdir(snaps):
            continue
        ref = os.path.join(repo, "refs", "main")
        if os.path.isfile(ref):
            with open(ref) as f:
                d = os.path.join(snaps, f.read().strip())
            if os.path.isdir(d):
                return d
        revs = sorted((os.path.join(snaps, r) for r in os.listdir(snaps)), key=os.path.getmtime, reverse=True)
        if revs:
            return revs[0]
    return None


def _checkpoint_tensors(path: str) -> Iterator[Tuple[str, np.ndarray]]:
    """(name, array) of every tensor in a checkpoint directory: ``*.safetensors``, else
    ``pytorch_model*.bin`` through ``torch.load(weights_only=True)`` (never unpickles code)."""
    st = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
    if st:
        from safetensors.numpy import load_file

        for f in st:
            yield from load_file(os.path.join(path, f)).items()
        return
    bins = sorted(f for f in os.listdir(path) if f.startswith("pytorch_model") and f.endswith(".bin"))
    if not bins:
        raise FileNotFoundError(f"{path} holds no model.safetensors or pytorch_model.bin")
    import torch

    for f in bins:
        sd = torch.load(os.path.join(path, f), map_location="cpu", weights_only=True)
        for k, v in sd.items():
            yield k, v.detach().to(torch.float32).numpy()


def checkpoint_state_dict(path: str, cfg: EncoderConfig) -> Dict[str, np.ndarray]:
    """Read a local Hugging Face checkpoint directory (safetensors or pytorch_model.bin).
    Only the names param_specs() lists are returned; a missing file or parameter raises."""
    if not path or not os.path.isdir(path):
        raise FileNotFoundError(f"checkpoint directory {path!r} does not exist")
    want = {n for n, _, _ in param_specs(cfg)}
    out: Dict[str, np.ndarray] = {}
    for k, v in _checkpoint_tensors(path):
        for cand in (k, k.replace("0.auto_model.", ""), k.replace("bert.", ""), "bert." + k):
            if cand in want:
                out[cand] = np.asarray(v, dtype=np.float32)
    missing = want - set(out)
    if missing:
        raise ValueError(f"checkpoint {path} lacks {len(missing)} parameters, e.g. {sorted(missing)[:3]}")
    return out


def encoder_weights(cfg: EncoderConfig, name: Optional[str],
                    synthetic: Optional[bool] = None) -> Tuple[Optional[Dict[str, np.ndarray]], Optional[str]]:
    """(state dict, model directory) for a model name, as the reference's ``from_pretrained``
    / ``SentenceTransformer(name)`` would load it (app/ml/embeddings.py:23-43): a local
    directory or a cached hub snapshot. Where the reference would fail to load — an
    unresolvable name offline — this raises too, unless synthetic weights are requested
    explicitly (``MRAG_SYNTHETIC_WEIGHTS=1``, or ``synthetic=True``: returns ``(None, None)``)."""
    d = resolve_model_dir(name)
    if d is not None:
        return checkpoint_state_dict(d, cfg), d
    if synthetic_allowed() if synthetic is None else synthetic:
        return None, None
    raise OSError(f"model {name!r} is neither a local checkpoint directory nor in the local Hugging Face cache "
                  f"(no network here); point MODEL_TEXT / MODEL_CLIP / RERANKER_MODEL at a checkpoint directory, "
                  f"or set {SYNTHETIC_ENV}=1 for deterministic synthetic weights (benchmarks, tests)")
