"""Drop-in for the reference's ``app/ml/embeddings.py`` on the GPU encoders.

Same functions, return conventions and module-global seams (reference :14-105):
``embed_text_batch`` -> float32 [N,384] unit rows ((0,384) for no input),
``embed_images_batch`` -> [N,512] ((0,512)), ``embed_query_for_images`` -> (512,)
(zeros for a blank query); lazily created singletons ``_TEXT_MODEL``,
``_CLIP_MODEL``, ``_CLIP_PROCESSOR`` that tests may monkeypatch.

Differences, all deliberate: the default models are the MI355X encoders
(app.encoders.models) — there is no CPU fallback, so without a GPU the first call
raises; model inputs are accepted as a mapping OR an attribute namespace (the
reference's ``model.get_image_features(**inputs)`` cannot unpack the SimpleNamespace
its own dummy processor returns — tests/test_embeddings.py fails on that); the GPU
image batch is max(batch_size, 256) (results do not depend on it).
"""
from __future__ import annotations

import os
import time
from pathlib import Path
from typing import Any, Mapping, Optional, Sequence

import numpy as np

from app.settings import settings

_TEXT_MODEL: Optional[Any] = None
_DECODE_GROUP_BATCHES = 1  # encoder batches per K13 decode launch (profiles/r5s18_ingest_group_ab.jsonl)
# The host half runs as one prepare_batch per group, two groups ahead — for path lists one library
# call (preprocess.NativePrepared; profiles/r5s37_native_ab.jsonl: 16.6-18.2k img/s against
# 11.4-12.8k for a per-file host half on the decode pool, three interleaved rounds)
_CLIP_MODEL: Optional[Any] = None
_CLIP_PROCESSOR: Optional[Any] = None


def _device() -> str:
    import torch

    return "cuda" if torch.cuda.is_available() else "cpu"


def _ensure_text_model():
    global _TEXT_MODEL
    if _TEXT_MODEL is None:
        from app.encoders.models import MiniLMSentenceModel

        _TEXT_MODEL = MiniLMSentenceModel(settings.models.text)
        _TEXT_MODEL.to(_device())
    return _TEXT_MODEL


def _ensure_clip():
    global _CLIP_MODEL
    if _CLIP_MODEL is None:
        from app.encoders.models import ClipModel

        _CLIP_MODEL = ClipModel(settings.models.clip)
        _CLIP_MODEL.to(_device())
    return _CLIP_MODEL


def _ensure_processor():
    global _CLIP_PROCESSOR
    if _CLIP_PROCESSOR is None:
        from app.encoders.models import ClipProcessor

        _CLIP_PROCESSOR = ClipProcessor(settings.models.clip)
    return _CLIP_PROCESSOR


def _normalize(embeddings: np.ndarray) -> np.ndarray:
    norms = np.linalg.norm(embeddings, axis=1, keepdims=True)
    norms[norms == 0] = 1.0
    return embeddings / norms


def _kwargs(inputs: Any) -> Mapping[str, Any]:
    if isinstance(inputs, Mapping):
        return inputs
    return {k: v for k, v in vars(inputs).items() if not k.startswith("_")}


def _to_numpy(x: Any) -> np.ndarray:
    if hasattr(x, "pooler_output"):  # transformers >= 5 returns a ModelOutput
        x = x.pooler_output
    if hasattr(x, "detach"):
        return x.detach().cpu().float().numpy()
    return np.asarray(x, dtype=np.float32)


def embed_text_batch(texts: Sequence[str], batch_size: int = 32) -> np.ndarray:
    """Embed text with MiniLM and return L2-normalised float32 rows."""
    if not texts:
        return np.empty((0, 384), dtype=np.float32)
    model = _ensure_text_model()
    embeddings = model.encode(list(texts), batch_size=batch_size, convert_to_tensor=True, device=_device(),
                              show_progress_bar=False)
    return _normalize(_to_numpy(embeddings))


def embed_images_batch(paths: Sequence[Path], batch_size: int = 8) -> np.ndarray:
    """Embed images with CLIP's vision tower and return normalised float32 rows."""
    if not paths:
        return np.empty((0, 512), dtype=np.float32)
    return _normalize(np.vstack(list(_image_feature_batches(paths, batch_size))))


def embed_images_batches(paths: Sequence[Path], batch_size: int = 8, idle=None):
    """``embed_images_batch`` one encoder batch at a time: yields the normalised rows of each
    batch in order, while the next batches' files are read and decoded on the pipeline's threads.
    The rows equal embed_images_batch's: ``_normalize`` reduces each row on its own. ``idle``: a
    callable run while this thread would wait for the next decoded batch, repeatedly as long as it
    returns True (index_image_nodes builds the store's rows there: on this thread, so its Python
    does not contend for the interpreter lock with the pipeline's own threads)."""
    for raw in _image_feature_batches(paths, batch_size, idle):
        yield _normalize(raw)


def _image_feature_batches(paths: Sequence[Path], batch_size: int, idle=None):
    """The vision tower's unnormalised features, one array per encoder batch."""
    if not paths:
        return
    from PIL import Image

    from app.encoders.models import ClipModel, ClipProcessor

    model = _ensure_clip()
    processor = _ensure_processor()
    native = isinstance(model, ClipModel) and isinstance(processor, ClipProcessor)
    step = max(batch_size, 256) if native else batch_size
    paths = list(paths)
    if native and os.environ.get("MRAG_HOST_RESIZE") != "1":
        # three stages in flight: the host prepares group g + 2 (file reads, probes, PNG inflate,
        # Pillow for what the GPU decoders do not take), a second thread decodes group g + 1 on the
        # GPU (K13 / K14, its own stream), and this thread resizes (K0) and encodes group g
        from concurrent.futures import ThreadPoolExecutor

        import torch

        group = _DECODE_GROUP_BATCHES * step
        starts = list(range(0, len(paths), group))
        from app.encoders.models import _device_index

        dstream = torch.cuda.Stream(torch.device("cuda", _device_index()))

        with ThreadPoolExecutor(max_workers=1) as prep_ex, ThreadPoolExecutor(max_workers=1) as dec_ex:
            preps = {}
            decs = {}

            def prep(i):
                if i < len(starts) and i not in preps:
                    preps[i] = prep_ex.submit(processor.decode, paths[starts[i]:starts[i] + group])

            def dec(i):
                if i < len(starts) and i not in decs:
                    prep(i)
                    fut = preps[i]

                    def run():
                        prepared = fut.result()
                        with torch.cuda.stream(dstream):
                            return len(prepared), processor.decode_device(prepared)

                    decs[i] = dec_ex.submit(run)

            for i in range(len(starts)):
                dec(i)
                dec(i + 1)
                prep(i + 2)
                fut_i = decs.pop(i)
                if idle is not None:
                    while not fut_i.done() and idle():
                        time.sleep(0)  # lets the pipeline's threads take the interpreter lock
                n_i, imgs = fut_i.result()
                preps.pop(i, None)
                for c0 in range(0, n_i, step):
                    inputs = processor.from_device(imgs, c0, step)
                    yield _to_numpy(model.get_image_features(**_kwargs(inputs)))
                del imgs
        return
    for start in range(0, len(paths), step):
        batch_paths = paths[start:start + step]
        if native:
            inputs = processor(images=batch_paths, return_tensors="pt")  # decodes in a thread pool
        else:
            images = [Image.open(p).convert("RGB") for p in batch_paths]
            inputs = processor(images=images, return_tensors="pt")
            for img in images:
                img.close()
        if hasattr(inputs, "to"):
            inputs = inputs.to(_device())
        yield _to_numpy(model.get_image_features(**_kwargs(inputs)))


def embed_query_for_images(query: str) -> np.ndarray:
    """Encode a text query into the CLIP text space for image retrieval."""
    if not query.strip():
        return np.zeros((512,), dtype=np.float32)
    model = _ensure_clip()
    processor = _ensure_processor()
    inputs = processor(text=[query], return_tensors="pt", padding=True)
    if hasattr(inputs, "to"):
        inputs = inputs.to(_device())
    array = _to_numpy(model.get_text_features(**_kwargs(inputs)))
    return _normalize(array)[0]


__all__ = ["embed_text_batch", "embed_images_batch", "embed_images_batches", "embed_query_for_images"]
