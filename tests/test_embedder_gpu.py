"""``Embedder`` (reference app/embedding/embedder.py:15-68) through the GPU towers, against the
oracle on the same synthetic weights: MiniLM rows (unit, ST Normalize), raw CLIP text features
and raw CLIP image features — the latter against the reference-produced golden
(``golden_clip_image.npz::expected_unnormalized``, from the reference's own CLIP call)."""
from __future__ import annotations

import os

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN, record_numerics
from test_encoders_gpu import ABS_MAX, COS_ERR_MAX, REL_L2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def embedder(cuda):
    from app.embedding.embedder import Embedder

    return Embedder()


def test_embed_text(embedder):
    from app.encoders.tokenize import WordPieceTokenizer
    from oracle.models import bert_model, minilm_embeds

    texts = ["a photo of a cat on a mat", "retrieval augmented generation on gpus", "x"]
    got = embedder.embed_text(texts)
    ids, mask = WordPieceTokenizer(None, max_len=256)(texts)
    exp = minilm_embeds(bert_model(0), ids, mask)
    row = record_numerics("embedder_embed_text", got, exp)
    assert got.shape == (3, 384) and got.dtype == np.float32
    assert row["max_1_minus_cos"] <= COS_ERR_MAX and row["max_abs_diff"] <= ABS_MAX, row


def test_embed_text_for_images(embedder):
    from app.encoders.tokenize import ClipTokenizer
    from oracle.models import clip_model, clip_text_embeds

    texts = ["a dog", "two cats sleeping on a red sofa"]
    got = embedder.embed_text_for_images(texts)
    ids, mask = ClipTokenizer(None)(texts)
    exp = clip_text_embeds(clip_model(0), ids, mask, normalize=False)
    row = record_numerics("embedder_embed_text_for_images", got, exp, unit=False)
    assert got.shape == (2, 512) and row["max_rel_l2"] <= REL_L2, row


def test_embed_images(embedder, tmp_path):
    g = np.load(os.path.join(GOLDEN, "golden_clip_image.npz"))
    paths = []
    for i, a in enumerate([g["raw_0"], g["images_u8"][1], g["raw_2"]]):  # as the reference's own run
        p = tmp_path / f"im{i}.png"
        Image.fromarray(a).save(p)
        paths.append(str(p))
    got = embedder.embed_images(paths)
    row = record_numerics("embedder_embed_images", got, g["expected_unnormalized"], unit=False)
    assert got.shape == (len(paths), 512) and row["max_rel_l2"] <= REL_L2, row
    with pytest.raises(FileNotFoundError):
        embedder.embed_images([str(tmp_path / "missing.png")])
