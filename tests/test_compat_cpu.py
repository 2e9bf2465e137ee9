"""The reference's API contract (tests/test_embeddings.py, test_retrieve.py,
test_index_build.py, test_cache.py — same dummies, same monkeypatch seams) run
against the drop-in layer, plus host-side pieces: image preprocessing vs
transformers' CLIPImageProcessor, the splitter, tokenisers and the store helpers vs
the reference's own outputs. CPU only."""
from __future__ import annotations

import json
import os
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import GOLDEN


# ---------------------------------------------------------------- embeddings seams
class _DummyTextModel:
    def to(self, device):
        return self

    def encode(self, texts, batch_size=None, convert_to_tensor=None, device=None, show_progress_bar=None):
        return torch.ones((len(texts), 384), dtype=torch.float32)


class _DummyClipModel:
    def to(self, device):
        return self

    def get_image_features(self, **inputs):
        return torch.ones((inputs["pixel_values"].shape[0], 512), dtype=torch.float32)

    def get_text_features(self, **inputs):
        return torch.ones((inputs["input_ids"].shape[0], 512), dtype=torch.float32)


class _DummyProcessor:
    def to(self, device):
        return self

    def __call__(self, *, images=None, text=None, return_tensors="pt", padding=None):
        class _NS(SimpleNamespace):
            def to(self, device):
                return self

        if images is not None:
            return _NS(pixel_values=torch.ones((len(images), 3, 224, 224)))
        return _NS(input_ids=torch.ones((len(text), 77), dtype=torch.int64),
                   attention_mask=torch.ones((len(text), 77), dtype=torch.int64))


def test_embed_text_batch_normalized(monkeypatch):
    from app.ml import embeddings

    monkeypatch.setattr(embeddings, "_TEXT_MODEL", _DummyTextModel())
    v = embeddings.embed_text_batch(["hello", "world"])
    assert v.shape == (2, 384) and np.allclose(np.linalg.norm(v, axis=1), 1.0)


def test_embed_images_batch(monkeypatch, tmp_path: Path):
    """The reference fails this test (it ** -unpacks a SimpleNamespace); the drop-in passes."""
    from app.ml import embeddings

    monkeypatch.setattr(embeddings, "_CLIP_MODEL", _DummyClipModel())
    monkeypatch.setattr(embeddings, "_CLIP_PROCESSOR", _DummyProcessor())
    paths = []
    for i, color in enumerate([(255, 255, 255), (0, 0, 0)]):
        p = tmp_path / f"img_{i}.png"
        Image.fromarray(np.full((32, 32, 3), color, dtype=np.uint8)).save(p)
        paths.append(p)
    v = embeddings.embed_images_batch(paths)
    assert v.shape == (2, 512) and np.allclose(np.linalg.norm(v, axis=1), 1.0)


def test_embed_query_for_images(monkeypatch):
    from app.ml import embeddings

    monkeypatch.setattr(embeddings, "_CLIP_MODEL", _DummyClipModel())
    monkeypatch.setattr(embeddings, "_CLIP_PROCESSOR", _DummyProcessor())
    v = embeddings.embed_query_for_images("test query")
    assert v.shape == (512,) and np.linalg.norm(v) == pytest.approx(1.0, rel=1e-6)
    assert np.all(embeddings.embed_query_for_images("   ") == 0)


def test_empty_inputs():
    from app.ml import embeddings

    assert embeddings.embed_text_batch([]).shape == (0, 384)
    assert embeddings.embed_images_batch([]).shape == (0, 512)
    assert embeddings.embed_text_batch([]).dtype == np.float32


# ---------------------------------------------------------------- retrieval seams
class DummyStore:
    def __init__(self, text_rows, image_rows):
        self._t, self._i = text_rows, image_rows

    def search_text(self, user_id, vec, top_k):
        return self._t[:top_k]

    def search_image(self, user_id, vec, top_k):
        return self._i[:top_k]


class DummyMetadata:
    def __init__(self, chunks):
        self._c = chunks

    def get_chunk(self, chunk_id):
        return self._c.get(chunk_id)


class DummyCrossEncoder:
    def predict(self, pairs):
        return np.linspace(0.1, 0.9, len(pairs))


@pytest.fixture(autouse=True)
def _clear():
    from app.cache import clear_all_caches

    clear_all_caches()
    yield
    clear_all_caches()


def _patch_retrieve(monkeypatch, store, meta, ce, version=1):
    from app.ml import retrieve

    monkeypatch.setattr(retrieve, "_LANCEDB_STORE", store)
    monkeypatch.setattr(retrieve, "_METADATA_STORE", meta)
    monkeypatch.setattr(retrieve, "embed_text_batch", lambda texts: np.ones((1, 384), dtype=np.float32))
    monkeypatch.setattr(retrieve, "embed_query_for_images", lambda q: np.ones(512, dtype=np.float32))
    monkeypatch.setattr(retrieve, "_get_cross_encoder", lambda: ce)
    monkeypatch.setattr(retrieve, "get_index_version", lambda user_id: version)
    return retrieve


def test_retrieve_fusion_matches_reference(monkeypatch):
    """tests/test_retrieve.py::test_retrieve_fusion asserts fused[0] == 't1', which the
    reference itself fails on numpy 2.x (float32 z-score rounding makes i1 first).
    The drop-in must reproduce the reference's actual output (golden_fusion.json)."""
    from app.storage.schema import Chunk

    store = DummyStore([{"chunk_id": "t1", "score": 0.8, "meta": {}}, {"chunk_id": "t2", "score": 0.6, "meta": {}}],
                       [{"chunk_id": "i1", "score": 0.7, "meta": {}}])
    chunks = {
        "t1": Chunk(id="t1", document_id="doc1", modality="text", text="alpha", meta={}),
        "t2": Chunk(id="t2", document_id="doc2", modality="text", text="beta", meta={}),
        "i1": Chunk(id="i1", document_id="doc3", modality="image", meta={"file_path": "/tmp/img.jpg"}),
    }
    retrieve = _patch_retrieve(monkeypatch, store, DummyMetadata(chunks), DummyCrossEncoder())
    fused = retrieve.retrieve("user", "example query")
    ref = json.load(open(os.path.join(GOLDEN, "golden_fusion.json")))["cases"][0]["fused"]
    assert [f["chunk_id"] for f in fused] == [f["chunk_id"] for f in ref]
    assert [f["combined_score"] for f in fused] == [f["combined_score"] for f in ref]


def test_retrieval_cache_invalidation(monkeypatch):
    retrieve = _patch_retrieve(monkeypatch, DummyStore([], []), DummyMetadata({}), False, version=1)
    retrieve.retrieve("user", "question")
    monkeypatch.setattr(retrieve, "get_index_version", lambda user_id: 2)
    assert retrieve.retrieve("user", "question") == []


def test_fusion_golden_cases():
    from app.ml.retrieve import _fuse_results, _z_scores

    d = json.load(open(os.path.join(GOLDEN, "golden_fusion.json")))
    for c in d["cases"]:
        assert _z_scores([it["score"] for it in c["text"]]) == c["z_text"]
        assert _fuse_results([dict(i) for i in c["text"]], [dict(i) for i in c["image"]]) == c["fused"]


# ---------------------------------------------------------------- index build seams
class _DummyStore:
    def __init__(self):
        self.text_rows, self.image_rows = [], []

    def upsert_text_vectors(self, rows):
        self.text_rows.extend(rows)

    def upsert_image_vectors(self, rows):
        self.image_rows.extend(rows)


def test_index_text_nodes(monkeypatch, tmp_path):
    from app.ml import index_build

    store = _DummyStore()
    monkeypatch.setattr(index_build, "_LANCEDB_STORE", store)
    monkeypatch.setattr(index_build, "_VERSION_FILE", tmp_path / "versions.json")
    monkeypatch.setattr(index_build, "embed_text_batch", lambda texts: np.ones((len(texts), 384), dtype=np.float32))
    nodes = [{"id": "doc-1", "text": "This is a short document for testing purposes.", "metadata": {"source": "pdf"}}]
    indexed = index_build.index_text_nodes("user-1", nodes)
    assert indexed and store.text_rows and (tmp_path / "versions.json").exists()
    assert index_build.get_index_version("user-1") == 1
    row = store.text_rows[0]
    assert row.document_id == "doc-1" and row.meta["user_id"] == "user-1" and row.meta["modality"] == "text"
    assert index_build.index_text_nodes("user-1", [{"id": "x", "text": "   "}]) == []


def test_index_image_nodes(monkeypatch, tmp_path):
    from app.ml import index_build

    store = _DummyStore()
    monkeypatch.setattr(index_build, "_LANCEDB_STORE", store)
    monkeypatch.setattr(index_build, "_VERSION_FILE", tmp_path / "versions.json")
    monkeypatch.setattr(index_build, "embed_images_batch", lambda paths: np.ones((len(list(paths)), 512), np.float32))
    f = tmp_path / "image.png"
    f.write_bytes(b"fake")
    nodes = [{"id": "img-1", "metadata": {"file_path": str(f), "doc_id": "doc-1", "source": "youtube"}},
             {"id": "img-2", "metadata": {"file_path": str(tmp_path / "missing.png")}}]
    indexed = index_build.index_image_nodes("user-1", nodes)
    assert [i["chunk_id"] for i in indexed] == ["img-1"] and len(store.image_rows) == 1
    assert isinstance(store.image_rows[0].embedding, list)  # a foreign store gets the reference's lists


def test_normalize_rows_bit_identical_to_normalize():
    """LanceDBStore._normalize_rows (the array path index_*_nodes take into this store) gives the
    bytes of the reference's per-vector _normalize (app/storage/lancedb_store.py:63-69) on every
    row: un-normalised, tiny, huge, zero and NaN rows."""
    from app.storage.lancedb_store import LanceDBStore

    rng = np.random.default_rng(3)
    e = rng.standard_normal((300, 512)).astype(np.float32) * rng.uniform(1e-3, 1e3, (300, 1)).astype(np.float32)
    e[5] = 0
    e[6, 3] = np.nan
    e[7] *= np.float32(1e-20)
    e[8] *= np.float32(1e18)
    got = LanceDBStore._normalize_rows(e)
    assert got.dtype == np.float32
    for i in range(len(e)):
        want = np.asarray(LanceDBStore._normalize(e[i].tolist()), dtype=np.float32)
        assert want.tobytes() == got[i].tobytes(), i


def test_prepare_rows_array_equals_list_path():
    """The array path's payloads equal _prepare_rows' (the reference's helper) field for field, the
    vectors byte for byte; the store dispatches numpy-row embeddings to it and lists to the
    reference's helper."""
    from app.storage.lancedb_store import LanceDBStore, VectorRow

    rng = np.random.default_rng(4)
    e = rng.standard_normal((64, 384)).astype(np.float32)
    rows = [VectorRow(chunk_id=f"c{i}", user_id="u", document_id=f"d{i}", modality="text", embedding=e[i],
                      meta={"i": i, "s": "x"}) for i in range(64)]
    payloads, vectors = LanceDBStore._prepare_rows_array(rows)
    ref = LanceDBStore._prepare_rows([VectorRow(**{**r.__dict__, "embedding": r.embedding.tolist()}) for r in rows])
    for p, q, v in zip(payloads, ref, vectors):
        assert {k: p[k] for k in p if k != "embedding"} == {k: q[k] for k in q if k != "embedding"}
        assert np.asarray(q["embedding"], np.float32).tobytes() == v.tobytes() == p["embedding"].tobytes()

    class _T:
        def upsert(self, payloads, vectors=None):
            self.got = (payloads, vectors)

    store = LanceDBStore.__new__(LanceDBStore)
    t = _T()
    store._upsert(t, rows)
    assert t.got[1] is not None and t.got[1].tobytes() == vectors.tobytes()
    store._upsert(t, [VectorRow(**{**r.__dict__, "embedding": r.embedding.tolist()}) for r in rows])
    assert t.got[1] is None and t.got[0] == ref


# ---------------------------------------------------------------- cache
def test_query_embedding_cache():
    from app.cache import get_query_embeddings, set_query_embeddings

    set_query_embeddings(" test Query ", np.ones(384, np.float32), np.ones(512, np.float32), ttl=1)
    assert get_query_embeddings("test query") is not None


def test_retrieval_cache_version_invalidation():
    from app.cache import get_retrieval_results, set_retrieval_results

    set_retrieval_results("user", "q", 1, [1])
    assert get_retrieval_results("user", "Q", 1) == [1]
    assert get_retrieval_results("user", "Q", 2) is None


# ---------------------------------------------------------------- store helpers vs reference outputs
def test_store_helpers_match_reference():
    from app.storage.lancedb_store import LanceDBStore

    g = np.load(os.path.join(GOLDEN, "golden_normalize.npz"))
    for i in range(3):
        np.testing.assert_array_equal(np.asarray(LanceDBStore._normalize(g[f"vec{i}"]), np.float32),
                                      g[f"vec{i}_expected"])
    d = json.load(open(os.path.join(GOLDEN, "golden_format.json")))
    assert LanceDBStore._format_results(d["rows"]) == d["expected"]
    assert LanceDBStore._where_clause("user_id", "o'brien") == "user_id == 'o''brien'"


def test_embeddings_normalize_matches_reference():
    from app.ml.embeddings import _normalize

    g = np.load(os.path.join(GOLDEN, "golden_normalize.npz"))
    np.testing.assert_array_equal(_normalize(g["x"].copy()), g["expected"])


# ---------------------------------------------------------------- host preprocessing
@pytest.mark.parametrize("hw", [(224, 224), (256, 320), (480, 200), (33, 57), (224, 500)])
def test_preprocess_matches_clip_image_processor(hw):
    from transformers import CLIPImageProcessor

    from app.encoders.preprocess import to_u8_224

    rng = np.random.default_rng(hw[0] * 1000 + hw[1])
    img = Image.fromarray(rng.integers(0, 256, (*hw, 3), dtype=np.uint8))
    ref = CLIPImageProcessor(do_rescale=False, do_normalize=False)(images=img, return_tensors="np")["pixel_values"][0]
    np.testing.assert_array_equal(to_u8_224(img), ref.transpose(1, 2, 0).round().astype(np.uint8))


def test_golden_images_preprocess():
    from app.encoders.preprocess import to_u8_224

    g = np.load(os.path.join(GOLDEN, "golden_clip_image.npz"))
    np.testing.assert_array_equal(to_u8_224(Image.fromarray(g["raw_2"])), g["images_u8"][2])
    np.testing.assert_array_equal(to_u8_224(Image.fromarray(g["raw_0"])), g["images_u8"][0])


# ---------------------------------------------------------------- splitter / tokenisers
def test_splitter_contract():
    from app.ml.splitter import Document, SentenceSplitter

    sp = SentenceSplitter(chunk_size=20, chunk_overlap=10)
    text = " ".join(f"Sentence number {i} has a few words." for i in range(30))
    nodes = sp.get_nodes_from_documents([Document(text=text, metadata={"source": "pdf", "page_no": 3}, doc_id="d")])
    assert len(nodes) > 5
    assert all(len(n.text.split()) <= 20 for n in nodes)
    assert nodes[0].get_content("all").startswith("source: pdf\npage_no: 3\n\n")
    # overlap: the last whole sentence (7 words <= 10) of a chunk opens the next one
    assert nodes[1].text.split()[:7] == nodes[0].text.split()[-7:]
    assert len({n.node_id for n in nodes}) == len(nodes) and all(n.ref_doc_id == "d" for n in nodes)


def test_tokenizers_fallback():
    from app.encoders.tokenize import ClipTokenizer, WordPieceTokenizer

    ids, mask = WordPieceTokenizer()(["Hello, world!", "a much longer sentence with more words"])
    assert ids[0, 0] == 101 and ids[0, mask[0].sum() - 1] == 102 and mask.shape == ids.shape
    ids, mask = ClipTokenizer()(["a photo of a cat"])
    assert ids[0, 0] == 49406 and ids[0, -1] == 49407 and mask.all()
    with pytest.raises(ValueError):
        ClipTokenizer()([" ".join(["word"] * 100)])
    long_ids, _ = WordPieceTokenizer()([" ".join(["word"] * 400)])
    assert long_ids.shape[1] == 256


def test_splitter_algorithm_properties():
    """llama_index SentenceSplitter restatement (§8f row 4; unpinned without tiktoken/nltk):
    with a pluggable whitespace tokenizer every chunk fits the (metadata-aware) budget,
    chunks cover the text in order, each chunk after the first opens with at most
    chunk_overlap tokens of its predecessor's tail, and an over-long unpunctuated run is
    split down to words."""
    from app.ml.splitter import Document, SentenceSplitter

    tok = str.split
    sp = SentenceSplitter(chunk_size=12, chunk_overlap=4, tokenizer=tok)
    rng = np.random.default_rng(0)
    sents = [" ".join(f"w{j}" for j in rng.integers(0, 99, int(rng.integers(2, 9)))) + "." for _ in range(40)]
    text = " ".join(sents[:20]) + "\n\n\n" + " ".join(sents[20:]) + " " + " ".join(f"x{i}" for i in range(30))
    chunks = sp.split_text(text)
    assert all(len(tok(c)) <= 12 for c in chunks)
    words = tok(text)
    pos = 0
    for i, c in enumerate(chunks):  # each chunk = overlap (<= 4 tokens) + new words, in order
        cw = tok(c)
        start = words.index(cw[0], max(0, pos - 4))
        assert words[start:start + len(cw)] == cw
        assert pos - start <= 4
        pos = start + len(cw)
    assert pos == len(words)
    meta = {"source": "pdf", "page_no": 3}
    nodes = sp.get_nodes_from_documents([Document(text=text, metadata=meta, doc_id="d")])
    budget = 12 - len(tok("source: pdf\npage_no: 3"))
    # a new chunk always takes its first split on top of the carried overlap (<= 4 tokens)
    assert all(len(tok(n.text)) <= budget + 4 for n in nodes) and max(len(tok(n.text)) for n in nodes) > budget
    with pytest.raises(ValueError):
        sp.split_text_metadata_aware("a b c", "k: " + " ".join(["v"] * 20))


def test_fuse_scores_matches_reference_fusion():
    """The batched, vectorised fusion (app.retrieval.fuse_scores: BASELINE config 5's last
    step) equals the drop-in's per-query ``_fuse_results`` — itself pinned against the
    reference's outputs (golden_fusion.json) — on ragged, tied and constant lists."""
    from app.ml import retrieve as r
    from app.retrieval import fuse_scores

    rng = np.random.default_rng(5)
    Q, kt, ki = 60, 50, 12
    ts = np.sort(rng.normal(0.3, 0.05, (Q, kt)).astype(np.float32), axis=1)[:, ::-1].copy()
    im = np.sort(rng.normal(0.2, 0.03, (Q, ki)).astype(np.float32), axis=1)[:, ::-1].copy()
    ts[3, 20:] = -np.inf  # fewer hits than k
    im[4, 5:] = -np.inf
    im[5, :] = -np.inf  # no image hits
    ts[6, :] = np.float32(0.5)  # zero std -> zeros
    ts[7, 1:3] = ts[7, 0]  # ties
    im[8, :] = -np.inf
    im[8, 0] = np.float32(0.9)  # single hit: std 0
    pick, comb = fuse_scores(ts, im, final_n=4)
    for q in range(Q):
        texts = [{"chunk_id": f"t{j}", "score": 1.0 - float(np.float32(1.0) - s)}
                 for j, s in enumerate(ts[q]) if np.isfinite(s)]
        imgs = [{"chunk_id": f"i{j}", "score": 1.0 - float(np.float32(1.0) - s)}
                for j, s in enumerate(im[q]) if np.isfinite(s)]
        ref = r._fuse_results(texts, imgs)
        got = []
        for p in pick[q]:
            if p < 0:
                continue
            got.append(f"t{p}" if p < kt else f"i{p - kt}")
        assert got == [e["chunk_id"] for e in ref], q
        np.testing.assert_array_equal(comb[q][: len(ref)], [e["combined_score"] for e in ref])


def test_batched_chunk_lookup_equals_per_hit(tmp_path):
    """retrieve's hit lookup (one SQLite statement through MetadataStore.get_chunks) returns what the
    reference's per-hit get_chunk does, in hit order: missing ids -> None, duplicates repeated,
    more than one statement's worth of ids."""
    from app.ml import retrieve as r
    from app.storage.schema import Chunk, MetadataStore

    store = MetadataStore(str(tmp_path / "m.sqlite3"))
    store.upsert_chunks([Chunk(id=f"c{i}", document_id="d", modality="text" if i % 3 else "image",
                               text=None if i % 7 == 0 else f"t{i}", page_no=i, meta={"k": i}) for i in range(1200)])

    class PerHit:
        def get_chunk(self, chunk_id):
            return store.get_chunk(chunk_id)

    hits = [{"chunk_id": f"c{i}"} for i in [5, 1199, 3, 5, 77, 4000, 0, *range(100, 1150)]]
    old = r._METADATA_STORE
    try:
        r._METADATA_STORE = store
        batched = r._chunks_for(hits)
        r._METADATA_STORE = PerHit()
        per_hit = r._chunks_for(hits)
    finally:
        r._METADATA_STORE = old
    assert [c.model_dump() if c else None for c in batched] == [c.model_dump() if c else None for c in per_hit]
    assert batched[5] is None and batched[0] is not None


def test_paths_exist_equals_pathlib(tmp_path):
    """index_image_nodes' existence filter (one mrag_paths_exist call) gives Path(s).exists() for
    every kind of path the reference's per-node check sees."""
    from pathlib import Path

    from app.ml.index_build import _paths_exist

    f = tmp_path / "a.png"
    f.write_bytes(b"x")
    (tmp_path / "d").mkdir()
    (tmp_path / "loop").symlink_to(tmp_path / "loop")
    cases = [str(f), str(tmp_path / "missing.png"), "", ".", str(tmp_path / "d"), str(f) + "/x",
             str(tmp_path) + "//a.png", "a\0b", str(tmp_path / "loop"), str(tmp_path / "d" / ".." / "a.png")]
    assert _paths_exist(cases) == [Path(s).exists() for s in cases]
