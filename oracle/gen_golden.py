#!/usr/bin/env python3
"""Generate tests/golden/* by running the REFERENCE's own code (test infrastructure).

Run in this container only (needs /root/reference):  python oracle/gen_golden.py

The reference is imported from /root/reference with sys.modules stubs for the three
packages it imports that are not installed (sentence_transformers, lancedb,
llama_index — none of their arithmetic is exercised: the stubs only satisfy imports;
SURVEY.md §8c). It runs in this process under the package name `app`, which is why
the product's weight generator is loaded by file path (oracle.models.weights_module).

Fixtures written (each < 1 MB):
  golden_clip_image.npz  reference embed_images_batch() (app/ml/embeddings.py:73-91) on
                         PNG files; a real CLIPModel with the synthetic weights; the
                         processor is transformers' CLIPImageProcessor (openai defaults)
  golden_clip_text.npz   CLIPModel.get_text_features on token ids + reference _normalize
  golden_minilm.npz      reference embed_text_batch() (:52-70) with a BertModel +
                         mean-pool + Normalize model object (ST restated: not installed)
  golden_normalize.npz   reference embeddings._normalize / LanceDBStore._normalize
  golden_fusion.json     reference retrieve._z_scores / _fuse_results
  golden_format.json     reference LanceDBStore._format_results
  golden_knn.npz         oracle.knn on seeded corpora (lance is not installed; the
                         oracle itself is pinned against scikit-learn in the tests)
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")


def _install_stubs():
    st = types.ModuleType("sentence_transformers")

    class SentenceTransformer:  # never constructed: the tests set _TEXT_MODEL
        def __init__(self, *a, **k):
            raise RuntimeError("stub")

    class CrossEncoder(SentenceTransformer):
        pass

    st.SentenceTransformer = SentenceTransformer
    st.CrossEncoder = CrossEncoder
    sys.modules["sentence_transformers"] = st

    ldb = types.ModuleType("lancedb")

    class _Table:
        def create_index(self, **k):
            raise RuntimeError("stub")

    class _DB:
        def table_names(self):
            return []

        def create_table(self, name, schema=None):
            return _Table()

        def open_table(self, name):
            return _Table()

    ldb.connect = lambda path: _DB()
    sys.modules["lancedb"] = ldb

    li = types.ModuleType("llama_index")
    core = types.ModuleType("llama_index.core")
    np_ = types.ModuleType("llama_index.core.node_parser")
    sc = types.ModuleType("llama_index.core.schema")

    class SentenceSplitter:
        def __init__(self, *a, **k):
            pass

    class Document:
        def __init__(self, *a, **k):
            pass

    np_.SentenceSplitter = SentenceSplitter
    sc.Document = Document
    li.core = core
    core.node_parser = np_
    core.schema = sc
    for name, mod in (("llama_index", li), ("llama_index.core", core), ("llama_index.core.node_parser", np_),
                      ("llama_index.core.schema", sc)):
        sys.modules[name] = mod


def main():
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="mrag_golden_")
    os.environ["LANCEDB_DIR"] = tmp
    _install_stubs()
    sys.path.insert(0, REF)
    sys.path.insert(0, HERE)  # oracle modules importable as top-level (models, knn)
    import torch
    from PIL import Image
    from transformers import CLIPImageProcessor

    import models as om  # oracle/models.py
    import knn as ok  # oracle/knn.py
    from app.ml import embeddings as ref_emb  # the reference
    from app.ml import retrieve as ref_ret
    from app.storage.lancedb_store import LanceDBStore as RefStore

    torch.manual_seed(0)
    rng = np.random.default_rng(2)

    # ---------------- CLIP image: reference embed_images_batch on PNG files
    clip = om.clip_model(seed=0)

    class _ClipWrap:  # transformers 5.x returns ModelOutput; the reference expects a tensor
        def __init__(self, m):
            self.m = m

        def to(self, device):
            return self

        def get_image_features(self, **inputs):
            return self.m.get_image_features(**inputs).pooler_output

        def get_text_features(self, **inputs):
            return self.m.get_text_features(**inputs).pooler_output

    proc = CLIPImageProcessor()  # openai/clip-vit-base-patch32 preprocessing defaults
    shapes = [(224, 224), (224, 224), (256, 320)]
    paths, raw = [], []
    for i, (hh, ww) in enumerate(shapes):
        a = rng.integers(0, 256, (hh, ww, 3), dtype=np.uint8)
        p = os.path.join(tmp, f"img{i}.png")
        Image.fromarray(a).save(p)
        paths.append(p)
        raw.append(a)
    ref_emb._CLIP_MODEL = _ClipWrap(clip)
    ref_emb._CLIP_PROCESSOR = proc
    with torch.no_grad():
        img_out = ref_emb.embed_images_batch(paths)
    # the u8 224x224 images the processor produced after resize / centre crop
    noscale = CLIPImageProcessor(do_rescale=False, do_normalize=False)
    u8 = np.stack([noscale(images=Image.open(p).convert("RGB"), return_tensors="np")["pixel_values"][0]
                   .transpose(1, 2, 0).round().astype(np.uint8) for p in paths])
    unnorm = om.clip_image_embeds(clip, u8, normalize=False)
    np.savez_compressed(os.path.join(OUT, "golden_clip_image.npz"), images_u8=u8, raw_0=raw[0], raw_2=raw[2],
                        expected=img_out.astype(np.float32), expected_unnormalized=unnorm.astype(np.float32))

    # ---------------- CLIP text: ids (BOS 49406 ... EOS 49407, EOS-padded)
    T = 16
    lens = [16, 9, 5, 12]
    ids = np.full((len(lens), T), 49407, dtype=np.int64)
    mask = np.zeros((len(lens), T), dtype=np.int64)
    for b, L in enumerate(lens):
        ids[b, 0] = 49406
        ids[b, 1:L - 1] = rng.integers(300, 49000, L - 2)
        ids[b, L - 1] = 49407
        mask[b, :L] = 1
    with torch.no_grad():
        txt = clip.get_text_features(input_ids=torch.from_numpy(ids), attention_mask=torch.from_numpy(mask)).pooler_output
    txt_norm = ref_emb._normalize(txt.float().numpy())
    np.savez_compressed(os.path.join(OUT, "golden_clip_text.npz"), ids=ids.astype(np.int32),
                        mask=mask.astype(np.int32), expected=txt_norm.astype(np.float32),
                        expected_unnormalized=txt.float().numpy())

    # ---------------- MiniLM: reference embed_text_batch with an ST-equivalent model object
    bert = om.bert_model(seed=0)
    mlens = [8, 23, 64, 13, 31, 40, 9, 57]
    Tm = max(mlens)
    mids = np.zeros((len(mlens), Tm), dtype=np.int64)
    mmask = np.zeros((len(mlens), Tm), dtype=np.int64)
    for b, L in enumerate(mlens):
        mids[b, 0] = 101
        mids[b, 1:L - 1] = rng.integers(1000, 30000, L - 2)
        mids[b, L - 1] = 102
        mmask[b, :L] = 1
    table = {f"#{i}": i for i in range(len(mlens))}

    class _MiniLM:  # SentenceTransformer.encode restated: BertModel -> mean pool -> Normalize
        def to(self, device):
            return self

        def encode(self, texts, batch_size=32, convert_to_tensor=True, device=None, show_progress_bar=None):
            rows = [table[t] for t in texts]
            e = om.minilm_embeds(bert, mids[rows], mmask[rows], normalize=False)
            t = torch.nn.functional.normalize(torch.from_numpy(e), p=2, dim=1, eps=1e-12)
            return t

    ref_emb._TEXT_MODEL = _MiniLM()
    with torch.no_grad():
        mini = ref_emb.embed_text_batch(list(table))
    np.savez_compressed(os.path.join(OUT, "golden_minilm.npz"), ids=mids.astype(np.int32),
                        mask=mmask.astype(np.int32), expected=mini.astype(np.float32),
                        expected_unnormalized=om.minilm_embeds(bert, mids, mmask, normalize=False))

    # ---------------- normalisers
    x = (rng.standard_normal((33, 512)) * rng.uniform(0.01, 10, (33, 1))).astype(np.float32)
    x[5] = 0.0
    vecs = [rng.standard_normal(384).astype(np.float32) * 3, np.zeros(512, np.float32),
            rng.standard_normal(512).astype(np.float32)]
    np.savez_compressed(os.path.join(OUT, "golden_normalize.npz"), x=x, expected=ref_emb._normalize(x.copy()),
                        **{f"vec{i}": v for i, v in enumerate(vecs)},
                        **{f"vec{i}_expected": np.asarray(RefStore._normalize(v), np.float32) for i, v in enumerate(vecs)})

    # ---------------- fusion / format
    cases = []
    fr = np.random.default_rng(7)
    base_t = [{"chunk_id": "t1", "score": 0.8}, {"chunk_id": "t2", "score": 0.6}]
    base_i = [{"chunk_id": "i1", "score": 0.7}]
    rr = [dict(base_t[0], rerank_score=0.1), dict(base_t[1], rerank_score=0.9)]
    cases.append({"text": rr, "image": base_i})
    for _ in range(6):
        nt, ni = int(fr.integers(0, 9)), int(fr.integers(0, 5))
        t = [{"chunk_id": f"t{j}", "score": float(fr.uniform(0, 1))} for j in range(nt)]
        for j in range(min(nt, int(fr.integers(0, 5)))):
            t[j]["rerank_score"] = float(fr.normal())
        im = [{"chunk_id": f"i{j}", "score": float(fr.uniform(0, 1))} for j in range(ni)]
        cases.append({"text": t, "image": im})
    cases.append({"text": [{"chunk_id": "a", "score": 0.5}, {"chunk_id": "b", "score": 0.5}], "image": []})
    out_cases = []
    for c in cases:
        out_cases.append({"text": c["text"], "image": c["image"],
                          "z_text": ref_ret._z_scores([it["score"] for it in c["text"]]),
                          "fused": ref_ret._fuse_results([dict(i) for i in c["text"]], [dict(i) for i in c["image"]])})
    with open(os.path.join(OUT, "golden_fusion.json"), "w") as f:
        json.dump({"final_n": 4, "cases": out_cases}, f, indent=1)
    rows = [{"chunk_id": f"c{i}", "_distance": float(np.float32(fr.uniform(0, 1.2))), "meta": json.dumps({"i": i})}
            for i in range(7)]
    with open(os.path.join(OUT, "golden_format.json"), "w") as f:
        json.dump({"rows": rows, "expected": RefStore._format_results(rows)}, f, indent=1)

    # ---------------- kNN (oracle, pinned against sklearn in tests/test_oracle_pinning.py)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _data import clustered_corpus, labels_for, sha, unit_rows

    knn = {}
    for tag, (n, d, seed, nq, k) in {"a": (4096, 512, 0, 64, 10), "b": (4096, 384, 1, 64, 50),
                                    "c": (3000, 128, 2, 17, 12)}.items():
        X = unit_rows(n, d, seed) if tag != "c" else clustered_corpus(n, d, seed, dup_frac=0.2)
        lab = labels_for(n, 5, seed + 100)
        Q = unit_rows(nq, d, seed + 200)
        s, r = ok.flat_cosine_topk(X, lab, Q, k, label_filter=-1)
        s2, r2 = ok.flat_cosine_topk(X, lab, Q, k, label_filter=3)
        knn.update({f"{tag}_shape": np.array([n, d, seed, nq, k]), f"{tag}_sha": np.array(sha(X, lab, Q)),
                    f"{tag}_scores": s, f"{tag}_rows": r, f"{tag}_scores_f3": s2, f"{tag}_rows_f3": r2})
    np.savez_compressed(os.path.join(OUT, "golden_knn.npz"), **knn)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
