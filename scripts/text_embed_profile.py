#!/usr/bin/env python3
"""embed_text_batch over the bench's index_text_nodes chunks (1,000 synthetic documents split by
SentenceSplitter(512/64)): the whole call, the tokeniser alone and the GPU encodes alone (token ids
already on the device), median of five."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from app.ml import embeddings as emb_mod  # noqa: E402
from app.ml import index_build as ib  # noqa: E402
from app.ml.splitter import Document  # noqa: E402

docs = bench._synthetic_documents(1000)
nodes = ib._SPLITTER.get_nodes_from_documents([Document(text=d["text"], metadata=d["metadata"], doc_id=d["id"]) for d in docs])
texts = [n.get_content(metadata_mode="all") for n in nodes]
model = emb_mod._ensure_text_model()
emb_mod.embed_text_batch(texts[:300])
torch.cuda.synchronize()


def med(f, n=5):
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        t = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return round(sorted(ts)[n // 2], 2)


order = np.argsort([-len(s) for s in texts], kind="stable")
batches = [order[s:s + 256] for s in range(0, len(order), 256)]
toks = [model.tokenizer([texts[i] for i in idx]) for idx in batches]
dev = torch.device("cuda", 0)
dtoks = [(torch.from_numpy(a).to(dev), torch.from_numpy(m).to(dev)) for a, m in toks]
h = model._pool.acquire()


def gpu_only():
    for ids, mask in dtoks:
        h.embed_tokens(ids, mask, normalize=True)


out = {"chunks": len(texts), "tokens_per_batch": [int(m.sum()) for _, m in toks],
       "padded_T": [int(a.shape[1]) for a, _ in toks],
       "embed_text_batch_ms": med(lambda: emb_mod.embed_text_batch(texts)),
       "tokenizer_ms": med(lambda: [model.tokenizer([texts[i] for i in idx]) for idx in batches]),
       "gpu_encodes_ms": med(gpu_only)}
model._pool.release(h)
print(json.dumps(out))
