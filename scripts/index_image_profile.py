#!/usr/bin/env python3
"""index_image_nodes against embed_images_batch on the bench's 2,048 ingest files, interleaved call
by call on one box, with index_image_nodes split into its phases (wall ms, wrappers around the
module's own functions): the existence check, the embed (first batch, all batches), the upsert,
the version bump. One JSON line per call pair, then the medians."""
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import bench  # noqa: E402  (MRAG_SYNTHETIC_WEIGHTS)
from app.ml import embeddings as emb_mod  # noqa: E402
from app.ml import index_build as ib  # noqa: E402
from app.storage.lancedb_store import LanceDBStore  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
d = tempfile.mkdtemp(prefix="mrag_idx_prof_")
T = {}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            T[name] = T.get(name, 0.0) + (time.perf_counter() - t0) * 1e3
    return w


def timed_gen(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        first = True
        for x in fn(*a, **k):
            if first:
                T[name + "_first"] = (time.perf_counter() - t0) * 1e3
                first = False
            t1 = time.perf_counter()
            yield x
            T[name + "_consumer"] = T.get(name + "_consumer", 0.0) + (time.perf_counter() - t1) * 1e3
        T[name] = (time.perf_counter() - t0) * 1e3 - T.get(name + "_consumer", 0.0)
    return w


ib._paths_exist = timed("paths_exist", ib._paths_exist)
ib.embed_images_batches = timed_gen("embed", ib.embed_images_batches)
LanceDBStore._upsert_image_payloads = timed("upsert", LanceDBStore._upsert_image_payloads)
ib._bump_version = timed("bump", ib._bump_version)
from app.storage import corpus_files as cf  # noqa: E402
from app.storage import lancedb_store as ls  # noqa: E402
from app.vector_store import FlatIndex  # noqa: E402

cf.CorpusFiles.append = timed("upsert.files_append", cf.CorpusFiles.append)
ls._Table._sync = timed("upsert.sync", ls._Table._sync)
ls._Table._append_rows = timed("upsert.append_rows", ls._Table._append_rows)
FlatIndex.add = timed("upsert.append_rows.gpu_add", FlatIndex.add)
try:
    paths = bench._write_images(d, n)
    with bench._BenchStore() as bs:
        emb_mod.embed_images_batch(paths[:256])
        bs.ib.index_image_nodes("u0", [{"id": f"w{i}", "metadata": {"file_path": p}} for i, p in enumerate(paths[:256])])
        rows = []
        for c in range(rounds):
            bench._sync()
            t0 = time.perf_counter()
            emb_mod.embed_images_batch(paths)
            bench._sync()
            t_embed = (time.perf_counter() - t0) * 1e3
            nodes = [{"id": f"img{c}_{i}", "metadata": {"file_path": p, "doc_id": f"doc{i >> 4}", "source": "bench"}}
                     for i, p in enumerate(paths)]
            T.clear()
            bench._sync()
            t0 = time.perf_counter()
            ib.index_image_nodes("u0", nodes)
            bench._sync()
            t_index = (time.perf_counter() - t0) * 1e3
            r = {"embed_images_batch_ms": round(t_embed, 2), "index_image_nodes_ms": round(t_index, 2),
                 "ratio": round(t_embed / t_index, 3), **{k: round(v, 2) for k, v in T.items()}}
            rows.append(r)
            print(json.dumps(r), flush=True)
        med = lambda k: sorted(x[k] for x in rows)[len(rows) // 2]  # noqa: E731
        print(json.dumps({"median_embed_ms": med("embed_images_batch_ms"), "median_index_ms": med("index_image_nodes_ms"),
                          "ratio_of_medians": round(med("embed_images_batch_ms") / med("index_image_nodes_ms"), 3)}))
finally:
    shutil.rmtree(d, ignore_errors=True)
