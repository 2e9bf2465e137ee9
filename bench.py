#!/usr/bin/env python3
"""Headline benchmark: brute-force cosine kNN on 1M x 512 per GPU, top-k = 10.

Metric (BASELINE.json): "CLIP img-embeds/sec/GPU; kNN queries/sec on 1M×512 at
top-k=10, 1/2/4/8 GPUs". ``value`` is the kNN leg: whole-job queries/s, where one
query = one 512-d query scanned against one GPU's 1M-row shard (BASELINE config 3
at N=1; config 4's row-sharded layout at N>1: rank r holds global rows
[r*2^20, (r+1)*2^20), every step answers the same 1000 queries against all N*2^20
rows and ends with an RCCL all-gather of the per-shard top-k + the K11 merge).
Weak scaling: per-GPU work is fixed as N grows; value = N * 1000 * steps / t.

A step = one ``FlatIndex.search`` of 1000 queries (inputs already in HBM): query
prep, the K7 sample pre-pass (1/16 of the tiles, running maxima only) that seeds the
per-query threshold, the K7 fp16 MFMA scan, K8 merge + exact f64 rescore +
certificate, the (normally empty) collect pass, and for N>1 the all-gather + merge. The CLIP
ViT-B/32 leg (config 2) is reported beside it as ``clip`` when the encoder
library is present.

Run: python bench.py [--gpus N --steps K --warmup W]; N>1 under
torch.distributed.run (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

# synthetic encoder weights (random-init architecture; no hub checkpoints offline)
os.environ.setdefault("MRAG_SYNTHETIC_WEIGHTS", "1")
# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (HIP's default 4): with
# the bench's in-flight legs (three CLIP batches, two kNN searches, four config-5 steps of two
# branches, the image lanes' streams) two streams sharing a queue serialise. 8 queues when the
# environment does not say (set before the runtime starts); an explicit setting wins, and the GPU
# pool's boxes export 4, so the driver's runs use 4 (the line records it as "hip_hw_queues").
# With the CLIP leg's streams made at start-up and the image lanes on the handle's own streams
# the legs measure alike at 4 and 8 (profiles/r6s26_r6s27_hw_queues.txt; 16 cost config 5 ~8 %).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

ROWS_PER_GPU = 1 << 20
DIM = 512
NQ = 1000
TOPK = 10
MFMA_FP16_PEAK_TFLOPS = 2500.0  # dense fp16/bf16 MFMA, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0


def _dist_setup():
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one process per GPU; more ranks than GPUs (a rehearsal of the N > 1 path on a smaller box,
    # MRAG_DIST_BACKEND=gloo) share them round-robin. device_count() does not initialise the GPU.
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("MRAG_DIST_BACKEND", "nccl")  # "nccl" is RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def _max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _barrier(world: int):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def _cgroup_cpus():
    """CPUs the cgroup quota grants this process (cgroup v2 cpu.max), or None without a quota."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota == "max":
            return None
        return max(1, -(-int(quota) // int(period)))
    except Exception:
        return None


def _usable_cores() -> int:
    """Host cores the CPU baselines use: every core in this process's affinity mask, capped by
    the cgroup CPU quota when one is set (the GPU box's affinity lists the whole node while the
    job's share is a fraction of it; more threads than the quota only time-slice)."""
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    q = _cgroup_cpus()
    return min(cores, q) if q else cores


def _use_all_cores():
    """torch intra-op threads and the BLAS pool at _usable_cores() for a CPU baseline."""
    import torch

    n = _usable_cores()
    torch.set_num_threads(n)
    try:
        from threadpoolctl import threadpool_limits

        threadpool_limits(limits=n, user_api="blas")
    except Exception:
        pass
    return n


def _host_info():
    """Host cores this process may use, torch's intra-op threads, the BLAS numpy links."""
    import torch

    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    blas, blas_threads = "unknown", None
    try:
        from threadpoolctl import threadpool_info

        for i in threadpool_info():
            if i.get("user_api") == "blas":
                blas, blas_threads = f"{i.get('internal_api')} {i.get('version')}", i.get("num_threads")
                break
    except Exception:
        pass
    return {"affinity_cores": cores, "cgroup_cpus": _cgroup_cpus(), "usable_cores": _usable_cores(),
            "torch_threads": int(torch.get_num_threads()), "blas": blas, "blas_threads": blas_threads}


def _median_rate(fn, units: int, reps: int = 5):
    """Median over `reps` timed calls of fn() (after one warm call): units per second."""
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return units / ts[len(ts) // 2], ts


def cpu_baseline(seconds_budget: float = 20.0):
    """SURVEY §8(d) CPU path on the GPU box's host cores, bounded sample of the config-3
    workload: f32 brute force over the same 1M x 512 corpus shape, median of 5. Two
    implementations, the faster one is the baseline: numpy ``q @ X.T`` + ``argpartition`` +
    ordering of the k (the survey's recipe) and torch-CPU ``mm`` + ``topk`` (intra-op
    threaded selection). The exact f64 oracle stays the checker only (tests)."""
    import numpy as np
    import torch

    _use_all_cores()

    rng = np.random.default_rng(0)
    x = rng.standard_normal((ROWS_PER_GPU, DIM), dtype=np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    q = rng.standard_normal((NQ, DIM), dtype=np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)

    def np_search(qb):
        s = qb @ x.T
        part = np.argpartition(-s, TOPK - 1, axis=1)[:, :TOPK]
        ps = np.take_along_axis(s, part, axis=1)
        o = np.argsort(-ps, axis=1, kind="stable")
        return np.take_along_axis(ps, o, 1), np.take_along_axis(part, o, 1)

    xt = torch.from_numpy(x)

    def torch_search(qb):
        return torch.topk(torch.from_numpy(qb) @ xt.T, TOPK, dim=1)

    # size the batch so that 6 timed calls of the slower variant fit the budget
    t0 = time.perf_counter()
    np_search(q[:16])
    per_q = (time.perf_counter() - t0) / 16
    nb = int(min(NQ, max(16, seconds_budget / 12 / max(per_q, 1e-5))))
    r_np, t_np = _median_rate(lambda: np_search(q[:nb]), nb)
    r_t, t_t = _median_rate(lambda: torch_search(q[:nb]), nb)
    best = max(r_np, r_t)
    info = _host_info()
    return {
        "value": round(best, 2),
        "unit": "queries/s (1M x 512 f32 corpus, top-10)",
        "cores": info["torch_threads"] if r_t >= r_np else (info["blas_threads"] or info["affinity_cores"]),
        "host": info,
        "kind": "port",
        "variants_queries_per_s": {"numpy_matmul_argpartition": round(r_np, 2), "torch_mm_topk": round(r_t, 2)},
        "sample": f"{nb} of the 1000 queries against the same 1M x 512 corpus shape (f32, unit rows), median of 5 "
                  f"timed batches per variant (numpy {np.median(t_np):.2f} s, torch {np.median(t_t):.2f} s per batch); "
                  f"value = the faster variant",
    }


def clip_cpu_baseline(seconds_budget: float = 12.0):
    """oracle.models CLIP ViT-B/32 image tower (transformers, torch-CPU fp32) on the host
    cores, bounded sample of the config-2 workload: random 224x224 images, median of 5
    timed batches (batch size chosen to fit the budget)."""
    import numpy as np
    import torch

    _use_all_cores()

    from oracle.models import clip_image_embeds, clip_model

    model = clip_model(0)
    imgs = np.random.default_rng(2).integers(0, 256, (64, 224, 224, 3), dtype=np.uint8)
    t0 = time.perf_counter()
    clip_image_embeds(model, imgs[:8])
    per = (time.perf_counter() - t0) / 8
    nb = int(min(64, max(8, seconds_budget / 6 / max(per, 1e-4))))
    rate, ts = _median_rate(lambda: clip_image_embeds(model, imgs[:nb]), nb)
    return {"value": round(rate, 2), "unit": "images/s", "cores": int(torch.get_num_threads()), "kind": "port",
            "host": _host_info(),
            "sample": f"transformers CLIPModel.get_image_features fp32 on batches of {nb} random 224x224 images, "
                      f"median of 5 ({ts[len(ts) // 2]:.2f} s per batch)"}


def _traffic_from_profiles():
    """HBM bytes per K7 launch from the committed rocprofv3 PMC pass (or None)."""
    path = os.path.join(ROOT, "profiles", "knn_scan_pmc.json")
    try:
        with open(path) as f:
            return float(json.load(f)["hbm_bytes_per_launch"])
    except Exception:
        return None


def _early_streams(dev, n: int):
    """n HIP streams made (and each given one tiny kernel) before the bench's other legs create
    and destroy theirs. HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by
    default); streams taken late in the run from torch's pool landed two of the CLIP leg's three
    on one queue for some pool positions (78k vs 86k img/s on one box,
    profiles/r6s24_clip_stream_position.txt). A serving process makes its request streams once at
    start-up, as these are."""
    import torch

    ss = [torch.cuda.Stream(device=dev) for _ in range(n)]
    for s in ss:
        with torch.cuda.stream(s):
            torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize(dev)
    return ss


def clip_leg(steps: int, warmup: int, streams=None):
    """CLIP ViT-B/32 image embeds/s on one GPU (config 2: batch 256, fp16)."""
    try:
        from app.encoders import bench_clip_images
    except Exception:
        return None
    out = bench_clip_images(steps=steps, warmup=warmup, streams=streams)  # three batches in flight
    # one batch at a time on a stream from torch's pool, as before: its image lanes fork onto the
    # handle's own lane stream, which shared a hardware queue with the start-up stream in three of
    # four runs (53k instead of 74k img/s, profiles/r6s26_r6s27_hw_queues.txt)
    one = bench_clip_images(steps=steps, warmup=warmup, inflight=1)
    out["one_batch_in_flight"] = {"images_per_s": one["value"], "ms_per_batch": one["ms_per_batch"]}
    return out


def call_pattern_leg(index, q, reps: int = 200):
    """The reference's own call pattern over the same 1M x 512 shard: retrieve_text /
    retrieve_images issue ONE query per search (app/ml/retrieve.py:53,84 ->
    app/storage/lancedb_store.py:103-123). Timed here, one GPU, beside `value` (never as it):

    * ``device_q{1,8}``: FlatIndex.search of 1 / 8 device-resident queries on a stream (the scan
      streams the corpus once per search: K7s, the 64-query scan instance), with the K7 launch
      time from the in-library HIP events -> HBM GB/s of the corpus read (N * D * 2 bytes);
    * ``host_q1``: numpy query in, numpy results out (PCIe both ways);
    * ``dropin_search_image``: ``LanceDBStore.search_image(user_id, vec.tolist(), 10)`` through
      the drop-in module on a 1M-row table (Python list in, formatted hit dicts out)."""
    import numpy as np
    import torch

    out = {}
    dev = q.device
    stream = torch.cuda.Stream(device=dev)
    for nq in (1, 8):
        qq = q[:nq].contiguous()
        with torch.cuda.stream(stream):
            for _ in range(10):
                index.search(qq, TOPK)
            stream.synchronize()
            index.profile(1)
            t0 = time.perf_counter()
            for _ in range(reps):
                index.search(qq, TOPK)
            stream.synchronize()
            dt = (time.perf_counter() - t0) / reps
            scan_ms, n = index.profile(0)
        scan_s = scan_ms / max(n, 1) / 1e3
        gbs = ROWS_PER_GPU * DIM * 2 / scan_s / 1e9 if scan_s > 0 else 0.0
        out[f"device_q{nq}"] = {"ms_per_search": round(dt * 1e3, 4), "queries_per_s": round(nq / dt, 1),
                                "scan_ms": round(scan_s * 1e3, 4), "scan_hbm_gbs": round(gbs, 1),
                                "scan_hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
    qh = q[:1].cpu().numpy()
    for _ in range(10):
        index.search(qh, TOPK)
    t0 = time.perf_counter()
    for _ in range(reps):
        index.search(qh, TOPK)
    dt = (time.perf_counter() - t0) / reps
    out["host_q1"] = {"ms_per_search": round(dt * 1e3, 4), "queries_per_s": round(1 / dt, 1)}

    # the drop-in store over the same GPU index: one table of 1M rows of user "u0"
    os.environ["MRAG_STORE_PERSIST"] = "0"
    import tempfile

    from app.storage.lancedb_store import LanceDBStore

    store = LanceDBStore(tempfile.mkdtemp(prefix="mrag_bench_store_"))
    t = store._image_table
    t.index, t.dim = index, DIM
    t.chunk_ids = [f"c{i}" for i in range(ROWS_PER_GPU)]
    t.metas = ["{}"] * ROWS_PER_GPU
    t.labels = {"u0": 0}
    vec = q[0].cpu().numpy().tolist()
    hits = store.search_image("u0", vec, TOPK)
    for _ in range(10):
        store.search_image("u0", vec, TOPK)
    t0 = time.perf_counter()
    for _ in range(reps):
        store.search_image("u0", vec, TOPK)
    dt = (time.perf_counter() - t0) / reps
    out["dropin_search_image"] = {"ms_per_call": round(dt * 1e3, 4), "calls_per_s": round(1 / dt, 1),
                                  "hits": len(hits)}
    t.index = None  # the bench owns the index
    out["note"] = ("one query per search, the reference's call pattern (retrieve_text / retrieve_images); "
                   "scan_hbm_gbs = 1M x 512 fp16 corpus bytes / K7 launch time (HIP events)")
    return out


RETRIEVE_TEXT_DIM = 384
RETRIEVE_META_ROWS = 1 << 16  # chunk rows in the SQLite catalog per modality (row i -> chunk i mod this)


def _sync():
    import torch

    torch.cuda.synchronize()


def _per_call_ms(fn, args_list):
    """Mean wall ms of fn(*a) over args_list, the device drained before and after."""
    _sync()
    t0 = time.perf_counter()
    for a in args_list:
        fn(*a)
    _sync()
    return (time.perf_counter() - t0) / max(1, len(args_list)) * 1e3


def retrieve_pattern_leg(image_index, reps: int = 100):
    """The reference's per-query path end to end, through the drop-in modules
    (app/ml/retrieve.py:41-100 with _get_embeddings :120-129): ``retrieve_text(user, query)``
    = MiniLM on [query] (B = 1) + CLIP-text on the query (B = 1) + ``search_text`` (top-50) over
    a 1M x 384 table + one SQLite ``get_chunk`` per hit + result dicts; then
    ``retrieve_images(user, query)`` for the same query = (query embeddings from the cache, as in
    the reference) + ``search_image`` (top-12) over the 1M x 512 table + lookups. Every query is
    a distinct string, so the embedding and result caches miss as on fresh queries. Synthetic
    weights; the tokenisers are the offline ones. The split times each part alone over the same
    kind of query (wall ms, device drained around each)."""
    import numpy as np
    import tempfile

    import torch

    os.environ["MRAG_STORE_PERSIST"] = "0"
    from app.ml import embeddings as emb_mod
    from app.ml import retrieve as rmod
    from app.settings import settings
    from app.storage.lancedb_store import LanceDBStore
    from app.storage.schema import MetadataStore
    from app.vector_store import FlatIndex

    dev = torch.device("cuda", image_index.device if hasattr(image_index, "device") else 0)
    d = tempfile.mkdtemp(prefix="mrag_bench_retrieve_")
    store = LanceDBStore(d)
    g = torch.Generator(device=dev).manual_seed(4000)
    xt = torch.randn((ROWS_PER_GPU, RETRIEVE_TEXT_DIM), generator=g, device=dev)
    text_index = FlatIndex(RETRIEVE_TEXT_DIM, device=dev.index or 0)
    text_index.add(xt)
    del xt
    for t, ix, dim, pre in ((store._text_table, text_index, RETRIEVE_TEXT_DIM, "t"),
                            (store._image_table, image_index, DIM, "i")):
        t.index, t.dim = ix, dim
        t.chunk_ids = [f"{pre}{i % RETRIEVE_META_ROWS}" for i in range(ROWS_PER_GPU)]
        t.metas = ['{"page_no": 1}'] * ROWS_PER_GPU
        t.labels = {"u0": 0}
    meta = MetadataStore(os.path.join(d, "metadata.sqlite3"))
    c = meta._c()
    for pre, mod in (("t", "text"), ("i", "image")):
        c.executemany("INSERT INTO chunks VALUES (?,?,?,?,?,?,?,?,?,?)",
                      ((f"{pre}{i}", f"doc{i >> 8}", mod, f"passage {i} of the synthetic corpus" if mod == "text" else None,
                        i & 31, None, None, None, "{}", "") for i in range(RETRIEVE_META_ROWS)))
    c.commit()
    saved = (rmod._LANCEDB_STORE, rmod._METADATA_STORE)
    rmod._LANCEDB_STORE, rmod._METADATA_STORE = store, meta
    words = ["gpu", "vector", "search", "image", "caption", "lecture", "slide", "graph", "diagram", "model",
             "embedding", "retrieval", "page", "figure", "table", "network", "matrix", "energy", "cell", "river"]
    rng = np.random.default_rng(5)

    def queries(n, tag):
        return [f"{tag} {i} " + " ".join(rng.choice(words, 8)) for i in range(n)]

    kt, ki = settings.retrieval.index_topk_text, settings.retrieval.index_topk_image
    try:
        for q in queries(10, "warm"):  # model load, first launches, workspace growth
            rmod.retrieve_text("u0", q)
            rmod.retrieve_images("u0", q)
        qs = queries(reps, "q")
        t_text = _per_call_ms(lambda q: rmod.retrieve_text("u0", q), [(q,) for q in qs])
        t_img = _per_call_ms(lambda q: rmod.retrieve_images("u0", q), [(q,) for q in qs])
        hits_t = len(rmod.retrieve_text("u0", qs[0]))
        hits_i = len(rmod.retrieve_images("u0", qs[0]))
        # the parts alone (fresh strings: no cache)
        qs2 = queries(reps, "s")
        t_minilm = _per_call_ms(lambda q: emb_mod.embed_text_batch([q]), [(q,) for q in qs2])
        t_clipt = _per_call_ms(lambda q: emb_mod.embed_query_for_images(q), [(q,) for q in qs2])
        tv = emb_mod.embed_text_batch([qs2[0]])[0].tolist()
        iv = emb_mod.embed_query_for_images(qs2[0]).tolist()
        t_st = _per_call_ms(lambda: store.search_text("u0", tv, kt), [()] * reps)
        t_si = _per_call_ms(lambda: store.search_image("u0", iv, ki), [()] * reps)
        ids_t = [h["chunk_id"] for h in store.search_text("u0", tv, kt)]
        t_lk = _per_call_ms(lambda: meta.get_chunks(ids_t), [()] * reps)  # what retrieve_text runs
        t_lk1 = _per_call_ms(lambda: [meta.get_chunk(cid) for cid in ids_t], [()] * reps)  # the reference's per-hit form
    finally:
        rmod._LANCEDB_STORE, rmod._METADATA_STORE = saved
        for t in (store._text_table, store._image_table):
            t.index = None  # the bench owns the image index; the text index is closed here
        text_index.close()
        meta.close()
    return {
        "retrieve_text_ms": round(t_text, 4),
        "retrieve_images_ms": round(t_img, 4),
        "query_pair_ms": round(t_text + t_img, 4),
        "queries_per_s": round(1e3 / (t_text + t_img), 1),
        "hits": {"text": hits_t, "image": hits_i},
        "split_ms": {"minilm_b1_embed_text_batch": round(t_minilm, 4),
                     "clip_text_b1_embed_query_for_images": round(t_clipt, 4),
                     f"search_text_top{kt}_1Mx384": round(t_st, 4),
                     f"search_image_top{ki}_1Mx512": round(t_si, 4),
                     f"sqlite_get_chunks_x{len(ids_t)}": round(t_lk, 4),
                     f"sqlite_get_chunk_per_hit_x{len(ids_t)}": round(t_lk1, 4)},
        "workload": f"{reps} distinct synthetic queries; text table {ROWS_PER_GPU} x {RETRIEVE_TEXT_DIM}, image table "
                    f"{ROWS_PER_GPU} x {DIM} (one user), SQLite catalog of {RETRIEVE_META_ROWS} chunks per modality; "
                    f"top_k text {kt} / image {ki}",
        "note": "reference call pattern: retrieve_text then retrieve_images per query (retrieve() minus rerank/fusion); "
                "wall time per call on the host, device drained; split = each part alone",
    }


def _write_images(d: str, n: int, seed: int = 9):
    """n synthetic photos-like files (3/4 JPEG q90, 1/4 PNG), sizes cycling 640x480 / 800x600 /
    1024x768 / 480x640: a smooth field + coarse noise upsampled (decodes like natural images,
    not like white noise)."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image

    sizes = [(640, 480), (800, 600), (1024, 768), (480, 640)]

    def one(i):
        rng = np.random.default_rng((seed, i))
        w, h = sizes[i % len(sizes)]
        coarse = rng.integers(0, 256, (h // 16 + 1, w // 16 + 1, 3), dtype=np.uint8)
        img = Image.fromarray(coarse).resize((w, h), Image.BILINEAR)
        fine = rng.integers(-4, 5, (h, w, 3))
        a = np.clip(np.asarray(img, dtype=np.int16) + fine, 0, 255).astype(np.uint8)
        p = os.path.join(d, f"img{i:05d}.{'png' if i % 4 == 3 else 'jpg'}")
        Image.fromarray(a).save(p, quality=90) if p.endswith("jpg") else Image.fromarray(a).save(p)
        return p

    with ThreadPoolExecutor(max_workers=min(16, _usable_cores())) as ex:
        return list(ex.map(one, range(n)))


def ingest_leg(n_images: int = 2048):
    """``embed_images_batch`` over a folder of image files (app/ml/embeddings.py:73-91, the
    ingest path behind index_image_nodes): baseline JPEGs decoded on the GPU (K13, byte-identical
    to Pillow), the PNGs inflated on the host thread pool and reconstructed on the GPU (K14), K0
    resize + crop on the GPU,
    ViT-B/32, L2 normalise; encoder batches of 256, one K13 launch per batch, the next batch
    prepared on the host while the GPU works on the current one. Reported: img/s of the whole call
    and each stage alone over the same files (and Pillow decoding every file, the host decode K13
    replaces)."""
    import shutil
    import tempfile

    import numpy as np

    import gc

    from app.encoders.preprocess import (decode_batch, decode_workers, prepare_batch, resize_images,
                                         upload_decode)
    from app.ml import embeddings as emb_mod

    d = tempfile.mkdtemp(prefix="mrag_bench_ingest_")
    try:
        paths = _write_images(d, n_images)
        nbytes = sum(os.path.getsize(p) for p in paths)
        emb_mod.embed_images_batch(paths[:256])  # warm: model + workspaces
        _sync()
        calls = []  # the first full call also grows the pinned staging buffers; then two more
        for _ in range(3):
            t0 = time.perf_counter()
            out = emb_mod.embed_images_batch(paths)
            _sync()
            calls.append(time.perf_counter() - t0)
        t_all = sorted(calls)[1]
        workers = decode_workers()  # the pool embed_images_batch prepares on (app/encoders/preprocess.py)
        group = emb_mod._DECODE_GROUP_BATCHES * 256
        # the stages alone, over the same files: host prepare (reads, probes, the PNGs' inflate),
        # K13 / K14 decode of each group (+ the copy of any host-decoded image), K0 per batch, ViT
        t0 = time.perf_counter()
        prepared = [prepare_batch(paths[i:i + group]) for i in range(0, len(paths), group)]
        t_prep = time.perf_counter() - t0
        def _kinds(g):  # 1 JPEG (K13), 2 PNG (K14) per file of a prepared group, either host half
            if hasattr(g, "kind"):
                return g.kind.tolist()
            return [0 if j is None else {"jpeg": 1, "png": 2}[j[0]] for j, _ in g]

        k13_files = sum(k.count(1) for k in map(_kinds, prepared))
        k14_files = sum(k.count(2) for k in map(_kinds, prepared))
        _sync()
        t0 = time.perf_counter()
        groups = [upload_decode(g) for g in prepared]
        _sync()
        t_k13 = time.perf_counter() - t0
        t0 = time.perf_counter()
        u8 = [resize_images(g, i, 256) for g in groups for i in range(0, len(g), 256)]
        _sync()
        t_rs = time.perf_counter() - t0
        del groups, prepared
        model = emb_mod._ensure_clip()
        _sync()
        t0 = time.perf_counter()
        for b in u8:
            model.get_image_features(images_u8=b)
        _sync()
        t_vit = time.perf_counter() - t0
        t0 = time.perf_counter()
        decode_batch(paths)  # every file with Pillow on the pool: the host decode K13 replaces
        t_pil = time.perf_counter() - t0
        ok = bool(np.allclose(np.linalg.norm(out, axis=1), 1.0, atol=1e-5))
        index_image = index_image_leg(paths, n_images / t_all)
    finally:
        shutil.rmtree(d, ignore_errors=True)
        # the drop-in's CLIP handles go, so later legs' handles are the process's only ones (a sole
        # image handle splits a large batch into two lanes, encoder.hip)
        emb_mod._CLIP_MODEL = None
        gc.collect()
    return index_image, {
        "images_per_s": round(n_images / t_all, 1),
        "ms_per_256": round(t_all / n_images * 256 * 1e3, 3),
        "calls_images_per_s": [round(n_images / t, 1) for t in calls],
        "stages_alone_images_per_s": {"host_prepare": round(n_images / t_prep, 1),
                                      "k13_k14_decode_device": round(n_images / t_k13, 1),
                                      "k0_resize_crop_device": round(n_images / t_rs, 1),
                                      "vit_b32_tower": round(n_images / t_vit, 1),
                                      "pillow_decode_every_file_host": round(n_images / t_pil, 1)},
        "files_decoded_by_k13": k13_files,
        "files_reconstructed_by_k14": k14_files,
        "decode_group_images": group,
        "decode_threads": workers,
        "unit_rows": ok,
        "workload": f"{n_images} synthetic files (3/4 JPEG q90, 1/4 PNG; 640x480 .. 1024x768; "
                    f"{nbytes / 1e6:.1f} MB on disk), embed_images_batch(paths) in batches of 256; "
                    f"images_per_s = median of three calls",
    }


class _BenchStore:
    """app.ml.index_build pointed at a fresh persistent LanceDBStore in a temp directory (the drop-in
    store: Parquet + fp32 segments on disk, rows on the GPU), restored on exit."""

    def __enter__(self):
        import tempfile
        from pathlib import Path

        from app.ml import index_build as ib
        from app.storage.lancedb_store import LanceDBStore

        self.ib, self.dir = ib, tempfile.mkdtemp(prefix="mrag_bench_index_")
        self.saved = (ib._LANCEDB_STORE, ib._VERSION_FILE, os.environ.get("MRAG_STORE_PERSIST"))
        os.environ["MRAG_STORE_PERSIST"] = "1"  # the retrieve leg turns persistence off for its tables
        self.store = LanceDBStore(self.dir)
        ib._LANCEDB_STORE, ib._VERSION_FILE = self.store, Path(self.dir) / "index_versions.json"
        return self

    def __exit__(self, *exc):
        import shutil

        ib = self.ib
        ib._LANCEDB_STORE, ib._VERSION_FILE, persist = self.saved
        if persist is None:
            os.environ.pop("MRAG_STORE_PERSIST", None)
        else:
            os.environ["MRAG_STORE_PERSIST"] = persist
        for t in (self.store._text_table, self.store._image_table):
            if t.index is not None:
                t.index.close()
                t.index = None
        shutil.rmtree(self.dir, ignore_errors=True)


def _split_store(store_table, rows, modality: str):
    """The store half of an index_*_nodes call alone, over the call's own rows: the array prepare
    (_prepare_rows_array: the reference's _normalize bytes + json meta), the Parquet / fp32 segment
    append, and the GPU add (each part on fresh chunk ids)."""
    import tempfile

    import numpy as np

    from app.storage.corpus_files import CorpusFiles
    from app.storage.lancedb_store import LanceDBStore
    from app.vector_store import FlatIndex

    t0 = time.perf_counter()
    payloads, vectors = LanceDBStore._prepare_rows_array(rows)
    t_prep = time.perf_counter() - t0
    d = tempfile.mkdtemp(prefix="mrag_bench_seg_")
    try:
        cf = CorpusFiles(d)
        t0 = time.perf_counter()
        cf.append(vectors, payloads)
        t_files = time.perf_counter() - t0
    finally:
        import shutil

        shutil.rmtree(d, ignore_errors=True)
    ix = FlatIndex(vectors.shape[1], device=store_table.device)
    ix.add(vectors[:64], np.zeros(64, np.int32))
    _sync()
    t0 = time.perf_counter()
    ix.add(vectors, np.zeros(len(vectors), np.int32))
    _sync()
    t_add = time.perf_counter() - t0
    ix.close()
    return {f"prepare_rows_array_{modality}": round(t_prep * 1e3, 3), "parquet_f32_segment_append": round(t_files * 1e3, 3),
            "gpu_add": round(t_add * 1e3, 3)}


def index_image_leg(paths, embed_rate: float):
    """``index_image_nodes`` (app/ml/index_build.py -> reference app/ml/index_build.py:106-155) over
    the ingest leg's files into a fresh persistent store: the existence checks, the embed, the
    rows, the store's normalisation + json meta, the fp32 segment + Parquet append, the GPU add
    and the version bump. Median of seven calls on fresh chunk ids, each paired with an
    embed_images_batch call of the same files (the ratio's denominator), and the store half's
    parts alone over the same rows."""
    from app.ml import embeddings as emb_mod
    from app.storage.lancedb_store import VectorRow

    n = len(paths)
    with _BenchStore() as bs:
        bs.ib.index_image_nodes("u0", [{"id": f"w{i}", "metadata": {"file_path": p}} for i, p in enumerate(paths[:256])])
        calls, embeds = [], []  # after a warm call (table creation, the first Parquet write, workspaces)
        for c in range(7):  # each call paired with an embed_images_batch call of the same files
            _sync()
            t0 = time.perf_counter()
            emb_mod.embed_images_batch(paths)
            _sync()
            embeds.append(time.perf_counter() - t0)
            nodes = [{"id": f"img{c}_{i}", "metadata": {"file_path": p, "doc_id": f"doc{i >> 4}", "source": "bench"}}
                     for i, p in enumerate(paths)]
            _sync()
            t0 = time.perf_counter()
            out = bs.ib.index_image_nodes("u0", nodes)
            _sync()
            calls.append(time.perf_counter() - t0)
            assert len(out) == n
        t_call, t_embed = sorted(calls)[3], sorted(embeds)[3]
        import numpy as np

        emb = np.random.default_rng(1).standard_normal((n, 512)).astype(np.float32)
        rows = [VectorRow(chunk_id=f"s{i}", user_id="u0", document_id=f"doc{i >> 4}", modality="image",
                          embedding=emb[i], meta={"file_path": p, "doc_id": f"doc{i >> 4}", "user_id": "u0",
                                                  "modality": "image", "source": "bench"})
                for i, p in enumerate(paths)]
        split = _split_store(bs.store._image_table, rows, "image")
        rows_total = len(bs.store._image_table.index)
    store_ms = sum(split.values())
    return {
        "images_per_s": round(n / t_call, 1),
        "calls_images_per_s": [round(n / t, 1) for t in calls],
        "embed_images_batch_images_per_s": round(n / t_embed, 1),
        "ratio_to_embed_images_batch": round(t_embed / t_call, 3),
        "ratio_to_ingest_leg": round(n / t_call / embed_rate, 3),
        "split_ms": dict(split, embed_images_batch=round(t_embed * 1e3, 3)),
        "store_half_frac_of_call": round(store_ms / (t_call * 1e3), 3),
        "rows_in_table": rows_total,
        "workload": f"index_image_nodes('u0', {n} nodes) over the ingest leg's files, fresh persistent store, "
                    "fresh chunk ids per call, after one warm call of 256; median of seven calls, each after an "
                    "embed_images_batch call of the same files (the ratio's denominator, median of those five); "
                    "split = each part alone",
    }


def _synthetic_documents(n: int, seed: int = 11):
    import numpy as np

    words = ["gpu", "vector", "search", "image", "caption", "lecture", "slide", "graph", "diagram", "model",
             "embedding", "retrieval", "page", "figure", "table", "network", "matrix", "energy", "cell", "river",
             "the", "of", "and", "a", "to", "in", "is", "for", "on", "with"]
    rng = np.random.default_rng(seed)
    docs = []
    for i in range(n):
        sents = []
        for _ in range(int(rng.integers(6, 40))):
            w = rng.choice(words, int(rng.integers(6, 18)))
            sents.append(" ".join(w).capitalize() + ".")
        docs.append({"id": f"doc{i}", "text": " ".join(sents), "metadata": {"source": "pdf", "page_no": int(i % 50)}})
    return docs


def index_text_leg(n_docs: int = 1000):
    """``index_text_nodes`` (reference app/ml/index_build.py:46-103) over n_docs synthetic documents
    (6-40 sentences each) into a fresh persistent store: SentenceSplitter(512/64) with the
    metadata prefix, embed_text_batch (MiniLM-L6 on the GPU), VectorRows, upsert_text_vectors, the
    version bump. Median of three calls on fresh document ids, and each part alone."""
    from app.ml import index_build as ib
    from app.ml.splitter import Document
    from app.storage.lancedb_store import VectorRow

    with _BenchStore() as bs:
        ib.index_text_nodes("u0", _synthetic_documents(64, seed=99))  # warm: model, workspaces
        calls, chunks = [], 0
        for c in range(3):
            docs = _synthetic_documents(n_docs)
            for d in docs:
                d["id"] = f"c{c}_{d['id']}"
            _sync()
            t0 = time.perf_counter()
            out = ib.index_text_nodes("u0", docs)
            _sync()
            calls.append(time.perf_counter() - t0)
            chunks = len(out)
        t_call = sorted(calls)[1]
        docs = _synthetic_documents(n_docs)
        documents = [Document(text=d["text"], metadata=dict(d["metadata"]), doc_id=d["id"]) for d in docs]
        t0 = time.perf_counter()
        nodes = ib._SPLITTER.get_nodes_from_documents(documents)
        texts = [nd.get_content(metadata_mode="all") for nd in nodes]
        t_split = time.perf_counter() - t0
        _sync()
        t0 = time.perf_counter()
        emb = ib.embed_text_batch(texts)
        _sync()
        t_embed = time.perf_counter() - t0
        rows = [VectorRow(chunk_id=f"s{i}", user_id="u0", document_id=f"doc{i}", modality="text", embedding=emb[i],
                          meta={"doc_id": f"doc{i}", "user_id": "u0", "modality": "text", "source": "pdf"})
                for i in range(len(texts))]
        split = _split_store(bs.store._text_table, rows, "text")
    return {
        "documents_per_s": round(n_docs / t_call, 1),
        "chunks_per_s": round(chunks / t_call, 1),
        "chunks_per_call": chunks,
        "calls_documents_per_s": [round(n_docs / t, 1) for t in calls],
        "split_ms": dict(split, sentence_splitter=round(t_split * 1e3, 3), embed_text_batch=round(t_embed * 1e3, 3)),
        "store_half_frac_of_call": round(sum(split.values()) / (t_call * 1e3), 3),
        "workload": f"index_text_nodes('u0', {n_docs} synthetic documents of 6-40 sentences), fresh persistent store, "
                    "fresh document ids per call; median of three calls; split = each part alone",
    }


FUSION_ROWS_PER_GPU = 1 << 19  # config 5: 4M text + 4M image rows over 8 GPUs
FUSION_T = 16                   # synthetic query length (tokens, incl. specials)
_ORACLE_MODELS = {}


def _oracle_model(name):
    if name not in _ORACLE_MODELS:
        import oracle.models as om

        _ORACLE_MODELS[name] = getattr(om, name)(0)
    return _ORACLE_MODELS[name]


def _fusion_queries(dev, nq):
    """The leg's synthetic query batch: MiniLM ids ([CLS] ... [SEP]) and CLIP ids (BOS ... EOS)."""
    import torch

    gq = torch.Generator(device=dev).manual_seed(7)  # same batch on every rank
    ids_m = torch.randint(1000, 30000, (nq, FUSION_T), generator=gq, device=dev, dtype=torch.int32)
    ids_m[:, 0], ids_m[:, -1] = 101, 102
    ids_c = torch.randint(1, 49405, (nq, FUSION_T), generator=gq, device=dev, dtype=torch.int32)
    ids_c[:, 0], ids_c[:, -1] = 49406, 49407
    return ids_m, torch.ones_like(ids_m), ids_c


def fusion_flops_per_query(world: int) -> dict:
    """Algorithmic FLOP of one config-5 query: both query towers at T = FUSION_T (linear
    layers + attention + CLIP projection) and the two scans over the whole corpus."""
    from app.encoders import CLIP_TEXT_B32, MINILM_L6, text_flops_per_sequence

    enc = text_flops_per_sequence(MINILM_L6, FUSION_T) + text_flops_per_sequence(CLIP_TEXT_B32, FUSION_T)
    scan = 2.0 * world * FUSION_ROWS_PER_GPU * (MINILM_L6.hidden + CLIP_TEXT_B32.proj_dim)
    return {"encoders": enc, "scans": scan, "total": enc + scan}


def fusion_cpu_baseline(seconds_budget: float = 20.0):
    """CPU restatement of the config-5 query path (retrieve minus rerank) on the host cores, on
    a bounded sample: oracle MiniLM + CLIP-text towers (transformers, torch-CPU fp32) on the
    leg's synthetic ids, f32 torch-CPU mm + topk over 2^19 x 384 + 2^19 x 512 corpora (one
    GPU's shard), the reference's fusion (oracle.fusion = app/ml/retrieve.py:158-195) per
    query. Median of 5 timed batches."""
    import numpy as np
    import torch

    _use_all_cores()

    from oracle.fusion import fuse_results
    from oracle.models import clip_text_embeds, minilm_embeds

    bert, clip = _oracle_model("bert_model"), _oracle_model("clip_model")
    rng = np.random.default_rng(11)
    xt = torch.from_numpy(rng.standard_normal((FUSION_ROWS_PER_GPU, 384), dtype=np.float32))
    xi = torch.from_numpy(rng.standard_normal((FUSION_ROWS_PER_GPU, 512), dtype=np.float32))
    xt /= xt.norm(dim=1, keepdim=True)
    xi /= xi.norm(dim=1, keepdim=True)
    ids_m, mask, ids_c = (t.cpu().numpy() for t in _fusion_queries(torch.device("cpu"), 256))
    from app.settings import settings

    kt, ki, fn = settings.retrieval.index_topk_text, settings.retrieval.index_topk_image, settings.retrieval.final_n

    def run(n):
        tv = torch.from_numpy(minilm_embeds(bert, ids_m[:n], mask[:n]))
        iv = torch.from_numpy(clip_text_embeds(clip, ids_c[:n], np.ones_like(ids_c[:n])))
        st, rt = torch.topk(tv @ xt.T, kt, dim=1)
        si, ri = torch.topk(iv @ xi.T, ki, dim=1)
        for q in range(n):
            th = [{"chunk_id": int(r), "score": float(s)} for s, r in zip(st[q].tolist(), rt[q].tolist())]
            ih = [{"chunk_id": int(r), "score": float(s)} for s, r in zip(si[q].tolist(), ri[q].tolist())]
            fuse_results(th, ih, fn)

    t0 = time.perf_counter()
    run(8)
    per = (time.perf_counter() - t0) / 8
    nb = int(min(256, max(8, seconds_budget / 6 / max(per, 1e-5))))
    rate, ts = _median_rate(lambda: run(nb), nb)
    return {"value": round(rate, 2), "unit": "queries/s (one GPU's shard: 2^19 x 384 text + 2^19 x 512 image rows)",
            "cores": int(torch.get_num_threads()), "kind": "port", "host": _host_info(),
            "sample": f"{nb} synthetic {FUSION_T}-token queries: transformers MiniLM + CLIP-text fp32, torch mm + topk "
                      f"(k={kt}/{ki}) over the two corpora, oracle.fusion per query; median of 5 "
                      f"({ts[len(ts) // 2]:.2f} s per batch)"}


def fusion_leg(world: int, rank: int, local: int, steps: int, warmup: int):
    """BASELINE config 5: mixed text+image retrieval of a 1000-query batch, end to end on
    the GPUs: both query towers (MiniLM-L6 -> 384-d, CLIP text -> 512-d) on synthetic token
    ids, each rank encoding its slice of the batch (all-gathered over RCCL at N > 1), then
    the text (k = 50) and image (k = 12) searches over row-sharded corpora of 2^19 x 384 +
    2^19 x 512 rows per GPU (4M + 4M at 8 GPUs) with the per-shard all-gather + merge, the
    reference's z-score fusion (rerank off, final_n = 4) on the GPU (K12, bit-identical to
    app.retrieval.fuse_scores) on rank 0, and the fused picks copied to the host.
    value = queries/s over the whole corpus."""
    import torch
    import torch.distributed as dist

    from app.encoders import CLIP_TEXT_B32, MINILM_L6, GpuEncoder
    from app.retrieval import fuse_scores_gpu
    from app.settings import settings
    from app.vector_store import FlatIndex
    from app.vector_store.sharded import ShardedFlatIndex

    dev = torch.device("cuda", local)
    kt, ki = settings.retrieval.index_topk_text, settings.retrieval.index_topk_image
    final_n = settings.retrieval.final_n
    shards = []
    for dim, seed in ((MINILM_L6.hidden, 2000), (CLIP_TEXT_B32.proj_dim, 3000)):
        g = torch.Generator(device=dev).manual_seed(seed + rank)
        x = torch.randn((FUSION_ROWS_PER_GPU, dim), generator=g, device=dev)
        ix = FlatIndex(dim, device=local)
        ix.add(x)
        del x
        shards.append(ShardedFlatIndex(ix, row_offset=rank * FUSION_ROWS_PER_GPU))
    torch.cuda.empty_cache()
    text_sh, img_sh = shards
    ids_m, mask, ids_c = _fusion_queries(dev, NQ)
    per = (NQ + world - 1) // world
    lo, hi = rank * per, min(NQ, (rank + 1) * per)
    def gather(v):
        if world == 1:
            return v
        buf = torch.zeros((per, v.shape[1]), dtype=v.dtype, device=dev)
        buf[: v.shape[0]] = v
        if dist.get_backend() == "nccl":
            out = torch.empty((world * per, v.shape[1]), dtype=v.dtype, device=dev)
            dist.all_gather_into_tensor(out, buf)
        else:  # gloo rehearsal
            parts = [torch.empty_like(buf) for _ in range(world)]
            dist.all_gather(parts, buf)
            out = torch.cat(parts)
        return out[:NQ]

    # The leg runs on its own streams: device-pointer encoder calls are then stream-ordered (no
    # host sync per call; on the default stream the library synchronises every call). The text
    # branch (MiniLM -> text search) and the image branch (CLIP text -> image search) are
    # independent until the fusion; on one GPU the image branch runs in a second host thread on
    # a second stream (a search returns to the host once its certificate is read, which would
    # otherwise serialise the branches), and `slots` steps are in flight at once, each slot with
    # its own encoder handles (workspaces) and streams (the indexes give every search its own
    # workspace), so kernels that leave CUs idle (attention, LayerNorm, K8, partial GEMM rounds)
    # overlap with other branches' and steps' work, as a serving process with concurrent query
    # batches runs them. At N > 1 everything stays in one thread: the collectives share one
    # communicator and must be issued in the same order on every rank. MRAG_FUSION_STREAMS=1
    # serialises the branches, MRAG_FUSION_INFLIGHT sets the steps in flight (A/B timing; four
    # measured +4.1 / +1.3 / +2.8 % over two in three interleaved pairs on one box in round 4,
    # profiles/r4s24_fusion_inflight_ab.txt, and -3.9 / +2.0 / +0.7 % in round 5,
    # profiles/r5_fusion_inflight_ab.txt: no difference beyond the noise; four kept).
    two = world == 1 and os.environ.get("MRAG_FUSION_STREAMS", "2") != "1"
    slots = max(1, int(os.environ.get("MRAG_FUSION_INFLIGHT", "4"))) if two else 1
    from concurrent.futures import ThreadPoolExecutor

    class Slot:
        def __init__(self):
            self.minilm = GpuEncoder(MINILM_L6, device=local)
            self.clipt = GpuEncoder(CLIP_TEXT_B32, device=local)
            self.leg = torch.cuda.Stream(device=dev)
            self.img = torch.cuda.Stream(device=dev) if two else self.leg
            self.pool = ThreadPoolExecutor(max_workers=1) if two else None

        def image_branch(self):
            with torch.cuda.stream(self.img):
                iv = gather(self.clipt.embed_tokens(ids_c[lo:hi]))
                return img_sh.search(iv, ki)

        def step(self):
            with torch.cuda.stream(self.leg):
                if self.pool is not None:
                    self.img.wait_stream(self.leg)  # the previous step's fusion read its outputs
                    fut = self.pool.submit(self.image_branch)
                else:
                    si, ri = self.image_branch()
                tv = gather(self.minilm.embed_tokens(ids_m[lo:hi], mask[lo:hi]))
                st, rt = text_sh.search(tv, kt)
                if self.pool is not None:
                    si, ri = fut.result()
                    self.leg.wait_stream(self.img)
                if rank == 0:
                    pick, _ = fuse_scores_gpu(st, si, final_n)
                    return pick.cpu()
                return None

    slot_list = [Slot() for _ in range(slots)]
    runner = ThreadPoolExecutor(max_workers=slots) if slots > 1 else None
    last = [None]

    def run(nsteps):
        if runner is None:
            for _ in range(nsteps):
                last[0] = slot_list[0].step()
            return

        def share(j):
            out = None
            for _ in range(nsteps // slots + (1 if j < nsteps % slots else 0)):
                out = slot_list[j].step()
            return out

        outs = list(runner.map(share, range(slots)))
        last[0] = next((o for o in outs if o is not None), last[0])

    torch.cuda.synchronize()
    run(max(warmup, slots))
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    _barrier(world)
    dt = _max_over_ranks(time.perf_counter() - t0, world)
    pick = last[0]
    one_dt = None
    if runner is not None:  # the one-step-at-a-time rate (branches still on two streams)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            slot_list[0].step()
        torch.cuda.synchronize()
        one_dt = time.perf_counter() - t0
    for sl in slot_list:
        if sl.pool is not None:
            sl.pool.shutdown()
    if runner is not None:
        runner.shutdown()
    if rank != 0:
        return None
    fl = fusion_flops_per_query(world)
    achieved = fl["total"] * NQ * steps / dt / 1e12
    return {
        "metric": "mixed text+image retrieve queries/s (BASELINE config 5)",
        "value": round(NQ * steps / dt, 1),
        "unit": "queries/s (each query: MiniLM + CLIP-text encode, text top-50 + image top-12 over the whole "
                "sharded corpus, z-score fusion to 4, picks on the host)",
        "steps": steps,
        "ms_per_step": round(dt / steps * 1e3, 3),
        "workload": f"{NQ} synthetic {FUSION_T}-token queries; corpora {FUSION_ROWS_PER_GPU} x 384 text + "
                    f"{FUSION_ROWS_PER_GPU} x 512 image rows per GPU ({world * FUSION_ROWS_PER_GPU} + "
                    f"{world * FUSION_ROWS_PER_GPU} total), synthetic weights, rerank off",
        "top_k": {"text": kt, "image": ki, "final_n": final_n},
        "steps_in_flight": slots,
        "one_step_in_flight": None if one_dt is None else {"queries_per_s": round(NQ * steps / one_dt, 1),
                                                          "ms_per_step": round(one_dt / steps * 1e3, 3)},
        "fused_hits_last_step": int((pick >= 0).sum()),
        # queries whose fp16 top-k the certificate could not prove in the last search of each index
        # (they take the exact collect pass: correct, one more scan of their query group)
        "uncertified_last_search": {"text": text_sh.local.last_stats()[0], "image": img_sh.local.last_stats()[0]},
        "roofline": {"bound": "mfma", "scope": "whole step (towers + both scans; fusion and copies add no FLOP)",
                     "achieved": round(achieved, 2), "peak": MFMA_FP16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / MFMA_FP16_PEAK_TFLOPS, 4),
                     "algorithmic_flops_per_query": fl},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-clip", action="store_true")
    ap.add_argument("--no-fusion", action="store_true")
    ap.add_argument("--no-call-pattern", action="store_true")
    ap.add_argument("--no-retrieve-pattern", action="store_true",
                    help="skip the per-query retrieve_text / retrieve_images leg")
    ap.add_argument("--no-ingest", action="store_true", help="skip the embed_images_batch-from-files leg")
    ap.add_argument("--knn-streams", type=int, default=2,
                    help="kNN searches in flight (host threads / streams); 1 = one at a time")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world, rank, local = _dist_setup()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device("cuda", local)
    clip_streams = _early_streams(dev, 3) if rank == 0 and not args.no_clip else None

    from app.vector_store import FlatIndex

    # shard r of the 8M x 512 corpus (config 4): seed (0, r), generated on device
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn((ROWS_PER_GPU, DIM), generator=g, device=dev)
    x = x / x.norm(dim=1, keepdim=True)
    index = FlatIndex(DIM, device=local)
    index.add(x)
    del x
    torch.cuda.empty_cache()
    gq = torch.Generator(device=dev).manual_seed(1)
    q = torch.randn((NQ, DIM), generator=gq, device=dev)  # same queries on every rank
    row_offset = rank * ROWS_PER_GPU

    from app.vector_store.sharded import ShardedFlatIndex

    sharded = ShardedFlatIndex(index, row_offset=row_offset)

    # Searches in flight: KNN_STREAMS host threads, each searching on its own stream (the
    # library gives each search its own workspace), so one search's K8 / certificate read-back
    # / host round trip overlaps the next one's scan, as a serving process with concurrent
    # batches runs them. The collective steps (all-gather + K11 merge, N > 1) stay on this
    # thread, in step order on every rank. --knn-streams 1 = one search at a time.
    nstreams = max(1, args.knn_streams)
    streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
    pool = None
    if nstreams > 1:
        from concurrent.futures import ThreadPoolExecutor

        pool = ThreadPoolExecutor(max_workers=nstreams)

    def local_search(i):
        with torch.cuda.stream(streams[i % nstreams]):
            return sharded.search_local(q, TOPK)

    def run(nsteps):
        if pool is None:
            for i in range(nsteps):
                sharded.combine(local_search(i), TOPK)
            return
        futs = [pool.submit(local_search, i) for i in range(nsteps)]
        for f in futs:
            sharded.combine(f.result(), TOPK)

    def timed(nsteps):
        torch.cuda.synchronize()
        _barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(nsteps)
        torch.cuda.synchronize()
        _barrier(world)
        return time.perf_counter() - t0

    run(args.warmup)
    # K7's launch time (roofline) from HIP events around the scan, taken while ONE search is in
    # flight, so that a launch's span holds no other search's kernels; that run's rate is
    # reported beside value as "one_search_in_flight"
    nstreams_saved, pool_saved = nstreams, pool
    nstreams, pool = 1, None
    index.profile(1)
    serial_dt = _max_over_ranks(timed(args.steps), world)
    scan_ms, scan_n = index.profile(0)
    unc, _ = index.last_stats()
    nstreams, pool = nstreams_saved, pool_saved
    dt = _max_over_ranks(timed(args.steps), world) if nstreams > 1 else serial_dt
    if pool is not None:
        pool.shutdown()

    # N > 1: what the communicator is, which devices the ranks drove, and the collective part of a
    # step (all-gather of the per-shard (f64 score, row) lists + the K11 merge) timed alone
    comm = None
    if world > 1:
        backend = dist.get_backend()
        ranks = [None] * world
        props = torch.cuda.get_device_properties(local)
        dist.all_gather_object(ranks, {"rank": rank, "local_device": local, "name": props.name,
                                       "pci_bus": getattr(props, "pci_bus_id", None),
                                       "host": os.uname().nodename})
        loc = sharded.search_local(q, TOPK)
        for _ in range(3):
            sharded.combine(loc, TOPK)
        reps = max(10, args.steps)
        torch.cuda.synchronize()
        _barrier(world)
        t0 = time.perf_counter()
        for _ in range(reps):
            sharded.combine(loc, TOPK)
        torch.cuda.synchronize()
        comm_dt = _max_over_ranks(time.perf_counter() - t0, world)
        comm = {"backend": backend, "collective": "RCCL" if backend == "nccl" else backend,
                "world": dist.get_world_size(), "devices": ranks,
                "distinct_devices": len({(r["host"], r["pci_bus"], r["local_device"]) for r in ranks}),
                "allgather_merge_ms_per_step": round(comm_dt / reps * 1e3, 4),
                "allgather_bytes_per_rank": NQ * TOPK * 16}

    ms_per_step = dt / args.steps * 1e3
    value = world * NQ * args.steps / dt
    avg_scan_s = (scan_ms / max(scan_n, 1)) / 1e3
    flops_per_launch = 2.0 * NQ * ROWS_PER_GPU * DIM
    achieved_tflops = flops_per_launch / avg_scan_s / 1e12 if avg_scan_s > 0 else 0.0

    # the reference's call pattern hands host buffers over: same search with numpy queries in
    # and numpy results out (PCIe both ways + the final sync), reported beside value, never as it
    host_path = None
    if world == 1:
        qh = q.cpu().numpy()
        index.search(qh, TOPK)
        t0 = time.perf_counter()
        n_host = max(3, args.steps // 2)
        for _ in range(n_host):
            index.search(qh, TOPK)
        dt_host = time.perf_counter() - t0
        host_path = {"queries_per_s": round(NQ * n_host / dt_host, 1), "ms_per_search": round(dt_host / n_host * 1e3, 4),
                     "note": "numpy queries in / numpy results out (PCIe-inclusive, host buffers); not `value`"}

    call_pattern = None
    if world == 1 and not args.no_call_pattern:
        call_pattern = call_pattern_leg(index, q, reps=max(50, 10 * args.steps))
    if world == 1 and not args.no_retrieve_pattern:
        call_pattern = call_pattern or {}
        call_pattern["retrieve"] = retrieve_pattern_leg(index, reps=max(50, 5 * args.steps))

    fusion = None
    if not args.no_fusion:  # config 5 (all ranks take part: sharded corpora + all-gathers)
        del sharded
        index.close()
        torch.cuda.empty_cache()
        fusion = fusion_leg(world, rank, local, steps=max(20, args.steps), warmup=4)
        if fusion is not None and not args.no_cpu_baseline and world == 1:
            fusion["cpu_baseline"] = fusion_cpu_baseline()

    if rank == 0:
        out = {
            "metric": "CLIP img-embeds/sec/GPU; kNN queries/sec on 1M×512 at top-k=10, 1/2/4/8 GPUs",
            "value": round(value, 3),
            "unit": "queries/s (1000-query batches, each query scanned against a 1M x 512 shard per GPU, top-10; aggregate over GPUs)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp16 MFMA scan + f64 exact rescore",
            "data": "synthetic (N(0,1) rows L2-normalised, seeded; queries N(0,1))",
            "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "config": {
                "workload": "BASELINE config 3 (N=1) / config 4 (N>1): brute-force cosine top-10, 1M x 512 rows per GPU, 1000-query batch",
                "rows_per_gpu": ROWS_PER_GPU,
                "total_rows": ROWS_PER_GPU * world,
                "dim": DIM,
                "queries_per_step": NQ,
                "top_k": TOPK,
                "parallelism": f"row-sharded x{world}" + (f" + {comm['collective']} all-gather of per-shard top-k"
                                                          if comm else ""),
                "query_vector_pairs_per_s": round(value * ROWS_PER_GPU, 1),
                "uncertified_queries_last_step": unc,
                "searches_in_flight": nstreams,
                "one_search_in_flight": {"queries_per_s": round(world * NQ * args.steps / serial_dt, 1),
                                         "ms_per_step": round(serial_dt / args.steps * 1e3, 4)},
            },
            "roofline": {
                "kernel": "knn_scan3_kernel<512, 0, 4> (K7 v3 main scan, MFMA 16x16x32; the 1/16 sample pre-pass is a separate launch, inside ms_per_step)",
                "bound": "mfma",
                "achieved": round(achieved_tflops, 2),
                "peak": MFMA_FP16_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved_tflops / MFMA_FP16_PEAK_TFLOPS, 4),
                "traffic": _traffic_from_profiles(),
                "traffic_source": "profiles/knn_scan_pmc.json: rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs) "
                                  "of this kernel on the committed tree, 2 x FETCH_SIZE (gfx950) + WRITE_SIZE per launch; "
                                  "counters cannot be read inside this process",
                "avg_launch_ms": round(avg_scan_s * 1e3, 4),
                "algorithmic_flops_per_launch": flops_per_launch,
                "algorithmic_bytes_per_launch": ROWS_PER_GPU * DIM * 2 + NQ * DIM * 2,
            },
        }
        if world == 1 and not args.no_ingest:
            index_image, ingest = ingest_leg()
            out["call_pattern"] = dict(call_pattern or {}, ingest_embed_images_batch=ingest,
                                       index_image_nodes=index_image, index_text_nodes=index_text_leg())
            call_pattern = out["call_pattern"]
        if not args.no_clip:
            clip = clip_leg(steps=max(30, args.steps), warmup=3, streams=clip_streams)  # single-GPU leg, rank 0; 30+ batches: three in flight reach steady state
            if clip is not None:
                if not args.no_cpu_baseline:
                    clip["cpu_baseline"] = clip_cpu_baseline()
                out["clip"] = clip
        if comm is not None:
            out["comm"] = comm
        if host_path is not None:
            out["host_buffer_path"] = host_path
        if call_pattern is not None:
            out["call_pattern"] = call_pattern
        if fusion is not None:
            out["fusion"] = fusion
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()  # ranks > 0 wait while rank 0 runs the single-GPU CLIP leg
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
