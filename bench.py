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
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
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


def _host_cores():
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    try:
        from threadpoolctl import threadpool_info

        blas = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        blas = cores
    return int(min(cores, blas))


def cpu_baseline(seconds_budget: float = 15.0):
    """The oracle (exact f64 numpy flat cosine, oracle/knn.py) on the host cores, on a
    bounded sample of the same workload: the 1M x 512 corpus and as many of the 1000
    queries as fit ~budget seconds (two-point timing: fixed corpus pass + per query)."""
    import numpy as np

    from oracle.knn import flat_cosine_topk

    rng = np.random.default_rng(0)
    x = rng.standard_normal((ROWS_PER_GPU, DIM), dtype=np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    q = rng.standard_normal((NQ, DIM), dtype=np.float32)
    lab = np.zeros(ROWS_PER_GPU, dtype=np.int32)
    flat_cosine_topk(x, lab, q[:1], TOPK)  # warm (page-in, BLAS init)
    t0 = time.perf_counter()
    flat_cosine_topk(x, lab, q[:8], TOPK)
    t8 = time.perf_counter() - t0
    t0 = time.perf_counter()
    flat_cosine_topk(x, lab, q[:32], TOPK)
    t32 = time.perf_counter() - t0
    per_q = max((t32 - t8) / 24.0, 1e-4)
    nq = int(min(NQ, max(32, (seconds_budget - t8) / per_q)))
    t0 = time.perf_counter()
    flat_cosine_topk(x, lab, q[:nq], TOPK)
    dt = time.perf_counter() - t0
    return {
        "value": round(nq / dt, 3),
        "unit": "queries/s (1M x 512 shard, top-10)",
        "cores": _host_cores(),
        "kind": "port",
        "sample": f"oracle.knn.flat_cosine_topk (exact f64 numpy, chunked) on {nq} of the 1000 queries against "
                  f"the same 1M x 512 corpus shape, {dt:.1f} s",
    }


def clip_cpu_baseline(seconds_budget: float = 10.0):
    """oracle.models CLIP ViT-B/32 image tower (transformers, torch-CPU fp32) on the host
    cores, bounded sample of the config-2 workload: random 224x224 images in batches of 16
    (generated per batch), as many batches as fit ~budget seconds (at most 2048 images)."""
    import numpy as np
    import torch

    from oracle.models import clip_image_embeds, clip_model

    model = clip_model(0)
    rng = np.random.default_rng(2)

    def batch():
        return rng.integers(0, 256, (16, 224, 224, 3), dtype=np.uint8)

    clip_image_embeds(model, batch())
    t0 = time.perf_counter()
    clip_image_embeds(model, batch())
    t16 = time.perf_counter() - t0
    n_batches = int(min(128, max(1, seconds_budget / max(t16, 1e-3))))
    t0 = time.perf_counter()
    for _ in range(n_batches):
        clip_image_embeds(model, batch())
    dt = time.perf_counter() - t0
    n_images = 16 * n_batches
    return {"value": round(n_images / dt, 2), "unit": "images/s", "cores": int(torch.get_num_threads()),
            "kind": "port", "sample": f"transformers CLIPModel.get_image_features fp32 on {n_images} random "
                                       f"224x224 images, batches of 16, {dt:.1f} s"}


def _traffic_from_profiles():
    """HBM bytes per K7 launch from the committed rocprofv3 PMC pass (or None)."""
    path = os.path.join(ROOT, "profiles", "knn_scan_pmc.json")
    try:
        with open(path) as f:
            return float(json.load(f)["hbm_bytes_per_launch"])
    except Exception:
        return None


def clip_leg(steps: int, warmup: int):
    """CLIP ViT-B/32 image embeds/s on one GPU (config 2: batch 256, fp16)."""
    try:
        from app.encoders import bench_clip_images
    except Exception:
        return None
    return bench_clip_images(steps=steps, warmup=warmup)


FUSION_ROWS_PER_GPU = 1 << 19  # config 5: 4M text + 4M image rows over 8 GPUs
FUSION_T = 16                   # synthetic query length (tokens, incl. specials)


def fusion_leg(world: int, rank: int, local: int, steps: int, warmup: int):
    """BASELINE config 5: mixed text+image retrieval of a 1000-query batch, end to end on
    the GPUs: both query towers (MiniLM-L6 -> 384-d, CLIP text -> 512-d) on synthetic token
    ids, each rank encoding its slice of the batch (all-gathered over RCCL at N > 1), then
    the text (k = 50) and image (k = 12) searches over row-sharded corpora of 2^19 x 384 +
    2^19 x 512 rows per GPU (4M + 4M at 8 GPUs) with the per-shard all-gather + merge, and
    the reference's z-score fusion (rerank off, final_n = 4) on rank 0
    (app.retrieval.fuse_scores, vectorised). value = queries/s over the whole corpus."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from app.encoders import CLIP_TEXT_B32, MINILM_L6, GpuEncoder
    from app.retrieval import fuse_scores
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
    gq = torch.Generator(device=dev).manual_seed(7)  # same batch on every rank
    ids_m = torch.randint(1000, 30000, (NQ, FUSION_T), generator=gq, device=dev, dtype=torch.int32)
    ids_m[:, 0], ids_m[:, -1] = 101, 102  # [CLS] ... [SEP]
    mask = torch.ones_like(ids_m)
    ids_c = torch.randint(1, 49405, (NQ, FUSION_T), generator=gq, device=dev, dtype=torch.int32)
    ids_c[:, 0], ids_c[:, -1] = 49406, 49407  # <|startoftext|> ... <|endoftext|>
    per = (NQ + world - 1) // world
    lo, hi = rank * per, min(NQ, (rank + 1) * per)
    minilm = GpuEncoder(MINILM_L6, device=local)
    clipt = GpuEncoder(CLIP_TEXT_B32, device=local)

    def gather(v):
        if world == 1:
            return v
        buf = torch.zeros((per, v.shape[1]), dtype=v.dtype, device=dev)
        buf[: v.shape[0]] = v
        out = torch.empty((world * per, v.shape[1]), dtype=v.dtype, device=dev)
        dist.all_gather_into_tensor(out, buf)
        return out[:NQ]

    def step():
        tv = gather(minilm.embed_tokens(ids_m[lo:hi], mask[lo:hi]))
        iv = gather(clipt.embed_tokens(ids_c[lo:hi]))
        st, rt = text_sh.search(tv, kt)
        si, ri = img_sh.search(iv, ki)
        if rank == 0:
            pick, _ = fuse_scores(st.cpu().numpy(), si.cpu().numpy(), final_n)
            return pick
        return None

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        pick = step()
    torch.cuda.synchronize()
    _barrier(world)
    dt = _max_over_ranks(time.perf_counter() - t0, world)
    if rank != 0:
        return None
    return {
        "metric": "mixed text+image retrieve queries/s (BASELINE config 5)",
        "value": round(NQ * steps / dt, 1),
        "unit": "queries/s (each query: MiniLM + CLIP-text encode, text top-50 + image top-12 over the whole "
                "sharded corpus, z-score fusion to 4)",
        "steps": steps,
        "ms_per_step": round(dt / steps * 1e3, 3),
        "workload": f"{NQ} synthetic {FUSION_T}-token queries; corpora {FUSION_ROWS_PER_GPU} x 384 text + "
                    f"{FUSION_ROWS_PER_GPU} x 512 image rows per GPU ({world * FUSION_ROWS_PER_GPU} + "
                    f"{world * FUSION_ROWS_PER_GPU} total), synthetic weights, rerank off",
        "top_k": {"text": kt, "image": ki, "final_n": final_n},
        "fused_hits_last_step": int((pick >= 0).sum()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-clip", action="store_true")
    ap.add_argument("--no-fusion", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world, rank, local = _dist_setup()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device("cuda", local)

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

    def step():
        return sharded.search(q, TOPK)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    index.profile(1)
    _barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    dt = time.perf_counter() - t0
    scan_ms, scan_n = index.profile(0)
    unc, _ = index.last_stats()
    dt = _max_over_ranks(dt, world)

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

    fusion = None
    if not args.no_fusion:  # config 5 (all ranks take part: sharded corpora + all-gathers)
        del sharded
        index.close()
        torch.cuda.empty_cache()
        fusion = fusion_leg(world, rank, local, steps=max(5, args.steps // 2), warmup=2)

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
            "config": {
                "workload": "BASELINE config 3 (N=1) / config 4 (N>1): brute-force cosine top-10, 1M x 512 rows per GPU, 1000-query batch",
                "rows_per_gpu": ROWS_PER_GPU,
                "total_rows": ROWS_PER_GPU * world,
                "dim": DIM,
                "queries_per_step": NQ,
                "top_k": TOPK,
                "parallelism": f"row-sharded x{world}" + (" + RCCL all-gather of per-shard top-k" if world > 1 else ""),
                "query_vector_pairs_per_s": round(value * ROWS_PER_GPU, 1),
                "uncertified_queries_last_step": unc,
            },
            "roofline": {
                "kernel": "knn_scan3_kernel<512, 0, 0, 4> (K7 v3 main scan, MFMA 16x16x32; the 1/16 sample pre-pass is a separate launch, inside ms_per_step)",
                "bound": "mfma",
                "achieved": round(achieved_tflops, 2),
                "peak": MFMA_FP16_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved_tflops / MFMA_FP16_PEAK_TFLOPS, 4),
                "traffic": _traffic_from_profiles(),
                "avg_launch_ms": round(avg_scan_s * 1e3, 4),
                "algorithmic_flops_per_launch": flops_per_launch,
                "algorithmic_bytes_per_launch": ROWS_PER_GPU * DIM * 2 + NQ * DIM * 2,
            },
        }
        if not args.no_clip:
            clip = clip_leg(steps=max(5, args.steps // 2), warmup=2)  # single-GPU leg, rank 0
            if clip is not None:
                if not args.no_cpu_baseline:
                    clip["cpu_baseline"] = clip_cpu_baseline()
                out["clip"] = clip
        if host_path is not None:
            out["host_buffer_path"] = host_path
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
