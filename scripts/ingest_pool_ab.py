#!/usr/bin/env python3
"""embed_images_batch over the bench's ingest files with the host decode pool at 8 / 12 / 16 / 24
threads (the process's CPU quota is 16 on a one-GPU box), interleaved twice: img/s and CPU s."""
import json, os, shutil, sys, tempfile, time
from concurrent.futures import ThreadPoolExecutor
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import torch  # noqa: E402
import bench  # noqa: E402
from app.encoders import preprocess  # noqa: E402
from app.ml import embeddings as emb  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
d = tempfile.mkdtemp(prefix="mrag_pool_ab_")
try:
    paths = bench._write_images(d, n)
    emb.embed_images_batch(paths[:256])
    emb.embed_images_batch(paths)
    torch.cuda.synchronize()
    for rnd in range(2):
        for k in (8, 12, 16, 24):
            preprocess._POOL = ThreadPoolExecutor(max_workers=k, thread_name_prefix="mrag-decode")
            emb.embed_images_batch(paths[:256])
            c0, t0 = os.times(), time.perf_counter()
            emb.embed_images_batch(paths)
            torch.cuda.synchronize()
            t, c1 = time.perf_counter() - t0, os.times()
            print(json.dumps({"round": rnd, "pool": k, "images_per_s": round(n / t, 1),
                              "cpu_s": round(c1.user - c0.user + c1.system - c0.system, 2),
                              "decode_workers_default": preprocess.decode_workers()}), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
