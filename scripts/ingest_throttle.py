#!/usr/bin/env python3
"""CPU-quota throttling of this process's cgroup during embed_images_batch (cpu.stat deltas:
nr_periods, nr_throttled, throttled_usec) over the bench's ingest files, three calls."""
import json, os, shutil, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import torch  # noqa: E402
import bench  # noqa: E402
from app.ml import embeddings as emb  # noqa: E402


def stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (l.split() for l in f)}
    except Exception:
        return {}


n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
d = tempfile.mkdtemp(prefix="mrag_thr_")
try:
    paths = bench._write_images(d, n)
    emb.embed_images_batch(paths[:256])
    emb.embed_images_batch(paths)
    torch.cuda.synchronize()
    try:
        quota = open("/sys/fs/cgroup/cpu.max").read().strip()
    except Exception:
        quota = None
    for rnd in range(3):
        s0, c0, t0 = stat(), os.times(), time.perf_counter()
        emb.embed_images_batch(paths)
        torch.cuda.synchronize()
        t, c1, s1 = time.perf_counter() - t0, os.times(), stat()
        print(json.dumps({"round": rnd, "images_per_s": round(n / t, 1), "wall_ms": round(t * 1e3, 1),
                          "cpu_s": round(c1.user - c0.user + c1.system - c0.system, 2), "cpu.max": quota,
                          **{k: s1.get(k, 0) - s0.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec")}}),
              flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
