#!/usr/bin/env python3
"""The device-decode stage alone (upload_decode of NativePrepared groups of 256 of the bench's
ingest files, as embed_images_batch's decode thread runs it): wall ms per group, over 3 x 8 groups;
run under rocprofv3 --kernel-trace --memory-copy-trace --stats to split it into kernels, copies
and host work."""
import json, os, shutil, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import torch  # noqa: E402
import bench  # noqa: E402
from app.encoders import preprocess as pp  # noqa: E402

n = 2048
d = tempfile.mkdtemp(prefix="mrag_split_")
try:
    paths = bench._write_images(d, n)
    groups = [pp.NativePrepared(paths[i:i + 256]) for i in range(0, n, 256)]
    for g in groups[:2]:
        pp.upload_decode(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        for g in groups:
            x = pp.upload_decode(g)
            del x
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(json.dumps({"lib": os.path.basename(os.environ.get("MRAG_LIB", "libmrag.so")), "groups": 24, "ms_per_group": round(t / 24 * 1e3, 3), "images_per_s": round(24 * 256 / t, 1)}))
finally:
    shutil.rmtree(d, ignore_errors=True)
