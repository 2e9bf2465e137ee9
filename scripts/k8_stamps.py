#!/usr/bin/env python3
"""K8 (merge / rescore / certify) phase times from the stamp build:

    make -C multimodal-rag-for-image-text-search_amd stamp
    MRAG_LIB=multimodal-rag-for-image-text-search_amd/lib/libmrag_k7stamp.so python scripts/k8_stamps.py

Wave 0 of each merge workgroup stamps s_memtime (shader clock cycles) at: [0] start, [1] its own key fold done, [2] wave 0's
fold of the other waves done, [3] after the barrier, [4] rescoring done, [5] candidate sort
done, [6] end. Printed: mean span per phase over the workgroups, Q = 1 and Q = 1000 on 1M x 512."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
assert "k7stamp" in os.environ.get("MRAG_LIB", ""), "set MRAG_LIB to the stamp build"

import torch  # noqa: E402

from app import _native  # noqa: E402
from app.vector_store import FlatIndex  # noqa: E402

NST, MAXB = 8, 4096
lib = _native.load()
fn = lib.mrag_debug_k8_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
fn.restype = ctypes.c_int
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(7)
x = torch.randn((1 << 20, 512), generator=g, device=dev)
ix = FlatIndex(512)
ix.add(x)
del x
for nq in (1, 1000):
    q = torch.randn((nq, 512), generator=g, device=dev)
    for _ in range(5):
        res = ix.search(q, 10)
    torch.cuda.synchronize()
    import hashlib
    check = hashlib.sha1(b"".join(t.cpu().numpy().tobytes() for t in res)).hexdigest()[:12]
    buf = np.zeros(MAXB * NST, np.uint64)
    assert fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), MAXB * NST) == 0
    st = buf.reshape(MAXB, NST)[:nq].astype(np.int64)
    span = np.diff(st[:, :7], axis=1)
    names = ["own_fold", "wave0_fold", "barrier", "rescore", "cand_sort", "out_cert"]
    print(json.dumps({"nq": nq, "mean_ticks": {n: round(float(v), 1) for n, v in zip(names, span.mean(0))},
                      "total_ticks": round(float((st[:, 6] - st[:, 0]).mean()), 1), "results_sha1": check,
                      "lib": os.path.basename(os.environ["MRAG_LIB"])}), flush=True)
