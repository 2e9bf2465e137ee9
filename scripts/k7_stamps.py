#!/usr/bin/env python3
"""K7 segment stamps (diagnostic build): where a tile's cycles go.

    make -C multimodal-rag-for-image-text-search_amd stamp
    MRAG_LIB=multimodal-rag-for-image-text-search_amd/lib/libmrag_k7stamp.so python scripts/k7_stamps.py

The stamp build sums, per wave, the shader-clock spans (s_memtime) of each tile's segments:
[0] tile top -> end of the k-steps that issue the next tile's LDS-DMA, [1] -> last MFMA issued,
[2] the tail (masking, vmcnt(0), theta), [3] the end-of-tile barrier, [5] group-test fires,
[6] cycles inside the fired insert bodies. Printed per segment: mean
cycles per tile over the waves and the 10th / 90th percentile, next to the MFMA floor (16
cycles per 16x16x32 MFMA, MI355X_MICROARCH.md). Runs the bench's config 3 (1M x 512, Q = 1000,
k = 10; the 256-query instance) and Q = 1 (K7s, 64-query instance). The stamps cost cycles
themselves (the guide quotes ~+11 % wave cycles), so compare segments, not totals, with the
production build."""
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

NST, MAXW = 8, 1 << 16
lib = _native.load()
fn = lib.mrag_debug_k7_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
fn.restype = ctypes.c_int


def read():
    buf = np.zeros(MAXW * NST, np.uint64)
    _native.check(fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), buf.size), "stamps")
    return buf.reshape(MAXW, NST)


def summarize(name, st, mfma_per_tile):
    t = st[:, 4].astype(np.float64)
    live = t > 0
    seg = st[live, :4].astype(np.float64) / t[live, None]
    out = {"case": name, "waves": int(live.sum()), "tiles_per_wave": float(t[live].mean()),
           "mfma_floor_cycles_per_tile": 16 * mfma_per_tile}
    names = ["dma_ksteps", "rest_ksteps", "tail_vmcnt", "barrier"]
    for i, n in enumerate(names):
        col = seg[:, i]
        out[n] = {"mean": round(col.mean(), 1), "p10": round(np.percentile(col, 10), 1),
                  "p90": round(np.percentile(col, 90), 1)}
    out["total_mean"] = round(seg.sum(1).mean(), 1)
    # group-test fires (an insert body ran) per tile and their cycles, and the per-SIMD view
    # (wave w of every workgroup): who waits at the barrier, who fires
    out["fires_per_tile"] = round(float((st[live, 5] / t[live]).mean()), 3)
    out["fire_cycles_per_tile"] = round(float((st[live, 6] / t[live]).mean()), 1)
    w = np.nonzero(live)[0] % 4
    out["by_wave"] = {int(i): {"barrier": round(float(seg[w == i, 3].mean()), 1),
                               "total": round(float(seg[w == i].sum(1).mean()), 1),
                               "fires_per_tile": round(float((st[live, 5] / t[live])[w == i].mean()), 3)}
                      for i in range(4)}
    print(json.dumps(out), flush=True)


dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn((1 << 20, 512), generator=g, device=dev)
x = x / x.norm(dim=1, keepdim=True)
ix = FlatIndex(512)
ix.add(x)
del x
q = torch.randn((1000, 512), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
for _ in range(10):
    ix.search(q, 10)
torch.cuda.synchronize()
read()  # clear
ix.search(q, 10)
torch.cuda.synchronize()
summarize("Q1000_k10_QB4", read(), 256)
for _ in range(10):
    ix.search(q[:1].contiguous(), 10)
torch.cuda.synchronize()
read()
ix.search(q[:1].contiguous(), 10)
torch.cuda.synchronize()
summarize("Q1_k10_QB1", read(), 64)
