"""Diagnose kNN parity on the collect-pass-heavy case.

Same data as tests/test_knn_gpu.py::test_collect_pass_many_failing_queries (30k clustered
512-d rows, 640 queries, k = 50), searched under several batchings / depths that select
different kernels, each compared with the exact oracle. Prints one JSON line per case and, for
mismatching queries, which rows are missing / extra with their exact scores and scan
coordinates (tile, main-scan split, collect split).

Needs the diagnostic library (the mrag_debug_knn_last_collect export is not in the shipped one):
    make -C multimodal-rag-for-image-text-search_amd stamp
    MRAG_LIB=multimodal-rag-for-image-text-search_amd/lib/libmrag_k7stamp.so python scripts/knn_collect_diag.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT, os.path.join(ROOT, "tests")]

from _data import clustered_corpus  # noqa: E402
from oracle.knn import cosine_scores  # noqa: E402


def main():
    from app.vector_store import FlatIndex

    x = clustered_corpus(30000, 512, 11, n_clusters=8, spread=0.01, dup_frac=0.2)
    q = x[np.random.default_rng(5).integers(0, len(x), 640)] + 0.001
    cos = cosine_scores(x, q)
    order = np.lexsort((np.broadcast_to(np.arange(len(x)), cos.shape), -cos), axis=1)
    ix = FlatIndex(512)
    ix.add(x)

    import ctypes

    from app import _native

    lib = _native.load()
    dbg = lib.mrag_debug_knn_last_collect
    dbg.restype = ctypes.c_int

    def last_collect(nqc):
        info = np.zeros(8, np.int32)
        fl = np.full(nqc, -1, np.int32)
        cc = np.full(nqc, -1, np.int32)
        th = np.full(nqc, np.nan, np.float32)
        rc = dbg(ix._h, info.ctypes.data_as(ctypes.c_void_p), fl.ctypes.data_as(ctypes.c_void_p),
                 cc.ctypes.data_as(ctypes.c_void_p), th.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(nqc))
        assert rc == 0
        return info, fl, cc, th

    def run(name, k, chunk):
        outs_s, outs_r, uncs = [], [], []
        coll = {}
        for i in range(0, len(q), chunk):
            s, r, s64 = ix.search(q[i:i + chunk], k, with_f64=True)
            outs_s.append(s64)
            outs_r.append(r)
            uncs.append(ix.last_stats())
            info, fl, cc, th = last_collect(len(q[i:i + chunk]))
            uncs[-1] = uncs[-1] + (info.tolist(),)
            for slot in range(int(info[5])):
                qq = i + int(fl[slot])
                coll[qq] = (slot, int(cc[slot]), float(th[fl[slot]]))
        s64 = np.concatenate(outs_s)
        r = np.concatenate(outs_r)
        kk = min(k, 50)
        ref = order[:, :kk]
        bad = np.nonzero(np.any(r[:, :kk] != ref, axis=1))[0]
        rec = {"case": name, "k": k, "chunk": chunk, "unc_retries": uncs, "bad_queries": int(bad.size)}
        det = []
        for qi in bad[:6]:
            g = r[qi, :kk]
            o = ref[qi]
            ek = cos[qi, o[-1]]
            missing = [int(v) for v in o if v not in set(g.tolist())]
            extra = [int(v) for v in g if v not in set(o.tolist())]
            first = int(np.argmax(g != o))
            ekr = cos[qi, o[kk - 1]]
            cinfo = coll.get(int(qi))
            need = int((cos[qi] >= (cinfo[2] if cinfo else ekr - 1.05e-3) + 1.05e-3).sum()) if cinfo else None
            det.append({
                "collect_slot_cnt_thresh": cinfo, "thresh_minus_ek_plus_eps": (cinfo[2] - (ekr - 1.05e-3)) if cinfo else None,
                "rows_exact_ge_thresh_plus_eps": need,
                "q": int(qi), "first_diff_pos": first, "e_k": float(ek),
                "n_missing": len(missing), "n_extra": len(extra),
                "missing": [(m, float(cos[qi, m]), m // 64) for m in missing[:8]],
                "extra": [(e, float(cos[qi, e]) if e >= 0 else None, e // 64) for e in extra[:8]],
                "gpu_s64_vs_exact_at_first": (float(s64[qi, first]), float(cos[qi, g[first]]) if g[first] >= 0 else None),
                "order_only": sorted(g.tolist()) == sorted(o.tolist()),
            })
        rec["detail"] = det
        print(json.dumps(rec), flush=True)
        return r

    ra = run("full_640_k50", 50, 640)
    rb = run("full_640_k50_again", 50, 640)
    print(json.dumps({"case": "repeat_identical", "same": bool(np.array_equal(ra, rb))}), flush=True)
    run("chunks_256_k50", 50, 256)
    run("chunks_320_k50", 50, 320)
    run("chunks_64_k50_K7s", 50, 64)
    run("full_640_k65_v1", 65, 640)
    run("full_640_k32", 32, 640)
    run("full_640_k40", 40, 640)
    run("full_640_k64", 64, 640)
    run("full_640_k10", 10, 640)


if __name__ == "__main__":
    main()
