"""Kernel-level check of the LayerNorm-fold GEMM epilogues (mrag_debug_gemm_ln) against torch,
with duplicated rows placed at different positions (tile, wave row, 16-row block, lane) to show
whether a row's result depends on where it sits."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import torch  # noqa: E402

from app import _native  # noqa: E402

lib = _native.load()
f = lib.mrag_debug_gemm_ln
vp, i32 = ctypes.c_void_p, ctypes.c_int32
f.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, vp, i32, i32, ctypes.c_float, vp, vp, vp, vp, vp, vp]
f.restype = ctypes.c_int
dev = torch.device("cuda", 0)
P = lambda t: None if t is None else t.data_ptr()  # noqa: E731


def run(A, W, b, C, epi, st_in=None, p_in=0, d=0, eps=1e-5, cs=None, lg=None, lb=None, c16=None, st_out=None):
    M, K = A.shape
    N = W.shape[0]
    rc = f(P(A), P(W), P(b), P(C), M, N, K, epi, P(st_in), p_in, d, eps, P(cs), P(lg), P(lb), P(c16), P(st_out), None)
    assert rc == 0, lib.mrag_last_error()
    torch.cuda.synchronize()


def case(M, N, K, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    A = (torch.randn(M, K, generator=g, device=dev) * 0.5).half()
    C0 = torch.randn(M, N, generator=g, device=dev) + 0.3
    # duplicate row 5 of A / C0 at several positions
    dup = [5, 21, 37, 70, 133, 200, 300, M - 1]
    dup = [r for r in dup if r < M]
    A[dup] = A[5].clone()
    C0[dup] = C0[5].clone()
    W = (torch.randn(N, K, generator=g, device=dev) * 0.05).half()
    b = torch.randn(N, generator=g, device=dev) * 0.1
    out = {"M": M, "N": N, "K": K}
    # EPI_STATS (19) vs plain residual (3)
    C3 = C0.clone()
    run(A, W, b, C3, 3)
    C = C0.clone()
    c16 = torch.empty(M, N, dtype=torch.float16, device=dev)
    st = torch.zeros(M, N // 64, 2, device=dev)
    run(A, W, b, C, 16 | 3, c16=c16, st_out=st)
    out["stats_C_equal_res"] = bool(torch.equal(C, C3))
    out["c16_equal"] = bool(torch.equal(c16, C.half()))
    ref = C.double().view(M, N // 64, 64)
    out["st_sum_err"] = float((st[..., 0].double() - ref.sum(-1)).abs().max() / ref.abs().sum(-1).max())
    m2 = ((ref - ref.mean(-1, keepdim=True)) ** 2).sum(-1)
    out["st_m2_err"] = float((st[..., 1].double() - m2).abs().max() / m2.max())
    out["dup_C"] = bool(all(torch.equal(C[r], C[5]) for r in dup))
    out["dup_st"] = bool(all(torch.equal(st[r], st[5]) for r in dup))
    bad = [r for r in dup if not torch.equal(st[r], st[5])]
    out["dup_st_bad_rows"] = bad
    if bad:
        out["st_row5"] = st[5].tolist()[:3]
        out["st_bad"] = st[bad[0]].tolist()[:3]
    # EPI_FOLD (8) consuming those statistics: out = r (A' W'^T - mu cs) + b with A' = c16
    D = N
    W2 = (torch.randn(384, D, generator=g, device=dev) * 0.05).half()
    cs = W2.float().sum(1)
    b2 = torch.randn(384, generator=g, device=dev) * 0.1
    O = torch.empty(c16.shape[0], 384, dtype=torch.float16, device=dev)
    run(c16, W2, b2, O, 8, st_in=st, p_in=N // 64, d=D, eps=1e-5, cs=cs)
    Cd = C.double()
    mu = Cd.mean(1)
    r = 1.0 / torch.sqrt(((Cd - mu[:, None]) ** 2).mean(1) + 1e-5)
    refO = (r[:, None] * (c16.double() @ W2.double().t() - mu[:, None] * cs.double()[None, :]) + b2.double())
    out["fold_err"] = float((O.double() - refO).abs().max())
    out["dup_fold"] = bool(all(torch.equal(O[rr], O[5]) for rr in dup))
    out["dup_fold_bad_rows"] = [rr for rr in dup if not torch.equal(O[rr], O[5])]
    # EPI_RESLN (51): C = LN(C) + acc + b
    lg = torch.rand(N, generator=g, device=dev) + 0.5
    lb = torch.randn(N, generator=g, device=dev) * 0.1
    Cr = C.clone()
    c16b = torch.empty_like(c16)
    st2 = torch.zeros_like(st)
    run(A, W, b, Cr, 32 | 16 | 3, st_in=st, p_in=N // 64, d=D, eps=1e-5, lg=lg, lb=lb, c16=c16b, st_out=st2)
    lnC = (C.double() - mu[:, None]) * r[:, None] * lg.double() + lb.double()
    refR = lnC + (A.double() @ W.double().t()) + b.double()
    out["resln_err"] = float((Cr.double() - refR).abs().max())
    out["dup_resln"] = bool(all(torch.equal(Cr[rr], Cr[5]) for rr in dup))
    print(json.dumps(out), flush=True)


for M, N, K in [(80, 512, 512), (300, 768, 768), (300, 512, 2048), (3050, 768, 768), (3050, 768, 3072),
                (16000, 512, 512), (520, 384, 1536)]:
    case(M, N, K)
