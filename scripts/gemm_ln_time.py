"""Timing of the LayerNorm-fold GEMM epilogues against the plain ones on the encoder shapes
(one launch at a time, HIP events, median of 20)."""
import ctypes
import json
import os
import sys

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

SHAPES = {"qkv": (12800, 2304, 768, "fold"), "fc1": (12800, 3072, 768, "fold"), "fc2": (12800, 768, 3072, "res"),
          "out": (12800, 768, 768, "res"), "t_qkv": (16000, 1536, 512, "fold"), "t_out": (16000, 512, 512, "res"),
          "t_fc1": (16000, 2048, 512, "fold"), "t_fc2": (16000, 512, 2048, "res"), "m_qkv": (16000, 1152, 384, "fold"),
          "m_out": (16000, 384, 384, "res"), "m_fc1": (16000, 1536, 384, "fold"), "m_fc2": (16000, 384, 1536, "res")}


def timed(fn, reps=20):
    ts = []
    for _ in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts = sorted(ts[3:])
    return round(ts[len(ts) // 2], 1)


for name in (sys.argv[1:] or list(SHAPES)):
    M, N, K, kind = SHAPES[name]
    A = (torch.rand(M, K, device=dev) * 2 - 1).half()
    W = (torch.rand(N, K, device=dev) * 0.1 - 0.05).half()
    b = torch.rand(N, device=dev) * 0.1
    out = {"shape": name, "M": M, "N": N, "K": K}
    if kind == "fold":
        C = torch.empty(M, N, dtype=torch.float16, device=dev)
        st = torch.rand(M, K // 64, 2, device=dev) + 1.0
        cs = torch.rand(N, device=dev)
        for epi in (0, 1, 2):
            out[f"epi{epi}"] = timed(lambda: f(P(A), P(W), P(b), P(C), M, N, K, epi, None, 0, 0, 0.0, None, None, None,
                                              None, None, None))
            out[f"epi{epi}|fold"] = timed(lambda: f(P(A), P(W), P(b), P(C), M, N, K, epi | 8, P(st), K // 64, K, 1e-5,
                                                   P(cs), None, None, None, None, None))
    else:
        C = torch.rand(M, N, device=dev)
        c16 = torch.empty(M, N, dtype=torch.float16, device=dev)
        st = torch.rand(M, N // 64, 2, device=dev) + 1.0
        st2 = torch.empty_like(st)
        lg, lb = torch.rand(N, device=dev), torch.rand(N, device=dev)
        out["res"] = timed(lambda: f(P(A), P(W), P(b), P(C), M, N, K, 3, None, 0, 0, 0.0, None, None, None, None, None,
                                     None))
        out["res|stats"] = timed(lambda: f(P(A), P(W), P(b), P(C), M, N, K, 19, None, 0, 0, 0.0, None, None, None,
                                           P(c16), P(st2), None))
        if N % 256 != 0:
            out["res|stats|resln"] = timed(lambda: f(P(A), P(W), P(b), P(C), M, N, K, 51, P(st), N // 64, N, 1e-5, None,
                                                     P(lg), P(lb), P(c16), P(st2), None))
    print(json.dumps(out), flush=True)
