#!/usr/bin/env python3
"""Per-GEMM roofline of the encoder towers' GEMM shapes: each shape through
the C ABI (`mrag_gemm_nt`, the same kernel choice as inside the towers) timed with HIP events over
20 back-to-back launches that rotate three activation / output buffer sets (so A and C stream from
HBM rather than the 256 MB MALL, as in a tower where LayerNorm and attention run in between).
FLOP = 2 M N K; bytes = A (f16) + W (f16) + bias + C (f16 out, or f32 read + write for the residual
epilogue). Roofline floor = max(FLOP / 2.5 PF, bytes / 8 TB/s); frac_of_bound = floor / time."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

from app import _native  # noqa: E402

PEAK_TF, HBM_GBS = 2500.0, 8000.0
EPI_NAME = {0: "f16", 1: "f16 quick_gelu", 2: "f16 gelu_erf", 3: "f32 residual +=", 4: "f32"}
SHAPES = [  # (tower, gemm, M, N, K, epilogue)
    ("vit_b32 B=256", "qkv", 12800, 2304, 768, 0), ("vit_b32 B=256", "out", 12800, 768, 768, 3),
    ("vit_b32 B=256", "fc1", 12800, 3072, 768, 1), ("vit_b32 B=256", "fc2", 12800, 768, 3072, 3),
    ("clip_text config5", "qkv", 16000, 1536, 512, 0), ("clip_text config5", "out", 16000, 512, 512, 3),
    ("clip_text config5", "fc1", 16000, 2048, 512, 1), ("clip_text config5", "fc2", 16000, 512, 2048, 3),
    ("minilm config5", "qkv", 16000, 1152, 384, 0), ("minilm config5", "out", 16000, 384, 384, 3),
    ("minilm config5", "fc1", 16000, 1536, 384, 2), ("minilm config5", "fc2", 16000, 384, 1536, 3),
]

import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sets", type=int, default=3, help="activation / output buffer sets rotated")
ap.add_argument("--operands", choices=["randn", "small", "zeros"], default="randn",
                help="activation values: N(0,1), N(0,1) x 1e-3, or zeros (switching activity A/B)")
ap.add_argument("--only", default="", help="comma-separated tower:gemm names")
ap.add_argument("--epi", type=int, default=-1, help="override every shape's epilogue (A/B of the epilogue cost)")
args = ap.parse_args()
if args.only:
    keep = set(args.only.split(","))
    SHAPES = [s for s in SHAPES if f"{s[0].split()[0]}:{s[1]}" in keep]
lib = _native.load()
lib.mrag_gemm_nt.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int32] * 4 + [ctypes.c_void_p]
lib.mrag_gemm_nt.restype = ctypes.c_int
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
for tower, name, M, N, K, epi in SHAPES:
    if args.epi >= 0:
        epi = args.epi
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).half()
    bias = torch.randn(N, device=dev, generator=g) * 0.01
    sets = []
    for _ in range(args.sets):
        A = torch.randn(M, K, device=dev, generator=g)
        A = (A * (1e-3 if args.operands == "small" else 0.0 if args.operands == "zeros" else 1.0)).half()
        C = torch.randn(M, N, device=dev, generator=g) if epi in (3, 4) else torch.empty(M, N, device=dev).half()
        sets.append((A, C))
    stream = torch.cuda.current_stream(dev)

    def launch(i):
        A, C = sets[i % len(sets)]
        rc = lib.mrag_gemm_nt(A.data_ptr(), W.data_ptr(), bias.data_ptr(), C.data_ptr(), M, N, K, epi,
                              stream.cuda_stream)
        assert rc == 0, _native.load().mrag_last_error()

    for i in range(6):
        launch(i)
    torch.cuda.synchronize()
    reps = []
    for r in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(20):
            launch(i)
        e1.record(stream)
        torch.cuda.synchronize()
        reps.append(e0.elapsed_time(e1) * 1e3 / 20)
    t_us = sorted(reps)[2]
    flop = 2.0 * M * N * K
    cbytes = M * N * 8 if epi == 3 else M * N * (4 if epi == 4 else 2)
    nbytes = M * K * 2 + N * K * 2 + N * 4 + cbytes
    t_mfma, t_hbm = flop / (PEAK_TF * 1e12) * 1e6, nbytes / (HBM_GBS * 1e9) * 1e6
    floor = max(t_mfma, t_hbm)
    print(json.dumps({"sets": args.sets, "operands": args.operands, "tower": tower, "gemm": name, "M": M, "N": N, "K": K, "epilogue": EPI_NAME[epi],
                      "us": round(t_us, 2), "tflops": round(flop / t_us / 1e6, 1),
                      "mfma_frac": round(flop / t_us / 1e6 / PEAK_TF, 3), "hbm_gbs": round(nbytes / t_us / 1e3, 1),
                      "bound": "mfma" if t_mfma >= t_hbm else "hbm", "floor_us": round(floor, 2),
                      "frac_of_bound": round(floor / t_us, 3)}), flush=True)
    del sets, W, bias
    torch.cuda.empty_cache()
