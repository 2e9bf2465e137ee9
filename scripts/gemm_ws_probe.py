#!/usr/bin/env python3
"""K3w probe: time of one GEMM launch against M (tiles per workgroup) for a fixed N, K, per
kernel — the fixed cost (weights into AGPRs, first fill, drain) and the per-tile slope."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

from app.encoders import gemm_nt  # noqa: E402

N, K, epi = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
kernels = sys.argv[4].split(",") if len(sys.argv) > 4 else ["k3w", "k3d", "k3"]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
W = (torch.randn(N, K, device=dev, generator=g) * 0.02).half()
bias = torch.randn(N, device=dev, generator=g) * 0.01
Ms = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [2560, 5120, 10240, 16000, 32000]
for M in Ms:
    A = [(torch.randn(M, K, device=dev, generator=g)).half() for _ in range(3)]
    C = [torch.empty(M, N, device=dev).half() for _ in range(3)]
    row = {"N": N, "K": K, "epi": epi, "M": M, "tiles_of_64": M // 64}
    for kern in kernels:
        if kern == "k3d" and N % 256:
            continue
        try:
            for i in range(4):
                gemm_nt(A[i % 3], W, bias, C[i % 3], epi, kernel=kern)
            torch.cuda.synchronize()
            ts = []
            for rep in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(20):
                    gemm_nt(A[i % 3], W, bias, C[i % 3], epi, kernel=kern)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 20)
            row[kern + "_us"] = round(sorted(ts)[2], 2)
        except Exception as e:  # a kernel that does not take the shape
            row[kern + "_us"] = str(e)[:80]
    print(json.dumps(row), flush=True)
