"""Dump K3 GEMM outputs for a set of shapes x epilogues (seeded operands) to an .npz, so two
processes with different kernel-selection env vars can be compared bit for bit."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import torch  # noqa: E402

from app.encoders import gemm_nt  # noqa: E402

CASES = [(12800, 2304, 768, 0), (12800, 3072, 768, 1), (12800, 768, 3072, 3), (12800, 768, 768, 3),
         (12850, 768, 768, 4), (4000, 1536, 512, 2), (1100, 512, 2048, 3), (2560, 1024, 64, 0), (1030, 256, 128, 1),
         (16000, 512, 512, 3), (16000, 512, 2048, 3), (16000, 2048, 512, 1)]
out = {}
for ci, (M, N, K, epi) in enumerate(CASES):
    g = torch.Generator(device="cuda").manual_seed(ci)
    A = (torch.rand(M, K, generator=g, device="cuda") * 2 - 1).half()
    W = (torch.rand(N, K, generator=g, device="cuda") * 2 - 1).half()
    bias = torch.rand(N, generator=g, device="cuda") - 0.5
    if epi >= 3:
        C = torch.rand(M, N, generator=g, device="cuda")
    else:
        C = torch.zeros(M, N, device="cuda", dtype=torch.float16)
    gemm_nt(A, W, bias, C, epi)
    out[f"c{ci}"] = C.float().cpu().numpy()
    ref = A.float() @ W.float().t() + bias
    print(ci, (M, N, K, epi), "max|C| %.3g" % float(C.float().abs().max()), flush=True)
np.savez(sys.argv[1], **out)
