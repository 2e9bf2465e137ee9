"""K12 (csrc/fusion.hip, mrag_fuse_scores): the reference's z-score fusion on the GPU,
bit-identical to the host restatement ``app.retrieval.fuse_scores`` (pinned against the
reference's ``_fuse_results`` by tests/test_compat_cpu.py) and to ``oracle.fusion`` on the
hit dicts: picks equal, combined f64 scores equal bit for bit. Cases: full lists, missing hits
(-inf padding), one-hit lists (std 0), empty lists, exact score ties, k up to 300."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _lists(rng, q, k, fill):
    s = -np.sort(-rng.uniform(-0.2, 0.9, (q, k)).astype(np.float32), axis=1)
    s[: q // 8] = np.round(s[: q // 8], 2)  # exact ties inside a list
    n = rng.integers(0, k + 1, q) if fill else np.full(q, k)
    n[:3] = [0, 1, min(2, k)]
    s[np.arange(k)[None, :] >= n[:, None]] = -np.inf
    return s


@pytest.mark.parametrize("kt,ki,final_n", [(50, 12, 4), (10, 10, 4), (300, 7, 9), (1, 1, 4), (130, 140, 20)])
def test_fusion_gpu_equals_host(cuda, kt, ki, final_n):
    import torch

    from app.retrieval import fuse_scores, fuse_scores_gpu
    from oracle.fusion import fuse_results

    rng = np.random.default_rng(kt * 1000 + ki)
    q = 700
    ts, im = _lists(rng, q, kt, True), _lists(rng, q, ki, True)
    ts[5], im[5] = ts[4], im[4]  # identical queries
    hp, hc = fuse_scores(ts, im, final_n)
    gp, gc = fuse_scores_gpu(torch.from_numpy(ts).to(cuda), torch.from_numpy(im).to(cuda), final_n)
    gp, gc = gp.cpu().numpy(), gc.cpu().numpy()
    np.testing.assert_array_equal(gp, hp)
    np.testing.assert_array_equal(gc, hc)  # NaN == NaN for empty slots
    one = np.float32(1.0)
    for i in range(0, q, 23):  # the reference's dict-based fusion on a sample
        th = [{"i": j, "score": float(1.0 - float(one - s))} for j, s in enumerate(ts[i]) if np.isfinite(s)]
        ih = [{"i": kt + j, "score": float(1.0 - float(one - s))} for j, s in enumerate(im[i]) if np.isfinite(s)]
        ref = fuse_results(th, ih, final_n)
        assert [r["i"] for r in ref] == [int(p) for p in gp[i] if p >= 0], i
        assert [r["combined_score"] for r in ref] == [float(c) for c, p in zip(gc[i], gp[i]) if p >= 0], i
