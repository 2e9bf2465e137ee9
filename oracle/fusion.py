"""z-score fusion of text and image hits, restated (test oracle only).

Reference: ``app/ml/retrieve.py:158-195`` (`_fuse_results`, `_z_scores`): per-list
z-scores computed from a float32 array (mean/std in float32, then Python floats), zero
std -> all zeros; text items score mean(z_cos, z_rerank); sort desc; keep final_n.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import numpy as np


def z_scores(values: Sequence[Optional[float]]) -> List[float]:
    numeric = [v for v in values if v is not None]
    if not numeric:
        return []
    arr = np.array(numeric, dtype=np.float32)
    mean = float(arr.mean())
    std = float(arr.std())
    if std == 0:
        return [0.0 for _ in values]
    return [float((v - mean) / std) if v is not None else 0.0 for v in values]


def fuse_results(text_results: List[Dict[str, Any]], image_results: List[Dict[str, Any]], final_n: int = 4):
    items: List[Dict[str, Any]] = []
    t_cos = z_scores([it["score"] for it in text_results])
    t_rr_vals = [it.get("rerank_score") for it in text_results if "rerank_score" in it]
    t_rr = z_scores(t_rr_vals) if t_rr_vals else []
    i_cos = z_scores([it["score"] for it in image_results])
    for idx, it in enumerate(text_results):
        z = []
        if t_cos:
            z.append(t_cos[idx])
        if t_rr and idx < len(t_rr):
            z.append(t_rr[idx])
        items.append({**it, "combined_score": float(np.mean(z)) if z else it["score"]})
    for idx, it in enumerate(image_results):
        items.append({**it, "combined_score": float(i_cos[idx] if i_cos else it["score"])})
    items.sort(key=lambda e: e["combined_score"], reverse=True)
    return items[:final_n]
