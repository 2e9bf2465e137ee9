"""GPU flat cosine index — the engine behind ``app.storage.lancedb_store``.

Replaces the lancedb (Rust) flat scan the reference reaches through
``app/storage/lancedb_store.py:103-123`` and the per-row delete+append upsert at
``:87-101``. The arithmetic runs in ``libmrag.so`` (``csrc/knn.hip``): an fp16 MFMA
scan with per-lane top-k, exact f64 rescoring against the f32 master rows and a
certificate that proves the returned rows are the exact top-k.

``FlatIndex`` accepts numpy arrays (host pointers: the library copies in/out) or
torch CUDA tensors (device pointers, torch's current stream) — results come back
in the same kind.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple, Union

import numpy as np

from app import _native

ArrayLike = Union[np.ndarray, "torch.Tensor"]  # noqa: F821

MAX_DIM = 4096  # K7/K8 fused scan up to 512; K7g (knn_generic.hip) above
MAX_K = 65536
LABEL_ANY = _native.MRAG_LABEL_ANY
LABEL_DELETED = _native.MRAG_LABEL_DELETED


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _stream_ptr(t) -> int:
    import torch

    return int(torch.cuda.current_stream(t.device).cuda_stream)


class FlatIndex:
    """Exact flat cosine index of fixed ``dim`` on one GPU (one Lance table or one shard).

    Row ids are assigned densely in insertion order; ``delete`` tombstones rows
    (their ids are not reused). Each row carries an int32 label (the host maps
    ``user_id`` strings to labels); ``search(..., label=L)`` is the reference's
    ``where("user_id == ...")`` prefilter.
    """

    def __init__(self, dim: int, device: int = 0) -> None:
        if not (1 <= int(dim) <= MAX_DIM):
            raise ValueError(f"dim must be in 1..{MAX_DIM}, got {dim}")
        self.dim = int(dim)
        self.device = int(device)
        h = ctypes.c_void_p()
        _native.call("mrag_knn_create", self.dim, self.device, ctypes.byref(h))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _native.load().mrag_knn_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        n = ctypes.c_int64(0)
        _native.call("mrag_knn_size", self._h, ctypes.byref(n))
        return int(n.value)

    # ------------------------------------------------------------------ writes
    def add(self, rows: ArrayLike, labels: Union[ArrayLike, int, None] = 0) -> int:
        """Append rows ``[n, dim]`` (f32) with labels; returns the first new row id."""
        first = ctypes.c_int64(0)
        if _is_torch(rows):
            import torch

            r = rows.detach().to(dtype=torch.float32).contiguous()
            if r.ndim != 2 or r.shape[1] != self.dim:
                raise ValueError(f"rows must be [n, {self.dim}], got {tuple(r.shape)}")
            n = r.shape[0]
            if labels is None or isinstance(labels, int):
                lab = torch.full((n,), int(labels or 0), dtype=torch.int32, device=r.device)
            else:
                lab = torch.as_tensor(labels).to(device=r.device, dtype=torch.int32).contiguous()
                if tuple(lab.shape) != (n,):
                    raise ValueError(f"labels must be [{n}], got {tuple(lab.shape)}")
            if n and bool((lab < 0).any()):
                raise ValueError("labels must be >= 0")
            torch.cuda.current_stream(r.device).synchronize()
            _native.call("mrag_knn_add", self._h, r.data_ptr(), lab.data_ptr(), n,
                         _native.MRAG_PTR_DEVICE, ctypes.byref(first))
            return int(first.value)
        r = np.ascontiguousarray(rows, dtype=np.float32)
        if r.ndim != 2 or r.shape[1] != self.dim:
            raise ValueError(f"rows must be [n, {self.dim}], got {r.shape}")
        n = r.shape[0]
        if labels is None or isinstance(labels, (int, np.integer)):
            lab = np.full((n,), int(labels or 0), dtype=np.int32)
        else:
            lab = np.ascontiguousarray(labels, dtype=np.int32)
            if lab.shape != (n,):
                raise ValueError("labels must be [n]")
        if np.any(lab < 0):
            raise ValueError("labels must be >= 0")
        _native.call("mrag_knn_add", self._h, r.ctypes.data, lab.ctypes.data, n,
                     _native.MRAG_PTR_HOST, ctypes.byref(first))
        return int(first.value)

    def set_labels(self, rows: Sequence[int], label: int) -> None:
        ids = np.ascontiguousarray(np.asarray(rows, dtype=np.int64).reshape(-1))
        if ids.size == 0:
            return
        _native.call("mrag_knn_set_labels", self._h, ids.ctypes.data, ids.size, int(label))

    def delete(self, rows: Sequence[int]) -> None:
        self.set_labels(rows, LABEL_DELETED)

    # ------------------------------------------------------------------ search
    def search(self, queries: ArrayLike, k: int, label: int = LABEL_ANY, row_offset: int = 0,
               with_f64: bool = False):
        """k best rows per query: ``(scores f32 [nq,k], rows int64 [nq,k][, scores f64])``.

        Empty slots (fewer matching rows than k) have score ``-inf`` and row ``-1``.
        """
        k = int(k)
        if _is_torch(queries):
            import torch

            q = queries.detach().to(dtype=torch.float32).contiguous()
            if q.ndim == 1:
                q = q.unsqueeze(0)
            if q.shape[1] != self.dim:
                raise ValueError(f"queries must be [nq, {self.dim}]")
            nq = q.shape[0]
            s = torch.empty((nq, k), dtype=torch.float32, device=q.device)
            r = torch.empty((nq, k), dtype=torch.int64, device=q.device)
            s64 = torch.empty((nq, k), dtype=torch.float64, device=q.device) if with_f64 else None
            _native.call("mrag_knn_search", self._h, q.data_ptr(), nq, k, int(label), int(row_offset),
                         s.data_ptr(), s64.data_ptr() if s64 is not None else None, r.data_ptr(),
                         _native.MRAG_PTR_DEVICE, _stream_ptr(q))
            return (s, r, s64) if with_f64 else (s, r)
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        if q.shape[1] != self.dim:
            raise ValueError(f"queries must be [nq, {self.dim}], got {q.shape}")
        nq = q.shape[0]
        s = np.empty((nq, k), dtype=np.float32)
        r = np.empty((nq, k), dtype=np.int64)
        s64 = np.empty((nq, k), dtype=np.float64) if with_f64 else None
        _native.call("mrag_knn_search", self._h, q.ctypes.data, nq, k, int(label), int(row_offset),
                     s.ctypes.data, s64.ctypes.data if s64 is not None else None, r.ctypes.data,
                     _native.MRAG_PTR_HOST, None)
        return (s, r, s64) if with_f64 else (s, r)

    def profile(self, enable: int = -1) -> Tuple[float, int]:
        """Scan-kernel timing (HIP events on the search stream): enable=1 reset+on,
        0 off, -1 read. Returns (total scan ms, timed launches)."""
        ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
        _native.call("mrag_knn_profile", self._h, int(enable), ctypes.byref(ms), ctypes.byref(n))
        return float(ms.value), int(n.value)

    def last_stats(self) -> Tuple[int, int]:
        """(uncertified queries, collect retries) of the last search."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        _native.call("mrag_knn_last_stats", self._h, ctypes.byref(a), ctypes.byref(b))
        return int(a.value), int(b.value)


def topk_merge(scores64, rows, k: int):
    """Merge per-shard lists ``[nlists, nq, k]`` (torch CUDA f64 / int64) into the
    global top-k under (score desc, row asc): K11 in ``csrc/knn.hip``."""
    import torch

    if scores64.ndim != 3 or rows.shape != scores64.shape:
        raise ValueError("expected [nlists, nq, k] scores and rows")
    nl, nq, kk = scores64.shape
    if kk != k:
        raise ValueError("k mismatch")
    s64 = scores64.contiguous()
    r = rows.contiguous()
    out_s = torch.empty((nq, k), dtype=torch.float32, device=s64.device)
    out_s64 = torch.empty((nq, k), dtype=torch.float64, device=s64.device)
    out_r = torch.empty((nq, k), dtype=torch.int64, device=s64.device)
    _native.call("mrag_topk_merge", s64.data_ptr(), r.data_ptr(), nl, nq, k, out_s.data_ptr(),
                 out_s64.data_ptr(), out_r.data_ptr(), _stream_ptr(s64))
    return out_s, out_r, out_s64


def l2norm_rows(x):
    """K6: the reference's numpy ``_normalize`` (app/ml/embeddings.py:46-49) on the GPU,
    bit-identical. ``x``: torch CUDA f32 [rows, dim]; returns a new tensor."""
    import torch

    t = x.detach().to(dtype=torch.float32).contiguous()
    if t.ndim != 2:
        raise ValueError("expected [rows, dim]")
    y = torch.empty_like(t)
    _native.call("mrag_l2norm_rows", t.data_ptr(), y.data_ptr(), t.shape[0], t.shape[1], _stream_ptr(t))
    return y


__all__ = ["FlatIndex", "topk_merge", "l2norm_rows", "LABEL_ANY", "LABEL_DELETED"]
