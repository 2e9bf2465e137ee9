"""ctypes binding of ``libmrag.so`` (the C ABI declared in ``include/mrag.h``).

The library is built in-tree (``make -C multimodal-rag-for-image-text-search_amd``
or ``__graft_entry__.build()``) for gfx950. There is deliberately no CPU fallback:
if the library or a GPU is missing, every entry point raises.

torch is imported before the library is loaded so that the process uses one HIP
runtime (torch ships ``libamdhip64.so.7``; libmrag links the same soname).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MRAG_LIB", os.path.join(PKG_DIR, "lib", "libmrag.so"))

MRAG_OK = 0
MRAG_PTR_HOST = 0
MRAG_PTR_DEVICE = 1
MRAG_LABEL_ANY = -1
MRAG_LABEL_DELETED = -2

_c_int = ctypes.c_int32
_c_i64 = ctypes.c_int64
_vp = ctypes.c_void_p

# name -> (restype, argtypes); every symbol include/mrag.h declares.
SIGNATURES = {
    "mrag_last_error": (ctypes.c_char_p, []),
    "mrag_version": (ctypes.c_char_p, []),
    "mrag_get_device_count": (_c_int, [ctypes.POINTER(_c_int)]),
    "mrag_l2norm_rows": (_c_int, [_vp, _vp, _c_i64, _c_int, _vp]),
    "mrag_knn_create": (_c_int, [_c_int, _c_int, ctypes.POINTER(_vp)]),
    "mrag_knn_destroy": (_c_int, [_vp]),
    "mrag_knn_add": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, ctypes.POINTER(_c_i64)]),
    "mrag_knn_set_labels": (_c_int, [_vp, _vp, _c_i64, _c_int]),
    "mrag_knn_size": (_c_int, [_vp, ctypes.POINTER(_c_i64)]),
    "mrag_knn_search": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_int, _c_i64, _vp, _vp, _vp, _c_int, _vp]),
    "mrag_knn_last_stats": (_c_int, [_vp, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)]),
    "mrag_knn_profile": (_c_int, [_vp, _c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_i64)]),
    "mrag_topk_merge": (_c_int, [_vp, _vp, _c_int, _c_i64, _c_int, _vp, _vp, _vp, _vp]),
    "mrag_fuse_scores": (_c_int, [_vp, _c_int, _vp, _c_int, _c_i64, _c_int, _vp, _vp, _vp]),
    "mrag_image_resize_crop": (_c_int, [_vp, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_int),
                                        ctypes.POINTER(_c_int), _c_int, _c_int, _vp, _vp]),
    "mrag_jpeg_probe": (_c_int, [ctypes.c_char_p, _c_i64, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int)]),
    "mrag_jpeg_decode": (_c_int, [_vp, _vp, _c_int, _vp, _vp, _c_int, _vp]),
    "mrag_png_probe": (_c_int, [ctypes.c_char_p, _c_i64, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int),
                                ctypes.POINTER(_c_i64)]),
    "mrag_png_inflate": (_c_int, [ctypes.c_char_p, _c_i64, _vp, _c_i64, ctypes.POINTER(_c_int)]),
    "mrag_png_unfilter": (_c_int, [_vp, _vp, _c_int, _vp, _vp, _c_int, _vp]),
    "mrag_files_prepare": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_i64, ctypes.POINTER(_vp)]),
    "mrag_files_info": (_c_int, [_vp, _vp, _vp, _vp]),
    "mrag_files_bytes": (_c_int, [_vp, _c_int, ctypes.POINTER(_vp), ctypes.POINTER(_c_i64)]),
    "mrag_files_decode": (_c_int, [_vp, _vp, _vp, _c_int, _vp]),
    "mrag_files_free": (_c_int, [_vp]),
    "mrag_paths_exist": (_c_int, [_vp, _c_int, _c_int, _vp]),
    "mrag_hash_tokenize": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp]),
}

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    """A libmrag entry point returned a non-zero status."""


def load() -> ctypes.CDLL:
    """Load libmrag.so once (raises if it is missing: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (one HIP runtime per process: torch's)

        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libmrag.so not found at {LIB_PATH}; build it with __graft_entry__.build() "
                "or `make -C multimodal-rag-for-image-text-search_amd`"
            )
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (restype, argtypes) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = restype
            fn.argtypes = argtypes
        _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != MRAG_OK:
        msg = load().mrag_last_error().decode(errors="replace")
        raise NativeError(f"{what or 'libmrag'} failed (status {rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def device_count() -> int:
    n = _c_int(0)
    rc = load().mrag_get_device_count(ctypes.byref(n))
    return int(n.value) if rc == MRAG_OK else 0
