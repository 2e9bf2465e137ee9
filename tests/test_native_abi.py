"""The C-ABI library loads on a CPU-only machine and exports every symbol that
include/mrag.h declares (no compute calls: there is no GPU here)."""
from __future__ import annotations

import ctypes
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "mrag.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mrag_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from app import _native

    lib = _native.load()
    names = _declared()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # every declared symbol has a Python binding signature somewhere in the package
    assert set(_native.SIGNATURES) <= set(names)


def test_error_path_without_gpu():
    from app import _native

    lib = _native.load()
    assert lib.mrag_version().startswith(b"mrag")
    h = ctypes.c_void_p()
    rc = lib.mrag_knn_create(0, 0, ctypes.byref(h))  # dim 0 is rejected before any HIP call
    assert rc == 1 and b"dim" in lib.mrag_last_error()
