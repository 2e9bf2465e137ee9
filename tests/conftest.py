"""Test configuration: markers, import paths, shared fixtures.

``-m "not gpu"`` (CPU, here): oracle vs golden vectors, host logic, C-ABI exports.
``-m gpu`` (MI355X box): parity of the HIP path (through the C ABI) against the oracle.
GPU tests never skip on a missing GPU — they fail, so a broken box cannot pass.
"""
from __future__ import annotations

import os
import sys
import tempfile

import pytest

# the compat layer reads LANCEDB_DIR at import time (as the reference's settings do)
os.environ.setdefault("LANCEDB_DIR", tempfile.mkdtemp(prefix="mrag_lancedb_"))
# no hub weights offline: the drop-in encoders raise on an unresolvable model name unless
# synthetic weights are requested explicitly (tests that check the raise unset this)
os.environ.setdefault("MRAG_SYNTHETIC_WEIGHTS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libmrag.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def cuda():
    import torch

    assert torch.cuda.is_available(), "GPU test on a machine without a visible GPU"
    from app import _native

    _native.load()
    return torch.device("cuda:0")


# ---- numerics log: observed errors of the fp16 GPU path against the fp32 oracle --------
# Tests record (name, max 1-cos, max |diff|, ...) here; the table is printed at the end of
# the run (visible in the GPU test log whether the tests pass or fail) and written to
# gpurun_out/numerics_r02.json when that directory exists.
NUMERICS = []


def record_numerics(name: str, got, exp, unit: bool = True, **extra):
    import numpy as np

    g = np.asarray(got, np.float64)
    e = np.asarray(exp, np.float64)
    row = {"name": name, "rows": int(g.shape[0]) if g.ndim else 1}
    if g.ndim == 2 and g.shape[0]:
        cos = np.sum(g * e, 1) / np.maximum(np.linalg.norm(g, axis=1) * np.linalg.norm(e, axis=1), 1e-300)
        row["max_1_minus_cos"] = float((1.0 - cos).max())
        row["mean_1_minus_cos"] = float((1.0 - cos).mean())
        if not unit:
            row["max_rel_l2"] = float((np.linalg.norm(g - e, axis=1) / np.linalg.norm(e, axis=1)).max())
    if g.size:
        row["max_abs_diff"] = float(np.abs(g - e).max())
    row.update(extra)
    NUMERICS.append(row)
    return row


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if not NUMERICS:
        return
    import json

    terminalreporter.section("numerics (GPU fp16 path vs fp32 oracle)")
    for r in NUMERICS:
        terminalreporter.write_line(json.dumps(r))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "numerics_r02.json"), "w") as f:
            json.dump(NUMERICS, f, indent=1)
