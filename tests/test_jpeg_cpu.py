"""K13's decode arithmetic (csrc/jpeg_core.h + jpeg_parse.h: the functions the device kernels
call) run on the CPU and compared with Pillow (the reference's decoder) byte for byte; the
library's host-side probe classifies supported / unsupported files. No GPU."""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from _jpeg_cases import (damaged_cases, jpeg_bytes, overlong_run_cases, photo, pillow_rgb, supported_cases,
                         unsupported_cases)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd", "csrc")


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    so = str(tmp_path_factory.mktemp("jpeg") / "jpeg_host_check.so")
    subprocess.run([hipcc, "-O2", "-fPIC", "-shared", f"-I{CSRC}", os.path.join(ROOT, "scripts", "jpeg_host_check.hip"),
                    "-o", so], check=True, capture_output=True, timeout=300)
    lib = ctypes.CDLL(so)
    lib.jpeg_host_decode.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    lib.jpeg_host_decode_mode.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int]
    lib.jpeg_host_par_check.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p]
    return lib


def _decode(lib, b: bytes, par: int = 0):
    wh = np.zeros(2, np.int32)
    cap = 64 << 20
    out = np.zeros(cap, np.uint8)
    r = lib.jpeg_host_decode_mode(b, len(b), out.ctypes.data, cap, wh.ctypes.data, par)
    if r != 1:
        return None
    w, h = int(wh[0]), int(wh[1])
    return out[:w * h * 3].reshape(h, w, 3)


def test_core_matches_pillow(host_check):
    for name, b in supported_cases():
        got = _decode(host_check, b)
        assert got is not None, name
        np.testing.assert_array_equal(got, pillow_rgb(b), err_msg=name)


def test_parallel_entropy_decode_equals_sequential(host_check):
    """K13a's lane emulation (jpeg_parse.h decode_segment_par: the kernel's passes, lane by lane)
    gives the sequential decoder's coefficients on every case, including files whose chunks need
    several resynchronisation rounds (high quality, noise, small chunks), restart intervals and
    large photos; and Pillow's pixels through the rest of the pipeline."""
    cases = supported_cases() + [(f"big{i}", jpeg_bytes(photo(h, w, 100 + i), quality=q, subsampling=sub))
                                 for i, (h, w, q, sub) in enumerate([(768, 1024, 90, 2), (768, 1024, 95, 0),
                                                                     (480, 640, 75, 1)])]
    rounds = []
    for name, b in cases:
        st = np.zeros(2, np.int32)
        assert host_check.jpeg_host_par_check(b, len(b), st.ctypes.data) == 1, name
        rounds.append(int(st[0]))
    assert max(rounds) >= 2  # the resynchronisation rounds are exercised, not only pass 1
    for name, b in cases[::7] + cases[-3:]:
        np.testing.assert_array_equal(_decode(host_check, b, par=1), pillow_rgb(b), err_msg=name)


def test_parallel_entropy_decode_truncated_and_padded(host_check):
    """Truncated entropy-coded data (the decoder feeds zeros, as libjpeg does) and trailing bytes
    after the last MCU: the lane emulation still equals the sequential decoder."""
    b = jpeg_bytes(photo(480, 640, 9), quality=90, subsampling=2)
    eoi = len(b) - 2
    st = np.zeros(2, np.int32)
    for cut in (eoi - 1, eoi - 5000, eoi - 30000):
        t = b[:cut] + b"\xff\xd9"
        assert host_check.jpeg_host_par_check(t, len(t), st.ctypes.data) == 1, cut
    extra = b[:eoi] + bytes(range(1, 200)) + b"\xff\xd9"
    assert host_check.jpeg_host_par_check(extra, len(extra), st.ctypes.data) == 1


def test_damaged_files_as_pillow(host_check):
    """Damaged files: whatever K13 decodes (sequential and lane-parallel entropy decoding) equals
    Pillow; a file Pillow refuses (truncated without a marker) K13 refuses too, so the caller's
    Pillow path raises as the reference does."""
    decoded = 0
    for name, b in damaged_cases():
        try:
            ref = pillow_rgb(b)
        except OSError:
            ref = None
        for par in (0, 1):
            got = _decode(host_check, b, par=par)
            if ref is None:
                assert got is None, name
            elif got is not None:
                decoded += 1
                np.testing.assert_array_equal(got, ref, err_msg=f"{name} par={par}")
    assert decoded >= 20  # the damaged files K13 takes are exercised, not only refused


def test_overlong_ac_run_as_pillow(host_check):
    """an AC run past coefficient 63 (k = 64..78 after a ZRL chain) lands on natural
    index 63, as libjpeg-turbo's padded jpeg_natural_order[] puts it; sequential and lane-parallel
    entropy decoding both give Pillow's pixels."""
    for name, b in overlong_run_cases():
        for par in (0, 1):
            got = _decode(host_check, b, par=par)
            assert got is not None, name
            np.testing.assert_array_equal(got, pillow_rgb(b), err_msg=f"{name} par={par}")


def test_core_refuses_unsupported(host_check):
    for name, b in unsupported_cases():
        assert _decode(host_check, b) is None, name


def test_library_probe():
    from app import _native

    lib = _native.load()
    w, h = ctypes.c_int32(0), ctypes.c_int32(0)
    for name, b in supported_cases()[:12]:
        assert lib.mrag_jpeg_probe(b, len(b), ctypes.byref(w), ctypes.byref(h)) == 1, name
        assert (h.value, w.value) == pillow_rgb(b).shape[:2], name
    for name, b in unsupported_cases():
        assert lib.mrag_jpeg_probe(b, len(b), ctypes.byref(w), ctypes.byref(h)) == 0, name
    png = b"\x89PNG\r\n\x1a\n" + b"\0" * 32
    assert lib.mrag_jpeg_probe(png, len(png), ctypes.byref(w), ctypes.byref(h)) == 0
