"""Synthetic JPEG files for the K13 tests (generated with Pillow, the reference's decoder): photo-
like content (a smooth field + upsampled coarse noise + fine noise) and white noise, every
quality / subsampling / size class the decoder distinguishes, optimised Huffman tables, restart
intervals, grayscale; plus files K13 must refuse (progressive, CMYK, 4:4:0-like, tiny chroma)."""
from __future__ import annotations

import io

import numpy as np
from PIL import Image


def photo(h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    coarse = rng.integers(0, 256, (h // 16 + 1, w // 16 + 1, 3), dtype=np.uint8)
    img = np.asarray(Image.fromarray(coarse).resize((w, h), Image.BILINEAR), dtype=np.int16)
    return np.clip(img + rng.integers(-4, 5, (h, w, 3)), 0, 255).astype(np.uint8)


def jpeg_bytes(a: np.ndarray, **kw) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, "JPEG", **kw)
    return buf.getvalue()


def supported_cases():
    """(name, bytes) K13 decodes: Pillow's output is the expected RGB array."""
    out = []
    sizes = [(480, 640), (768, 1024), (9, 17), (65, 33), (57, 101), (224, 224), (3, 7), (201, 300), (5, 5)]
    for i, (h, w) in enumerate(sizes):
        a = photo(h, w, 10 + i)
        n = np.random.default_rng(40 + i).integers(0, 256, (h, w, 3), dtype=np.uint8)
        for q in (50, 90, 100):
            for sub in (0, 1, 2):
                out.append((f"photo{h}x{w}_q{q}_s{sub}", jpeg_bytes(a, quality=q, subsampling=sub)))
        out.append((f"noise{h}x{w}_q90_s2", jpeg_bytes(n, quality=90, subsampling=2)))
        out.append((f"gray{h}x{w}_q85", jpeg_bytes(a[..., 0], quality=85)))
    a = photo(480, 640, 3)
    out.append(("optimized_huffman", jpeg_bytes(a, quality=85, optimize=True)))
    out.append(("restart_blocks3", jpeg_bytes(a, quality=85, restart_marker_blocks=3)))
    out.append(("restart_rows1", jpeg_bytes(a, quality=85, restart_marker_rows=1)))
    out.append(("q1", jpeg_bytes(a, quality=1)))
    return out


def unsupported_cases():
    a = photo(96, 128, 5)
    return [("progressive", jpeg_bytes(a, quality=85, progressive=True)),
            ("cmyk", _cmyk(a)),
            ("tiny_chroma_w3", jpeg_bytes(photo(5, 3, 6), quality=90, subsampling=2))]


def _cmyk(a: np.ndarray) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(a).convert("CMYK").save(buf, "JPEG", quality=85)
    return buf.getvalue()


def damaged_cases():
    """(name, bytes) of damaged files: cut inside the entropy-coded data and closed with EOI (libjpeg
    finishes the MCU in progress with zero bits and leaves the rest zero), cut with nothing after
    (Pillow raises "image file is truncated"), an RST0 / RST7 spliced in (in a restart-interval
    file: out of order, libjpeg resynchronises), for plain and restart-interval files."""
    out = []
    for seed, (h, w, sub, kw) in enumerate([(480, 640, 2, {}), (301, 223, 0, {}), (480, 640, 1, {"restart_marker_rows": 1}),
                                            (200, 300, 2, {"restart_marker_blocks": 3})]):
        b = jpeg_bytes(photo(h, w, 50 + seed), quality=90, subsampling=sub, **kw)
        for frac in (0.1, 0.5, 0.95, 0.999):
            cut = int(len(b) * frac)
            out.append((f"f{seed}_cut{frac}_eoi", b[:cut] + b"\xff\xd9"))
            out.append((f"f{seed}_cut{frac}", b[:cut]))
            out.append((f"f{seed}_rst0_at{frac}", b[:cut] + b"\xff\xd0" + b[cut:]))
            out.append((f"f{seed}_rst7_at{frac}", b[:cut] + b"\xff\xd7" + b[cut:]))
    return out


def _segments(b: bytes):
    """(marker, payload start, payload end) of every marker segment before the scan data."""
    i = 2
    while i + 4 <= len(b):
        marker, seglen = b[i + 1], int.from_bytes(b[i + 2:i + 4], "big")
        yield marker, i + 4, i + 2 + seglen
        if marker == 0xDA:
            return
        i += 2 + seglen


def _huffman_codes(b: bytes):
    """{(table class, id): {symbol: (code, length)}} from the file's DHT segments (canonical codes,
    JPEG Annex C)."""
    tables = {}
    for marker, lo, hi in _segments(b):
        if marker != 0xC4:
            continue
        p = lo
        while p < hi:
            tc, th = b[p] >> 4, b[p] & 15
            counts = b[p + 1:p + 17]
            syms = b[p + 17:p + 17 + sum(counts)]
            code, k, codes = 0, 0, {}
            for length in range(1, 17):
                for _ in range(counts[length - 1]):
                    codes[syms[k]] = (code, length)
                    code, k = code + 1, k + 1
                code <<= 1
            tables[(tc, th)] = codes
            p += 17 + sum(counts)
    return tables


def overlong_run_cases():
    """Grayscale files whose entropy-coded data holds AC runs past coefficient 63 (corrupt data:
    after a ZRL chain a run/size token lands on k = 64..78). libjpeg-turbo writes such a value to
    natural index 63 (jpeg_natural_order[] carries 16 extra 63 entries, jdhuff.c); every other
    block decodes normally. The scan is re-encoded with the file's own (standard) Huffman tables."""
    base = jpeg_bytes(photo(16, 24, 7)[..., 0], quality=90)
    codes = _huffman_codes(base)
    dc, ac = codes[(0, 0)], codes[(1, 0)]
    sos_end = max(hi for m, lo, hi in _segments(base) if m == 0xDA)

    def amp(v):  # (size category, extra bits) of a coefficient value (F.1.2.1)
        n = abs(v).bit_length()
        return n, (v if v > 0 else v + (1 << n) - 1)

    out = []
    # one token list per block of the 3 x 2 blocks: (table, symbol, value or None)
    plans = {
        "overlong_r15_s2": [[("dc", 5), ("ac", 0xF0), ("ac", 0xF0), ("ac", 0xF0), ("acv", 15, 3)],
                            [("dc", 0), ("acv", 0, 1), ("ac", 0x00)]],
        "overlong_k60_then_76": [[("dc", -3), ("ac", 0xF0), ("ac", 0xF0), ("ac", 0xF0), ("acv", 10, -2),
                                  ("acv", 15, 7)], [("dc", 2), ("acv", 2, -1), ("ac", 0x00)]],
        "overlong_exact_63": [[("dc", 1), ("ac", 0xF0), ("ac", 0xF0), ("ac", 0xF0), ("acv", 14, 9)],
                              [("dc", 0), ("ac", 0x00)]],
    }
    for name, plan in plans.items():
        bits = []

        def put(code, length):
            bits.extend((code >> (length - 1 - j)) & 1 for j in range(length))

        for blk in range(6):
            for tok in plan[blk % len(plan)]:
                if tok[0] == "dc":
                    cat, extra = amp(tok[1]) if tok[1] else (0, 0)
                    put(*dc[cat])
                    if cat:
                        put(extra, cat)
                elif tok[0] == "ac":
                    put(*ac[tok[1]])
                else:
                    cat, extra = amp(tok[2])
                    put(*ac[(tok[1] << 4) | cat])
                    put(extra, cat)
        bits.extend([1] * (-len(bits) % 8))
        data = bytearray()
        for i in range(0, len(bits), 8):
            v = int("".join(map(str, bits[i:i + 8])), 2)
            data.append(v)
            if v == 0xFF:
                data.append(0)
        out.append((name, base[:sos_end] + bytes(data) + b"\xff\xd9"))
    return out


def pillow_rgb(b: bytes) -> np.ndarray:
    with Image.open(io.BytesIO(b)) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)
