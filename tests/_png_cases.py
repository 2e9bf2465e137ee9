"""Synthetic PNG files for the K14 tests (written by Pillow, the reference's decoder): every colour
type K14 reconstructs, sizes around the 64-row band and the prefetch distance, photo-like and noise
content (Pillow's encoder picks the filter per row, so all five filters occur), zlib levels 0
(stored blocks) to 9, several IDAT chunks; plus files K14 must leave to Pillow."""
from __future__ import annotations

import io
import zlib

import numpy as np
from PIL import Image

from _jpeg_cases import photo


def png_bytes(a: np.ndarray, mode: str, **kw) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(a, mode).save(buf, "PNG", **kw)
    return buf.getvalue()


def _content(h: int, w: int, seed: int, noise: bool) -> np.ndarray:
    if noise:
        return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    return photo(h, w, seed)


def _chunk(t: bytes, d: bytes) -> bytes:
    return len(d).to_bytes(4, "big") + t + d + zlib.crc32(t + d).to_bytes(4, "big")


def filtered_png(pix: np.ndarray, ctype: int, filters=None, idat_size: int = 1 << 15) -> bytes:
    """A PNG written here (not by Pillow) with a chosen filter per scanline — by default filter
    r % 5 on row r, so None, Sub, Up, Average and Paeth all occur — split into IDAT chunks of
    idat_size bytes. pix: h x w x bpp u8 (bpp 1, 2, 3, 4 for colour types 0, 4, 2, 6)."""
    h, w, bpp = pix.shape
    x = pix.reshape(h, w * bpp).astype(np.int32)
    rows = []
    for r in range(h):
        ft = (r % 5) if filters is None else filters[r % len(filters)]
        up = x[r - 1] if r > 0 else np.zeros(w * bpp, np.int32)
        left = np.concatenate([np.zeros(bpp, np.int32), x[r, :-bpp]])
        ul = np.concatenate([np.zeros(bpp, np.int32), up[:-bpp]])
        if ft == 0:
            pred = 0
        elif ft == 1:
            pred = left
        elif ft == 2:
            pred = up
        elif ft == 3:
            pred = (left + up) // 2
        else:
            p = left + up - ul
            pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
        rows.append(bytes([ft]) + ((x[r] - pred) & 0xFF).astype(np.uint8).tobytes())
    z = zlib.compress(b"".join(rows), 6)
    ihdr = w.to_bytes(4, "big") + h.to_bytes(4, "big") + bytes([8, ctype, 0, 0, 0])
    idats = b"".join(_chunk(b"IDAT", z[i:i + idat_size]) for i in range(0, len(z), idat_size))
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + idats + _chunk(b"IEND", b"")


def supported_cases():
    out = []
    for i, (h, w) in enumerate([(1, 1), (5, 3), (70, 9), (130, 257), (300, 201)]):
        for ctype, bpp in ((0, 1), (4, 2), (2, 3), (6, 4)):
            pix = np.random.default_rng(80 + i).integers(0, 256, (h, w, bpp), dtype=np.uint8)
            if i % 2:
                pix = np.repeat(photo(h, w, 90 + i), 2, axis=-1)[..., :bpp].copy()
            out.append((f"filters{h}x{w}_ct{ctype}", filtered_png(pix, ctype, idat_size=997)))
    sizes = [(1, 1), (3, 7), (9, 17), (64, 5), (65, 33), (130, 70), (201, 300), (480, 640), (7, 1500)]
    for i, (h, w) in enumerate(sizes):
        for noise in (False, True):
            rgb = _content(h, w, 20 + i, noise)
            alpha = np.random.default_rng(60 + i).integers(0, 256, (h, w, 1), dtype=np.uint8)
            tag = f"{'noise' if noise else 'photo'}{h}x{w}"
            out.append((f"{tag}_RGB", png_bytes(rgb, "RGB")))
            out.append((f"{tag}_RGBA", png_bytes(np.concatenate([rgb, alpha], -1), "RGBA")))
            out.append((f"{tag}_L", png_bytes(rgb[..., 1].copy(), "L")))
            out.append((f"{tag}_LA", png_bytes(np.concatenate([rgb[..., :1], alpha], -1), "LA")))
    a = photo(480, 640, 3)
    for lvl in (0, 1, 9):
        out.append((f"level{lvl}", png_bytes(a, "RGB", compress_level=lvl)))
    out.append(("optimize", png_bytes(a, "RGB", optimize=True)))
    return out


def unsupported_cases():
    a = photo(40, 50, 7)
    pal = Image.fromarray(a).convert("P", palette=Image.ADAPTIVE, colors=200)
    b_pal = io.BytesIO()
    pal.save(b_pal, "PNG")
    b16 = io.BytesIO()
    Image.fromarray(a[..., 0].astype(np.uint16) * 257).save(b16, "PNG")
    bw = io.BytesIO()
    Image.fromarray(a[..., 0] > 128).save(bw, "PNG")
    good = png_bytes(a, "RGB")
    bad_crc = bytearray(good)
    bad_crc[40] ^= 0x55  # the chunk type after IHDR: an unknown chunk with a bad CRC
    return [("palette", b_pal.getvalue()), ("gray16", b16.getvalue()), ("bilevel", bw.getvalue()),
            ("bad_crc", bytes(bad_crc))]


def bad_idat_crc_case():
    """A PNG whose IDAT chunk CRC is wrong but whose data is intact: Pillow does not check IDAT
    CRCs and decodes it, so K14 takes it too."""
    a = photo(40, 50, 9)
    good = bytearray(png_bytes(a, "RGB"))
    pos = 8
    while good[pos + 4:pos + 8] != b"IDAT":
        pos += 12 + int.from_bytes(good[pos:pos + 4], "big")
    n = int.from_bytes(good[pos:pos + 4], "big")
    good[pos + 8 + n] ^= 0xFF  # first byte of that chunk's CRC
    return bytes(good)


def truncated_stream_case():
    """A PNG whose zlib stream ends before the last scanline, with valid CRCs (probe 1, inflate 0)."""
    a = photo(40, 50, 8)
    raw = b"".join(b"\x00" + a[r].tobytes() for r in range(40))
    data = zlib.compress(raw[:len(raw) // 2])
    ihdr = (50).to_bytes(4, "big") + (40).to_bytes(4, "big") + bytes([8, 2, 0, 0, 0])
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", data) + _chunk(b"IEND", b"")


def split_idat_case(tail_complete: bool = False) -> bytes:
    """A PNG whose IDAT chunks are not consecutive (a tEXt chunk between two runs). Pillow reads
    only the first run (PngImageFile.load_read stops at the other chunk) and raises "image file is
    truncated" when scanlines are still missing, so K14 must leave such a file to Pillow.
    tail_complete: the first run already holds the whole stream (the second IDAT is empty), which
    Pillow decodes — K14 refuses it as well and Pillow decides."""
    pix = _content(40, 30, 3, False)
    b = filtered_png(pix, 2, idat_size=1 << 20 if tail_complete else 300)
    sig, rest = b[:8], b[8:]
    chunks, p = [], 0
    while p < len(rest):
        n = int.from_bytes(rest[p:p + 4], "big")
        chunks.append(rest[p:p + 12 + n])
        p += 12 + n
    idat = [i for i, c in enumerate(chunks) if c[4:8] == b"IDAT"]
    text = _chunk(b"tEXt", b"k\0v")
    if tail_complete:
        chunks.insert(idat[-1] + 1, text + _chunk(b"IDAT", b""))
    else:
        assert len(idat) >= 2
        chunks.insert(idat[0] + 1, text)
    return sig + b"".join(chunks)


def pillow_rgb(b: bytes) -> np.ndarray:
    with Image.open(io.BytesIO(b)) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)
