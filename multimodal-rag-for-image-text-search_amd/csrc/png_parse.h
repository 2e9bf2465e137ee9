// png_parse.h — host side of K14: chunk parsing (PNG specification sections 5 and 11: signature,
// length / type / data / CRC-32 chunks, IHDR first, IDAT data concatenated into one zlib stream)
// and the zlib inflate of the IDAT stream into the filtered scanlines. Used by csrc/png.hip and
// scripts/png_host_check.cpp.
#pragma once

#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "inflate.h"
#include "png_core.h"

namespace mrag_png {

struct PngParsed {
  int32_t width = 0, height = 0, bpp = 0, ctype = -1;
  std::vector<std::pair<int64_t, int64_t>> idat;  // (offset, length) of every IDAT chunk's data
  int64_t raw_bytes = 0;                           // h x (1 + w x bpp)
  std::string why;
};

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

inline bool png_fail(PngParsed& P, const char* why) {
  P.why = why;
  return false;
}

// Parse one file; true when K14 decodes it. check_crc: verify the CRC-32 of every chunk but IDAT
// (the probe does; a file with a bad one goes to Pillow, which raises for it).
inline bool png_parse(const uint8_t* d, int64_t n, PngParsed& P, bool check_crc) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  if (n < 8 || std::memcmp(d, sig, 8) != 0) return png_fail(P, "not a PNG");
  int64_t pos = 8;
  bool ihdr = false, iend = false, idat_gap = false;
  while (pos + 12 <= n) {
    const int64_t len = be32(d + pos);
    const uint8_t* type = d + pos + 4;
    if (len > 0x7fffffff || pos + 12 + len > n) return png_fail(P, "truncated chunk");
    const uint8_t* data = d + pos + 8;
    // Pillow checks the CRC of every chunk it reads except IDAT (PngImageFile.load_read skips
    // those four bytes): the same here, so a file goes to Pillow exactly when Pillow would raise
    if (check_crc && std::memcmp(type, "IDAT", 4) != 0) {
      const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), type, (uInt)(4 + len));
      if (crc != be32(data + len)) return png_fail(P, "bad CRC");
    }
    if (std::memcmp(type, "IHDR", 4) == 0) {
      if (ihdr || pos != 8 || len != 13) return png_fail(P, "IHDR");
      P.width = (int32_t)be32(data);
      P.height = (int32_t)be32(data + 4);
      const int depth = data[8], ct = data[9];
      if (be32(data) == 0 || be32(data + 4) == 0 || be32(data) > (uint32_t)PNG_MAXW || be32(data + 4) > 65535u)
        return png_fail(P, "size");
      if (depth != 8) return png_fail(P, "bit depth other than 8");
      if (ct != 0 && ct != 2 && ct != 4 && ct != 6) return png_fail(P, "palette colour type");
      if (data[10] != 0 || data[11] != 0) return png_fail(P, "compression / filter method");
      if (data[12] != 0) return png_fail(P, "interlaced");
      P.ctype = ct;
      P.bpp = ct == 0 ? 1 : ct == 2 ? 3 : ct == 4 ? 2 : 4;
      ihdr = true;
    } else if (!ihdr) {
      return png_fail(P, "IHDR not first");
    } else if (std::memcmp(type, "IDAT", 4) == 0) {
      // Pillow reads only the first run of consecutive IDAT chunks (PngImageFile.load_read stops
      // at the next other chunk: "image file is truncated" if scanlines are still missing), so a
      // file with a second run goes to Pillow, which decides what it is
      if (idat_gap) return png_fail(P, "IDAT chunks not consecutive");
      P.idat.emplace_back(pos + 8, len);
    } else if (std::memcmp(type, "IEND", 4) == 0) {
      iend = true;
      break;
    } else if (!P.idat.empty()) {
      idat_gap = true;
    }
    pos += 12 + len;
  }
  if (!ihdr || P.idat.empty()) return png_fail(P, "no image data");
  (void)iend;  // a missing IEND after complete image data is no error for Pillow either
  P.raw_bytes = (int64_t)P.height * (1 + (int64_t)P.width * P.bpp);
  return true;
}

// Inflate the IDAT stream into raw with zlib (the reference implementation of the format).
inline bool png_inflate_zlib(const uint8_t* d, const PngParsed& P, uint8_t* raw) {
  z_stream z;
  std::memset(&z, 0, sizeof(z));
  if (inflateInit(&z) != Z_OK) return false;
  z.next_out = raw;
  int64_t left = P.raw_bytes;
  bool ok = false, stop = false;
  for (size_t i = 0; i < P.idat.size() && !stop; ++i) {
    z.next_in = const_cast<Bytef*>(d + P.idat[i].first);
    z.avail_in = (uInt)P.idat[i].second;
    while (z.avail_in > 0) {
      const uInt out_take = (uInt)(left > (1 << 30) ? (1 << 30) : left);
      z.avail_out = out_take;
      const int rc = inflate(&z, Z_NO_FLUSH);
      left -= out_take - z.avail_out;
      if (left == 0) {  // every scanline inflated; an error zlib found after them (a bad code, the
        ok = rc == Z_OK || rc == Z_STREAM_END || rc == Z_BUF_ERROR;  // Adler-32) is one for Pillow too
        stop = true;
        break;
      }
      if (rc != Z_OK) {  // stream end before the last scanline, corrupt data, or no progress
        stop = true;
        break;
      }
    }
  }
  inflateEnd(&z);
  return ok;
}

// Inflate the IDAT stream into raw (P.raw_bytes bytes): the IDAT data concatenated and inflated by
// fast_inflate (inflate.h), zlib when that reports an error (so a stream is refused only when
// zlib refuses it). False when the stream is corrupt or ends early, or a scanline's filter byte is
// not 0..4 (the caller then lets Pillow decode the file).
inline bool png_inflate(const uint8_t* d, const PngParsed& P, uint8_t* raw) {
  static thread_local std::vector<uint8_t> z;
  size_t n = 0;
  for (const auto& c : P.idat) n += (size_t)c.second;
  z.resize(n);
  size_t o = 0;
  for (const auto& c : P.idat) {
    std::memcpy(z.data() + o, d + c.first, (size_t)c.second);
    o += (size_t)c.second;
  }
  if (!fast_inflate(z.data(), n, raw, (size_t)P.raw_bytes) && !png_inflate_zlib(d, P, raw)) return false;
  const int64_t stride = 1 + (int64_t)P.width * P.bpp;
  for (int64_t r = 0; r < P.height; ++r)
    if (raw[r * stride] > 4) return false;
  return true;
}

}  // namespace mrag_png
