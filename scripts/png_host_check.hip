// Host run of K14's arithmetic (csrc/png_core.h + png_parse.h), for checking it against Pillow
// byte for byte on any machine (tests/test_png_cpu.py): the chunk parse, the zlib inflate and the
// scanline reconstruction + RGB conversion the device kernel performs, executed on the CPU.
// Test infrastructure: nothing in the library calls it.
//   hipcc -O2 -fPIC -shared -I<pkg>/csrc scripts/png_host_check.hip -o <out>.so -lz
#include <cstdint>
#include <vector>

#include "png_parse.h"

using namespace mrag_png;

// 1: decoded into rgb (w * h * 3 bytes, capacity cap); 0: not for K14; -1: rgb too small.
extern "C" int png_host_decode(const uint8_t* d, int64_t n, uint8_t* rgb, int64_t cap, int32_t* wh) {
  PngParsed P;
  if (!png_parse(d, n, P, true)) return 0;
  wh[0] = P.width;
  wh[1] = P.height;
  if (cap < (int64_t)P.width * P.height * 3) return -1;
  std::vector<uint8_t> raw((size_t)P.raw_bytes);
  if (!png_inflate(d, P, raw.data())) return 0;
  unfilter_rgb_host(raw.data(), P.width, P.height, P.bpp, rgb);
  return 1;
}

// fast_inflate alone (tests compare it with Python's zlib): 1 when out_len bytes were produced.
extern "C" int png_fast_inflate(const uint8_t* in, int64_t in_len, uint8_t* out, int64_t out_len) {
  return fast_inflate(in, (size_t)in_len, out, (size_t)out_len) ? 1 : 0;
}

// zlib's inflate of the same stream into out (timing comparison)
extern "C" int png_zlib_inflate(const uint8_t* in, int64_t in_len, uint8_t* out, int64_t out_len) {
  z_stream z;
  std::memset(&z, 0, sizeof(z));
  if (inflateInit(&z) != Z_OK) return 0;
  z.next_in = const_cast<Bytef*>(in);
  z.avail_in = (uInt)in_len;
  z.next_out = out;
  z.avail_out = (uInt)out_len;
  const int rc = inflate(&z, Z_NO_FLUSH);
  const bool ok = z.avail_out == 0 && (rc == Z_OK || rc == Z_STREAM_END || rc == Z_BUF_ERROR);
  inflateEnd(&z);
  return ok ? 1 : 0;
}
