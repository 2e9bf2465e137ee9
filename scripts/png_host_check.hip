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
