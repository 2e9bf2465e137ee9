// Host run of K13's decode arithmetic (csrc/jpeg_core.h + jpeg_parse.h), for checking it against
// Pillow byte for byte on any machine (tests/test_jpeg_cpu.py): the same functions the device
// kernels call, executed on the CPU. Test infrastructure: nothing in the library calls it.
//   hipcc -O2 -fPIC -shared -I<pkg>/csrc scripts/jpeg_host_check.hip -o <out>.so
#include <cstdint>
#include <cstring>
#include <vector>

#include "jpeg_parse.h"

using namespace mrag_jpeg;

// 1: decoded into rgb (w * h * 3 bytes, capacity cap); 0: unsupported; -1: rgb too small.
extern "C" int jpeg_host_decode(const uint8_t* d, int64_t n, uint8_t* rgb, int64_t cap, int32_t* wh) {
  Parsed P;
  if (!parse(d, n, P)) return 0;
  const Image& im = P.img;
  wh[0] = im.width;
  wh[1] = im.height;
  if (cap < (int64_t)im.width * im.height * 3) return -1;
  std::vector<int16_t> coef((size_t)P.coef_blocks * 64, 0);
  std::vector<uint8_t> padded((size_t)n + 64, 0);  // Bits reads up to 32 B past a segment
  std::memcpy(padded.data(), d, (size_t)n);
  for (const Segment& s : P.segs) decode_segment(im, padded.data() + s.off, s.len, s.mcu0, s.mcus, coef.data());
  std::vector<uint8_t> planes((size_t)P.plane_bytes, 0);
  for (int c = 0; c < im.ncomp; ++c)
    for (int64_t b = 0; b < (int64_t)im.comp[c].bw * im.comp[c].bh; ++b) idct_block(im, coef.data(), planes.data(), c, b);
  for (int y = 0; y < im.height; ++y)
    for (int x = 0; x < im.width; ++x) color_pixel(im, planes.data(), x, y, rgb + ((int64_t)y * im.width + x) * 3);
  return 1;
}

// Entropy decoding only (into caller memory of coef_blocks * 64 int16): for timing the host share.
extern "C" int64_t jpeg_host_entropy(const uint8_t* d, int64_t n, int16_t* coef, int64_t cap_blocks) {
  Parsed P;
  if (!parse(d, n, P) || P.coef_blocks > cap_blocks) return -1;
  std::vector<uint8_t> padded((size_t)n + 64, 0);
  std::memcpy(padded.data(), d, (size_t)n);
  std::memset(coef, 0, (size_t)P.coef_blocks * 128);
  for (const Segment& s : P.segs) decode_segment(P.img, padded.data() + s.off, s.len, s.mcu0, s.mcus, coef);
  return P.coef_blocks;
}
