// Host run of K13's decode arithmetic (csrc/jpeg_core.h + jpeg_parse.h), for checking it against
// Pillow byte for byte on any machine (tests/test_jpeg_cpu.py): the same functions the device
// kernels call, executed on the CPU. Test infrastructure: nothing in the library calls it.
//   hipcc -O2 -fPIC -shared -I<pkg>/csrc scripts/jpeg_host_check.hip -o <out>.so
#include <cstdint>
#include <cstring>
#include <vector>

#include "jpeg_parse.h"

using namespace mrag_jpeg;

// Every segment unstuffed into a 16-byte aligned, zero-padded copy, as jpeg.hip stages it for K13a.
static void decode_par(const Parsed& P, const uint8_t* d, int16_t* coef, int* max_rounds, int* lanes) {
  for (const Segment& s : P.segs) {
    std::vector<uint8_t> u((size_t)s.len + 32, 0);
    const int64_t ulen = unstuff(d + s.off, s.len, u.data());
    const int r = decode_segment_par(P.img, u.data(), (uint32_t)ulen, s.mcu0, s.mcus, coef);
    if (max_rounds && r > *max_rounds) *max_rounds = r;
    if (lanes) {
      int nl;
      uint32_t chunk;
      par_geom((uint32_t)ulen * 8u, nl, chunk);
      *lanes += nl;
    }
  }
}

// 1: decoded into rgb (w * h * 3 bytes, capacity cap); 0: unsupported; -1: rgb too small.
// par = 1: entropy decoding by the K13a lane emulation instead of the sequential decoder.
extern "C" int jpeg_host_decode_mode(const uint8_t* d, int64_t n, uint8_t* rgb, int64_t cap, int32_t* wh, int par);
extern "C" int jpeg_host_decode(const uint8_t* d, int64_t n, uint8_t* rgb, int64_t cap, int32_t* wh) {
  return jpeg_host_decode_mode(d, n, rgb, cap, wh, 0);
}
extern "C" int jpeg_host_decode_mode(const uint8_t* d, int64_t n, uint8_t* rgb, int64_t cap, int32_t* wh, int par) {
  Parsed P;
  if (!parse(d, n, P)) return 0;
  const Image& im = P.img;
  wh[0] = im.width;
  wh[1] = im.height;
  if (cap < (int64_t)im.width * im.height * 3) return -1;
  std::vector<int16_t> coef((size_t)P.coef_blocks * 64, 0);
  std::vector<uint8_t> padded((size_t)n + 64, 0);  // Bits reads up to 32 B past a segment
  std::memcpy(padded.data(), d, (size_t)n);
  if (par)
    decode_par(P, d, coef.data(), nullptr, nullptr);
  else
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

// Coefficients of the sequential decoder vs the K13a lane emulation: 1 identical, 0 different,
// -1 unsupported. stats[0] = most resynchronisation rounds of a segment, stats[1] = lanes used.
extern "C" int jpeg_host_par_check(const uint8_t* d, int64_t n, int32_t* stats) {
  Parsed P;
  if (!parse(d, n, P)) return -1;
  std::vector<uint8_t> padded((size_t)n + 64, 0);
  std::memcpy(padded.data(), d, (size_t)n);
  std::vector<int16_t> a((size_t)P.coef_blocks * 64, 0), b((size_t)P.coef_blocks * 64, 0);
  for (const Segment& s : P.segs) decode_segment(P.img, padded.data() + s.off, s.len, s.mcu0, s.mcus, a.data());
  int rounds = 0, lanes = 0;
  decode_par(P, d, b.data(), &rounds, &lanes);
  stats[0] = rounds;
  stats[1] = lanes;
  return a == b ? 1 : 0;
}
