// png_core.h — K14: PNG scanline reconstruction shared by the device kernel (png.hip) and the host
// check (scripts/png_host_check.cpp), so the kernel's arithmetic is compared with Pillow on any
// machine.
//
// Reference call: the reference decodes every image file with Pillow
// (app/ml/embeddings.py:82-89, Image.open(path).convert("RGB")). A PNG's pixels are the zlib
// stream of its IDAT chunks, inflated (host, zlib: png_parse.h), then per scanline one filter byte
// and w x bpp filtered bytes; reconstruction (PNG specification, section 9 "Filtering") undoes
// filter 0 None, 1 Sub, 2 Up, 3 Average, 4 Paeth bytewise modulo 256 from the reconstructed left
// pixel a, the pixel above b and the one above-left c (0 outside the image). Pillow's
// convert("RGB") then keeps R, G, B of RGB / RGBA (alpha dropped, not composited) and replicates
// L of L / LA. Supported: bit depth 8, colour types 0 (L), 2 (RGB), 4 (LA), 6 (RGBA), not
// interlaced; anything else is decoded by Pillow on the host, as the reference does.
#pragma once

#include <cstdint>

namespace mrag_png {

constexpr int PNG_MAXW = 8192;  // widest image K14 takes (one band carry row of packed pixels in LDS)

// one byte: filter ft, filtered x, reconstructed left a / above b / above-left c. Branch-free (the
// lanes of a wave reconstruct rows with different filters): every predictor, then a select.
// Paeth's distances |p - a|, |p - b|, |p - c| with p = a + b - c are |b - c|, |a - c|, |a + b - 2c|.
__host__ __device__ inline uint32_t recon_byte(int ft, uint32_t x, uint32_t a, uint32_t b, uint32_t c) {
  const int ia = (int)a, ib = (int)b, ic = (int)c;
  const int pa = ib > ic ? ib - ic : ic - ib;
  const int pb = ia > ic ? ia - ic : ic - ia;
  const int t = ia + ib - 2 * ic;
  const int pc = t < 0 ? -t : t;
  const uint32_t paeth = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
  const uint32_t p = ft == 1 ? a : ft == 2 ? b : ft == 3 ? ((a + b) >> 1) : ft == 4 ? paeth : 0u;
  return (x + p) & 0xFFu;
}

// one pixel of bpp (1..4) bytes packed little-endian (channel 0 in the low byte)
__host__ __device__ inline uint32_t recon_pixel(int ft, uint32_t x, uint32_t a, uint32_t b, uint32_t c, int bpp) {
  uint32_t r = 0;
  for (int k = 0; k < 4; ++k) {
    if (k >= bpp) break;
    const int s = 8 * k;
    r |= recon_byte(ft, (x >> s) & 0xFF, (a >> s) & 0xFF, (b >> s) & 0xFF, (c >> s) & 0xFF) << s;
  }
  return r;
}

// Pillow's convert("RGB") of one reconstructed pixel: L / LA replicate L, RGB / RGBA keep R, G, B
__host__ __device__ inline void to_rgb(uint32_t px, int bpp, uint8_t* o) {
  if (bpp <= 2) {
    o[0] = o[1] = o[2] = (uint8_t)(px & 0xFF);
  } else {
    o[0] = (uint8_t)(px & 0xFF);
    o[1] = (uint8_t)((px >> 8) & 0xFF);
    o[2] = (uint8_t)((px >> 16) & 0xFF);
  }
}

// the bpp filtered bytes of one pixel, packed
__host__ __device__ inline uint32_t load_pixel(const uint8_t* p, int bpp) {
  uint32_t v = p[0];
  if (bpp > 1) v |= (uint32_t)p[1] << 8;
  if (bpp > 2) v |= (uint32_t)p[2] << 16;
  if (bpp > 3) v |= (uint32_t)p[3] << 24;
  return v;
}

// Sequential reconstruction of a whole image (host check): raw = h rows of 1 + w * bpp bytes.
inline void unfilter_rgb_host(const uint8_t* raw, int w, int h, int bpp, uint8_t* rgb) {
  const int64_t stride = 1 + (int64_t)w * bpp;
  uint32_t* prev = new uint32_t[(size_t)w + 1]();
  uint32_t* cur = new uint32_t[(size_t)w + 1]();
  for (int r = 0; r < h; ++r) {
    const uint8_t* row = raw + r * stride;
    const int ft = row[0];
    for (int j = 0; j < w; ++j) {
      const uint32_t a = j > 0 ? cur[j - 1] : 0, b = r > 0 ? prev[j] : 0, c = (r > 0 && j > 0) ? prev[j - 1] : 0;
      cur[j] = recon_pixel(ft, load_pixel(row + 1 + (int64_t)j * bpp, bpp), a, b, c, bpp);
      to_rgb(cur[j], bpp, rgb + ((int64_t)r * w + j) * 3);
    }
    uint32_t* t = prev;
    prev = cur;
    cur = t;
  }
  delete[] prev;
  delete[] cur;
}

}  // namespace mrag_png
