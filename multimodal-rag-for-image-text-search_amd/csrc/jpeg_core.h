// jpeg_core.h — K13: baseline JPEG decode arithmetic shared by the device kernels (jpeg.hip) and
// the host check (scripts/jpeg_host_check.hip), so the kernels are validated byte for byte
// against Pillow on any machine.
//
// Reference call: the reference decodes every image file with Pillow
// (app/ml/embeddings.py:82-89, Image.open(path).convert("RGB")); Pillow 12.2 decodes JPEG with
// libjpeg-turbo's defaults: Huffman entropy decoding, the "islow" integer IDCT (LL&M, 13-bit
// constants, 2 guard bits in pass 1), "fancy" triangular chroma upsampling (h2v1 / h2v2) with edge
// replication, and the fixed-point YCbCr -> RGB tables (16-bit). Those published algorithms are
// restated here; the output is the RGB array Pillow returns, byte for byte
// (tests/test_jpeg_cpu.py, tests/test_jpeg_gpu.py).
//
// Supported here: baseline / extended sequential Huffman, 8-bit, one interleaved scan, 1 or 3
// components, chroma 4:4:4, 4:2:2 (h2v1) and 4:2:0 (h2v2), restart intervals. Anything else is
// reported unsupported by the parser (jpeg.hip) and the caller decodes that file on the host
// with Pillow, exactly as the reference does.
#pragma once

#include <cstdint>

namespace mrag_jpeg {

constexpr int MAX_COMP = 3;

// Canonical Huffman table: a 9-bit lookahead (len << 8 | symbol, len 0 = longer code; two 16-bit
// entries per word) and the maxcode / value-offset arrays of the slow path (JPEG Annex F.2.2.3),
// symbols four per word. Packed so that the four tables of an image (5.6 KB) and the entropy
// bytes the device decoder streams stay in the scalar cache, which two CUs share.
struct Huff {
  uint32_t look2[256];
  int32_t maxcode[18];  // maxcode[l]: largest code of length l (-1 if none); [17] sentinel
  int32_t valoff[17];   // index into vals of the first code of length l, minus that code
  uint32_t vals4[64];
  __host__ __device__ uint32_t look(uint32_t i) const { return (look2[i >> 1] >> ((i & 1) * 16)) & 0xFFFF; }
  __host__ __device__ uint32_t val(uint32_t i) const { return (vals4[i >> 2] >> ((i & 3) * 8)) & 0xFF; }
};

struct Comp {
  int32_t h, v;              // sampling factors
  int32_t tq, td, ta;        // quant / DC / AC table ids
  int32_t bw, bh;            // blocks per row / column in the coefficient plane (MCU padded)
  int32_t dw, dh;            // downsampled width / height (samples)
  int64_t coef_off;          // first block of this component in the image's coefficient buffer
  int64_t plane_off;         // first sample of this component's plane (bw*8 x bh*8)
};

// One image: everything the device needs, built by the host parser.
struct Image {
  int32_t width, height, ncomp;
  int32_t hmax, vmax;
  int32_t mcux, mcuy;         // MCUs per row / column
  int32_t restart;            // restart interval in MCUs (0 = none)
  int32_t nseg;               // entropy-coded segments (restart intervals)
  int32_t seg0;               // first entry of this image in the segment table
  int32_t blocks_per_mcu;
  Comp comp[MAX_COMP];
  uint16_t quant[4][64];      // natural order
  Huff dc[2], ac[2];
  int64_t ecs_off;            // this image's entropy-coded bytes in the batch buffer
  int64_t coef_off;           // first block (64 int16) in the batch coefficient buffer
  int64_t plane_off;          // first sample in the batch plane buffer
  int64_t rgb_off;            // first byte of the H x W x 3 output
};

// Natural (row-major) index of the k-th zig-zag coefficient (four per word, see Huff).
__host__ __device__ inline int zigzag(int k) {
  constexpr uint32_t z4[16] = {0x10080100u, 0x0a030209u, 0x19201811u, 0x05040b12u, 0x211a130cu, 0x22293028u,
                               0x060d141bu, 0x1c150e07u, 0x38312a23u, 0x242b3239u, 0x170f161du, 0x332c251eu,
                               0x2d343b3au, 0x2e271f26u, 0x363d3c35u, 0x3f3e372fu};
  return (int)((z4[k >> 2] >> ((k & 3) * 8)) & 0xFF);
}

// Bit reader over one entropy-coded segment (byte stuffing 0xFF00 -> 0xFF; a marker or the end
// of the segment feeds zero bits, as libjpeg does for truncated data). Bytes come through a
// 16-byte window with the next 16 bytes already requested: on the device the decoder is one
// serial chain, so a load per byte would expose the memory latency on every byte. The source
// must be readable 32 bytes past the segment end (the callers pad their buffers).
struct Bits {
  const uint8_t* base;  // 16-byte aligned, at or before the segment's first byte
  int64_t off0;         // segment start - base
  int64_t n, pos;       // segment length, next byte (segment-relative)
  int64_t wbase;        // window start (base-relative, multiple of 16)
  uint64_t w0, w1, x0, x1;
  uint64_t buf;
  int32_t cnt;
  __host__ __device__ void load16(int64_t at, uint64_t& a, uint64_t& b) const {
#if defined(__HIP_DEVICE_COMPILE__)
    // device: the decoder is wave-uniform, so the window comes through the scalar cache; the
    // coefficient stores are vector stores, and the two no longer share a wait counter
    typedef const __attribute__((address_space(4))) uint64_t* cptr;
    const cptr q = (cptr)(base + at);
#else
    const uint64_t* q = (const uint64_t*)(base + at);
#endif
    a = q[0];
    b = q[1];
  }
  __host__ __device__ void init(const uint8_t* data, int64_t len) {
    base = (const uint8_t*)((uintptr_t)data & ~(uintptr_t)15);
    off0 = data - base;
    n = len;
    pos = 0;
    wbase = 0;
    load16(0, w0, w1);
    load16(16, x0, x1);
    buf = 0;
    cnt = 0;
  }
  __host__ __device__ uint32_t byte_at(int64_t rel) {  // rel: at most 2 past the last call's
    const int64_t a = off0 + rel;
    // one advance at most (fill reads byte by byte): the window load is not waited for until
    // the window after it is needed
    if (a >= wbase + 16) {
      w0 = x0;
      w1 = x1;
      wbase += 16;
      load16(wbase + 16, x0, x1);
    }
    const int k = (int)(a - wbase);
    return (uint32_t)((k < 8 ? (w0 >> (8 * k)) : (w1 >> (8 * (k - 8)))) & 0xFF);
  }
  __host__ __device__ void fill() {  // cnt > 56 on return
    while (cnt <= 56) {
      uint32_t b = 0;
      if (pos < n) {
        b = byte_at(pos);
        if (b == 0xFF) {
          const uint32_t b2 = pos + 1 < n ? byte_at(pos + 1) : 0xD9u;
          if (b2 == 0x00) {
            pos += 2;
          } else {
            b = 0;  // marker: stay on it, zeros from here
            n = pos;
          }
        } else {
          ++pos;
        }
      }
      buf |= (uint64_t)b << (56 - cnt);
      cnt += 8;
    }
  }
  __host__ __device__ uint32_t peek(int k) { return (uint32_t)(buf >> (64 - k)); }
  __host__ __device__ void skip(int k) {
    buf <<= k;
    cnt -= k;
  }
  __host__ __device__ uint32_t get(int k) {  // k <= 16, after fill()
    if (k == 0) return 0;
    const uint32_t v = peek(k);
    skip(k);
    return v;
  }
  __host__ __device__ int decode(const Huff& h) {
    if (cnt < 16) fill();
    const uint32_t e = h.look(peek(9));
    if (e >> 8) {
      skip((int)(e >> 8));
      return (int)(e & 0xFF);
    }
    int l = 10;
    int32_t code = (int32_t)peek(10);
    while (l <= 16 && code > h.maxcode[l]) {
      ++l;
      code = (int32_t)peek(l);
    }
    if (l > 16) {  // corrupt code: libjpeg warns and returns 0
      skip(16);
      return 0;
    }
    skip(l);
    return (int)h.val((uint32_t)(code + h.valoff[l]) & 0xFF);
  }
};

// (x, s) -> signed coefficient (JPEG F.2.2.1 EXTEND)
__host__ __device__ inline int extend(int x, int s) { return s == 0 ? 0 : (x < (1 << (s - 1)) ? x - (1 << s) + 1 : x); }

// Decode one 8x8 block: DC predictor in/out, coefficients (natural order, not dequantized) out.
// An AC run past index 63 (corrupt data) is dropped, as libjpeg drops it.
__host__ __device__ inline void decode_block(Bits& br, const Huff& dc, const Huff& ac, int& pred, int16_t* coef) {
  const int s = br.decode(dc);
  if (br.cnt < 16) br.fill();
  const int diff = extend((int)br.get(s), s);
  pred += diff;
  coef[0] = (int16_t)pred;
  for (int k = 1; k < 64;) {
    const int rs = br.decode(ac);
    const int r = rs >> 4, sz = rs & 15;
    if (sz) {
      k += r;
      if (br.cnt < 16) br.fill();
      const int v = extend((int)br.get(sz), sz);
      if (k < 64) coef[zigzag(k)] = (int16_t)v;
      ++k;
    } else {
      if (r != 15) break;  // EOB
      k += 16;
    }
  }
}

// islow IDCT of one block (coefficients natural order, quant natural order) -> 8x8 samples with
// libjpeg's range limiting (index masked to 10 bits, then the post-IDCT table).
__host__ __device__ inline uint8_t idct_limit(int32_t x) {
  const int idx = x & 1023;
  if (idx < 128) return (uint8_t)(idx + 128);
  if (idx < 512) return 255;
  if (idx < 896) return 0;
  return (uint8_t)(idx - 896);
}

__host__ __device__ inline void idct_islow(const int16_t* coef, const uint16_t* q, uint8_t* out, int64_t stride) {
  constexpr int CB = 13, P1 = 2;
  // libjpeg's JLONG is 64-bit on LP64 hosts: the products are formed in int64 and the pass-1
  // results truncated to int, as its workspace is
  typedef int64_t L;
  constexpr L F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
              F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) {
    const int16_t* in = coef + c;
    const uint16_t* qq = q + c;
    if (in[8] == 0 && in[16] == 0 && in[24] == 0 && in[32] == 0 && in[40] == 0 && in[48] == 0 && in[56] == 0) {
      const int32_t dc = (int32_t)in[0] * (int32_t)qq[0] * (1 << P1);
      for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
      continue;
    }
    L z2 = (L)((int32_t)in[16] * qq[16]), z3 = (L)((int32_t)in[48] * qq[48]);
    L z1 = (z2 + z3) * F0541;
    L tmp2 = z1 + z3 * (-F1847);
    L tmp3 = z1 + z2 * F0765;
    z2 = (int32_t)in[0] * qq[0];
    z3 = (int32_t)in[32] * qq[32];
    L tmp0 = (z2 + z3) * (1 << CB);
    L tmp1 = (z2 - z3) * (1 << CB);
    const L tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = (int32_t)in[56] * qq[56];
    tmp1 = (int32_t)in[40] * qq[40];
    tmp2 = (int32_t)in[24] * qq[24];
    tmp3 = (int32_t)in[8] * qq[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    L z4 = tmp1 + tmp3;
    const L z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int SH = CB - P1;
    constexpr L RD = (L)1 << (SH - 1);
    ws[0 * 8 + c] = (int32_t)((tmp10 + tmp3 + RD) >> SH);
    ws[7 * 8 + c] = (int32_t)((tmp10 - tmp3 + RD) >> SH);
    ws[1 * 8 + c] = (int32_t)((tmp11 + tmp2 + RD) >> SH);
    ws[6 * 8 + c] = (int32_t)((tmp11 - tmp2 + RD) >> SH);
    ws[2 * 8 + c] = (int32_t)((tmp12 + tmp1 + RD) >> SH);
    ws[5 * 8 + c] = (int32_t)((tmp12 - tmp1 + RD) >> SH);
    ws[3 * 8 + c] = (int32_t)((tmp13 + tmp0 + RD) >> SH);
    ws[4 * 8 + c] = (int32_t)((tmp13 - tmp0 + RD) >> SH);
  }
  for (int r = 0; r < 8; ++r) {
    const int32_t* w = ws + r * 8;
    uint8_t* o = out + r * stride;
    if (w[1] == 0 && w[2] == 0 && w[3] == 0 && w[4] == 0 && w[5] == 0 && w[6] == 0 && w[7] == 0) {
      constexpr int SH0 = P1 + 3;
      const uint8_t v = idct_limit((int32_t)(((L)w[0] + ((L)1 << (SH0 - 1))) >> SH0));
      for (int c = 0; c < 8; ++c) o[c] = v;
      continue;
    }
    L z2 = w[2], z3 = w[6];
    L z1 = (z2 + z3) * F0541;
    L tmp2 = z1 + z3 * (-F1847);
    L tmp3 = z1 + z2 * F0765;
    L tmp0 = ((L)w[0] + (L)w[4]) * (1 << CB);
    L tmp1 = ((L)w[0] - (L)w[4]) * (1 << CB);
    const L tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    L z4 = tmp1 + tmp3;
    const L z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int SH = CB + P1 + 3;
    constexpr L RD = (L)1 << (SH - 1);
    o[0] = idct_limit((int32_t)((tmp10 + tmp3 + RD) >> SH));
    o[7] = idct_limit((int32_t)((tmp10 - tmp3 + RD) >> SH));
    o[1] = idct_limit((int32_t)((tmp11 + tmp2 + RD) >> SH));
    o[6] = idct_limit((int32_t)((tmp11 - tmp2 + RD) >> SH));
    o[2] = idct_limit((int32_t)((tmp12 + tmp1 + RD) >> SH));
    o[5] = idct_limit((int32_t)((tmp12 - tmp1 + RD) >> SH));
    o[3] = idct_limit((int32_t)((tmp13 + tmp0 + RD) >> SH));
    o[4] = idct_limit((int32_t)((tmp13 - tmp0 + RD) >> SH));
  }
}

// One upsampled chroma sample at output (x, y) of a component with factors (ch, cv) against
// (hmax, vmax): 1 (no upsampling), h2v1 or h2v2 fancy upsampling of plane `pl` (stride ps, the
// component's downsampled dw x dh, edges replicated).
__host__ __device__ inline int chroma_at(const uint8_t* pl, int64_t ps, int dw, int dh, int hx, int vy, int x,
                                         int y) {
  if (hx == 1 && vy == 1) return pl[(int64_t)y * ps + x];
  if (hx == 2 && vy == 1) {  // h2v1: output column x from input column x >> 1
    const int ic = x >> 1;
    const uint8_t* r = pl + (int64_t)y * ps;
    const int t = r[ic];
    if ((x & 1) == 0) {
      if (ic == 0) return t;
      return (t * 3 + r[ic - 1] + 1) >> 2;
    }
    if (ic == dw - 1) return t;
    return (t * 3 + r[ic + 1] + 2) >> 2;
  }
  // h2v2: nearest input row iy = y >> 1, next nearest above (even y) or below (odd y)
  const int iy = y >> 1;
  const int ny = (y & 1) ? (iy + 1 < dh ? iy + 1 : dh - 1) : (iy > 0 ? iy - 1 : 0);
  const uint8_t* r0 = pl + (int64_t)iy * ps;
  const uint8_t* r1 = pl + (int64_t)ny * ps;
  const int ic = x >> 1;
  const int th = r0[ic] * 3 + r1[ic];
  if ((x & 1) == 0) {
    if (ic == 0) return (th * 4 + 8) >> 4;
    const int la = r0[ic - 1] * 3 + r1[ic - 1];
    return (th * 3 + la + 8) >> 4;
  }
  if (ic == dw - 1) return (th * 4 + 7) >> 4;
  const int nx = r0[ic + 1] * 3 + r1[ic + 1];
  return (th * 3 + nx + 7) >> 4;
}

__host__ __device__ inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// libjpeg's fixed-point YCbCr -> RGB (jdcolor.c tables, SCALEBITS 16), one pixel.
__host__ __device__ inline void ycc_rgb(int y, int cb, int cr, uint8_t* rgb) {
  constexpr int64_t ONE_HALF = 1 << 15;
  const int64_t xcb = cb - 128, xcr = cr - 128;
  const int r_off = (int)((91881 * xcr + ONE_HALF) >> 16);
  const int b_off = (int)((116130 * xcb + ONE_HALF) >> 16);
  const int g_off = (int)(((-22554) * xcb + ONE_HALF + (-46802) * xcr) >> 16);
  rgb[0] = clamp255(y + r_off);
  rgb[1] = clamp255(y + g_off);
  rgb[2] = clamp255(y + b_off);
}

// Block b (0 .. bw*bh - 1) of component c: dequantise + islow IDCT into the component's plane
// (bw*8 x bh*8 samples, MCU padding included).
__host__ __device__ inline void idct_block(const Image& im, const int16_t* coef, uint8_t* planes, int c, int64_t b) {
  const Comp& k = im.comp[c];
  const int64_t by = b / k.bw, bx = b - by * k.bw;
  const int64_t ps = (int64_t)k.bw * 8;
  idct_islow(coef + (k.coef_off + b) * 64, im.quant[k.tq], planes + k.plane_off + by * 8 * ps + bx * 8, ps);
}

// Output pixel (x, y): Y at full resolution, Cb / Cr upsampled by the image's (hmax, vmax), then
// YCbCr -> RGB; one component: Y replicated (Pillow's L -> RGB).
__host__ __device__ inline void color_pixel(const Image& im, const uint8_t* planes, int x, int y, uint8_t* rgb) {
  const Comp& k0 = im.comp[0];
  const int yv = planes[k0.plane_off + (int64_t)y * k0.bw * 8 + x];
  if (im.ncomp == 1) {
    rgb[0] = rgb[1] = rgb[2] = (uint8_t)yv;
    return;
  }
  const Comp& k1 = im.comp[1];
  const Comp& k2 = im.comp[2];
  const int cb = chroma_at(planes + k1.plane_off, (int64_t)k1.bw * 8, k1.dw, k1.dh, im.hmax, im.vmax, x, y);
  const int cr = chroma_at(planes + k2.plane_off, (int64_t)k2.bw * 8, k2.dw, k2.dh, im.hmax, im.vmax, x, y);
  ycc_rgb(yv, cb, cr, rgb);
}

}  // namespace mrag_jpeg
