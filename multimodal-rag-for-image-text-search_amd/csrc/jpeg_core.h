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
  int64_t data_bits, used;  // bits of real data put in buf / bits consumed
  bool at_end;              // the data has ended (a marker or the segment end): zeros follow
  // libjpeg's insufficient_data: a token took bits past the end of the data
  __host__ __device__ bool insufficient() const { return at_end && used > data_bits; }
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
    data_bits = used = 0;
    at_end = false;
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
            data_bits += 8;
          } else {
            b = 0;  // marker: stay on it, zeros from here
            n = pos;
            at_end = true;
          }
        } else {
          ++pos;
          data_bits += 8;
        }
      } else {
        at_end = true;
      }
      buf |= (uint64_t)b << (56 - cnt);
      cnt += 8;
    }
  }
  __host__ __device__ uint32_t peek(int k) { return (uint32_t)(buf >> (64 - k)); }
  __host__ __device__ void skip(int k) {
    buf <<= k;
    cnt -= k;
    used += k;
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
// An AC run past index 63 (corrupt data: k up to 63 + 15) lands on natural index 63, as in libjpeg,
// whose jpeg_natural_order[] carries 16 extra entries of 63 for exactly this (jdhuff.c).
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
      coef[k < 64 ? zigzag(k) : 63] = (int16_t)v;
      ++k;
    } else {
      if (r != 15) break;  // EOB
      k += 16;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Parallel entropy decoding of one segment (K13a). The segment's bytes are unstuffed on the host
// (0xFF00 -> 0xFF; the first 0xFF not followed by 0x00 ends the data, as Bits treats it), so a bit
// position is a plain offset, and zero bits follow the data (Bits feeds zeros there too).
// The bits are cut into one chunk per lane. The decoder state at a token boundary is
// (bit position, block of the MCU b, coefficient index k); a token (Huffman code + its extra
// bits) belongs to the chunk its first bit lies in. Every lane first decodes its chunk from its
// first bit with a guessed state (b = 0, k = 0) and records its exit (the state at the first token
// boundary at or past the chunk end) and checkpoints (the state and running counts at the first
// token boundary past NCP fixed positions). A Huffman stream resynchronises: a decode started at
// a wrong position soon lands on the true token boundaries with the true (b, k), after which it is
// the true decode. Then, until no exit changes, every lane whose entry (its predecessor's exit)
// differs from the state it last decoded from decodes again from that entry, and stops at the
// first checkpoint whose state it meets (the rest of the chunk is then known); lane 0's entry is
// exact, so lane i is exact after at most i rounds (in practice one). Block counts and per-component
// DC-difference sums of each chunk, prefix-summed over the lanes, give every lane its first block
// and its DC predictors, and a final decode from the exact entries writes the coefficients:
// the same tokens, the same values, as decode_segment.
struct PState {
  uint32_t p;   // bit position of the next token
  uint32_t bk;  // block of the MCU << 8 | coefficient index (0 = the DC token is next)
};
struct PCheck {
  uint32_t p, bk;
  int32_t n[4];  // completed blocks, DC-difference sums of components 0..2 since the entry
};
constexpr int PAR_NCP = 4;         // checkpoints per chunk
#ifndef MRAG_PAR_LANES  // (overridable for A/B builds only; 256 x 4096: K13a 2.87 ms per ingest
#define MRAG_PAR_LANES 1024  // group, 512 x 2048: 1.94, 1024 x 1024: 1.67 — profiles/r5s41_*)
#define MRAG_PAR_MIN_BITS 1024
#endif
constexpr int PAR_LANES = MRAG_PAR_LANES;        // lanes (chunks) per segment at most
constexpr int PAR_MIN_BITS = MRAG_PAR_MIN_BITS;  // shortest chunk

// Per-image tables for the parallel decoder: the four Huffman tables and, per block of the MCU,
// its component and table ids.
struct PTabs {
  Huff h[4];           // dc0, dc1, ac0, ac1
  uint8_t tdc[8], tac[8], cmp[8];
  int32_t bpm;
};

// Component and table ids of every block of the MCU (the Huffman tables are copied separately).
__host__ __device__ inline void make_ptab_ids(const Image& im, PTabs& T) {
  int b = 0;
  for (int c = 0; c < im.ncomp; ++c) {
    const int nb = im.ncomp == 1 ? 1 : im.comp[c].h * im.comp[c].v;
    for (int i = 0; i < nb; ++i, ++b) {
      T.tdc[b] = (uint8_t)im.comp[c].td;
      T.tac[b] = (uint8_t)(2 + im.comp[c].ta);
      T.cmp[b] = (uint8_t)c;
    }
  }
  T.bpm = b;
}

// Lanes and chunk length for a segment of nbits bits; lane t covers [start, end), the last lane
// to the end of the data; checkpoints at NCP evenly spaced positions inside the chunk.
__host__ __device__ inline void par_geom(uint32_t nbits, int& nl, uint32_t& chunk) {
  const uint32_t want = (nbits + PAR_MIN_BITS - 1) / PAR_MIN_BITS;
  nl = want < 1 ? 1 : (want > (uint32_t)PAR_LANES ? PAR_LANES : (int)want);
  chunk = (nbits + (uint32_t)nl - 1) / (uint32_t)nl;
}
__host__ __device__ inline void par_lane(uint32_t nbits, int nl, uint32_t chunk, int t, uint32_t& start, uint32_t& end,
                                         uint32_t (&cpos)[PAR_NCP]) {
  const uint64_t s = (uint64_t)t * chunk;
  start = s < nbits ? (uint32_t)s : nbits;
  end = t == nl - 1 ? nbits : (start + chunk < nbits ? start + chunk : nbits);
  for (int j = 0; j < PAR_NCP; ++j) cpos[j] = start + (uint32_t)((uint64_t)(j + 1) * (end - start) / (PAR_NCP + 1));
}

// Bit reader over unstuffed bytes (big-endian 32-bit words, 16 bytes per load, the next 16 bytes
// requested one load ahead; bytes past the data read as zero).
struct PBits {
  const uint8_t* base;
  uint32_t nblk;           // 16-byte blocks holding data (the last one zero-padded)
  uint32_t blk;            // block of cur
  uint32_t cur[4], nxt[4];
  int j;                   // next word of cur
  uint64_t buf;            // MSB-aligned
  int cnt;
  __host__ __device__ static uint32_t bswap(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
  }
  __host__ __device__ void load(uint32_t i, uint32_t (&w)[4]) const {
    if (i < nblk) {
      const uint32_t* q = (const uint32_t*)(base + (size_t)i * 16);
      w[0] = bswap(q[0]);
      w[1] = bswap(q[1]);
      w[2] = bswap(q[2]);
      w[3] = bswap(q[3]);
    } else {
      w[0] = w[1] = w[2] = w[3] = 0;
    }
  }
  __host__ __device__ uint32_t take() {
    const uint32_t w = j == 0 ? cur[0] : j == 1 ? cur[1] : j == 2 ? cur[2] : cur[3];
    if (++j == 4) {
      cur[0] = nxt[0];
      cur[1] = nxt[1];
      cur[2] = nxt[2];
      cur[3] = nxt[3];
      ++blk;
      load(blk + 1, nxt);
      j = 0;
    }
    return w;
  }
  uint32_t nblk_bits;      // bits of data (8 x bytes)
  __host__ __device__ void init(const uint8_t* b, uint32_t nbytes, uint32_t p) {
    base = b;
    nblk_bits = nbytes * 8u;
    nblk = (nbytes + 15) / 16;
    blk = p >> 7;
    load(blk, cur);
    load(blk + 1, nxt);
    j = (int)((p >> 5) & 3);
    const uint64_t w0 = take(), w1 = take();
    const int sh = (int)(p & 31);
    buf = ((w0 << 32) | w1) << sh;
    cnt = 64 - sh;
  }
  __host__ __device__ void refill() {
    if (cnt <= 32) {
      buf |= (uint64_t)take() << (32 - cnt);
      cnt += 32;
    }
  }
};

enum { PAR_RECORD = 0, PAR_SYNC = 1, PAR_WRITE = 2 };

// Decode one chunk from state st (updated to the exit) until the next token would start at or
// past `end`. RECORD: counts since the entry into n, checkpoints cp[j] at the positions cpos[j].
// SYNC: the same, but on meeting a recorded checkpoint state, n becomes the chunk total implied by
// the record (tot_old) and the function returns true (exit unchanged; later checkpoints rebased).
// WRITE: coefficients of blocks g .. (g < gtot) into coef (block g of the segment = MCU
// mcu0 + g / bpm), DC predictors pred[]; stops early when g reaches gtot.
template <int MODE, class TAB>
__host__ __device__ inline bool par_run(const TAB& T, PBits& br, PState& st, uint32_t end, int32_t (&n)[4],
                                        PCheck* cp, int cstride, const uint32_t* cpos, const int32_t* tot_old,
                                        const Image* im, int16_t* coef, int64_t g, int64_t gtot, int mcu0,
                                        int32_t* pred) {
  uint32_t p = st.p;
  int b = (int)(st.bk >> 8), k = (int)(st.bk & 255);
  int jcp = 0;
  if (MODE != PAR_WRITE)
    while (jcp < PAR_NCP && cpos[jcp] <= p) ++jcp;  // checkpoints behind the entry are not ours
  int64_t blk = 0;
  int my = 0, mx = 0;
  auto locate = [&]() {
    const int64_t m = mcu0 + g / T.bpm;
    my = (int)(m / im->mcux);
    mx = (int)(m - (int64_t)my * im->mcux);
    const int c = T.cmp[b];
    const Comp& kc = im->comp[c];
    int first = 0;
    for (int q = 0; q < b; ++q) first += T.cmp[q] == c ? 1 : 0;
    const int v = first / kc.h, h = first - v * kc.h;
    blk = kc.coef_off + (int64_t)(my * kc.v + v) * kc.bw + (mx * kc.h + h);
  };
  if (MODE == PAR_WRITE) {
    if (g >= gtot) {
      st.p = p;
      return false;
    }
    locate();
  }
  const uint32_t nbits = br.nblk_bits;  // end of the data (WRITE: libjpeg's insufficient_data rule)
  bool crossed = false;
  while (MODE == PAR_WRITE ? (p < end && g < gtot) : p < end) {
    if (MODE != PAR_WRITE && jcp < PAR_NCP && p >= cpos[jcp]) {
      PCheck& c = cp[jcp * cstride];
      const uint32_t bk = (uint32_t)(b << 8 | k);
      if (MODE == PAR_SYNC && c.p == p && c.bk == bk) {
        // synchronised: from here on the decode is the recorded one
        int32_t d[4];
        for (int q = 0; q < 4; ++q) d[q] = n[q] - c.n[q];
        for (int q = 0; q < 4; ++q) n[q] = tot_old[q] + d[q];
        for (int jj = jcp; jj < PAR_NCP; ++jj)
          for (int q = 0; q < 4; ++q) cp[jj * cstride].n[q] += d[q];
        return true;
      }
      c.p = p;
      c.bk = bk;
      for (int q = 0; q < 4; ++q) c.n[q] = n[q];
      ++jcp;
    }
    br.refill();
    const uint32_t top = (uint32_t)(br.buf >> 32);
    const Huff& h = T.h[k == 0 ? T.tdc[b] : T.tac[b]];
    const uint32_t e = h.look(top >> 23);
    int l, sym;
    if (e >> 8) {
      l = (int)(e >> 8);
      sym = (int)(e & 0xFF);
    } else {
      l = 10;
      int32_t code = (int32_t)(top >> 22);
      while (l <= 16 && code > h.maxcode[l]) {
        ++l;
        code = (int32_t)(top >> (32 - l));
      }
      if (l > 16) {  // corrupt code: 16 bits dropped, symbol 0 (as Bits::decode)
        l = 16;
        sym = 0;
      } else {
        sym = (int)h.val((uint32_t)(code + h.valoff[l]) & 0xFF);
      }
    }
    const int s = k == 0 ? sym : (sym & 15);
    const uint32_t v = s ? (top << l) >> (32 - s) : 0u;
    br.buf <<= (l + s);
    br.cnt -= l + s;
    p += (uint32_t)(l + s);
    if (MODE == PAR_WRITE && p > nbits) crossed = true;
    if (k == 0) {
      const int diff = extend((int)v, s);
      const int c = T.cmp[b];
      if (MODE == PAR_WRITE) {
        pred[c] += diff;
        coef[blk * 64] = (int16_t)pred[c];
      } else {
        n[1 + c] += diff;
      }
      k = 1;
    } else {
      const int r = sym >> 4;
      if (s) {
        k += r;
        if (MODE == PAR_WRITE) coef[blk * 64 + (k < 64 ? zigzag(k) : 63)] = (int16_t)extend((int)v, s);
        ++k;
      } else if (r == 15) {
        k += 16;
      } else {
        k = 64;
      }
    }
    if (k >= 64) {
      k = 0;
      b = b + 1 == T.bpm ? 0 : b + 1;
      if (MODE == PAR_WRITE) {
        ++g;
        // a token of this MCU needed bits past the data: libjpeg completes the MCU with zero
        // bits and leaves the rest of the segment zero (jdhuff.c insufficient_data)
        if (crossed && b == 0) break;
        if (g < gtot) locate();
      } else {
        ++n[0];
      }
    }
  }
  st.p = p;
  st.bk = (uint32_t)(b << 8 | k);
  return false;
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

__host__ __device__ inline void idct_islow(const int16_t* coef_g, const uint16_t* q, uint8_t* out, int64_t stride) {
  constexpr int CB = 13, P1 = 2;
  int16_t coef[64];  // the block in registers: eight 16-byte loads, not 64 two-byte ones
  __builtin_memcpy(coef, coef_g, sizeof(coef));
  // libjpeg's JLONG is 64-bit on LP64 hosts: the products are formed in int64 and the pass-1
  // results truncated to int, as its workspace is
  typedef int64_t L;
  constexpr L F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
              F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
  int32_t ws[64];
#pragma unroll
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
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int32_t* w = ws + r * 8;
    uint8_t o[8];  // one 8-byte store per row
    if (w[1] == 0 && w[2] == 0 && w[3] == 0 && w[4] == 0 && w[5] == 0 && w[6] == 0 && w[7] == 0) {
      constexpr int SH0 = P1 + 3;
      const uint8_t v = idct_limit((int32_t)(((L)w[0] + ((L)1 << (SH0 - 1))) >> SH0));
      for (int c = 0; c < 8; ++c) o[c] = v;
      __builtin_memcpy(out + r * stride, o, 8);
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
    __builtin_memcpy(out + r * stride, o, 8);
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
