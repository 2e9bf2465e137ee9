// jpeg_parse.h — host side of K13: marker parsing, Huffman table construction, geometry and the
// entropy-coded segments of one JPEG file (ITU T.81 Annex B; libjpeg's geometry rules in
// jdinput.c: interleaved scans pad every component to whole MCUs, a one-component scan is
// non-interleaved with one block per MCU). Used by csrc/jpeg.hip and scripts/jpeg_host_check.hip.
#pragma once

#include <cstdint>
#include <array>
#include <cstring>
#include <string>
#include <vector>

#include "jpeg_core.h"

namespace mrag_jpeg {

struct Segment {
  int64_t off;  // first entropy-coded byte (in the file; the batch rebases it)
  int64_t len;
  int32_t img;
  int32_t mcu0, mcus;
};

struct Parsed {
  Image img{};
  std::vector<Segment> segs;
  int64_t ecs_begin = 0, ecs_end = 0;  // entropy-coded bytes of the scan in the file
  int64_t coef_blocks = 0, plane_bytes = 0;
  std::string why;  // reason when unsupported
};

// tc: 0 = DC table (symbols are magnitude categories 0..11 for 8-bit data), 1 = AC (run / size,
// size 0..10); a table with other symbols is refused (the file goes to Pillow), so a token is at
// most 16 + 11 bits.
inline bool build_huff(int tc, const uint8_t bits[17], const uint8_t* vals, int nvals, Huff& h) {
  std::memset(&h, 0, sizeof(h));
  if (nvals > 256) return false;
  for (int i = 0; i < nvals; ++i) {
    if (tc == 0 ? vals[i] > 11 : (vals[i] & 15) > 10) return false;
    h.vals4[i >> 2] |= (uint32_t)vals[i] << ((i & 3) * 8);
  }
  int32_t code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    const int n = bits[l];
    if (n == 0) {
      h.maxcode[l] = -1;
    } else {
      h.valoff[l] = k - code;
      for (int i = 0; i < n; ++i, ++k, ++code) {
        if (l <= 9) {
          const int shift = 9 - l;
          for (int s = 0; s < (1 << shift); ++s) {
            const uint32_t i = (uint32_t)((code << shift) | s);
            h.look2[i >> 1] |= (uint32_t)((l << 8) | vals[k]) << ((i & 1) * 16);
          }
        }
      }
      h.maxcode[l] = code - 1;
      if (code > (1 << l)) return false;  // over-subscribed
    }
    code <<= 1;
  }
  h.maxcode[17] = 0x7fffffff;
  return true;
}

inline bool fail(Parsed& P, const char* why) {
  P.why = why;
  return false;
}

// Parse one file. Returns true when K13 can decode it (else P.why says why and the caller decodes
// the file with Pillow on the host).
inline bool parse(const uint8_t* d, int64_t n, Parsed& P) {
  Image& im = P.img;
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return fail(P, "not a JPEG");
  bool sof = false, jfif = false, adobe = false;
  int adobe_transform = -1;
  int comp_id[MAX_COMP] = {0, 0, 0};
  bool qset[4] = {false, false, false, false}, dcset[2] = {false, false}, acset[2] = {false, false};
  int64_t pos = 2;
  while (true) {
    if (pos + 4 > n) return fail(P, "truncated before SOS");
    if (d[pos] != 0xFF) return fail(P, "marker expected");
    const int m = d[pos + 1];
    if (m == 0xFF) {
      ++pos;
      continue;
    }
    pos += 2;
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (m == 0xD9) return fail(P, "EOI before SOS");
    const int len = (d[pos] << 8) | d[pos + 1];
    if (len < 2 || pos + len > n) return fail(P, "bad segment length");
    const uint8_t* s = d + pos + 2;
    const int sl = len - 2;
    if (m == 0xC0 || m == 0xC1) {
      if (sl < 6 || s[0] != 8) return fail(P, "not 8-bit");
      im.height = (s[1] << 8) | s[2];
      im.width = (s[3] << 8) | s[4];
      im.ncomp = s[5];
      if (im.width <= 0 || im.height <= 0) return fail(P, "bad size");
      if (im.ncomp != 1 && im.ncomp != 3) return fail(P, "components");
      if (sl < 6 + 3 * im.ncomp) return fail(P, "SOF length");
      for (int c = 0; c < im.ncomp; ++c) {
        comp_id[c] = s[6 + 3 * c];
        im.comp[c].h = s[7 + 3 * c] >> 4;
        im.comp[c].v = s[7 + 3 * c] & 15;
        im.comp[c].tq = s[8 + 3 * c];
        if (im.comp[c].h < 1 || im.comp[c].v < 1 || im.comp[c].tq > 3) return fail(P, "SOF fields");
      }
      sof = true;
    } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return fail(P, "progressive / lossless / arithmetic");
    } else if (m == 0xC4) {
      int i = 0;
      while (i < sl) {
        const int tc = s[i] >> 4, th = s[i] & 15;
        if (i + 17 > sl) return fail(P, "DHT length");
        uint8_t bits[17] = {0};
        int total = 0;
        for (int l = 1; l <= 16; ++l) total += (bits[l] = s[i + l]);
        if (i + 17 + total > sl || tc > 1 || th > 1) return fail(P, "DHT table");
        Huff& h = tc == 0 ? im.dc[th] : im.ac[th];
        if (!build_huff(tc, bits, s + i + 17, total, h)) return fail(P, "bad Huffman table");
        (tc == 0 ? dcset : acset)[th] = true;
        i += 17 + total;
      }
    } else if (m == 0xDB) {
      int i = 0;
      while (i < sl) {
        const int pq = s[i] >> 4, tq = s[i] & 15;
        if (tq > 3 || pq > 1 || i + 1 + 64 * (pq + 1) > sl) return fail(P, "DQT");
        for (int k = 0; k < 64; ++k)
          im.quant[tq][zigzag(k)] = pq ? (uint16_t)((s[i + 1 + 2 * k] << 8) | s[i + 2 + 2 * k]) : s[i + 1 + k];
        qset[tq] = true;
        i += 1 + 64 * (pq + 1);
      }
    } else if (m == 0xDD) {
      if (sl < 2) return fail(P, "DRI");
      im.restart = (s[0] << 8) | s[1];
    } else if (m == 0xE0) {
      if (sl >= 5 && std::memcmp(s, "JFIF\0", 5) == 0) jfif = true;
    } else if (m == 0xEE) {
      if (sl >= 12 && std::memcmp(s, "Adobe", 5) == 0) {
        adobe = true;
        adobe_transform = s[11];
      }
    } else if (m == 0xDA) {
      if (!sof) return fail(P, "SOS before SOF");
      const int ns = s[0];
      if (ns != im.ncomp || sl < 1 + 2 * ns + 3) return fail(P, "not one interleaved scan");
      for (int k = 0; k < ns; ++k) {
        const int id = s[1 + 2 * k];
        int c = 0;
        while (c < im.ncomp && comp_id[c] != id) ++c;
        if (c != k) return fail(P, "scan component order");
        im.comp[c].td = s[2 + 2 * k] >> 4;
        im.comp[c].ta = s[2 + 2 * k] & 15;
        if (im.comp[c].td > 1 || im.comp[c].ta > 1 || !dcset[im.comp[c].td] || !acset[im.comp[c].ta])
          return fail(P, "scan tables");
        if (!qset[im.comp[c].tq]) return fail(P, "quant table");
      }
      const uint8_t* t = s + 1 + 2 * ns;
      if (t[0] != 0 || t[1] != 63 || t[2] != 0) return fail(P, "not a sequential scan");
      P.ecs_begin = pos + len;
      break;
    }
    pos += len;
  }
  // colour space as libjpeg decides it for three components (jdapimin.c default_decompress_parms)
  if (im.ncomp == 3) {
    bool rgb = false;
    if (jfif) rgb = false;
    else if (adobe) rgb = adobe_transform == 0;
    else rgb = comp_id[0] == 'R' && comp_id[1] == 'G' && comp_id[2] == 'B';
    if (rgb) return fail(P, "RGB-coded JPEG");
  }
  // geometry
  im.hmax = im.vmax = 1;
  for (int c = 0; c < im.ncomp; ++c) {
    im.hmax = im.comp[c].h > im.hmax ? im.comp[c].h : im.hmax;
    im.vmax = im.comp[c].v > im.vmax ? im.comp[c].v : im.vmax;
  }
  if (im.ncomp == 3) {
    const Comp& y = im.comp[0];
    if (y.h != im.hmax || y.v != im.vmax) return fail(P, "luma not at full resolution");
    for (int c = 1; c < 3; ++c)
      if (im.comp[c].h != 1 || im.comp[c].v != 1) return fail(P, "chroma sampling");
    if (!((im.hmax == 1 && im.vmax == 1) || (im.hmax == 2 && im.vmax == 1) || (im.hmax == 2 && im.vmax == 2)))
      return fail(P, "sampling other than 4:4:4 / 4:2:2 / 4:2:0");
  }
  int64_t blocks = 0, plane = 0;
  if (im.ncomp == 1) {
    Comp& c = im.comp[0];
    c.h = c.v = 1;
    im.hmax = im.vmax = 1;
    c.bw = (im.width + 7) / 8;
    c.bh = (im.height + 7) / 8;
    im.mcux = c.bw;
    im.mcuy = c.bh;
    im.blocks_per_mcu = 1;
  } else {
    im.mcux = (im.width + 8 * im.hmax - 1) / (8 * im.hmax);
    im.mcuy = (im.height + 8 * im.vmax - 1) / (8 * im.vmax);
    im.blocks_per_mcu = 0;
    for (int c = 0; c < 3; ++c) {
      im.comp[c].bw = im.mcux * im.comp[c].h;
      im.comp[c].bh = im.mcuy * im.comp[c].v;
      im.blocks_per_mcu += im.comp[c].h * im.comp[c].v;
    }
  }
  for (int c = 0; c < im.ncomp; ++c) {
    Comp& k = im.comp[c];
    k.dw = (int)(((int64_t)im.width * k.h + im.hmax - 1) / im.hmax);
    k.dh = (int)(((int64_t)im.height * k.v + im.vmax - 1) / im.vmax);
    // libjpeg-turbo's SIMD upsamplers treat a 2-sample chroma row differently from the C rule (measured
    // against Pillow: widths 3-4 at 4:2:x differ); such tiny images go to the host
    if (c > 0 && ((im.hmax == 2 && k.dw < 3) || (im.vmax == 2 && k.dh < 2))) return fail(P, "chroma narrower than 3");
    k.coef_off = blocks;
    k.plane_off = plane;
    blocks += (int64_t)k.bw * k.bh;
    plane += (int64_t)k.bw * 8 * k.bh * 8;
  }
  P.coef_blocks = blocks;
  P.plane_bytes = plane;
  // entropy-coded segments: split at RSTn, end at any other marker
  const int64_t total_mcus = (int64_t)im.mcux * im.mcuy;
  int64_t q = P.ecs_begin, seg_start = P.ecs_begin;
  std::vector<std::pair<int64_t, int64_t>> raw;
  while (true) {
    // next 0xFF (entropy-coded bytes are mostly not 0xFF: memchr, not a byte loop)
    const void* f = q < n ? std::memchr(d + q, 0xFF, (size_t)(n - q)) : nullptr;
    q = f ? (const uint8_t*)f - d : n;
    // the file ends inside the entropy-coded data (no marker after it, not even EOI): Pillow
    // raises "image file is truncated" for such a file, so it is left to Pillow
    if (q + 1 >= n) return fail(P, "truncated: the file ends inside the entropy-coded data");
    {
      const int b = d[q + 1];
      if (b == 0x00 || b == 0xFF) {
        q += b == 0x00 ? 2 : 1;
        continue;
      }
      if (b >= 0xD0 && b <= 0xD7) {
        // libjpeg expects RST0, RST1, ... in turn and resynchronises otherwise (jdmarker.c
        // read_restart_marker / jpeg_resync_to_restart): a file out of that order goes to Pillow
        if (im.restart > 0 && (b & 7) != (int)(raw.size() & 7)) return fail(P, "restart marker out of order");
        raw.emplace_back(seg_start, q - seg_start);
        q += 2;
        seg_start = q;
        continue;
      }
      raw.emplace_back(seg_start, q - seg_start);
      break;
    }
  }
  P.ecs_end = raw.back().first + raw.back().second;
  const int64_t per = im.restart > 0 ? im.restart : total_mcus;
  const int64_t nseg = (total_mcus + per - 1) / per;
  if (im.restart > 0 ? (int64_t)raw.size() != nseg : raw.size() < 1) return fail(P, "restart intervals != markers");
  P.segs.clear();
  for (int64_t i = 0; i < nseg; ++i) {
    Segment sg;
    sg.off = raw[i].first;
    sg.len = raw[i].second;
    sg.img = 0;
    sg.mcu0 = (int32_t)(i * per);
    sg.mcus = (int32_t)((i + 1) * per < total_mcus ? per : total_mcus - i * per);
    P.segs.push_back(sg);
  }
  im.nseg = (int32_t)nseg;
  return true;
}

// Decode one segment's MCUs into the image's coefficient buffer (zeroed by the caller): the same
// code runs in the device kernel (one wave per segment) and in the host check.
__host__ __device__ inline void decode_segment(const Image& im, const uint8_t* ecs, int64_t len, int mcu0, int mcus,
                                               int16_t* coef) {
  Bits br;
  br.init(ecs, len);
  int pred[MAX_COMP] = {0, 0, 0};
  for (int m = mcu0; m < mcu0 + mcus; ++m) {
    const int my = m / im.mcux, mx = m - my * im.mcux;
    for (int c = 0; c < im.ncomp; ++c) {
      const Comp& k = im.comp[c];
      for (int v = 0; v < k.v; ++v)
        for (int h = 0; h < k.h; ++h) {
          const int64_t blk = k.coef_off + (int64_t)(my * k.v + v) * k.bw + (mx * k.h + h);
          decode_block(br, im.dc[k.td], im.ac[k.ta], pred[c], coef + blk * 64);
        }
    }
    // libjpeg (jdhuff.c): once a token needed bits past the data (insufficient_data), the MCU is
    // completed with zero bits and the rest of the segment is left zero
    if (br.insufficient()) break;
  }
}

// Unstuffed bytes of one segment (K13a's input): 0xFF00 -> 0xFF; the first 0xFF not followed by
// 0x00 (or last in the segment) ends the data, where Bits starts feeding zeros. Returns the length.
inline int64_t unstuff(const uint8_t* src, int64_t len, uint8_t* dst) {
  uint8_t* o = dst;
  int64_t i = 0;
  while (i < len) {
    const void* f = std::memchr(src + i, 0xFF, (size_t)(len - i));
    const int64_t j = f ? (const uint8_t*)f - src : len;
    std::memcpy(o, src + i, (size_t)(j - i));
    o += j - i;
    if (j >= len) break;
    if (j + 1 < len && src[j + 1] == 0x00) {
      *o++ = 0xFF;
      i = j + 2;
    } else {
      break;
    }
  }
  return o - dst;
}

// Host emulation of K13a over one segment: the kernel's passes, lane by lane, with its barrier
// semantics (a round reads every exit before any lane rewrites its own). u: unstuffed bytes,
// readable and zero up to the next multiple of 16. Returns the number of resynchronisation
// rounds that changed an exit (the kernel runs one more to see that nothing changed). coef: the
// image's coefficient blocks, as decode_segment takes them.
inline int decode_segment_par(const Image& im, const uint8_t* u, uint32_t nbytes, int mcu0, int mcus, int16_t* coef) {
  PTabs T;
  T.h[0] = im.dc[0];
  T.h[1] = im.dc[1];
  T.h[2] = im.ac[0];
  T.h[3] = im.ac[1];
  make_ptab_ids(im, T);
  const uint32_t nbits = nbytes * 8u;
  int nl;
  uint32_t chunk;
  par_geom(nbits, nl, chunk);
  std::vector<PCheck> cps((size_t)PAR_NCP * PAR_LANES);
  std::vector<PState> ex(nl), entry(nl), myexit(nl);
  std::vector<std::array<int32_t, 4>> tot(nl);
  std::vector<std::array<uint32_t, 4>> cposv(nl);
  std::vector<uint32_t> endv(nl);
  for (int t = 0; t < nl; ++t) {
    uint32_t start, end, cpos[PAR_NCP];
    par_lane(nbits, nl, chunk, t, start, end, cpos);
    for (int j = 0; j < PAR_NCP; ++j) cposv[t][j] = cpos[j];
    endv[t] = end;
    PBits br;
    br.init(u, nbytes, start);
    PState st{start, 0};
    entry[t] = st;
    int32_t n[4] = {0, 0, 0, 0};
    par_run<PAR_RECORD>(T, br, st, end, n, &cps[t], PAR_LANES, cpos, nullptr, &im, nullptr, 0, 0, 0, nullptr);
    ex[t] = myexit[t] = st;
    for (int q = 0; q < 4; ++q) tot[t][q] = n[q];
  }
  int rounds = 0;
  while (true) {
    const std::vector<PState> snap = ex;
    bool changed = false;
    for (int t = 1; t < nl; ++t) {
      const PState e = snap[t - 1];
      if (e.p == entry[t].p && e.bk == entry[t].bk) continue;
      entry[t] = e;
      PState st = e;
      PBits br;
      br.init(u, nbytes, e.p);
      int32_t m[4] = {0, 0, 0, 0};
      const bool synced = par_run<PAR_SYNC>(T, br, st, endv[t], m, &cps[t], PAR_LANES, cposv[t].data(),
                                            tot[t].data(), &im, nullptr, 0, 0, 0, nullptr);
      for (int q = 0; q < 4; ++q) tot[t][q] = m[q];
      if (!synced && (st.p != myexit[t].p || st.bk != myexit[t].bk)) {
        myexit[t] = ex[t] = st;
        changed = true;
      }
    }
    if (!changed) break;
    ++rounds;
  }
  int32_t pre[4] = {0, 0, 0, 0};
  const int64_t gtot = (int64_t)mcus * T.bpm;
  for (int t = 0; t < nl; ++t) {
    PState st = t == 0 ? PState{0, 0} : ex[t - 1];
    PBits br;
    br.init(u, nbytes, st.p);
    int32_t pred[3] = {pre[1], pre[2], pre[3]};
    int32_t n[4] = {0, 0, 0, 0};
    par_run<PAR_WRITE>(T, br, st, t == nl - 1 ? 0xFFFFFFFFu : endv[t], n, nullptr, 0, nullptr, nullptr, &im,
                       coef, pre[0], gtot, mcu0, pred);
    for (int q = 0; q < 4; ++q) pre[q] += tot[t][q];
  }
  return rounds;
}

}  // namespace mrag_jpeg
