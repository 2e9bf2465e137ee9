// inflate.h — host-side DEFLATE / zlib decoder for K14's PNG path (RFC 1950 / RFC 1951), written
// for throughput: a 64-bit bit buffer refilled eight bytes at a time, two-level Huffman tables
// (a direct primary lookup, subtables for the longer codes) whose primary entries hold two
// literals when both codes fit in its bits (PNG scanlines after filtering are mostly literals with
// short codes: one lookup then writes two bytes), match copies in 8-byte words.
// It applies zlib's validity rules (inftrees.c: over-subscribed code sets and incomplete ones are
// errors, except a single code of length 1 for literal/length and distance codes; inflate.c:
// header check, no preset dictionary, HLIT <= 286, HDIST <= 30, a repeat with no previous length,
// lengths past the declared count, no end-of-block code, invalid symbols 286/287 and 30/31, a
// distance before the start of the output, a stored block whose LEN and NLEN disagree, block type
// 3). The output is the inflated bytes, so it equals zlib's for every stream zlib accepts
// (tests/test_png_cpu.py checks it against Python's zlib on thousands of streams); the caller
// falls back to zlib whenever this decoder reports an error, so a stream is refused only when zlib
// refuses it too. Once `out_len` bytes are produced it goes on as zlib does when the caller's
// output is full (Pillow's PNG decoder hands zlib exactly the image's bytes): codes that need no
// output are still decoded and checked (an invalid code, a distance before the start, block
// headers, and the Adler-32 trailer when the stream ends there); a symbol that needs output, or
// the end of the input, stops it without error.
#pragma once

#include <zlib.h>

#include <cstdint>
#include <cstring>

namespace mrag_png {

namespace infl {

constexpr int LBITS = 11, DBITS = 8;  // primary table bits (literal/length, distance)
// entry: bits 0-4 bits to consume (primary or whole code; a literal entry: all its literals),
// bit 5: subtable pointer, bit 6: invalid, bits 16-31: symbol or subtable offset.
// SUB entries: bits 8-15 subtable bits. LIT entries (literal/length table, symbol < 256): bits 8-12
// the first literal's code length, bit 13 PAIR (bits 16-23 the first literal, 24-31 the second)
constexpr uint32_t SUB = 1u << 5, BAD = 1u << 6, LIT = 1u << 7, PAIR = 1u << 13;

struct Table {
  uint32_t e[(1 << LBITS) + 32 * 1024];  // worst case: every primary slot owns a subtable
  int bits;
};

inline uint32_t rev(uint32_t code, int len) {
  uint32_t r = 0;
  for (int i = 0; i < len; ++i) r |= ((code >> i) & 1u) << (len - 1 - i);
  return r;
}

// Build a decode table from code lengths; kind 0 = code-length code, 1 = literal/length,
// 2 = distance (zlib inftrees.c rules). False on an over-subscribed or forbidden incomplete set.
inline bool build(Table& t, const uint8_t* lens, int n, int kind, int pbits) {
  int count[16] = {0};
  for (int i = 0; i < n; ++i) count[lens[i]]++;
  int max = 15;
  while (max >= 1 && count[max] == 0) --max;
  t.bits = pbits;
  const int psize = 1 << pbits;
  if (max == 0) {  // no codes: every lookup is an invalid code (an error only if it is used)
    for (int i = 0; i < psize; ++i) t.e[i] = BAD | 1u;
    return true;
  }
  int left = 1;
  for (int len = 1; len <= 15; ++len) {
    left <<= 1;
    left -= count[len];
    if (left < 0) return false;  // over-subscribed
  }
  if (left > 0 && (kind == 0 || max != 1)) return false;  // incomplete
  int next[16];
  next[1] = 0;
  for (int len = 1; len < 15; ++len) next[len + 1] = (next[len] + count[len]) << 1;
  for (int i = 0; i < psize; ++i) t.e[i] = BAD | 1u;  // an incomplete single-code set leaves holes
  int used = psize;
  // subtables: one per primary index whose codes are longer than pbits, sized for the longest
  int subbits[1 << LBITS];
  for (int i = 0; i < psize; ++i) subbits[i] = 0;
  // canonical codes in symbol order
  int code_of[320] = {0};
  {
    int nx[16];
    for (int i = 0; i < 16; ++i) nx[i] = next[i];
    for (int s = 0; s < n; ++s)
      if (lens[s]) code_of[s] = nx[lens[s]]++;
  }
  for (int s = 0; s < n; ++s) {
    const int len = lens[s];
    if (len > pbits) {
      const uint32_t r = rev((uint32_t)code_of[s], len);
      const int p = (int)(r & (uint32_t)(psize - 1));
      if (len - pbits > subbits[p]) subbits[p] = len - pbits;
    }
  }
  for (int p = 0; p < psize; ++p)
    if (subbits[p]) {
      t.e[p] = SUB | (uint32_t)pbits | ((uint32_t)subbits[p] << 8) | ((uint32_t)used << 16);
      for (int i = 0; i < (1 << subbits[p]); ++i) t.e[used + i] = BAD | 1u;
      used += 1 << subbits[p];
    }
  for (int s = 0; s < n; ++s) {
    const int len = lens[s];
    if (!len) continue;
    const uint32_t r = rev((uint32_t)code_of[s], len);
    if (len <= pbits) {
      const uint32_t lit = kind == 1 && s < 256 ? LIT | (uint32_t)len << 8 : 0u;
      for (uint32_t i = r; i < (uint32_t)psize; i += 1u << len) t.e[i] = (uint32_t)len | lit | ((uint32_t)s << 16);
    } else {
      const int p = (int)(r & (uint32_t)(psize - 1));
      const uint32_t base = t.e[p] >> 16;
      const int sb = (int)((t.e[p] >> 8) & 0xFF), rem = len - pbits;
      const uint32_t lit = kind == 1 && s < 256 ? LIT | (uint32_t)rem << 8 : 0u;
      for (uint32_t i = r >> pbits; i < (1u << sb); i += 1u << rem)
        t.e[base + i] = (uint32_t)rem | lit | ((uint32_t)s << 16);
    }
  }
  if (kind == 1) {  // literal pairs: index i's first code a literal of l1 bits, the next in the
    // remaining pbits - l1 bits (its entry at i >> l1 of the single-symbol table) a literal too
    uint32_t one[1 << LBITS];
    std::memcpy(one, t.e, sizeof(uint32_t) * (size_t)psize);
    for (int i = 0; i < psize; ++i) {
      const uint32_t e1 = one[i];
      if (!(e1 & LIT)) continue;
      const uint32_t l1 = e1 & 31, e2 = one[i >> l1];
      if ((e2 & LIT) && l1 + (e2 & 31) <= (uint32_t)pbits)
        t.e[i] = (l1 + (e2 & 31)) | LIT | PAIR | l1 << 8 | (e1 >> 16 & 0xFFu) << 16 | (e2 >> 16 & 0xFFu) << 24;
    }
  }
  return true;
}

constexpr uint16_t LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t DBASE[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf = 0;
  int cnt = 0;
  int64_t over = 0;  // bits consumed past the end of the input (zeros fed there)
  void refill() {
    if (end - p >= 8) {
      uint64_t w;
      std::memcpy(&w, p, 8);  // little-endian host
      buf |= w << cnt;
      p += (63 - cnt) >> 3;
      cnt |= 56;
    } else {
      while (cnt <= 56) {
        if (p < end) {
          buf |= (uint64_t)*p++ << cnt;
        } else {
          over += 8;  // virtual zero byte
        }
        cnt += 8;
      }
    }
  }
  void refill_fast() {  // at least 8 input bytes left
    uint64_t w;
    std::memcpy(&w, p, 8);
    buf |= w << cnt;
    p += (63 - cnt) >> 3;
    cnt |= 56;
  }
  uint32_t peek(int n) const { return (uint32_t)(buf & ((1ull << n) - 1)); }
  void drop(int n) {
    buf >>= n;
    cnt -= n;
  }
  uint32_t get(int n) {  // n <= 32, refilled by the caller
    const uint32_t v = peek(n);
    drop(n);
    return v;
  }
  bool overrun() const { return over > 0 && (int64_t)cnt < over; }  // consumed a virtual byte
};

// decode one symbol (buf holds >= 15 bits); -1 on an invalid code
inline int decode(Bits& b, const Table& t) {
  uint32_t e = t.e[b.peek(t.bits)];
  if (e & SUB) {
    const int sb = (int)((e >> 8) & 0xFF);
    b.drop(t.bits);
    e = t.e[(e >> 16) + b.peek(sb)];
  }
  if (e & BAD) return -1;
  if (e & LIT) {  // the first literal of the entry
    b.drop((int)(e >> 8 & 31));
    return (int)(e >> 16 & 0xFF);
  }
  b.drop((int)(e & 31));
  return (int)(e >> 16);
}

}  // namespace infl

// Inflate a zlib stream into out[0 .. out_len): true once out_len bytes are produced.
inline bool fast_inflate(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_len) {
  using namespace infl;
  if (in_len < 2) return false;
  const uint32_t cmf = in[0], flg = in[1];
  if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) return false;
  Bits b{in + 2, in + in_len};
  static thread_local Table lt, dt, ct;
  uint8_t* op = out;
  uint8_t* const oend = out + out_len;
  bool last = false;
  while (!last) {
    b.refill();
    last = b.get(1) != 0;
    const uint32_t type = b.get(2);
    if (b.overrun()) return op == oend;  // the input ends before the block header
    if (type == 0) {  // stored
      b.drop(b.cnt & 7);
      // give the whole bytes still in the bit buffer back to the input (the refills read the
      // input in order; zero bytes fed past its end are not given back)
      const int64_t real = b.cnt / 8 - b.over / 8;
      if (real < 0) return op == oend;  // the header bits ran past the input
      b.p -= real;
      b.buf = 0;
      b.cnt = 0;
      b.over = 0;
      if (b.end - b.p < 4) return op == oend;
      const uint32_t len = b.p[0] | (uint32_t)b.p[1] << 8, nlen = b.p[2] | (uint32_t)b.p[3] << 8;
      b.p += 4;
      if ((len ^ 0xFFFFu) != nlen) return false;
      const uint32_t rem = len;
      const size_t avail = (size_t)(b.end - b.p);
      const size_t take = rem < avail ? rem : avail;
      const size_t room = (size_t)(oend - op);
      if (take > room) {  // the output fills inside the block: zlib stops there, no error
        std::memcpy(op, b.p, room);
        return true;
      }
      std::memcpy(op, b.p, take);
      op += take;
      b.p += take;
      if (take < rem) return op == oend;  // the input ends inside the block
      continue;
    }
    if (type == 3) return false;
    if (type == 1) {
      uint8_t l[320];
      for (int i = 0; i < 144; ++i) l[i] = 8;
      for (int i = 144; i < 256; ++i) l[i] = 9;
      for (int i = 256; i < 280; ++i) l[i] = 7;
      for (int i = 280; i < 288; ++i) l[i] = 8;
      for (int i = 0; i < 32; ++i) l[288 + i] = 5;  // 30 and 31 complete the code; decoding them is an error
      if (!build(lt, l, 288, 1, LBITS) || !build(dt, l + 288, 32, 2, DBITS)) return false;
    } else {
      const int hlit = (int)b.get(5) + 257, hdist = (int)b.get(5) + 1, hclen = (int)b.get(4) + 4;
      if (b.overrun()) return op == oend;
      if (hlit > 286 || hdist > 30) return false;
      static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      uint8_t cl[19] = {0};
      for (int i = 0; i < hclen; ++i) {
        b.refill();
        cl[order[i]] = (uint8_t)b.get(3);
      }
      if (b.overrun()) return op == oend;
      if (!build(ct, cl, 19, 0, 7)) return false;
      uint8_t l[320];
      int i = 0;
      while (i < hlit + hdist) {
        b.refill();
        const int sym = decode(b, ct);
        if (b.overrun()) return op == oend;
        if (sym < 0) return false;
        if (sym < 16) {
          l[i++] = (uint8_t)sym;
          continue;
        }
        int rep, val = 0;
        if (sym == 16) {
          if (i == 0) return false;
          val = l[i - 1];
          rep = 3 + (int)b.get(2);
        } else if (sym == 17) {
          rep = 3 + (int)b.get(3);
        } else {
          rep = 11 + (int)b.get(7);
        }
        if (i + rep > hlit + hdist) return false;
        while (rep--) l[i++] = (uint8_t)val;
      }
      if (b.overrun()) return op == oend;
      if (l[256] == 0) return false;  // no end-of-block code
      if (!build(lt, l, hlit, 1, LBITS) || !build(dt, l + hlit, hdist, 2, DBITS)) return false;
    }
    // the block's symbols
    while (true) {
      // hot loop: >= 16 input bytes and >= 274 output bytes left, so no end checks; up to three
      // primary literal entries (one or two literals, <= LBITS bits each) per refill (>= 56 bits:
      // 3 x 11 + a length code with its extra bits, 20), each stored as two bytes; the general
      // symbol after them as below
      while (b.end - b.p >= 16 && oend - op >= 274) {
        b.refill_fast();
        uint32_t e = lt.e[b.peek(LBITS)];
        if (e & LIT) {
          auto put = [&](uint32_t x) {
            b.drop((int)(x & 31));
            const uint16_t two = (uint16_t)(x >> 16);
            std::memcpy(op, &two, 2);
            op += 1 + (x >> 13 & 1);
          };
          put(e);
          e = lt.e[b.peek(LBITS)];
          if (e & LIT) {
            put(e);
            e = lt.e[b.peek(LBITS)];
            if (e & LIT) {
              put(e);
              continue;
            }
          }
          if (b.cnt < 32) b.refill_fast();
        }
        if (e & SUB) {
          const int sb = (int)((e >> 8) & 0xFF);
          b.drop(LBITS);
          e = lt.e[(e >> 16) + b.peek(sb)];
        }
        if (e & BAD) return false;
        b.drop((int)(e & 31));
        const int sym = (int)(e >> 16);
        if (sym < 256) {
          *op++ = (uint8_t)sym;
          continue;
        }
        if (sym == 256) goto block_end;
        const int li = sym - 257;
        if (li >= 29) return false;
        const uint32_t len = LBASE[li] + b.get(LEXT[li]);
        b.refill_fast();
        const int ds = decode(b, dt);
        if (ds < 0 || ds >= 30) return false;
        const uint32_t dist = DBASE[ds] + b.get(DEXT[ds]);
        if (dist > (size_t)(op - out)) return false;
        const uint8_t* src = op - dist;
        if (dist >= 8) {  // room >= 274 >= len + 8
          uint8_t* d = op;
          for (uint32_t k = 0; k < len; k += 8, d += 8, src += 8) {
            uint64_t w;
            std::memcpy(&w, src, 8);
            std::memcpy(d, &w, 8);
          }
        } else {
          for (uint32_t k = 0; k < len; ++k) op[k] = src[k];
        }
        op += len;
      }
      b.refill();  // >= 57 bits: a literal/length code + extra (15 + 5) then a refill for the distance
      const int sym = decode(b, lt);
      if (b.overrun()) return op == oend;  // zlib waits for more input: an error only if bytes are missing
      if (sym < 0) return false;
      if (sym < 256) {
        if (op == oend) return true;
        *op++ = (uint8_t)sym;
        continue;
      }
      if (sym == 256) break;
      const int li = sym - 257;
      if (li >= 29) return false;  // 286, 287
      uint32_t len = LBASE[li] + b.get(LEXT[li]);
      b.refill();
      const int ds = decode(b, dt);
      if (b.overrun()) return op == oend;
      if (ds < 0 || ds >= 30) return false;
      const uint32_t dist = DBASE[ds] + b.get(DEXT[ds]);
      if (b.overrun()) return op == oend;
      if (dist > (size_t)(op - out)) return false;  // before the start of the output
      const size_t room = (size_t)(oend - op);
      bool done = false;
      if (len > room) {  // zlib stops inside the copy: no error
        len = (uint32_t)room;
        done = true;
      }
      const uint8_t* src = op - dist;
      if (dist >= 8 && room >= len + 8) {  // word copies (may write up to 7 bytes past, inside out)
        uint8_t* d = op;
        const uint8_t* s = src;
        for (uint32_t k = 0; k < len; k += 8, d += 8, s += 8) {
          uint64_t w;
          std::memcpy(&w, s, 8);
          std::memcpy(d, &w, 8);
        }
      } else {
        for (uint32_t k = 0; k < len; ++k) op[k] = src[k];
      }
      op += len;
      if (done) return true;
    }
  block_end:
    if (b.overrun()) return op == oend;
  }
  if (op != oend) return false;  // the stream ended before the image did
  // the Adler-32 of the whole output follows, byte-aligned: zlib checks it if it is there
  b.drop(b.cnt & 7);
  const int64_t real = b.cnt / 8 - b.over / 8;
  if (real < 0) return true;
  b.p -= real;
  if (b.end - b.p < 4) return true;
  const uint32_t want = (uint32_t)b.p[0] << 24 | (uint32_t)b.p[1] << 16 | (uint32_t)b.p[2] << 8 | b.p[3];
  return (uint32_t)adler32(adler32(0L, Z_NULL, 0), out, (uInt)out_len) == want;
}

}  // namespace mrag_png
