// tokenize.cpp — the offline stand-in tokeniser's ASCII fast path (app/encoders/tokenize.py: no
// local vocabulary, so token ids are hashed: lo + crc32(token) % (hi - lo) over BERT-style basic
// pre-tokens, `\w+|[^\w\s]` of the lowercased NFC text). For an ASCII text NFC is the identity,
// lowercasing maps A-Z only, `\w` is [0-9A-Za-z_] and `\s` is Python's str whitespace (\t \n \v \f
// \r, space, \x1c-\x1f): the same tokens and the same zlib crc32 as the Python path, without the
// interpreter, on this library's threads. Texts with a non-ASCII byte are left to the caller.
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include <zlib.h>

#include "common.h"

namespace {

inline bool is_word(unsigned char c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_';
}
inline bool is_space(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }

// crc32 of s[0 .. len) lowercased, in 256-byte pieces (a word may be as long as the text)
uint32_t crc_lower(const unsigned char* s, int64_t len) {
  unsigned char buf[256];
  uLong crc = crc32(0L, Z_NULL, 0);
  for (int64_t p = 0; p < len; p += 256) {
    const int m = (int)(len - p < 256 ? len - p : 256);
    for (int j = 0; j < m; ++j) {
      const unsigned char c = s[p + j];
      buf[j] = (c >= 'A' && c <= 'Z') ? (unsigned char)(c + 32) : c;
    }
    crc = crc32(crc, buf, (uInt)m);
  }
  return (uint32_t)crc;
}

}  // namespace

extern "C" int mrag_hash_tokenize(const char* const* texts, const int64_t* lens, int32_t n, int32_t lo, int32_t hi,
                                  int32_t max_tokens, int32_t threads, int32_t* ids, int32_t* counts) {
  MRAG_REQUIRE(n >= 0 && (n == 0 || (texts && lens && ids && counts)), "NULL argument");
  MRAG_REQUIRE(hi > lo && lo >= 0 && max_tokens > 0, "tokenize: bad id range or max_tokens");
  const uint32_t span = (uint32_t)(hi - lo);
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int i = next++; i < n; i = next++) {
      const unsigned char* s = (const unsigned char*)texts[i];
      const int64_t L = lens[i];
      int32_t* out = ids + (size_t)i * (size_t)max_tokens;
      int32_t c = 0;
      bool ascii = true;
      for (int64_t k = 0; k < L; ++k)
        if (s[k] >= 0x80) {
          ascii = false;
          break;
        }
      if (!ascii) {
        counts[i] = -1;
        continue;
      }
      int64_t k = 0;
      while (k < L && c < max_tokens) {
        const unsigned char ch = s[k];
        if (is_space(ch)) {
          ++k;
          continue;
        }
        int64_t e = k + 1;
        if (is_word(ch))
          while (e < L && is_word(s[e])) ++e;
        out[c++] = lo + (int32_t)(crc_lower(s + k, e - k) % span);
        k = e;
      }
      counts[i] = c;
    }
  };
  const int nth = threads > 1 ? (threads < n ? threads : n) : 1;
  std::vector<std::thread> th;
  try {
    th.reserve((size_t)nth);
    for (int t = 1; t < nth; ++t) th.emplace_back(work);
  } catch (...) {  // fewer helpers than asked: this thread and the started ones finish the work
  }
  work();
  for (auto& x : th) x.join();
  return MRAG_OK;
}
