// files.hip — the host half of image ingest in one call (reference: the per-file
// Image.open(path) of app/ml/embeddings.py:82-89): read a group of files on this library's own
// threads, classify each (K13 JPEG, K14 PNG, or other) and stage what the GPU decoders read — the
// JPEGs' entropy-coded segments unstuffed, the PNGs' scanlines inflated — in one pinned arena, so
// that mrag_files_decode does no per-file host work (staged.h): the work the Python decode pool
// did per file, now without the interpreter lock between files and off the decode call's path.
// Files classified "other" (and unreadable ones) are left to the caller, which decodes them with
// Pillow (or raises the reference's exception for them), so the result is the same as the
// per-file path's.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <sys/stat.h>

#include "common.h"
#include "jpeg_parse.h"
#include "png_parse.h"
#include "staged.h"

namespace {

// Host arenas: pinned (hipHostMalloc) when the runtime gives it, plain malloc otherwise (no GPU:
// the classification still works); freed arenas are kept for the next groups.
struct Arena {
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool pinned = false;
};
std::mutex g_pool_mu;
std::vector<Arena> g_pool;
constexpr size_t POOL_KEEP = 6;  // prepare runs up to two groups ahead of the decode

Arena arena_get(size_t bytes) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    int best = -1;
    for (int i = 0; i < (int)g_pool.size(); ++i)
      if (g_pool[i].cap >= bytes && (best < 0 || g_pool[i].cap < g_pool[best].cap)) best = i;
    if (best >= 0) {
      Arena a = g_pool[best];
      g_pool.erase(g_pool.begin() + best);
      return a;
    }
  }
  Arena a;
  a.cap = std::max<size_t>(bytes + bytes / 8, 1u << 20);  // headroom: the next group's sizes differ a little
  if (hipHostMalloc((void**)&a.p, a.cap, hipHostMallocDefault) == hipSuccess) {
    a.pinned = true;
  } else {
    (void)hipGetLastError();  // not sticky: a later launch check must not see it
    a.p = (uint8_t*)std::malloc(a.cap);
    if (!a.p) throw std::bad_alloc();
  }
  return a;
}

void arena_free(Arena& a) {
  if (a.pinned)
    (void)hipHostFree(a.p);
  else
    std::free(a.p);
  a = Arena{};
}

void arena_put(Arena a) {
  if (!a.p) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (g_pool.size() < POOL_KEEP) {
    g_pool.push_back(a);
    return;
  }
  // keep the largest: drop the smallest of the pool and a
  auto it = std::min_element(g_pool.begin(), g_pool.end(), [](const Arena& x, const Arena& y) { return x.cap < y.cap; });
  if (it->cap < a.cap) std::swap(*it, a);
  arena_free(a);
}

}  // namespace

struct mrag_files {
  int32_t n = 0;
  std::vector<std::vector<uint8_t>> data;  // file bytes
  std::vector<int32_t> kind, w, h, bpp;    // kind: 1 JPEG (K13), 2 PNG (K14), 0 other, -1 unreadable
  std::vector<mrag_jpeg::Parsed> jp;       // kind 1: the parse
  std::vector<mrag_png::PngParsed> pp;     // kind 2: the parse
  std::vector<int64_t> off;                // kind 1: first stage byte of its segments; kind 2: of its scanlines
  std::vector<uint32_t> nbits;             // unstuffed bits of every JPEG segment, file then segment order
  std::vector<int32_t> seg0;               // kind 1: its first entry in nbits
  int64_t jpeg_bytes = 0;                  // the JPEG part of the arena: [0, jpeg_bytes); the PNGs after it
  Arena arena;
  ~mrag_files() { arena_put(arena); }
};

namespace {

bool read_file(const char* path, std::vector<uint8_t>& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  bool ok = std::fseek(f, 0, SEEK_END) == 0;
  const long sz = ok ? std::ftell(f) : -1;
  ok = ok && sz >= 0 && std::fseek(f, 0, SEEK_SET) == 0;
  if (ok) {
    out.resize((size_t)sz);
    ok = sz == 0 || std::fread(out.data(), 1, (size_t)sz, f) == (size_t)sz;
  }
  std::fclose(f);
  return ok;
}

// read, then parse what K13 / K14 may take (kind 2 is provisional until the inflate succeeds)
// Pillow's decompression-bomb count (Image._decompression_bomb_check): above max_pixels it warns,
// above twice that it raises; either way the file is Pillow's (kind 0), as in the reference
bool over_limit(int64_t w, int64_t h, int64_t max_pixels) {
  return max_pixels >= 0 && std::max<int64_t>(1, w) * std::max<int64_t>(1, h) > max_pixels;
}

void classify(mrag_files& F, int i, const char* path, bool device_decode, int64_t max_pixels) {
  std::vector<uint8_t>& d = F.data[i];
  if (!read_file(path, d)) {
    F.kind[i] = -1;
    return;
  }
  F.kind[i] = 0;
  if (!device_decode) return;
  const int64_t n = (int64_t)d.size();
  if (n >= 2 && d[0] == 0xFF && d[1] == 0xD8) {
    if (mrag_jpeg::parse(d.data(), n, F.jp[i]) &&
        !over_limit(F.jp[i].img.width, F.jp[i].img.height, max_pixels)) {
      F.kind[i] = 1;
      F.w[i] = F.jp[i].img.width;
      F.h[i] = F.jp[i].img.height;
    }
    return;
  }
  if (mrag_png::png_parse(d.data(), n, F.pp[i], true) && !over_limit(F.pp[i].width, F.pp[i].height, max_pixels)) {
    F.kind[i] = 2;
    F.w[i] = F.pp[i].width;
    F.h[i] = F.pp[i].height;
    F.bpp[i] = F.pp[i].bpp;
  }
}

// write file i's staged bytes: the JPEG's segments unstuffed, or the PNG's scanlines inflated (a
// stream that does not inflate turns the file into kind 0: Pillow decides what it is)
void stage(mrag_files& F, int i) {
  uint8_t* base = F.arena.p;
  if (F.kind[i] == 1) {
    const mrag_jpeg::Parsed& P = F.jp[i];
    int64_t o = F.off[i];
    int q = F.seg0[i];
    for (const mrag_jpeg::Segment& sg : P.segs) {
      uint8_t* dst = base + o;
      const int64_t u = mrag_jpeg::unstuff(F.data[i].data() + sg.off, sg.len, dst);
      std::memset(dst + u, 0, (size_t)((u + 15) / 16 * 16 - u));
      F.nbits[q++] = (uint32_t)(u * 8);
      o += mrag_stage::jpeg_seg_stage_bytes(sg.len);
    }
  } else if (F.kind[i] == 2) {
    if (!mrag_png::png_inflate(F.data[i].data(), F.pp[i], base + F.off[i])) {
      F.kind[i] = 0;
      F.w[i] = F.h[i] = F.bpp[i] = 0;
    }
  }
}

template <class Fn>
bool on_threads(int n, int threads, Fn fn) {
  const int nth = std::max(1, std::min<int>(threads > 0 ? threads : 1, n));
  std::atomic<int> next{0};
  std::atomic<bool> thrown{false};
  auto work = [&]() {
    try {
      for (int i = next++; i < n; i = next++) fn(i);
    } catch (...) {
      thrown = true;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nth; ++t) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  return !thrown;
}

int prepare_impl(const char* const* paths, int32_t n, int32_t threads, int32_t device_decode, int64_t max_pixels,
                 mrag_files** out) {
  if (!out || n < 0 || (n > 0 && !paths)) return mrag::fail(MRAG_ERR_ARG, "NULL argument");
  *out = nullptr;
  auto* F = new mrag_files();
  auto fail_oom = [&]() {
    delete F;
    return mrag::fail(MRAG_ERR_OOM, "files: host allocation failed");
  };
  F->n = n;
  F->data.resize((size_t)n);
  F->kind.assign((size_t)n, 0);
  F->w.assign((size_t)n, 0);
  F->h.assign((size_t)n, 0);
  F->bpp.assign((size_t)n, 0);
  F->jp.resize((size_t)n);
  F->pp.resize((size_t)n);
  F->off.assign((size_t)n, 0);
  F->seg0.assign((size_t)n, 0);
  if (!on_threads(n, threads, [&](int i) { classify(*F, i, paths[i], device_decode != 0, max_pixels); })) return fail_oom();
  // the arena: every JPEG's segments (K13's stage layout, file order), then every PNG's scanlines
  int64_t pos = 0;
  int32_t nseg = 0;
  for (int i = 0; i < n; ++i)
    if (F->kind[i] == 1) {
      F->off[i] = pos;
      F->seg0[i] = nseg;
      for (const mrag_jpeg::Segment& sg : F->jp[i].segs) pos += mrag_stage::jpeg_seg_stage_bytes(sg.len);
      nseg += (int32_t)F->jp[i].segs.size();
    }
  F->jpeg_bytes = pos;
  for (int i = 0; i < n; ++i)
    if (F->kind[i] == 2) {
      F->off[i] = pos;
      pos += (F->pp[i].raw_bytes + 15) / 16 * 16;
    }
  F->nbits.assign((size_t)nseg, 0);
  if (pos > 0) F->arena = arena_get((size_t)pos);
  if (!on_threads(n, threads, [&](int i) { stage(*F, i); })) return fail_oom();
  for (int i = 0; i < n; ++i) {  // the parses of files K13 / K14 do not take are not needed again
    if (F->kind[i] != 1) std::vector<mrag_jpeg::Segment>().swap(F->jp[i].segs);
    if (F->kind[i] != 2) std::vector<std::pair<int64_t, int64_t>>().swap(F->pp[i].idat);
  }
  *out = F;
  return MRAG_OK;
}

int decode_impl(const mrag_files* F, uint8_t* out, const int64_t* out_offsets, int32_t device, void* stream) {
  MRAG_REQUIRE(F && out && out_offsets, "NULL argument");
  std::vector<const mrag_jpeg::Parsed*> jp;
  std::vector<int64_t> jo, po, roff;
  std::vector<int32_t> pd;
  for (int i = 0; i < F->n; ++i) {
    if (F->kind[i] == 1) {
      jp.push_back(&F->jp[i]);
      jo.push_back(out_offsets[i]);
    } else if (F->kind[i] == 2) {
      pd.push_back(F->w[i]);
      pd.push_back(F->h[i]);
      pd.push_back(F->bpp[i]);
      po.push_back(out_offsets[i]);
      roff.push_back(F->off[i] - F->jpeg_bytes);
    }
  }
  if (!jp.empty()) {
    const mrag_stage::JpegStaged st{jp.data(), F->arena.p, F->jpeg_bytes, F->nbits.data()};
    if (int rc = mrag_stage::jpeg_decode_staged(st, (int32_t)jp.size(), out, jo.data(), device, stream)) return rc;
  }
  if (!po.empty()) {
    const int64_t png_bytes = (int64_t)F->arena.cap - F->jpeg_bytes;
    int64_t used = 0;
    for (size_t k = 0; k < po.size(); ++k)
      used = std::max(used, roff[k] + (int64_t)pd[3 * k + 1] * (1 + (int64_t)pd[3 * k] * pd[3 * k + 2]));
    MRAG_REQUIRE(used <= png_bytes, "files: PNG stage overrun");
    if (int rc = mrag_stage::png_unfilter_staged(F->arena.p + F->jpeg_bytes, used, roff.data(), pd.data(),
                                                 (int32_t)po.size(), out, po.data(), device, stream))
      return rc;
  }
  return MRAG_OK;
}

}  // namespace

extern "C" {

// the C ABI: no C++ exception crosses it (a failed host allocation is MRAG_ERR_OOM)
int mrag_files_prepare(const char* const* paths, int32_t n, int32_t threads, int32_t device_decode,
                       int64_t max_pixels, mrag_files** out) {
  try {
    return prepare_impl(paths, n, threads, device_decode, max_pixels, out);
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "files: host allocation failed");
  }
}

int mrag_files_info(const mrag_files* F, int32_t* kind, int32_t* width, int32_t* height) {
  MRAG_REQUIRE(F && kind && width && height, "NULL argument");
  for (int i = 0; i < F->n; ++i) {
    kind[i] = F->kind[i];
    width[i] = F->w[i];
    height[i] = F->h[i];
  }
  return MRAG_OK;
}

int mrag_files_bytes(const mrag_files* F, int32_t i, const uint8_t** data, int64_t* size) {
  MRAG_REQUIRE(F && data && size && i >= 0 && i < F->n, "bad argument");
  *data = F->data[i].data();
  *size = (int64_t)F->data[i].size();
  return MRAG_OK;
}

int mrag_files_decode(const mrag_files* F, uint8_t* out, const int64_t* out_offsets, int32_t device, void* stream) {
  try {
    return decode_impl(F, out, out_offsets, device, stream);
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "files: host allocation failed");
  }
}

int mrag_files_free(mrag_files* F) {
  delete F;
  return MRAG_OK;
}

int mrag_paths_exist(const char* const* paths, int32_t n, int32_t threads, int32_t* out) {
  MRAG_REQUIRE(n >= 0 && (n == 0 || (paths && out)), "NULL argument");
  try {
    on_threads(n, threads, [&](int i) {
      const char* p = paths[i] && paths[i][0] ? paths[i] : ".";
      struct stat st;
      if (stat(p, &st) == 0) {
        out[i] = 1;
      } else {
        const int e = errno;
        out[i] = (e == ENOENT || e == ENOTDIR || e == EBADF || e == ELOOP) ? 0 : -1;
      }
    });
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "paths: host allocation failed");
  }
  return MRAG_OK;
}

}  // extern "C"
