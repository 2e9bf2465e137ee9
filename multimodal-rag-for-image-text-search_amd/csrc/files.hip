// files.hip — the host half of image ingest in one call (reference: the per-file
// Image.open(path) of app/ml/embeddings.py:82-89): read a group of files on this library's own
// threads, classify each (K13 JPEG, K14 PNG, or other), probe it and inflate the PNGs — the work
// the Python decode pool did per file, now without the interpreter lock between files. Files
// classified "other" (and unreadable ones) are left to the caller, which decodes them with Pillow
// (or raises the reference's exception for them), so the result is the same as the per-file path.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "jpeg_parse.h"
#include "png_parse.h"

struct mrag_files {
  int32_t n = 0;
  std::vector<std::vector<uint8_t>> data;  // file bytes
  std::vector<std::vector<uint8_t>> raw;   // PNG: inflated scanlines
  std::vector<int32_t> kind, w, h, bpp;    // kind: 1 JPEG (K13), 2 PNG (K14), 0 other, -1 unreadable
};

extern "C" int mrag_jpeg_decode(const uint8_t* const* files, const int64_t* sizes, int32_t n, uint8_t* out,
                                const int64_t* out_offsets, int32_t device, void* stream);
extern "C" int mrag_png_unfilter(const uint8_t* const* raws, const int32_t* dims, int32_t n, uint8_t* out,
                                 const int64_t* out_offsets, int32_t device, void* stream);

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

void classify(mrag_files& F, int i, const char* path, bool device_decode) {
  std::vector<uint8_t>& d = F.data[i];
  if (!read_file(path, d)) {
    F.kind[i] = -1;
    return;
  }
  F.kind[i] = 0;
  if (!device_decode) return;
  const int64_t n = (int64_t)d.size();
  if (n >= 2 && d[0] == 0xFF && d[1] == 0xD8) {
    mrag_jpeg::Parsed P;
    if (mrag_jpeg::parse(d.data(), n, P)) {
      F.kind[i] = 1;
      F.w[i] = P.img.width;
      F.h[i] = P.img.height;
    }
    return;
  }
  mrag_png::PngParsed P;
  if (mrag_png::png_parse(d.data(), n, P, true)) {
    F.raw[i].resize((size_t)P.raw_bytes);
    if (mrag_png::png_inflate(d.data(), P, F.raw[i].data())) {
      F.kind[i] = 2;
      F.w[i] = P.width;
      F.h[i] = P.height;
      F.bpp[i] = P.bpp;
    } else {
      std::vector<uint8_t>().swap(F.raw[i]);
    }
  }
}

}  // namespace

extern "C" {

int mrag_files_prepare(const char* const* paths, int32_t n, int32_t threads, int32_t device_decode, mrag_files** out) {
  if (!out || n < 0 || (n > 0 && !paths)) return mrag::fail(MRAG_ERR_ARG, "NULL argument");
  *out = nullptr;
  try {
    auto* F = new mrag_files();
    F->n = n;
    F->data.resize((size_t)n);
    F->raw.resize((size_t)n);
    F->kind.assign((size_t)n, 0);
    F->w.assign((size_t)n, 0);
    F->h.assign((size_t)n, 0);
    F->bpp.assign((size_t)n, 0);
    const int nth = std::max(1, std::min<int>(threads > 0 ? threads : 1, n));
    std::atomic<int> next{0};
    std::atomic<bool> thrown{false};
    auto work = [&]() {
      try {
        for (int i = next++; i < n; i = next++) classify(*F, i, paths[i], device_decode != 0);
      } catch (...) {
        thrown = true;
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nth; ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    if (thrown) {
      delete F;
      return mrag::fail(MRAG_ERR_OOM, "files: host allocation failed");
    }
    *out = F;
    return MRAG_OK;
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
  MRAG_REQUIRE(F && out && out_offsets, "NULL argument");
  try {
    std::vector<const uint8_t*> jf, pr;
    std::vector<int64_t> js, jo, po;
    std::vector<int32_t> pd;
    for (int i = 0; i < F->n; ++i) {
      if (F->kind[i] == 1) {
        jf.push_back(F->data[i].data());
        js.push_back((int64_t)F->data[i].size());
        jo.push_back(out_offsets[i]);
      } else if (F->kind[i] == 2) {
        pr.push_back(F->raw[i].data());
        pd.push_back(F->w[i]);
        pd.push_back(F->h[i]);
        pd.push_back(F->bpp[i]);
        po.push_back(out_offsets[i]);
      }
    }
    if (!jf.empty())
      if (int rc = mrag_jpeg_decode(jf.data(), js.data(), (int32_t)jf.size(), out, jo.data(), device, stream)) return rc;
    if (!pr.empty())
      if (int rc = mrag_png_unfilter(pr.data(), pd.data(), (int32_t)pr.size(), out, po.data(), device, stream)) return rc;
    return MRAG_OK;
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "files: host allocation failed");
  }
}

int mrag_files_free(mrag_files* F) {
  delete F;
  return MRAG_OK;
}

}  // extern "C"
