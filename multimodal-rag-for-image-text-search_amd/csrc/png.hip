// png.hip — K14: PNG scanline reconstruction + convert("RGB") on the GPU (decode ->
// resize -> crop on the device). Reference: app/ml/embeddings.py:82-89 decodes every file with
// Pillow (Image.open(path).convert("RGB")); png_core.h restates what Pillow's PNG decoder and
// convert do with 8-bit L / LA / RGB / RGBA non-interlaced files, so the bytes are Pillow's.
//
// The zlib inflate of the IDAT stream stays on the host (png_parse.h, mrag_png_inflate, called on
// the caller's decode threads); the filtered scanlines of a batch go to the device in one copy and
//   K14 png_unfilter_kernel  one workgroup per image, one wave per 64-row band (16 bands in flight,
//                            taller images in groups of 16 bands). Within a band, lane l
//                            reconstructs row r0 + l one pixel behind lane l - 1 (a skewed
//                            wavefront): the pixel above (b) arrives from lane l - 1's previous
//                            step by a DPP lane shift, the above-left one (c) is the lane's own
//                            previous b, the left one (a) its own previous pixel. Band k starts two
//                            64-step chunks after band k - 1, and its lane 0 reads the row above
//                            from the LDS ring band k - 1's lane 63 fills, so the bands of an
//                            image advance together on one diagonal (w + h steps instead of
//                            h / 64 x (w + 63)); the waves meet at one barrier per chunk. A lane
//                            loads four filtered pixels with one (unaligned) vector load, eight
//                            steps ahead, and stores their RGB bytes with one 12-byte store at the
//                            caller's offsets (the H x W x 3 layout K0 resizes from). One instance
//                            per pixel size (1 L, 2 LA, 3 RGB, 4 RGBA).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"
#include "png_parse.h"
#include "staged.h"

using namespace mrag_png;

namespace {

struct PngImg {
  int64_t raw_off, out_off;
  int32_t w, h, bpp, pad;
};

constexpr int PNG_WAVES = 16;   // bands (64 rows each) in flight per image
constexpr int PNG_RING = 256;   // columns of a band's bottom row kept for the band below

// pixels q = 0..3 (BPP bytes each, packed) out of 4 x BPP consecutive bytes held in BPP words
template <int BPP>
__device__ __forceinline__ uint32_t pixel_of(const uint32_t (&wd)[BPP], int q) {
  const int o = q * BPP, wq = o >> 2, sh = (o & 3) * 8;
  uint32_t v = wd[wq] >> sh;
  if (sh && wq + 1 < BPP) v |= wd[wq + 1] << (32 - sh);
  return BPP == 4 ? v : (v & ((1u << (8 * BPP)) - 1u));
}

template <int BPP>
__global__ __launch_bounds__(64 * PNG_WAVES) void png_unfilter_kernel(const PngImg* __restrict__ imgs,
                                                                      const uint8_t* __restrict__ raw,
                                                                      uint8_t* __restrict__ out) {
  __shared__ uint32_t carry[PNG_MAXW];                // bottom row of the previous band group
  __shared__ uint32_t ring[PNG_WAVES - 1][PNG_RING];  // bottom row of band k, read by band k + 1
  const PngImg im = imgs[blockIdx.x];
  if (im.bpp != BPP) return;  // whole workgroup: images of another pixel size are another launch's
  const int lane = threadIdx.x & 63;
  const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int w = im.w, h = im.h;
  const int64_t stride = 1 + (int64_t)w * BPP;
  const int bands = (h + 63) / 64;
  for (int g0 = 0; g0 < bands; g0 += PNG_WAVES) {
    const int nb = std::min(PNG_WAVES, bands - g0);
    const bool wact = k < nb;
    const int r = (g0 + k) * 64 + lane;
    const bool act = wact && r < h;
    const uint8_t* row = raw + im.raw_off + (int64_t)(act ? r : 0) * stride;
    const int ft = act ? row[0] : 0;
    const uint8_t* px = row + 1;
    uint8_t* o = out + im.out_off + (int64_t)(act ? r : 0) * w * 3;
    // four pixels (columns j0 .. j0 + 3) of this lane's row: one unaligned vector load inside
    // the row, pixel by pixel at its ends, 0 outside
    auto load4 = [&](int j0, uint32_t (&v)[4]) {
      if (act && j0 >= 0 && j0 + 3 < w) {
        uint32_t wd[BPP];
        __builtin_memcpy(wd, px + (int64_t)j0 * BPP, 4 * BPP);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = pixel_of<BPP>(wd, q);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = j0 + q;
          v[q] = (act && j >= 0 && j < w) ? load_pixel(px + (int64_t)j * BPP, BPP) : 0u;
        }
      }
    };
    // band k's local step s = global step - 128 k; column j = s - lane
    const int nchunks = (128 * (nb - 1) + w + 63 + 63) / 64;
    uint32_t xprev = 0, bprev = 0;
    uint32_t pre[2][4];  // the next two groups of four steps, loaded eight steps ahead
    load4(-lane, pre[0]);
    load4(4 - lane, pre[1]);
    for (int t = 0; t < nchunks; ++t) {
      const int s0 = 64 * t - 128 * k;  // a multiple of 64: the band runs from local step 0
      if (wact && s0 >= 0 && s0 < w + 63) {
        for (int i0 = 0; i0 < 64; i0 += 8) {
#pragma unroll
          for (int gq = 0; gq < 2; ++gq) {
            const int j0 = s0 + i0 + 4 * gq - lane;  // this lane's column at the group's first step
            uint32_t x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x[q] = pre[gq][q];
            load4(j0 + 8, pre[gq]);
            uint32_t rgbw[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int j = j0 + q;
              // lane l - 1 reconstructed row r - 1, column j, one step ago (lane 0: 0)
              const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xprev, 0x138, 0xf, 0xf, false);
              const bool inside = j >= 0 && j < w;
              uint32_t b = up;
              if (lane == 0) b = !inside ? 0u : k > 0 ? ring[k - 1][j & (PNG_RING - 1)] : g0 > 0 ? carry[j] : 0u;
              uint32_t v = 0;
              if (act && inside) {
                const uint32_t a = j > 0 ? xprev : 0u, c = j > 0 ? bprev : 0u;
                v = recon_pixel(ft, x[q], a, b, c, BPP);
                if (lane == 63) {
                  if (k < nb - 1) ring[k][j & (PNG_RING - 1)] = v;  // read two chunks later by band k + 1
                  else carry[j] = v;                                // read by the next band group
                }
                xprev = v;
                bprev = b;
              }
              rgbw[q] = BPP <= 2 ? (v & 0xFF) * 0x010101u : (v & 0xFFFFFFu);
            }
            // RGB of the four pixels: one 12-byte store inside the row, byte stores at its ends
            if (act && j0 >= 0 && j0 + 3 < w) {
              const uint32_t ow[3] = {rgbw[0] | rgbw[1] << 24, rgbw[1] >> 8 | rgbw[2] << 16, rgbw[2] >> 16 | rgbw[3] << 8};
              __builtin_memcpy(o + (int64_t)j0 * 3, ow, 12);
            } else if (act) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int j = j0 + q;
                if (j >= 0 && j < w) {
                  uint8_t* d = o + (int64_t)j * 3;
                  d[0] = (uint8_t)rgbw[q];
                  d[1] = (uint8_t)(rgbw[q] >> 8);
                  d[2] = (uint8_t)(rgbw[q] >> 16);
                }
              }
            }
          }
        }
      }
      __syncthreads();
    }
  }
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};
int ensure(DevBuf& b, size_t bytes) {
  if (bytes <= b.cap) return MRAG_OK;
  const size_t c = std::max(bytes, b.cap * 2);
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  MRAG_HIP(hipMalloc(&b.p, c));
  b.cap = c;
  return MRAG_OK;
}

// Per-device scratch, grown on demand and reused by every batch (calls serialise on its lock).
struct Ctx {
  std::mutex mu;
  DevBuf raw, imgs;
  uint8_t* stage = nullptr;  // pinned host staging of the filtered scanlines
  size_t stage_cap = 0;
};
Ctx g_ctx[64];

}  // namespace

extern "C" {

static int png_probe_impl(const uint8_t* data, int64_t size, int32_t* width, int32_t* height, int64_t* raw_bytes) {
  if (!data || !width || !height || !raw_bytes || size < 0) return -mrag::fail(MRAG_ERR_ARG, "NULL argument");
  PngParsed P;
  if (!png_parse(data, size, P, true)) {
    *width = *height = 0;
    *raw_bytes = 0;
    return 0;
  }
  *width = P.width;
  *height = P.height;
  *raw_bytes = P.raw_bytes;
  return 1;
}

static int png_inflate_impl(const uint8_t* data, int64_t size, uint8_t* raw, int64_t cap, int32_t* bpp) {
  if (!data || !raw || !bpp || size < 0) return -mrag::fail(MRAG_ERR_ARG, "NULL argument");
  PngParsed P;
  if (!png_parse(data, size, P, false)) return 0;
  if (cap < P.raw_bytes) return -mrag::fail(MRAG_ERR_ARG, "raw buffer of %lld bytes, %lld needed", (long long)cap,
                                            (long long)P.raw_bytes);
  if (!png_inflate(data, P, raw)) return 0;
  *bpp = P.bpp;
  return 1;
}

// staged == nullptr: raws[i] anywhere in host memory, copied here into the pinned stage; otherwise
// image i's scanlines at staged + raw_off[i], inside staged[0 .. staged_bytes) (staged.h)
static int png_unfilter_impl(const uint8_t* const* raws, const int32_t* dims, int32_t n, uint8_t* out,
                             const int64_t* out_offsets, int32_t device, void* stream, const uint8_t* staged,
                             int64_t staged_bytes, const int64_t* raw_off) {
  MRAG_REQUIRE(n >= 0, "negative batch");
  if (n == 0) return MRAG_OK;
  MRAG_REQUIRE((staged ? raw_off != nullptr : raws != nullptr) && dims && out && out_offsets, "NULL argument");
  MRAG_REQUIRE(device >= 0 && device < 64, "bad device %d", device);
  std::vector<PngImg> imgs((size_t)n);
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    const int w = dims[3 * i], h = dims[3 * i + 1], bpp = dims[3 * i + 2];
    MRAG_REQUIRE(staged || raws[i] != nullptr, "NULL image %d", i);
    MRAG_REQUIRE(w >= 1 && w <= PNG_MAXW && h >= 1 && h <= 65535 && bpp >= 1 && bpp <= 4,
                 "png %d: %d x %d, %d bytes per pixel unsupported", i, w, h, bpp);
    const int64_t bytes = (int64_t)h * (1 + (int64_t)w * bpp);
    if (staged)
      MRAG_REQUIRE(raw_off[i] >= 0 && raw_off[i] + bytes <= staged_bytes, "png %d: scanlines outside the stage", i);
    imgs[i] = PngImg{staged ? raw_off[i] : total, out_offsets[i], w, h, bpp, 0};
    total += bytes;
  }
  if (staged) total = staged_bytes;
  mrag::DeviceGuard g(device);
  Ctx& C = g_ctx[device];
  std::lock_guard<std::mutex> lk(C.mu);
  hipStream_t s = (hipStream_t)stream;
  if (!staged && total > (int64_t)C.stage_cap) {
    const size_t cap = std::max<size_t>((size_t)total, C.stage_cap * 2);
    if (int rc = mrag::blocking_wait(s)) return rc;
    if (C.stage) (void)hipHostFree(C.stage);
    C.stage = nullptr;
    C.stage_cap = 0;
    MRAG_HIP(hipHostMalloc((void**)&C.stage, cap, hipHostMallocDefault));
    C.stage_cap = cap;
  }
  if (!staged) {
    if (int rc = mrag::blocking_wait(s)) return rc;  // the previous batch's copy out of the stage is done
    const int nth =
        (int)std::max<int64_t>(1, std::min<int64_t>({8, (int64_t)std::thread::hardware_concurrency(), (n + 3) / 4}));
    std::vector<std::thread> th;
    auto copy = [&](int w0) {
      for (int i = w0; i < n; i += nth)
        std::memcpy(C.stage + imgs[i].raw_off, raws[i],
                    (size_t)((int64_t)imgs[i].h * (1 + (int64_t)imgs[i].w * imgs[i].bpp)));
    };
    for (int w0 = 1; w0 < nth; ++w0) th.emplace_back(copy, w0);
    copy(0);
    for (auto& t : th) t.join();
  }
  if (int rc = ensure(C.raw, (size_t)total)) return rc;
  if (int rc = ensure(C.imgs, sizeof(PngImg) * (size_t)n)) return rc;
  // an error return from here on first drains s: the copies read imgs on this stack frame and the
  // staging buffer, which the caller may hand back to its pool
  mrag::StreamDrain drain(s);
  MRAG_HIP(hipMemcpyAsync(C.raw.p, staged ? staged : C.stage, (size_t)total, hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemcpyAsync(C.imgs.p, imgs.data(), sizeof(PngImg) * (size_t)n, hipMemcpyHostToDevice, s));
  // one launch per pixel size present (a workgroup of another size returns at once)
  bool has[5] = {false, false, false, false, false};
  for (const PngImg& q : imgs) has[q.bpp] = true;
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)n), dim3(64 * PNG_WAVES), 0, s, (const PngImg*)C.imgs.p,
                       (const uint8_t*)C.raw.p, out);
  };
  if (has[1]) launch(png_unfilter_kernel<1>);
  if (has[2]) launch(png_unfilter_kernel<2>);
  if (has[3]) launch(png_unfilter_kernel<3>);
  if (has[4]) launch(png_unfilter_kernel<4>);
  MRAG_CHECK_LAUNCH();
  if (int rc = mrag::blocking_wait(s)) return rc;  // the descriptors live on this stack frame
  drain.armed = false;
  return MRAG_OK;
}

// the C ABI: no C++ exception crosses it (a failed host allocation is MRAG_ERR_OOM)
int mrag_png_probe(const uint8_t* data, int64_t size, int32_t* width, int32_t* height, int64_t* raw_bytes) {
  try {
    return png_probe_impl(data, size, width, height, raw_bytes);
  } catch (...) {
    return -mrag::fail(MRAG_ERR_OOM, "png probe: host allocation failed");
  }
}

int mrag_png_inflate(const uint8_t* data, int64_t size, uint8_t* raw, int64_t cap, int32_t* bpp) {
  try {
    return png_inflate_impl(data, size, raw, cap, bpp);
  } catch (...) {
    return -mrag::fail(MRAG_ERR_OOM, "png inflate: host allocation failed");
  }
}

int mrag_png_unfilter(const uint8_t* const* raws, const int32_t* dims, int32_t n, uint8_t* out,
                      const int64_t* out_offsets, int32_t device, void* stream) {
  try {
    return png_unfilter_impl(raws, dims, n, out, out_offsets, device, stream, nullptr, 0, nullptr);
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "png unfilter: host allocation failed");
  }
}

}  // extern "C"

int mrag_stage::png_unfilter_staged(const uint8_t* stage, int64_t bytes, const int64_t* raw_off, const int32_t* dims,
                                    int32_t n, uint8_t* out, const int64_t* out_offsets, int32_t device, void* stream) {
  try {
    return png_unfilter_impl(nullptr, dims, n, out, out_offsets, device, stream, stage, bytes, raw_off);
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "png unfilter: host allocation failed");
  }
}
