// imgprep.hip — K0: image resize (shortest edge -> size, bicubic) + centre crop on the GPU,
// bit-exact to the reference's CLIPImageProcessor PIL path (app/ml/embeddings.py:84-85 ->
// PIL.Image.resize(BICUBIC) + center_crop; restated on the host in
// app/encoders/preprocess.py:to_u8_224 and in oracle/imgprep.py).
//
// Pillow's 8-bit resampler (libImaging/Resample.c) is fixed point: per output position a
// window [xmin, xmin + n) of int32 taps (double weights normalised to sum 1, scaled by 2^22
// and rounded half away from zero), a horizontal pass (only if the width changes) and a
// vertical pass (only if the height changes), each `clamp((2^21 + sum u8 * tap) >> 22)` back
// to u8. The taps are computed here on the host in double exactly as Pillow does (this file
// is built with -ffp-contract=off); the GPU runs the two integer passes for the 224 x 224
// crop window only (each output pixel depends on its own taps alone, so this equals the full
// resize followed by the crop). A pass whose size does not change becomes one identity tap
// (2^21 + v * 2^22) >> 22 == v, i.e. the same bytes Pillow passes through untouched.
//
// Layout: images are u8 RGB HWC, concatenated (byte offsets); output u8 [n][size][size][3],
// which mrag_encoder_embed_images consumes (normalise + patchify fused there).
#include <array>
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "common.h"

namespace {

constexpr int PRECISION_BITS = 32 - 8 - 2;

struct ImgPlan {
  int64_t src_off;   // byte offset of the image in `pixels`
  int64_t tmp_off;   // byte offset of its horizontal-pass rows in the workspace
  int32_t w, h;      // source size
  int32_t y0, nrows; // source rows the crop needs (pass 1 input rows)
  int32_t hk, vk;    // taps per output column / row (table stride = 2 + taps)
  int32_t hoff, voff;  // int32 index of the column / row tables in `coef`
};

double bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Resample.c precompute_coeffs + normalize_coeffs_8bpc for output positions [o0, o0 + cnt)
// of an in_size -> out_size resize; appends rows of [xmin, n, tap_0 .. tap_{K-1}] to `tab`.
int coeffs(int in_size, int out_size, int o0, int cnt, std::vector<int32_t>& tab) {
  const double scale = (double)((float)in_size - 0.0f) / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  std::vector<double> k((size_t)ksize);
  for (int xx = o0; xx < o0 + cnt; ++xx) {
    const double center = 0.0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    for (int x = 0; x < xmax; ++x) {
      const double w = bicubic((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    tab.push_back(xmin);
    tab.push_back(xmax);
    for (int x = 0; x < ksize; ++x) {
      const double v = x < xmax ? k[x] : 0.0;
      tab.push_back(v < 0 ? (int32_t)(-0.5 + v * (1 << PRECISION_BITS)) : (int32_t)(0.5 + v * (1 << PRECISION_BITS)));
    }
  }
  return ksize;
}

// identity taps: output position o reads source position o0 + o
int identity(int o0, int cnt, std::vector<int32_t>& tab) {
  for (int o = 0; o < cnt; ++o) {
    tab.push_back(o0 + o);
    tab.push_back(1);
    tab.push_back(1 << PRECISION_BITS);
  }
  return 1;
}

__device__ __forceinline__ uint8_t clip8(int v) {
  const int s = v >> PRECISION_BITS;
  return (uint8_t)(s < 0 ? 0 : (s > 255 ? 255 : s));
}

// pass 1: rows [y0, y0 + nrows) of image blockIdx.y, crop columns -> tmp [nrows][size][3].
// Block: RH_ROWS source rows; thread: one output pixel (its three channels share each tap). The
// image's column tap table is staged in LDS when it fits (RH_LDS ints), else read from global.
// Each channel sums its taps in Pillow's order into an int32 (exact in any order anyway).
constexpr int RH_ROWS = 8;
constexpr int RH_LDS = 6144;

__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ px, const ImgPlan* __restrict__ plans,
                                                       const int32_t* __restrict__ coef, uint8_t* __restrict__ tmp,
                                                       int size) {
  __shared__ int32_t stab[RH_LDS];
  const ImgPlan pl = plans[blockIdx.y];
  const int r0 = blockIdx.x * RH_ROWS;
  if (r0 >= pl.nrows) return;  // whole block
  const int stride = 2 + pl.hk;
  const int nt = size * stride;
  const int32_t* gtab = coef + pl.hoff;
  const bool in_lds = nt <= RH_LDS;
  if (in_lds)
    for (int i = threadIdx.x; i < nt; i += blockDim.x) stab[i] = gtab[i];
  __syncthreads();
  auto rows = [&](const int32_t* tab) {
    for (int t = threadIdx.x; t < RH_ROWS * size; t += blockDim.x) {
      const int rr = t / size, x = t - rr * size, r = r0 + rr;
      if (r >= pl.nrows) break;
      const uint8_t* sp = px + pl.src_off + (int64_t)(pl.y0 + r) * pl.w * 3;
      const int32_t* e = tab + x * stride;
      const int xmin = e[0], n = e[1];
      sp += xmin * 3;
      int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
#pragma unroll 4
      for (int j = 0; j < n; ++j) {
        const int c = e[2 + j];
        s0 += (int)sp[3 * j] * c;
        s1 += (int)sp[3 * j + 1] * c;
        s2 += (int)sp[3 * j + 2] * c;
      }
      uint8_t* d = tmp + pl.tmp_off + ((int64_t)r * size + x) * 3;
      d[0] = clip8(s0);
      d[1] = clip8(s1);
      d[2] = clip8(s2);
    }
  };
  if (in_lds)
    rows(stab);
  else
    rows(gtab);
}

// pass 2: crop row blockIdx.x of image blockIdx.y from the pass-1 rows -> out [size][size][3]
__global__ __launch_bounds__(256) void resize_v_kernel(const ImgPlan* __restrict__ plans, const int32_t* __restrict__ coef,
                                                       const uint8_t* __restrict__ tmp, uint8_t* __restrict__ out,
                                                       int size) {
  const ImgPlan pl = plans[blockIdx.y];
  const int y = blockIdx.x;
  const int32_t* e = coef + pl.voff + y * (2 + pl.vk);
  const int ymin = e[0], n = e[1];
  const uint8_t* src = tmp + pl.tmp_off;
  uint8_t* dst = out + ((int64_t)blockIdx.y * size + y) * size * 3;
  for (int t = threadIdx.x; t < size * 3; t += blockDim.x) {
    int ss = 1 << (PRECISION_BITS - 1);
    for (int j = 0; j < n; ++j) ss += (int)src[(int64_t)(ymin + j) * size * 3 + t] * e[2 + j];
    dst[t] = clip8(ss);
  }
}

// Tap tables depend only on (in size, out size, first output, count): images of one size share
// them. A process-wide cache of the tables computed so far (bounded; cleared when full), so a
// batch computes only the sizes it has not met before.
using TapKey = std::array<int, 4>;
struct TapTable {
  std::vector<int32_t> tab;  // rows of [xmin, n, taps ...]
  int k;                     // taps per row
};
std::mutex g_tap_mu;
std::map<TapKey, TapTable> g_taps;

TapTable taps(int in_size, int out_size, int o0, int cnt) {
  const TapKey key{in_size, out_size, o0, cnt};
  std::lock_guard<std::mutex> lk(g_tap_mu);
  auto it = g_taps.find(key);
  if (it != g_taps.end()) return it->second;
  if (g_taps.size() >= 4096) g_taps.clear();
  TapTable t;
  t.k = out_size != in_size ? coeffs(in_size, out_size, o0, cnt, t.tab) : identity(o0, cnt, t.tab);
  g_taps.emplace(key, t);
  return t;
}

// grow-only device workspace (per process; calls are serialised by `mu`)
struct Workspace {
  std::mutex mu;
  void* p = nullptr;
  size_t cap = 0;
  int dev = -1;
};
Workspace g_ws;

}  // namespace

extern "C" int mrag_image_resize_crop(const uint8_t* pixels, const int64_t* offsets, const int32_t* widths,
                                      const int32_t* heights, int32_t n, int32_t size, uint8_t* out, void* stream) {
  MRAG_REQUIRE(n >= 0, "n=%d", n);
  if (n == 0) return MRAG_OK;
  MRAG_REQUIRE(pixels && offsets && widths && heights && out, "NULL pointer");
  MRAG_REQUIRE(size > 0 && size <= 4096, "size=%d", size);
  std::vector<ImgPlan> plans((size_t)n);
  std::vector<int32_t> coef;
  int64_t tmp_bytes = 0;
  int max_rows = 0;
  // tables of this call, one copy per distinct key: offset, taps, and for row tables the source
  // rows the crop reads (the table is stored relative to its first row)
  struct Placed {
    int32_t off, k, y0, nrows;
  };
  std::map<TapKey, Placed> placed_h, placed_v;
  auto place = [&](std::map<TapKey, Placed>& m, int in_size, int out_size, int o0, bool rows) -> Placed {
    const TapKey key{in_size, out_size, o0, size};
    auto it = m.find(key);
    if (it != m.end()) return it->second;
    TapTable t = taps(in_size, out_size, o0, size);
    Placed p{(int32_t)coef.size(), t.k, 0, 0};
    if (rows) {
      int y0 = 1 << 30, y1 = 0;
      for (int y = 0; y < size; ++y) {
        const int32_t* e = &t.tab[(size_t)y * (2 + t.k)];
        y0 = std::min(y0, (int)e[0]);
        y1 = std::max(y1, (int)(e[0] + e[1]));
      }
      for (int y = 0; y < size; ++y) t.tab[(size_t)y * (2 + t.k)] -= y0;
      p.y0 = y0;
      p.nrows = y1 - y0;
    }
    coef.insert(coef.end(), t.tab.begin(), t.tab.end());
    m.emplace(key, p);
    return p;
  };
  for (int i = 0; i < n; ++i) {
    const int w = widths[i], h = heights[i];
    MRAG_REQUIRE(w > 0 && h > 0 && offsets[i] >= 0, "image %d: bad size %dx%d / offset", i, w, h);
    // transformers get_resize_output_image_size(default_to_square=False): shortest edge -> size
    const int shrt = w <= h ? w : h, lng = w <= h ? h : w;
    const int nshort = size, nlong = (int)((double)size * lng / shrt);
    const int nw = w <= h ? nshort : nlong, nh = w <= h ? nlong : nshort;
    const int top = (nh - size) / 2, left = (nw - size) / 2;  // both >= 0: nlong >= size
    ImgPlan& pl = plans[(size_t)i];
    pl.src_off = offsets[i];
    pl.w = w;
    pl.h = h;
    const Placed ph = place(placed_h, w, nw, left, false);
    const Placed pv = place(placed_v, h, nh, top, true);
    pl.hoff = ph.off;
    pl.hk = ph.k;
    pl.voff = pv.off;
    pl.vk = pv.k;
    pl.y0 = pv.y0;
    pl.nrows = pv.nrows;
    pl.tmp_off = tmp_bytes;
    tmp_bytes += ((int64_t)pl.nrows * size * 3 + 255) / 256 * 256;
    max_rows = std::max(max_rows, pl.nrows);
    MRAG_REQUIRE(coef.size() < (1u << 31), "coefficient table too large");
  }
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> lock(g_ws.mu);
  int dev = 0;
  MRAG_HIP(hipGetDevice(&dev));
  const size_t plan_bytes = (size_t)n * sizeof(ImgPlan);
  const size_t coef_off = (plan_bytes + 255) / 256 * 256;
  const size_t tmp_off = coef_off + (coef.size() * 4 + 255) / 256 * 256;
  const size_t need = tmp_off + (size_t)tmp_bytes;
  if (need > g_ws.cap || dev != g_ws.dev) {
    if (g_ws.p) (void)hipFree(g_ws.p);
    g_ws.p = nullptr;
    g_ws.cap = 0;
    MRAG_HIP(hipMalloc(&g_ws.p, need));
    g_ws.cap = need;
    g_ws.dev = dev;
  }
  char* ws = (char*)g_ws.p;
  MRAG_HIP(hipMemcpyAsync(ws, plans.data(), plan_bytes, hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemcpyAsync(ws + coef_off, coef.data(), coef.size() * 4, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(resize_h_kernel, dim3((unsigned)((max_rows + RH_ROWS - 1) / RH_ROWS), (unsigned)n), dim3(256), 0, s, pixels,
                     (const ImgPlan*)ws, (const int32_t*)(ws + coef_off), (uint8_t*)(ws + tmp_off), size);
  MRAG_CHECK_LAUNCH();
  hipLaunchKernelGGL(resize_v_kernel, dim3((unsigned)size, (unsigned)n), dim3(256), 0, s, (const ImgPlan*)ws,
                     (const int32_t*)(ws + coef_off), (const uint8_t*)(ws + tmp_off), out, size);
  MRAG_CHECK_LAUNCH();
  // the host-side plan / coefficient vectors must outlive their copies
  if (int rc = mrag::blocking_wait(s)) return rc;
  return MRAG_OK;
}
