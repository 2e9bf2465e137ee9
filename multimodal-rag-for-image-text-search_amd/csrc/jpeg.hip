// jpeg.hip — K13: baseline JPEG decode on the GPU (decode -> resize -> crop on the
// device). Reference: app/ml/embeddings.py:82-89 decodes every file with Pillow
// (Image.open(path).convert("RGB")); the arithmetic restated in jpeg_core.h gives Pillow's bytes.
//
// A batch of files is parsed on the host (jpeg_parse.h: tables, geometry, entropy-coded segments;
// host threads, one file each), every segment's bytes are unstuffed into one pinned buffer and go
// to the device in one copy, and three kernels run:
//   K13a jpeg_huff_par_kernel  one workgroup per entropy-coded segment (a whole image, or one
//                           restart interval), one chunk of the segment's bits per lane (up to
//                           1024): self-synchronising parallel Huffman decode (jpeg_core.h,
//                           par_run) into zeroed int16 coefficient blocks, the same tokens and
//                           values as the sequential decoder (round 5 first shipped that one, one
//                           single-lane workgroup per segment: 70-78 ms per launch, the largest
//                           file's serial chain).
//   K13b jpeg_idct_kernel   one thread per 8x8 block: dequantise + islow IDCT into the planes.
//   K13c jpeg_color_kernel  one thread per four pixels of a row: fancy chroma upsampling +
//                           YCbCr -> RGB, H x W x 3 u8 at the caller's offset (the layout K0
//                           resizes from), 12 bytes per store.
// Files K13 does not support (progressive, arithmetic, CMYK, 4:4:0, tiny chroma) are reported by
// mrag_jpeg_probe and decoded on the host by the caller, as the reference decodes everything.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"
#include "jpeg_parse.h"
#include "staged.h"

using namespace mrag_jpeg;

namespace {

// one entropy-coded segment on the device: unstuffed bytes at uoff (16-byte aligned, zero to the
// next 16-byte boundary), nbits = 8 x their count
struct ParSeg {
  int64_t uoff;
  uint32_t nbits;
  int32_t img, mcu0, mcus;
};

// K13a: the passes of decode_segment_par (jpeg_parse.h, its host emulation), one lane per chunk.
__global__ __launch_bounds__(PAR_LANES) void jpeg_huff_par_kernel(const Image* __restrict__ imgs,
                                                                  const ParSeg* __restrict__ segs,
                                                                  const uint8_t* __restrict__ ecs,
                                                                  int16_t* __restrict__ coef) {
  __shared__ PTabs T;
  __shared__ PState ex[PAR_LANES];
  __shared__ PCheck cps[PAR_NCP * PAR_LANES];
  __shared__ int32_t scan[4][PAR_LANES];
  const ParSeg sg = segs[blockIdx.x];
  const Image* im = imgs + sg.img;
  const int t = threadIdx.x;
  {
    constexpr int W = (int)(4 * sizeof(Huff) / 4);
    const uint32_t* src = (const uint32_t*)&im->dc[0];
    uint32_t* dst = (uint32_t*)&T.h[0];
    for (int i = t; i < W; i += PAR_LANES) dst[i] = src[i];
    if (t == 0) make_ptab_ids(*im, T);
  }
  __syncthreads();
  int nl;
  uint32_t chunk;
  par_geom(sg.nbits, nl, chunk);
  const bool act = t < nl;
  uint32_t start = 0, end = 0, cpos[PAR_NCP];
  par_lane(sg.nbits, nl, chunk, act ? t : 0, start, end, cpos);
  const uint8_t* data = ecs + sg.uoff;
  const uint32_t nbytes = sg.nbits / 8;
  PBits br;
  PState entry{start, 0}, myexit{start, 0};
  int32_t tot[4] = {0, 0, 0, 0};
  if (act) {
    br.init(data, nbytes, start);
    PState st = entry;
    par_run<PAR_RECORD>(T, br, st, end, tot, cps + t, PAR_LANES, cpos, nullptr, im, nullptr, 0, 0, 0, nullptr);
    myexit = st;
    ex[t] = st;
  }
  while (true) {  // resynchronisation rounds, until no exit changes
    __syncthreads();
    bool redo = false;
    PState e{0, 0};
    if (act && t > 0) {
      e = ex[t - 1];
      redo = e.p != entry.p || e.bk != entry.bk;
    }
    __syncthreads();  // every exit read before any is rewritten
    int changed = 0;
    if (redo) {
      entry = e;
      PState st = e;
      br.init(data, nbytes, e.p);
      int32_t m[4] = {0, 0, 0, 0};
      const bool synced =
          par_run<PAR_SYNC>(T, br, st, end, m, cps + t, PAR_LANES, cpos, tot, im, nullptr, 0, 0, 0, nullptr);
      for (int q = 0; q < 4; ++q) tot[q] = m[q];
      if (!synced && (st.p != myexit.p || st.bk != myexit.bk)) {
        myexit = st;
        ex[t] = st;
        changed = 1;
      }
    }
    if (!__syncthreads_or(changed)) break;
  }
  // first block and DC predictors of every lane: exclusive prefix sums of the chunk totals
  for (int q = 0; q < 4; ++q) scan[q][t] = act ? tot[q] : 0;
  __syncthreads();
  for (int off = 1; off < PAR_LANES; off <<= 1) {
    int32_t v[4];
    for (int q = 0; q < 4; ++q) v[q] = t >= off ? scan[q][t - off] : 0;
    __syncthreads();
    for (int q = 0; q < 4; ++q) scan[q][t] += v[q];
    __syncthreads();
  }
  if (act) {
    int32_t pre[4];
    for (int q = 0; q < 4; ++q) pre[q] = scan[q][t] - tot[q];
    int32_t pred[3] = {pre[1], pre[2], pre[3]};
    PState st = entry;  // exact: lane 0 starts at bit 0, lane t at lane t - 1's final exit
    br.init(data, nbytes, st.p);
    int32_t n[4] = {0, 0, 0, 0};
    par_run<PAR_WRITE>(T, br, st, t == nl - 1 ? 0xFFFFFFFFu : end, n, nullptr, 0, nullptr, nullptr, im,
                       coef + im->coef_off * 64, pre[0], (int64_t)sg.mcus * T.bpm, sg.mcu0, pred);
  }
}

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const Image* __restrict__ imgs, const int16_t* __restrict__ coef,
                                                        uint8_t* __restrict__ planes) {
  const Image& im = imgs[blockIdx.y];
  int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int c = 0; c < im.ncomp; ++c) {
    const int64_t nb = (int64_t)im.comp[c].bw * im.comp[c].bh;
    if (b < nb) {
      idct_block(im, coef + im.coef_off * 64, planes + im.plane_off, c, b);
      return;
    }
    b -= nb;
  }
}

// K13c: four consecutive pixels of a row per thread, their 12 RGB bytes in one store
__global__ __launch_bounds__(256) void jpeg_color_kernel(const Image* __restrict__ imgs,
                                                         const uint8_t* __restrict__ planes, uint8_t* __restrict__ out) {
  const Image& im = imgs[blockIdx.y];
  const int qw = (im.width + 3) / 4;  // quads per row
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)qw * im.height) return;
  const int y = (int)(p / qw), x0 = (int)(p - (int64_t)y * qw) * 4;
  uint8_t rgb[12];
  const int nx = im.width - x0 < 4 ? im.width - x0 : 4;
  for (int q = 0; q < nx; ++q) color_pixel(im, planes + im.plane_off, x0 + q, y, rgb + 3 * q);
  uint8_t* o = out + im.rgb_off + ((int64_t)y * im.width + x0) * 3;
  if (nx == 4) {
    __builtin_memcpy(o, rgb, 12);
  } else {
    for (int i = 0; i < 3 * nx; ++i) o[i] = rgb[i];
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
  DevBuf ecs, imgs, segs, coef, planes;
  uint8_t* stage = nullptr;  // pinned host staging of the entropy-coded bytes
  size_t stage_cap = 0;
};
Ctx g_ctx[64];

}  // namespace

extern "C" {

static int jpeg_probe_impl(const uint8_t* data, int64_t size, int32_t* width, int32_t* height) {
  if (!data || !width || !height || size < 0) return -mrag::fail(MRAG_ERR_ARG, "NULL argument");  // not 1
  Parsed P;
  if (!parse(data, size, P)) {
    *width = *height = 0;
    return 0;
  }
  *width = P.img.width;
  *height = P.img.height;
  return 1;
}

// st == nullptr: parse the files and unstuff their segments here; otherwise the caller's staged
// parse and unstuffed bytes (staged.h; files / sizes unused)
static int jpeg_decode_impl(const uint8_t* const* files, const int64_t* sizes, int32_t n, uint8_t* out,
                            const int64_t* out_offsets, int32_t device, void* stream,
                            const mrag_stage::JpegStaged* st) {
  MRAG_REQUIRE(n >= 0, "negative batch");
  if (n == 0) return MRAG_OK;
  MRAG_REQUIRE((st ? (st->P && st->stage && st->nbits) : (files && sizes)) && out && out_offsets, "NULL argument");
  MRAG_REQUIRE(device >= 0 && device < 64, "bad device %d", device);
  if (!st)
    for (int i = 0; i < n; ++i) MRAG_REQUIRE(files[i] != nullptr && sizes[i] >= 0, "bad file %d", i);
  mrag::DeviceGuard g(device);
  Ctx& C = g_ctx[device];
  std::lock_guard<std::mutex> lk(C.mu);
  hipStream_t s = (hipStream_t)stream;

  // host threads over the files: parse, then (below) unstuff into the pinned stage
  const int nth = (int)std::max<int64_t>(1, std::min<int64_t>({8, (int64_t)std::thread::hardware_concurrency(), (n + 15) / 16}));
  std::atomic<bool> thrown{false};  // an exception (allocation) on a host thread: reported, not std::terminate
  auto parallel = [&](auto fn) {
    auto part = [&](int w) {
      try {
        for (int i = w; i < n; i += nth) fn(i);
      } catch (...) {
        thrown = true;
      }
    };
    std::vector<std::thread> th;
    for (int w = 1; w < nth; ++w) th.emplace_back(part, w);
    part(0);
    for (auto& x : th) x.join();
  };
  std::vector<Parsed> Pv;
  std::vector<const Parsed*> P((size_t)n);
  std::vector<char> ok((size_t)n, 1);
  if (st) {
    for (int i = 0; i < n; ++i) P[i] = st->P[i];
  } else {
    Pv.resize((size_t)n);
    parallel([&](int i) { ok[i] = parse(files[i], sizes[i], Pv[i]) ? 1 : 0; });
    if (thrown) return mrag::fail(MRAG_ERR_OOM, "jpeg: host allocation failed while parsing");
    for (int i = 0; i < n; ++i) P[i] = &Pv[i];
  }
  std::vector<Image> imgs((size_t)n);
  std::vector<ParSeg> segs;
  std::vector<int64_t> seg_src;  // raw segment start in its file
  std::vector<int64_t> seg_len;
  int64_t stage_bytes = 0, blocks = 0, planes = 0, max_blocks = 0, max_quads = 0;
  for (int i = 0; i < n; ++i) {
    if (!ok[i]) return mrag::fail(MRAG_ERR_ARG, "jpeg %d unsupported: %s", i, P[i]->why.c_str());
    Image& im = imgs[i] = P[i]->img;
    im.seg0 = (int32_t)segs.size();
    im.coef_off = blocks;
    im.plane_off = planes;
    im.rgb_off = out_offsets[i];
    for (const Segment& sg : P[i]->segs) {
      MRAG_REQUIRE(sg.len < (1ll << 28), "jpeg %d: entropy-coded segment of %lld bytes", i, (long long)sg.len);
      ParSeg ps;
      ps.uoff = stage_bytes;
      ps.nbits = 0;
      ps.img = i;
      ps.mcu0 = sg.mcu0;
      ps.mcus = sg.mcus;
      segs.push_back(ps);
      seg_src.push_back(sg.off);
      seg_len.push_back(sg.len);
      stage_bytes += mrag_stage::jpeg_seg_stage_bytes(sg.len);  // unstuffed <= raw; zero tail to 16 bytes
    }
    blocks += P[i]->coef_blocks;
    planes += P[i]->plane_bytes;
    max_blocks = std::max(max_blocks, P[i]->coef_blocks);
    max_quads = std::max(max_quads, (int64_t)(im.width + 3) / 4 * im.height);
  }
  const uint8_t* src = C.stage;
  if (st) {
    MRAG_REQUIRE(st->bytes == stage_bytes, "jpeg: staged %lld bytes, the layout needs %lld", (long long)st->bytes,
                 (long long)stage_bytes);
    for (size_t q = 0; q < segs.size(); ++q) segs[q].nbits = st->nbits[q];
    src = st->stage;
  } else if (stage_bytes > (int64_t)C.stage_cap) {
    const size_t cap = std::max<size_t>((size_t)stage_bytes, C.stage_cap * 2);
    if (int rc = mrag::blocking_wait(s)) return rc;  // a previous batch's copy may still read the old buffer
    if (C.stage) (void)hipHostFree(C.stage);
    C.stage = nullptr;
    C.stage_cap = 0;
    MRAG_HIP(hipHostMalloc((void**)&C.stage, cap, hipHostMallocDefault));
    C.stage_cap = cap;
  }
  if (!st) {
    // the previous batch's copy out of the staging buffer must be done before it is rewritten
    if (int rc = mrag::blocking_wait(s)) return rc;
    src = C.stage;
    parallel([&](int i) {
      for (int q = imgs[i].seg0, e = imgs[i].seg0 + (int)P[i]->segs.size(); q < e; ++q) {
        uint8_t* dst = C.stage + segs[q].uoff;
        const int64_t u = unstuff(files[i] + seg_src[q], seg_len[q], dst);
        std::memset(dst + u, 0, (size_t)((u + 15) / 16 * 16 - u));
        segs[q].nbits = (uint32_t)(u * 8);
      }
    });
    if (thrown) return mrag::fail(MRAG_ERR_OOM, "jpeg: host allocation failed while staging");
  }
  if (int rc = ensure(C.ecs, (size_t)stage_bytes)) return rc;
  if (int rc = ensure(C.imgs, sizeof(Image) * (size_t)n)) return rc;
  if (int rc = ensure(C.segs, sizeof(ParSeg) * segs.size())) return rc;
  if (int rc = ensure(C.coef, (size_t)blocks * 128)) return rc;
  if (int rc = ensure(C.planes, (size_t)planes)) return rc;
  // an error return from here on first drains s: the copies read imgs / segs on this stack frame
  // and the staging arena, which the caller may hand back to its pool
  mrag::StreamDrain drain(s);
  MRAG_HIP(hipMemcpyAsync(C.ecs.p, src, (size_t)stage_bytes, hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemcpyAsync(C.imgs.p, imgs.data(), sizeof(Image) * (size_t)n, hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemcpyAsync(C.segs.p, segs.data(), sizeof(ParSeg) * segs.size(), hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemsetAsync(C.coef.p, 0, (size_t)blocks * 128, s));
  hipLaunchKernelGGL(jpeg_huff_par_kernel, dim3((unsigned)segs.size()), dim3(PAR_LANES), 0, s, (const Image*)C.imgs.p,
                     (const ParSeg*)C.segs.p, (const uint8_t*)C.ecs.p, (int16_t*)C.coef.p);
  MRAG_CHECK_LAUNCH();
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((max_blocks + 255) / 256), (unsigned)n), dim3(256), 0, s,
                     (const Image*)C.imgs.p, (const int16_t*)C.coef.p, (uint8_t*)C.planes.p);
  MRAG_CHECK_LAUNCH();
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((max_quads + 255) / 256), (unsigned)n), dim3(256), 0, s,
                     (const Image*)C.imgs.p, (const uint8_t*)C.planes.p, out);
  MRAG_CHECK_LAUNCH();
  // the descriptors above live on this host stack frame: the copies must finish before return
  if (int rc = mrag::blocking_wait(s)) return rc;
  drain.armed = false;
  return MRAG_OK;
}

// the C ABI: no C++ exception crosses it (a failed host allocation is MRAG_ERR_OOM)
int mrag_jpeg_probe(const uint8_t* data, int64_t size, int32_t* width, int32_t* height) {
  try {
    return jpeg_probe_impl(data, size, width, height);
  } catch (...) {
    return -mrag::fail(MRAG_ERR_OOM, "jpeg probe: host allocation failed");
  }
}

int mrag_jpeg_decode(const uint8_t* const* files, const int64_t* sizes, int32_t n, uint8_t* out,
                     const int64_t* out_offsets, int32_t device, void* stream) {
  try {
    return jpeg_decode_impl(files, sizes, n, out, out_offsets, device, stream, nullptr);
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "jpeg decode: host allocation failed");
  }
}

}  // extern "C"

int mrag_stage::jpeg_decode_staged(const JpegStaged& st, int32_t n, uint8_t* out, const int64_t* out_offsets,
                                   int32_t device, void* stream) {
  try {
    return jpeg_decode_impl(nullptr, nullptr, n, out, out_offsets, device, stream, &st);
  } catch (...) {
    return mrag::fail(MRAG_ERR_OOM, "jpeg decode: host allocation failed");
  }
}
