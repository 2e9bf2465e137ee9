// jpeg.hip — K13: baseline JPEG decode on the GPU (decode -> resize -> crop on the
// device). Reference: app/ml/embeddings.py:82-89 decodes every file with Pillow
// (Image.open(path).convert("RGB")); the arithmetic restated in jpeg_core.h gives Pillow's bytes.
//
// A batch of files is parsed on the host (jpeg_parse.h: tables, geometry, entropy-coded segments),
// the entropy-coded bytes of all files go to the device in one copy, and three kernels run:
//   K13a jpeg_huff_kernel   one single-lane workgroup per entropy-coded segment (a whole image, or
//                           one restart interval): Huffman decode into zeroed int16 coefficient
//                           blocks. A one-thread workgroup makes every value wave-uniform, so the
//                           decoder runs on the scalar unit with its tables read through the
//                           scalar cache; segments run in parallel across CUs.
//   K13b jpeg_idct_kernel   one thread per 8x8 block: dequantise + islow IDCT into the planes.
//   K13c jpeg_color_kernel  one thread per output pixel: fancy chroma upsampling + YCbCr -> RGB,
//                           H x W x 3 u8 at the caller's offset (the layout K0 resizes from).
// Files K13 does not support (progressive, arithmetic, CMYK, 4:4:0, tiny chroma) are reported by
// mrag_jpeg_probe and decoded on the host by the caller, as the reference decodes everything.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"
#include "jpeg_parse.h"

using namespace mrag_jpeg;

namespace {

__global__ __launch_bounds__(1) void jpeg_huff_kernel(const Image* __restrict__ imgs, const Segment* __restrict__ segs,
                                                      const uint8_t* __restrict__ ecs, int16_t* __restrict__ coef) {
  const Segment sg = segs[blockIdx.x];
  const Image& im = imgs[sg.img];
  decode_segment(im, ecs + sg.off, sg.len, sg.mcu0, sg.mcus, coef + im.coef_off * 64);
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

__global__ __launch_bounds__(256) void jpeg_color_kernel(const Image* __restrict__ imgs,
                                                         const uint8_t* __restrict__ planes, uint8_t* __restrict__ out) {
  const Image& im = imgs[blockIdx.y];
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)im.width * im.height) return;
  const int y = (int)(p / im.width), x = (int)(p - (int64_t)y * im.width);
  uint8_t rgb[3];
  color_pixel(im, planes + im.plane_off, x, y, rgb);
  uint8_t* o = out + im.rgb_off + p * 3;
  o[0] = rgb[0];
  o[1] = rgb[1];
  o[2] = rgb[2];
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

int mrag_jpeg_probe(const uint8_t* data, int64_t size, int32_t* width, int32_t* height) {
  MRAG_REQUIRE(data && width && height && size >= 0, "NULL argument");
  Parsed P;
  if (!parse(data, size, P)) {
    *width = *height = 0;
    return 0;
  }
  *width = P.img.width;
  *height = P.img.height;
  return 1;
}

int mrag_jpeg_decode(const uint8_t* const* files, const int64_t* sizes, int32_t n, uint8_t* out,
                     const int64_t* out_offsets, int32_t device, void* stream) {
  MRAG_REQUIRE(n >= 0, "negative batch");
  if (n == 0) return MRAG_OK;
  MRAG_REQUIRE(files && sizes && out && out_offsets, "NULL argument");
  MRAG_REQUIRE(device >= 0 && device < 64, "bad device %d", device);
  mrag::DeviceGuard g(device);
  Ctx& C = g_ctx[device];
  std::lock_guard<std::mutex> lk(C.mu);
  hipStream_t s = (hipStream_t)stream;

  std::vector<Image> imgs((size_t)n);
  std::vector<Segment> segs;
  std::vector<int64_t> ecs_at((size_t)n);
  int64_t ecs_total = 0, blocks = 0, planes = 0, max_blocks = 0, max_pix = 0;
  for (int i = 0; i < n; ++i) {
    Parsed P;
    MRAG_REQUIRE(files[i] != nullptr, "NULL file %d", i);
    if (!parse(files[i], sizes[i], P)) return mrag::fail(MRAG_ERR_ARG, "jpeg %d unsupported: %s", i, P.why.c_str());
    Image& im = imgs[i] = P.img;
    im.seg0 = (int32_t)segs.size();
    im.ecs_off = ecs_total;
    im.coef_off = blocks;
    im.plane_off = planes;
    im.rgb_off = out_offsets[i];
    for (Segment sg : P.segs) {
      sg.off = sg.off - P.ecs_begin + ecs_total;
      sg.img = i;
      segs.push_back(sg);
    }
    ecs_at[i] = P.ecs_begin;
    ecs_total += P.ecs_end - P.ecs_begin;
    blocks += P.coef_blocks;
    planes += P.plane_bytes;
    max_blocks = std::max(max_blocks, P.coef_blocks);
    max_pix = std::max(max_pix, (int64_t)im.width * im.height);
  }
  if (ecs_total + 64 > (int64_t)C.stage_cap) {
    const size_t cap = std::max<size_t>((size_t)ecs_total + 64, C.stage_cap * 2);
    MRAG_HIP(hipStreamSynchronize(s));  // a previous batch's copy may still read the old buffer
    if (C.stage) (void)hipHostFree(C.stage);
    C.stage = nullptr;
    C.stage_cap = 0;
    MRAG_HIP(hipHostMalloc((void**)&C.stage, cap, hipHostMallocDefault));
    C.stage_cap = cap;
  }
  // the previous batch's copy out of the staging buffer must be done before it is rewritten
  MRAG_HIP(hipStreamSynchronize(s));
  for (int i = 0; i < n; ++i) {
    const int64_t len = (i + 1 < n ? imgs[i + 1].ecs_off : ecs_total) - imgs[i].ecs_off;
    std::memcpy(C.stage + imgs[i].ecs_off, files[i] + ecs_at[i], (size_t)len);
  }
  if (int rc = ensure(C.ecs, (size_t)ecs_total + 64)) return rc;  // Bits reads up to 32 B past a segment
  if (int rc = ensure(C.imgs, sizeof(Image) * (size_t)n)) return rc;
  if (int rc = ensure(C.segs, sizeof(Segment) * segs.size())) return rc;
  if (int rc = ensure(C.coef, (size_t)blocks * 128)) return rc;
  if (int rc = ensure(C.planes, (size_t)planes)) return rc;
  MRAG_HIP(hipMemcpyAsync(C.ecs.p, C.stage, (size_t)ecs_total, hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemcpyAsync(C.imgs.p, imgs.data(), sizeof(Image) * (size_t)n, hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemcpyAsync(C.segs.p, segs.data(), sizeof(Segment) * segs.size(), hipMemcpyHostToDevice, s));
  MRAG_HIP(hipMemsetAsync(C.coef.p, 0, (size_t)blocks * 128, s));
  hipLaunchKernelGGL(jpeg_huff_kernel, dim3((unsigned)segs.size()), dim3(1), 0, s, (const Image*)C.imgs.p,
                     (const Segment*)C.segs.p, (const uint8_t*)C.ecs.p, (int16_t*)C.coef.p);
  MRAG_CHECK_LAUNCH();
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((max_blocks + 255) / 256), (unsigned)n), dim3(256), 0, s,
                     (const Image*)C.imgs.p, (const int16_t*)C.coef.p, (uint8_t*)C.planes.p);
  MRAG_CHECK_LAUNCH();
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((max_pix + 255) / 256), (unsigned)n), dim3(256), 0, s,
                     (const Image*)C.imgs.p, (const uint8_t*)C.planes.p, out);
  MRAG_CHECK_LAUNCH();
  // the descriptors above live on this host stack frame: the copies must finish before return
  MRAG_HIP(hipStreamSynchronize(s));
  return MRAG_OK;
}

}  // extern "C"
