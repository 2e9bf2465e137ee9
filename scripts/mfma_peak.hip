// mfma_peak.hip — sustained fp16 MFMA rate of this MI355X (re-measure the
// 2.5 PFLOP/s spec on the box). 256-thread workgroups, 8 per CU over the launch, operands
// in registers, random data (the chip holds
// a lower clock on random operands than on zeros: MI355X_MICROARCH.md, DVFS give-back),
// four independent accumulators per wave, back-to-back issue, for both f16 shapes the
// kernels use (16x16x32 in the K7 v3 scan and the encoder GEMMs, 32x32x16 in K7 v1/v2).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/mfma_peak.hip -o scripts/mfma_peak
// Output: one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int SHAPE>  // 0: 16x16x32, 1: 32x32x16
__global__ __launch_bounds__(256) void mfma_loop(const half8* __restrict__ in, float* __restrict__ out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  half8 a0 = in[(t * 4 + 0) & 4095], a1 = in[(t * 4 + 1) & 4095];
  half8 b0 = in[(t * 4 + 2) & 4095], b1 = in[(t * 4 + 3) & 4095];
  if constexpr (SHAPE == 0) {
    f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, c3, 0, 0, 0);
      }
    }
    const f32x4 s = c0 + c1 + c2 + c3;
    out[t] = s[0] + s[1] + s[2] + s[3];
  } else {
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, c3, 0, 0, 0);
      }
    }
    const f32x16 s = c0 + c1 + c2 + c3;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v += s[r];
    out[t] = v;
  }
}

template <int SHAPE>
double run(const half8* in, float* out, int blocks, int iters, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(mfma_loop<SHAPE>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
  CK(hipDeviceSynchronize());
  std::vector<float> ms(reps);
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(mfma_loop<SHAPE>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[r], e0, e1));
  }
  std::sort(ms.begin(), ms.end());
  const double flop_per_mfma = SHAPE == 0 ? 2.0 * 16 * 16 * 32 : 2.0 * 32 * 32 * 16;
  const double flops = (double)blocks * 4 /*waves*/ * iters * 32 /*mfma per iter*/ * flop_per_mfma;
  return flops / (ms[reps / 2] * 1e-3) / 1e12;  // median, TFLOP/s
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::vector<_Float16> h(4096 * 8);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& v : h) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    v = (_Float16)(((double)(x >> 11) / 9007199254740992.0) * 2.0 - 1.0);
  }
  half8* in;
  float* out;
  CK(hipMalloc(&in, h.size() * 2));
  CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  CK(hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  const int blocks = cus * 8;  // 8 waves of work per CU in flight over the launch
  const int iters = 4000;       // ~20 ms per launch
  const double t16 = run<0>(in, out, blocks, iters, 9);
  const double t32 = run<1>(in, out, blocks, iters / 2, 9);
  printf("{\"device\": \"%s\", \"cus\": %d, \"f16_16x16x32_tflops\": %.1f, \"f16_32x32x16_tflops\": %.1f, "
         "\"spec_tflops\": 2500.0, \"operands\": \"random f16 in registers, 4 accumulators/wave, median of 9 launches\"}\n",
         prop.gcnArchName, cus, t16, t32);
  return 0;
}
