// K3h prototype (experiment, not in the library; harness shared with k3g.hip): C16 = A . W^T + bias with 256 x 128 x 64 tiles,
// 4 waves (2 x 2 of 128 x 64, one per SIMD), a 3-stage LDS ring (48 KiB per K-tile) filled by
// LDS-DMA two K-tiles ahead with a counted vmcnt, one barrier per K-tile. Same per-element order
// as the library's K3 / K3d (32-deep MFMA chunks in ascending k, one accumulator; weight fragment
// as MFMA operand A; block-pair column permutation), so the outputs must be bit-identical to
// mrag_gemm_nt(epilogue 0). Prints timings of both and the comparison.
// Build: hipcc --offload-arch=gfx950 -O3 -o k3g k3g.hip -L../multimodal-rag-for-image-text-search_amd/lib -lmrag
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" int mrag_gemm_nt(const void* A, const void* W, const float* bias, void* C, int32_t M, int32_t N, int32_t K,
                            int32_t epilogue, void* stream);

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
#define AS3 __attribute__((address_space(3)))

__device__ __forceinline__ void glds_x4(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_addr)
               : "memory");
}
__device__ __forceinline__ int swz_off(int j, int c) { return j * 128 + ((c ^ ((j >> 1) & 7)) * 16); }
__device__ __forceinline__ int g8_colperm(int jj) {
  const int jb = jj >> 4, f = (jj >> 2) & 3, r = jj & 3;
  return 8 * f + 4 * jb + r;
}

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int SLOT = 16384;  // half-tile slot: 128 LDS rows x 128 B
// K3h: K3d's slot ring (per 64-deep K-tile four 16 KiB slots A-h0, B-h0, B-h1, A-h1; two buffers;
// load stream L[i] = slot i & 3 of K-tile i >> 2; phase phi issues L[phi + 7] and waits for
// L[phi + 2]) driven by 4 waves of 128 x 128 (2 x 2, one per SIMD), one barrier per phase.
// Phase p of a K-tile computes quadrant (h, hh) of every wave's tile over BK = 64:
// p0 (h0, hh0) reads A-h0 + B-h0; p1 (h0, hh1) reads B-h1; p2 (h1, hh1) reads A-h1; p3 (h1, hh0)
// reads nothing.
#define VMC(n) case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) { VMC(0) VMC(4) VMC(8) VMC(12) VMC(16) VMC(20) default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
}

__global__ __launch_bounds__(256) void k3g_kernel(const _Float16* __restrict__ A, const _Float16* __restrict__ W,
                                                  const float* __restrict__ bias, _Float16* __restrict__ C, int M,
                                                  int N, int K, int order) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * SLOT];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));
  const int tiles_n = N / BN;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = T / tiles_n, tn = T - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int KT = K / BK, total = 4 * KT;
  (void)order;

  // this wave's 4 pieces of a slot: LDS rows j = 8 (4 w + q) + (lane >> 3), chunk pos lane & 7
  const _Float16* srcA[2][4];
  const _Float16* srcB[2][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = 8 * (4 * w + q) + (lane >> 3);
    const int c = (lane & 7) ^ ((j >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 128 * (j >> 6) + 64 * h + (j & 63);  // A slot h: wave-row j / 64, half h
      srcA[h][q] = A + (size_t)min(m0 + row, M - 1) * K + c * 8;
      const int jj = j & 63;
      const int col = 128 * (j >> 6) + 64 * h + (jj & ~31) + g8_colperm(jj & 31);  // B slot h
      srcB[h][q] = W + (size_t)(n0 + col) * K + c * 8;
    }
  }
  auto issue = [&](int i) {  // L[i]
    const int kt = i >> 2, sl = i & 3;
    const uint32_t dst = lds_base + (uint32_t)((kt & 1) * 4 * SLOT + sl * SLOT) + (uint32_t)(4 * w * 1024);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const _Float16* s = sl == 0 ? srcA[0][q] : sl == 1 ? srcB[0][q] : sl == 2 ? srcB[1][q] : srcA[1][q];
      glds_x4(s + kt * BK, dst + q * 1024);
    }
  };
  int offA[4][2], offB[4][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      offA[i][kk] = swz_off(64 * wr + 16 * i + fr, kk * 4 + fq);
      offB[i][kk] = swz_off(64 * wc + 16 * i + fr, kk * 4 + fq);
    }
  f32x4 acc[2][2][4][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][hh][i][j] = f32x4{};
  half8 fa[4][2], fb0[4][2], fb1[4][2];
  auto readA = [&](const char* s) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = *(const half8*)(s + offA[i][kk]);
  };
  auto readB = [&](const char* s, half8 (&fb)[4][2]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk] = *(const half8*)(s + offB[j][kk]);
  };
  auto mfma = [&](f32x4 (&a)[4][4], const half8 (&fb)[4][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) a[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j][kk], fa[i][kk], a[i][j], 0, 0, 0);
  };
  auto tail = [&](int phi) {  // issue L[phi + 7] was done; wait for L[phi + 2], barrier
    const int last = min(phi + 7, total - 1);
    vm_wait(phi + 2 <= last ? 4 * (last - phi - 2) : 0);
    __syncthreads();
  };
  // prologue: L[0..6]; L[0], L[1] landed
  {
    const int last = min(6, total - 1);
    for (int i = 0; i <= last; ++i) issue(i);
    vm_wait(4 * (last - 1 > 0 ? last - 1 : 0));
    __syncthreads();
  }
  for (int kt = 0; kt < KT; ++kt) {
    const char* buf = smem + (kt & 1) * 4 * SLOT;
    const int phi = 4 * kt;
    readA(buf + 0 * SLOT);  // p0: (h0, hh0)
    readB(buf + 1 * SLOT, fb0);
    if (phi + 7 < total) issue(phi + 7);
    mfma(acc[0][0], fb0);
    tail(phi);
    readB(buf + 2 * SLOT, fb1);  // p1: (h0, hh1)
    if (phi + 8 < total) issue(phi + 8);
    mfma(acc[0][1], fb1);
    tail(phi + 1);
    readA(buf + 3 * SLOT);  // p2: (h1, hh1)
    if (phi + 9 < total) issue(phi + 9);
    mfma(acc[1][1], fb1);
    tail(phi + 2);
    if (phi + 10 < total) issue(phi + 10);  // p3: (h1, hh0) from registers
    mfma(acc[1][0], fb0);
    tail(phi + 3);
  }
  // epilogue (f16): quadrant (h, hh), block i: row m0 + 128 wr + 64 h + 16 i + fr; block pair p
  // (blocks 2p, 2p + 1): columns n0 + 128 wc + 64 hh + 32 p + 8 fq + 0..7
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int n = n0 + 128 * wc + 64 * hh + 32 * p + 8 * fq;
        const f32x4 b0 = *(const f32x4*)(bias + n), b1 = *(const f32x4*)(bias + n + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + 128 * wr + 64 * h + 16 * i + fr;
          if (m < M) {
            f32x4 v0 = acc[h][hh][i][2 * p], v1 = acc[h][hh][i][2 * p + 1];
            half8 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v0[r] += b0[r];
              v1[r] += b1[r];
              o[r] = (_Float16)v0[r];
              o[4 + r] = (_Float16)v1[r];
            }
            *(half8*)(C + (size_t)m * N + n) = o;
          }
        }
      }
}

int main(int argc, char** argv) {
  struct Shape { const char* name; int M, N, K; };
  std::vector<Shape> shapes = {{"qkv", 12800, 2304, 768}, {"fc1", 12800, 3072, 768}, {"t_qkv", 16000, 1536, 512},
                               {"t_fc1", 16000, 2048, 512}, {"sq4k", 4096, 4096, 4096}};
  for (const auto& s : shapes) {
    const int M = s.M, N = s.N, K = s.K;
    std::vector<_Float16> hA((size_t)M * K), hW((size_t)N * K);
    std::vector<float> hb(N);
    srand(1);
    for (auto& x : hA) x = (_Float16)((rand() % 2001 - 1000) / 1000.0f);
    for (auto& x : hW) x = (_Float16)((rand() % 2001 - 1000) / 1000.0f);
    for (auto& x : hb) x = (rand() % 2001 - 1000) / 2000.0f;
    _Float16 *A, *Wd, *C1, *C2;
    float* b;
    hipMalloc(&A, hA.size() * 2);
    hipMalloc(&Wd, hW.size() * 2);
    hipMalloc(&b, N * 4);
    hipMalloc(&C1, (size_t)M * N * 2);
    hipMalloc(&C2, (size_t)M * N * 2);
    hipMemcpy(A, hA.data(), hA.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(Wd, hW.data(), hW.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(b, hb.data(), N * 4, hipMemcpyHostToDevice);
    const int tiles = ((M + BM - 1) / BM) * (N / BN);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int reps = 20;
    float ms_g = 0, ms_l = 0;
    float best = 1e30f;
    int best_order = 0;
    char orders[256] = "";
    for (int order : {0}) {
      for (int t = 0; t < 3; ++t) hipLaunchKernelGGL(k3g_kernel, dim3(tiles), dim3(256), 0, 0, A, Wd, b, C1, M, N, K, order);
      hipEventRecord(e0);
      for (int t = 0; t < reps; ++t) hipLaunchKernelGGL(k3g_kernel, dim3(tiles), dim3(256), 0, 0, A, Wd, b, C1, M, N, K, order);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      snprintf(orders + strlen(orders), sizeof(orders) - strlen(orders), "%s\"o%d\": %.1f", order ? ", " : "", order,
               ms * 1e3 / reps);
      if (ms < best) {
        best = ms;
        best_order = order;
      }
    }
    ms_g = best;
    for (int t = 0; t < 3; ++t) mrag_gemm_nt(A, Wd, b, C2, M, N, K, 0, nullptr);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int t = 0; t < reps; ++t) mrag_gemm_nt(A, Wd, b, C2, M, N, K, 0, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_l, e0, e1);
    std::vector<uint16_t> r1((size_t)M * N), r2((size_t)M * N);
    hipMemcpy(r1.data(), C1, r1.size() * 2, hipMemcpyDeviceToHost);
    hipMemcpy(r2.data(), C2, r2.size() * 2, hipMemcpyDeviceToHost);
    size_t diff = 0;
    for (size_t i = 0; i < r1.size(); ++i) diff += r1[i] != r2[i];
    const double fl = 2.0 * M * N * K;
    printf("{\"shape\": \"%s\", \"orders_us\": {%s}, \"best_order\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"k3g_us\": %.1f, \"lib_us\": %.1f, \"k3g_TF\": %.0f, "
           "\"lib_TF\": %.0f, \"elements_differing\": %zu, \"err\": \"%s\"}\n",
           s.name, orders, best_order, M, N, K, ms_g * 1e3 / reps, ms_l * 1e3 / reps, fl / (ms_g * 1e-3 / reps) / 1e12,
           fl / (ms_l * 1e-3 / reps) / 1e12, diff, hipGetErrorString(hipGetLastError()));
    fflush(stdout);
    hipFree(A);
    hipFree(Wd);
    hipFree(b);
    hipFree(C1);
    hipFree(C2);
  }
  return 0;
}
