// K3g prototype (experiment, not in the library): C16 = A . W^T + bias with 256 x 128 x 64 tiles,
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

constexpr int BM = 256, BN = 128, BK = 64;
constexpr int ST_BYTES = (BM + BN) * BK * 2;  // 48 KiB
constexpr int NST = 3;
constexpr int PPW = ST_BYTES / 1024 / 4;       // 12 pieces per wave per K-tile

template <int NP>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NP) : "memory"); }

__global__ __launch_bounds__(256) void k3g_kernel(const _Float16* __restrict__ A, const _Float16* __restrict__ W,
                                                  const float* __restrict__ bias, _Float16* __restrict__ C, int M,
                                                  int N, int K, int order) {
  __shared__ __attribute__((aligned(16))) char smem[NST * ST_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));
  const int tiles_n = N / BN;
  // blocks b, b + 8, ... (one XCD) take consecutive tile ids, tm-major
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tm, tn;
  if (order == 0) {  // tm-major
    tm = T / tiles_n;
    tn = T - tm * tiles_n;
  } else {  // grouped: blocks of G row panels, columns outer inside a group (G x tiles_n tiles)
    const int G = order, tiles_m = (M + BM - 1) / BM;
    const int gsz = G * tiles_n, grp = T / gsz, first = grp * G, gm = min(G, tiles_m - first);
    const int in = T - grp * gsz;
    tm = first + in % gm;
    tn = in / gm;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int KT = K / BK;

  // this wave's 12 pieces: P = 12 w + i; P < 32: A rows 8 P .. 8 P + 7, else W rows 8 (P - 32) ..
  const _Float16* src[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int P = PPW * w + i;
    const int rr = lane >> 3, pos = lane & 7;
    if (P < 32) {
      const int row = 8 * P + rr;
      const int c = pos ^ ((row >> 1) & 7);
      src[i] = A + (size_t)min(m0 + row, M - 1) * K + c * 8;
    } else {
      const int row = 8 * (P - 32) + rr;
      const int c = pos ^ ((row >> 1) & 7);
      const int col = (row & ~31) + g8_colperm(row & 31);
      src[i] = W + (size_t)(n0 + col) * K + c * 8;
    }
  }
  auto stage = [&](int kt) {
    const uint32_t dst = lds_base + (uint32_t)((kt % NST) * ST_BYTES) + (uint32_t)(PPW * w * 1024);
#pragma unroll
    for (int i = 0; i < PPW; ++i) glds_x4(src[i] + kt * BK, dst + i * 1024);
  };

  int offA[8][2], offW[4][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < 8; ++i) offA[i][kk] = swz_off(wr * 128 + 16 * i + fr, kk * 4 + fq);
#pragma unroll
    for (int j = 0; j < 4; ++j) offW[j][kk] = BM * 128 + swz_off(wc * 64 + 16 * j + fr, kk * 4 + fq);
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  stage(0);
  if (KT > 1) stage(1);
  if (KT > 1) wait_vm<PPW>(); else wait_vm<0>();
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 2 < KT) stage(kt + 2);
    const char* st = smem + (kt % NST) * ST_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      half8 a[8], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *(const half8*)(st + offW[j][kk]);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = *(const half8*)(st + offA[i][kk]);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < KT) wait_vm<PPW>(); else wait_vm<0>();  // K-tile kt + 1 landed (kt + 2 younger)
    __syncthreads();
  }
  // epilogue (f16): block pair p = blocks 2p, 2p + 1 -> columns n0 + 64 wc + 32 p + 8 fq + 0..7
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int n = n0 + wc * 64 + 32 * p + 8 * fq;
    const f32x4 b0 = *(const f32x4*)(bias + n), b1 = *(const f32x4*)(bias + n + 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + 16 * i + fr;
      if (m < M) {
        f32x4 v0 = acc[i][2 * p], v1 = acc[i][2 * p + 1];
        half8 h;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v0[r] += b0[r];
          v1[r] += b1[r];
          h[r] = (_Float16)v0[r];
          h[4 + r] = (_Float16)v1[r];
        }
        *(half8*)(C + (size_t)m * N + n) = h;
      }
    }
  }
}

int main(int argc, char** argv) {
  struct Shape { const char* name; int M, N, K; };
  std::vector<Shape> shapes = {{"qkv", 12800, 2304, 768}, {"fc1", 12800, 3072, 768}, {"t_qkv", 16000, 1536, 512},
                               {"t_fc1", 16000, 2048, 512}, {"m_qkv", 16000, 1152, 384}, {"sq4k", 4096, 4096, 4096}};
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
    for (int order : {0, 2, 4, 8}) {
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
