// encoder_kernels.hip — K1..K5: the transformer building blocks of the three encoders
// (CLIP ViT-B/32 image tower, CLIP text tower, MiniLM-L6 BERT), gfx950 only.
//
// Reference arithmetic (third-party, reached from app/ml/embeddings.py:62-105):
//   transformers/models/clip/modeling_clip.py  CLIPVisionEmbeddings (:202-218), CLIPAttention
//   (:280-335, scale head_dim^-0.5), CLIPMLP quick_gelu (:346-350), CLIPEncoderLayer pre-LN
//   (:362-383), pooling (:561-580, :650-651), projections (:674-675, :750-751);
//   transformers/models/bert/modeling_bert.py  embeddings + post-LN layers (:53-350).
//
// Layout: activations row-major [tokens][features]; the residual stream is f32, every GEMM
// input is f16 (LayerNorm writes the f16 copy), weights are f16 [out][in] (torch Linear
// layout, K contiguous for both GEMM operands), biases / LN params / embeddings f32.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "common.h"
#include "encoder_kernels.h"

#define AS3 __attribute__((address_space(3)))

namespace mrag_enc {

__device__ __forceinline__ void glds_x4(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

#define MRAG_VMCNT_CASE(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void vmcnt_wait(int n) {  // n wave-uniform, 0..63
  switch (n) {
    MRAG_VMCNT_CASE(1) MRAG_VMCNT_CASE(2) MRAG_VMCNT_CASE(3) MRAG_VMCNT_CASE(4) MRAG_VMCNT_CASE(5)
    MRAG_VMCNT_CASE(6) MRAG_VMCNT_CASE(7) MRAG_VMCNT_CASE(8) MRAG_VMCNT_CASE(9) MRAG_VMCNT_CASE(10)
    MRAG_VMCNT_CASE(11) MRAG_VMCNT_CASE(12) MRAG_VMCNT_CASE(13) MRAG_VMCNT_CASE(14) MRAG_VMCNT_CASE(15)
    MRAG_VMCNT_CASE(16) MRAG_VMCNT_CASE(17) MRAG_VMCNT_CASE(18) MRAG_VMCNT_CASE(19) MRAG_VMCNT_CASE(20)
    MRAG_VMCNT_CASE(21) MRAG_VMCNT_CASE(22) MRAG_VMCNT_CASE(23) MRAG_VMCNT_CASE(24) MRAG_VMCNT_CASE(25)
    MRAG_VMCNT_CASE(26) MRAG_VMCNT_CASE(27) MRAG_VMCNT_CASE(28) MRAG_VMCNT_CASE(29) MRAG_VMCNT_CASE(30)
    MRAG_VMCNT_CASE(31) MRAG_VMCNT_CASE(32) MRAG_VMCNT_CASE(33) MRAG_VMCNT_CASE(34) MRAG_VMCNT_CASE(35)
    MRAG_VMCNT_CASE(36) MRAG_VMCNT_CASE(37) MRAG_VMCNT_CASE(38) MRAG_VMCNT_CASE(39) MRAG_VMCNT_CASE(40)
    MRAG_VMCNT_CASE(41) MRAG_VMCNT_CASE(42) MRAG_VMCNT_CASE(43) MRAG_VMCNT_CASE(44) MRAG_VMCNT_CASE(45)
    MRAG_VMCNT_CASE(46) MRAG_VMCNT_CASE(47) MRAG_VMCNT_CASE(48) MRAG_VMCNT_CASE(49) MRAG_VMCNT_CASE(50)
    MRAG_VMCNT_CASE(51) MRAG_VMCNT_CASE(52) MRAG_VMCNT_CASE(53) MRAG_VMCNT_CASE(54) MRAG_VMCNT_CASE(55)
    MRAG_VMCNT_CASE(56) MRAG_VMCNT_CASE(57) MRAG_VMCNT_CASE(58) MRAG_VMCNT_CASE(59) MRAG_VMCNT_CASE(60)
    MRAG_VMCNT_CASE(61) MRAG_VMCNT_CASE(62) MRAG_VMCNT_CASE(63)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
#undef MRAG_VMCNT_CASE
// compile-time count: one s_waitcnt, never merged with the dynamic ladder above (which the
// compiler lowers to a compare/branch tree of ~20 scalar instructions per call)
template <int N>
__device__ __forceinline__ void vmcnt_wait_c() {
  static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---------------------------------------------------------------------------
// K3: C[m][n] (+)= act(sum_k A[m][k] W[n][k] + bias[n])   (the "NT" GEMM of nn.Linear)
//
// Both GEMM kernels use MFMA 16x16x32 f16 with the WEIGHT fragment as the MFMA's A operand
// and the activation fragment as its B operand, i.e. they compute C^T blocks: lane l holds
// output row m = (l & 15) and the four consecutive columns n = 4 (l >> 4) + r, r = 0..3,
// so the epilogue stores 8 B (f16) or 16 B (f32) per lane instead of one element.
// Operands are staged to LDS by LDS-DMA into 128-byte rows (64 k of one row) with 16-byte
// chunk c stored at position c ^ ((row >> 1) & 7) (source-address swizzle): every
// ds_read_b128 fragment read of 16 consecutive rows is bank-conflict free.
// Every output element is accumulated in the same order by both kernels (32-deep MFMA
// chunks in ascending k, one accumulator) and finished by the same gemm_store4, so a row's
// result does not depend on which kernel its batch size selected.
template <int EPI>
__device__ __forceinline__ float gemm_act(float x) {
  if constexpr (EPI == EPI_F16_QUICK_GELU) {
    // x * sigmoid(1.702 x) with hardware exp2 / rcp (~1 ulp each; the result is rounded to
    // fp16) instead of a full-precision divide
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.702f * 1.44269504088896341f * x));
  } else if constexpr (EPI == EPI_F16_GELU_ERF) {
    // erf by Abramowitz & Stegun 7.1.26 with hardware rcp / exp2: a fraction of the cost of the
    // libm erff in the epilogue. The erf error (<= 1.5e-7 absolute) gives a GELU error of at most
    // 0.5 |x| 1.5e-7 + rcp/exp2 ulps, i.e. an ABSOLUTE bound (~1e-6 at |x| = 8): below the fp16
    // rounding of outputs of magnitude >~ 2e-3, but several fp16 ulps in the far negative tail
    // where GELU(x) itself is ~1e-6 (tests/test_encoders_gpu.py::test_gelu_erf_epilogue_sweep)
    const float z = x * 0.70710678118654752f, az = fabsf(z);
    const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * az);
    const float poly =
        t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
    const float e = 1.0f - poly * __builtin_amdgcn_exp2f(-az * az * 1.44269504088896341f);
    return 0.5f * x * (1.0f + copysignf(e, z));
  } else {
    return x;
  }
}

// Finish four consecutive outputs C[m][n .. n + 3] = epilogue(v + bias) (K3).
template <int EPI>
__device__ __forceinline__ void gemm_store4(const GemmArgs& g, int m, int n, f32x4 v, const float* bn) {
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] += bn[r];
  const size_t o = (size_t)m * g.ldc + n;
  if constexpr (EPI == EPI_F16 || EPI == EPI_F16_QUICK_GELU || EPI == EPI_F16_GELU_ERF) {
    half4 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) h[r] = (_Float16)gemm_act<EPI>(v[r]);
    *(half4*)((_Float16*)g.C + o) = h;
  } else if constexpr (EPI == EPI_F32_RESIDUAL) {
    f32x4* p = (f32x4*)((float*)g.C + o);
    f32x4 c = *p;
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] += v[r];
    *p = c;
  } else {
    *(f32x4*)((float*)g.C + o) = v;
  }
}

// Eight consecutive outputs C[m][n .. n + 7] (K3d): one 16-byte store for the f16
// epilogues, two for the f32 ones — the same per-element arithmetic as gemm_store4.
template <int EPI>
__device__ __forceinline__ void gemm_store8(const GemmArgs& g, int m, int n, f32x4 v0, f32x4 v1, const float* bn) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v0[r] += bn[r];
    v1[r] += bn[4 + r];
  }
  const size_t o = (size_t)m * g.ldc + n;
  if constexpr (EPI == EPI_F16 || EPI == EPI_F16_QUICK_GELU || EPI == EPI_F16_GELU_ERF) {
    half8 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      h[r] = (_Float16)gemm_act<EPI>(v0[r]);
      h[4 + r] = (_Float16)gemm_act<EPI>(v1[r]);
    }
    *(half8*)((_Float16*)g.C + o) = h;
  } else if constexpr (EPI == EPI_F32_RESIDUAL) {
    f32x4* p = (f32x4*)((float*)g.C + o);
    f32x4 c0 = p[0], c1 = p[1];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c0[r] += v0[r];
      c1[r] += v1[r];
    }
    p[0] = c0;
    p[1] = c1;
  } else {
    f32x4* p = (f32x4*)((float*)g.C + o);
    p[0] = v0;
    p[1] = v1;
  }
}

// gemm_store8 for the f32 residual epilogue with the old C values already loaded (the epilogues
// load a batch of C blocks before storing any: a store may alias a later load, so loads issued
// block by block between the stores cost one memory round trip per block). Same arithmetic:
// C = C + (acc + bias).
__device__ __forceinline__ void gemm_store8_res(const GemmArgs& g, int m, int n, f32x4 v0, f32x4 v1,
                                                const float* bn, f32x4 c0, f32x4 c1) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v0[r] += bn[r];
    v1[r] += bn[4 + r];
    c0[r] += v0[r];
    c1[r] += v1[r];
  }
  f32x4* p = (f32x4*)((float*)g.C + (size_t)m * g.ldc + n);
  p[0] = c0;
  p[1] = c1;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // blocks bid, bid+8, ... share an XCD; give each XCD a contiguous range of tile ids
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// fragment offset (bytes) of row j, 16-byte chunk c, in a swizzled 128-byte-row LDS image
__device__ __forceinline__ int swz_off(int j, int c) { return j * 128 + ((c ^ ((j >> 1) & 7)) * 16); }

constexpr int GM = 128, GN = 128, GK = 64;
constexpr int GTHREADS = 256;
constexpr int STAGE_BYTES = (GM + GN) * GK * 2;  // 32 KiB

// K3 (small M: text queries, short batches, N not a multiple of 256): 128 x 128 x 64 block
// tile, 4 waves (2 x 2) of 64 x 64, 2 stages, one barrier per k-step; 2 workgroups per CU.
template <int EPI>
__global__ __launch_bounds__(GTHREADS) void gemm_nt_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  const int tiles_n = g.N / GN;
  // consecutive tile ids walk N for a fixed M panel; blocks b, b + 8, ... (one XCD under the
  // round-robin dispatch) take consecutive tile ids (xcd_remap), so the tiles_n tiles of an A
  // panel are fetched into ONE XCD's L2 instead of being dealt over tiles_n XCDs (speed only)
  const int T = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = T / tiles_n, tn = T - (T / tiles_n) * tiles_n;
  const int m0 = tm * GM, n0 = tn * GN;
  const int ksteps = g.K / GK;

  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int P = w * 8 + i;  // 1 KiB piece: 8 rows of 128 B
      const int rr = lane >> 3, pos = lane & 7;
      const int row = 8 * (P & 15) + rr;
      const int c = pos ^ ((row >> 1) & 7);
      const _Float16* src;
      if (P < 16) {
        const int m = min(m0 + row, g.M - 1);
        src = g.A + (size_t)m * g.lda + k0 + c * 8;
      } else {
        src = g.W + (size_t)(n0 + row) * g.ldw + k0 + c * 8;
      }
      glds_x4(src, lds_base + buf * STAGE_BYTES + P * 1024);
    }
  };

  f32x4 acc[4][4];  // [activation block i][weight block jb]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  int offA[4][2], offW[4][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      offA[i][kk] = swz_off(wr * 64 + 16 * i + fr, kk * 4 + fq);
      offW[i][kk] = GM * GK * 2 + swz_off(wc * 64 + 16 * i + fr, kk * 4 + fq);
    }

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int ks = 0; ks < ksteps; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < ksteps) stage(cur ^ 1, (ks + 1) * GK);
    const char* st = (const char*)smem + cur * STAGE_BYTES;
    half8 a[4][2], b[4][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i][kk] = *(const half8*)(st + offA[i][kk]);
        b[i][kk] = *(const half8*)(st + offW[i][kk]);
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j][kk], a[i][kk], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);  // MFMAs stay ahead of the stage wait + barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: bias as one 16-byte load per column block; for the residual, every old C block of
  // the wave in one batch of loads (rows clamped into the matrix) before the first store — loads
  // issued between stores that may alias them cost one memory round trip per block
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = f32x4{};
  if (g.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = *(const f32x4*)(g.bias + n0 + wc * 64 + 16 * j + 4 * fq);
  }
  f32x4 cv[4][4];
  if constexpr (EPI == EPI_F32_RESIDUAL) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mc = min(m0 + wr * 64 + 16 * i + fr, g.M - 1);
        cv[i][j] = *(const f32x4*)((const float*)g.C + (size_t)mc * g.ldc + n0 + wc * 64 + 16 * j + 4 * fq);
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + 16 * j + 4 * fq;
    const float bn[4] = {bv[j][0], bv[j][1], bv[j][2], bv[j][3]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * 64 + 16 * i + fr;
      if (m < g.M) {
        if constexpr (EPI == EPI_F32_RESIDUAL) {
          f32x4 c = cv[i][j], v = acc[i][j];
#pragma unroll
          for (int r = 0; r < 4; ++r) c[r] += v[r] + bn[r];
          *(f32x4*)((float*)g.C + (size_t)m * g.ldc + n) = c;
        } else {
          gemm_store4<EPI>(g, m, n, acc[i][j], bn);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K3s (M <= 64: one query per retrieve call, a single image): one wave per 16 output columns,
// so a GEMM spreads its weight stream over N / 16 CUs instead of K3's N / 128 workgroups (at
// M = 12 K3's residual GEMMs ran 12-15 us on 3-4 workgroups, each streaming 128 weight rows).
// An element's order is K3's: one accumulator, 32-deep MFMA 16x16x32 chunks in ascending k,
// the weight fragment as operand A, and the same epilogue, so a row's embedding does not depend
// on its batch size (tests/test_encoders_gpu.py batch-vs-alone tests).
// The wave streams k-pairs (64 k: 16 weight rows + 16 MB activation rows, 1 KiB LDS-DMA per
// 8 rows) through a ring of RP pairs in LDS, all LDS-DMA (no VGPRs held by loads in flight); a
// load lane takes row lane >> 3 and 16-byte chunk (lane & 7) ^ (lane >> 3) of its 8 rows (whole
// 128-byte lines per 8 lanes), so the fragment reads (8 rows of one chunk per 8 lanes) are
// bank-conflict free. The next pair's fragments are read before this pair's MFMAs.
template <int MB>
struct SkinnyGeom {
  static constexpr int PER = 2 + 2 * MB;                            // 1 KiB pieces per k-pair
  static constexpr int RP = MB == 1 ? 16 : (MB == 2 ? 10 : (MB == 3 ? 7 : 6));  // (RP - 1) PER < 64
  static constexpr int LDS = RP * PER * 1024;
  static_assert((RP - 1) * PER < 64, "vmcnt field");
};

template <int EPI, int MB>
__global__ __launch_bounds__(64) void gemm_skinny_kernel(GemmArgs g) {
  using G = SkinnyGeom<MB>;
  constexpr int PER = G::PER, RP = G::RP;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int lane = threadIdx.x;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));
  const int n0 = blockIdx.x * 16;
  const int npairs = g.K / 64;

  // load side: piece j of a pair = rows 8 (j & 1) .. + 8 of the weight block (j < 2) or of
  // activation block (j - 2) >> 1
  const int lr = lane >> 3, lc = (lane & 7) ^ (lane >> 3);
  const _Float16* src[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int row = 8 * (j & 1) + lr;
    if (j < 2) {
      src[j] = g.W + (size_t)(n0 + row) * g.ldw + lc * 8;
    } else {
      const int m = min(16 * ((j - 2) >> 1) + row, g.M - 1);
      src[j] = g.A + (size_t)m * g.lda + lc * 8;
    }
  }
  auto issue = [&](int p) {
    const uint32_t slot = lds_base + (uint32_t)((p % RP) * PER * 1024);
#pragma unroll
    for (int j = 0; j < PER; ++j) glds_x4(src[j] + p * 64, slot + j * 1024);
  };
  // read side: lane L holds row r = L & 15, chunk 4 q + (L >> 4) of k-step q of the pair
  const int r = lane & 15, r7 = r & 7;
  int offq[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) offq[q] = (r >> 3) * 1024 + (r7 * 8 + ((4 * q + (lane >> 4)) ^ r7)) * 16;

  half8 wf[2][2], af[2][MB][2];  // [register set][..][k-step q]
  auto read = [&](auto set_c, int p) {
    constexpr int S = decltype(set_c)::value;
    const char* slot = (const char*)smem + (p % RP) * PER * 1024;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      wf[S][q] = *(const half8*)(slot + offq[q]);
#pragma unroll
      for (int b = 0; b < MB; ++b) af[S][b][q] = *(const half8*)(slot + (2 + 2 * b) * 1024 + offq[q]);
    }
  };
  // pair p + 1 landed (pairs up to p + RP issued): the younger ones may stay in flight
  auto wait_next = [&](int p) {
    if (p + RP + 1 <= npairs) vmcnt_wait_c<(RP - 1) * PER>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x4 acc[MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) acc[b] = f32x4{};
  const int pro = min(RP, npairs);
  for (int p = 0; p < pro; ++p) issue(p);
  if (RP < npairs) vmcnt_wait_c<(RP - 1) * PER>();
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  read(std::integral_constant<int, 0>{}, 0);

  // step p: pair p's fragments (read a step ago) are in registers once their reads return, so its
  // slot is refilled with pair p + RP first; then pair p + 1's fragments are read under pair
  // p's MFMAs
  auto step = [&](auto set_c, int p) {
    constexpr int S = decltype(set_c)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (p + RP < npairs) issue(p + RP);
    if (p + 1 < npairs) wait_next(p);
    // unconditional (at p + 1 == npairs it reads a stale slot, never used), so that the MFMAs
    // below wait only for this set's reads on every path
    read(std::integral_constant<int, 1 - S>{}, p + 1);
    __builtin_amdgcn_sched_barrier(0);  // the reads go out before the MFMAs
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int b = 0; b < MB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[S][q], af[S][b][q], acc[b], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int p = 0; p < npairs; p += 2) {
    step(std::integral_constant<int, 0>{}, p);
    if (p + 1 < npairs) step(std::integral_constant<int, 1>{}, p + 1);
  }

  // epilogue (K3's): lane holds C[m = 16 b + r][n0 + 4 (lane >> 4) + 0..3]
  const int n = n0 + 4 * (lane >> 4);
  f32x4 bv = f32x4{};
  if (g.bias) bv = *(const f32x4*)(g.bias + n);
  const float bn[4] = {bv[0], bv[1], bv[2], bv[3]};
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    const int m = 16 * b + r;
    if (m < g.M) gemm_store4<EPI>(g, m, n, acc[b], bn);
  }
}

// ---------------------------------------------------------------------------
// K3d (M >= 1024, N % 256 == 0: the ViT batches): persistent, one workgroup per CU, 256 x 256
// x 64 tiles, 8 waves (2 M x 4 N, 128 x 64 each), an eight-phase pipeline whose LDS-DMA
// prefetch stays in flight across barriers and across tiles, two wave groups in ping-pong.
//
// A K-tile is staged as four 16 KiB half-tiles ("slots"), each 128 LDS rows x 128 B:
//   slot 0 A-h0: tile rows {0..63, 128..191}   slot 1 B-h0: tile cols {64w + 0..31}
//   slot 2 B-h1: tile cols {64w + 32..63}      slot 3 A-h1: tile rows {64..127, 192..255}
// (A = activations, B = weights) so that each of the four phases of a K-tile computes one
// 64 x 32 quadrant of every wave's 128 x 64 output over the full BK = 64 and reads exactly
// one new slot (phase 0 also B-h0): A-h0 + B-h0 -> (h0, hh0); B-h1 -> (h0, hh1); A-h1 ->
// (h1, hh1); nothing -> (h1, hh0). A slot is dead after its only read phase and is restaged
// one phase later with the K-tile two ahead (two LDS buffers x four slots = 128 KiB).
// Load stream L[i] = slot (i & 3) of the workgroup's (i >> 2)-th K-tile, counted over all
// its tiles; phase phi issues L[phi + 7] (the prologue L[0..6]) and waits until L[phi + 2]
// has landed — what phase phi + 1 reads — leaving the five younger half-tiles (10 LDS-DMA
// instructions per wave) in flight: one counted `s_waitcnt vmcnt`, never 0 in the loop.
// The epilogue of a tile (32 vector stores per wave) therefore runs while the next tile's
// first half-tiles land, and its stores drain under the next tile's MFMAs: the five waits
// after it count the stores among the younger operations.
// Phase: ds_reads -> issue -> vmcnt(N) + lgkmcnt(0) -> s_barrier -> MFMAs (setprio 1) ->
// s_barrier, with the two wave groups one barrier apart (ping-pong: on every SIMD one
// wave's MFMA segment overlaps the other wave's read segment). A wave's reads of phase phi
// are retired before the barrier that ends its read segment, which every wave passes before
// issuing phase phi + 1's LDS-DMA (WAR: a slot may be restaged one phase after its read);
// the vmcnt waits of phase phi precede the barrier ending the later group's read segment,
// which precedes every read of phase phi + 1 (RAW).
// Tiles: XCD x (blocks b = x mod 8) owns a contiguous range of tile ids (tm-major), taken
// round-robin by its workgroups, so an A panel and the weight panels stay in that L2.
// (The round-4 timing ablations of this kernel — profiles/r4_k3d_ablations.txt — were built
// from commit 227f50e with scripts/k3d_ablate.sh; they are not part of the product source.)
constexpr int G8_THREADS = 512;
constexpr int G8_BUF = 65536;      // one K-tile: two A and two B half-tile slots
constexpr int G8_BIAS_MAX = 4096;  // bias floats staged in LDS

// Tile geometry: 256 x 256 tiles, waves of 128 x 64 (a 128 x 384 geometry for N = 768 and a
// stream-K variant were measured slower: notes/gemm_experiments.md).
struct G8Geom {
  static constexpr int BM = 256, BN = 256;
  static constexpr int WM = BM / 2, WN = BN / 4;  // wave tile (2 x 4 waves)
  static constexpr int HM = WM / 2, HN = WN / 2;  // one phase's quadrant
  static constexpr int NI = HM / 16, NJ = HN / 16;
  static constexpr int SA = BM / 2 * 128, SB = BN / 2 * 128;  // A / B half-tile slot bytes
  static constexpr int PA = BM / 128, PB = BN / 128;          // 1 KiB LDS-DMA pieces per wave per slot
  static constexpr int slot_off(int sl) { return sl == 0 ? 0 : sl == 1 ? SA : sl == 2 ? SA + SB : SA + 2 * SB; }
  static constexpr int pieces(int sl) { return (sl == 0 || sl == 3) ? PA : PB; }
  static_assert(2 * SA + 2 * SB == G8_BUF, "a K-tile is 64 KiB");
  static_assert(NJ == 2, "column permutation below");
};
// tile column (within a wave-column half) of B LDS row jj: lane group f of the 16 x 16 MFMA
// block pair jb = 0, 1 owns 8 consecutive columns (one 16-byte f16 store)
__device__ __forceinline__ int g8_colperm(int jj) {
  const int jb = jj >> 4, f = (jj >> 2) & 3, r = jj & 3;
  return 8 * f + 4 * jb + r;
}


template <int EPI>
__global__ __launch_bounds__(G8_THREADS) void gemm_8p_kernel(GemmArgs g) {
  using GG = G8Geom;
  constexpr int BM = GG::BM, BN = GG::BN, WM = GG::WM, WN = GG::WN, HM = GG::HM, HN = GG::HN;
  constexpr int NI = GG::NI, NJ = GG::NJ, PA = GG::PA, PB = GG::PB;
  __shared__ __attribute__((aligned(16))) char smem[2 * G8_BUF + G8_BIAS_MAX * 4];
  float* sbias = (float*)(smem + 2 * G8_BUF);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  // this workgroup's tiles: lo + s + k * nbx, k = 0 .. my_n - 1
  const int tiles_n = g.N / BN;
  const int ntiles = ((g.M + BM - 1) / BM) * tiles_n;
  const int xcd = blockIdx.x & 7, sidx = blockIdx.x >> 3;
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3;
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int cnt = q8 + (xcd < r8 ? 1 : 0);
  const int my_n = sidx < cnt ? (cnt - sidx + nbx - 1) / nbx : 0;
  const int ktiles = g.K / GK;
  if (my_n == 0) return;  // whole workgroup, before any barrier
  // segment i of this workgroup: tile T, k-tiles [kb, ke)
  auto seg = [&](int i, int& T, int& kb, int& ke) {
    T = lo + sidx + i * nbx;
    kb = 0;
    ke = ktiles;
  };
  const int nseg = my_n;

  for (int i = threadIdx.x; i < g.N; i += G8_THREADS) sbias[i] = g.bias ? g.bias[i] : 0.f;
  __syncthreads();

  const int KH = 4 * ktiles;    // half-tiles per tile
  const int total = my_n * KH;  // half-tiles of the whole stream

  // staging: a slot with PX pieces per wave gets pieces PX w .. PX w + PX - 1 (8 LDS rows each)
  // from this wave; LDS row j = 8 (PX w + q) + (lane >> 3), chunk position lane & 7 holds
  // source chunk (lane & 7) ^ ((j >> 1) & 7).
  // A slot h: LDS row j holds tile row WM (j / HM) + HM h + j % HM (wave-row j / HM, half h).
  // B slot h: LDS row j = HN wc + 16 jb + 4 f + r holds tile column WN wc + HN h + g8_colperm(j % HN).
  int rowA[2][PA], colB[2][PB], coffA[PA], coffB[PB];
#pragma unroll
  for (int q = 0; q < PA; ++q) {
    const int j = 8 * (PA * w + q) + (lane >> 3);
    coffA[q] = ((lane & 7) ^ ((j >> 1) & 7)) * 8;
#pragma unroll
    for (int h = 0; h < 2; ++h) rowA[h][q] = WM * (j / HM) + HM * h + j % HM;
  }
#pragma unroll
  for (int q = 0; q < PB; ++q) {
    const int j = 8 * (PB * w + q) + (lane >> 3);
    coffB[q] = ((lane & 7) ^ ((j >> 1) & 7)) * 8;
#pragma unroll
    for (int h = 0; h < 2; ++h) colB[h][q] = WN * (j / HN) + HN * h + g8_colperm(j % HN);
  }
  // The stream is consumed strictly in order (prologue L[0..6], then L[phi + 7]); phase p of
  // a K-tile always issues slot (p + 3) & 3, a compile-time constant, so the loader keeps
  // its K-tile position incrementally and recomputes this lane's source-row element
  // offsets once per tile (no per-phase division or slot selection).
  int ld_kt, ld_ke, ld_T, ld_seg = 0, ld_par = 0;
  seg(0, ld_T, ld_kt, ld_ke);
  int gA[2][PA], gB[2][PB];  // element offsets (row * ld + chunk) for the tile being loaded
  auto load_tile_offsets = [&]() {
    const int tm = ld_T / tiles_n;
    const int m0 = tm * BM, n0 = (ld_T - tm * tiles_n) * BN;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int q = 0; q < PA; ++q) gA[h][q] = min(m0 + rowA[h][q], g.M - 1) * g.lda + coffA[q];
#pragma unroll
      for (int q = 0; q < PB; ++q) gB[h][q] = (n0 + colB[h][q]) * g.ldw + coffB[q];
    }
  };
  load_tile_offsets();
  auto stage_slot = [&](auto SL) {
    constexpr int sl = decltype(SL)::value;
    constexpr int PX = GG::pieces(sl);
    const int k0 = ld_kt * GK;
    const uint32_t dst = lds_base + (uint32_t)(ld_par * G8_BUF + GG::slot_off(sl)) + (uint32_t)(w * PX * 1024);
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const _Float16* src;
      if constexpr (sl == 0) src = g.A + gA[0][q];
      else if constexpr (sl == 1) src = g.W + gB[0][q];
      else if constexpr (sl == 2) src = g.W + gB[1][q];
      else src = g.A + gA[1][q];
      glds_x4(src + k0, dst + q * 1024);
    }
    if constexpr (sl == 3) {  // K-tile complete: advance the loader
      ld_par ^= 1;
      if (++ld_kt == ld_ke && ++ld_seg < nseg) {
        seg(ld_seg, ld_T, ld_kt, ld_ke);
        load_tile_offsets();
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  using S3 = std::integral_constant<int, 3>;

  int offA[NI][2], offB[NJ][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < NI; ++i) offA[i][kk] = swz_off(HM * wr + 16 * i + fr, kk * 4 + fq);
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) offB[jb][kk] = swz_off(HN * wc + 16 * jb + fr, kk * 4 + fq);
  }

  f32x4 acc[2][2][NI][NJ];  // [h][hh][i][jb]
  half8 fa[NI][2], fb0[NJ][2], fb1[NJ][2];
  auto readA = [&](const char* slot) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        fa[i][kk] = *(const half8*)(slot + offA[i][kk]);
      }
  };
  auto readB = [&](const char* slot, half8 (&fb)[NJ][2]) {
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        fb[jb][kk] = *(const half8*)(slot + offB[jb][kk]);
      }
  };
  auto mfma_q = [&](f32x4 (&a)[NI][NJ], const half8 (&fb)[NJ][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int jb = 0; jb < NJ; ++jb)
          a[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[jb][kk], fa[i][kk], a[i][jb], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int ST_FULL = ((EPI == EPI_F32_RESIDUAL || EPI == EPI_F32) ? 2 : 1) * 2 * 2 * NI;
  int st_phi = -100;  // last phase before the most recent epilogue
  int st_cnt = 0;     // vector stores that epilogue issued (wave-uniform)
  // end of a read segment: issue L[phi + 7] (slot SL), wait for L[phi + 2] (read by phase
  // phi + 1) and for this segment's own ds_reads, barrier
  // LDS-DMA instructions of L[i + 1 .. last] (the stream's slot i & 3 has pieces(i & 3) each)
  auto younger = [&](int i, int last) {
    int n = 0;
    for (int t = i + 1; t <= last; ++t) n += ((t & 3) == 0 || (t & 3) == 3) ? PA : PB;
    return n;
  };
  auto end_reads = [&](int phi, auto SL) {
    constexpr int sl = decltype(SL)::value;
    // steady state: L[phi + 3 .. phi + 7] in flight = every slot once + slot sl again
    constexpr int YSTEADY = 2 * PA + 2 * PB + GG::pieces(sl);
    const bool full = phi + 7 < total;  // five younger half-tiles in flight
    if (full) stage_slot(SL);
    const bool post = phi - st_phi <= 5;  // the last epilogue's stores are younger than L[phi + 2]
    if (__builtin_expect(full && !post, 1)) {
      vmcnt_wait_c<YSTEADY>();
    } else if (full && st_cnt == ST_FULL) {  // after a tile with every row valid
      vmcnt_wait_c<YSTEADY + ST_FULL>();
    } else if (full) {
      vmcnt_wait(YSTEADY + st_cnt);
    } else {
      vmcnt_wait(younger(phi + 2, total - 1) + (post ? st_cnt : 0));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
  };

  {  // prologue: L[0..6], then L[0], L[1] landed
    const int last = min(6, total - 1);
    stage_slot(S0{});
    if (last >= 1) stage_slot(S1{});
    if (last >= 2) stage_slot(S2{});
    if (last >= 3) stage_slot(S3{});
    if (last >= 4) stage_slot(S0{});
    if (last >= 5) stage_slot(S1{});
    if (last >= 6) stage_slot(S2{});
    vmcnt_wait(younger(1, last));  // L[0], L[1] landed
    bar();
  }
  // waves 4..7 (one per SIMD beside a wave of 0..3) run one barrier behind waves 0..3
  if (wr == 1) bar();
  int phi = 0;
  for (int sg = 0; sg < nseg; ++sg) {
    int T, kb, ke;
    seg(sg, T, kb, ke);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int jb = 0; jb < NJ; ++jb) acc[h][hh][i][jb] = f32x4{};
    for (int kt = kb; kt < ke; ++kt, phi += 4) {
      const char* buf = (const char*)smem + ((phi >> 2) & 1) * G8_BUF;
      readA(buf + GG::slot_off(0));  // phase 0: (h0, hh0)
      readB(buf + GG::slot_off(1), fb0);
      end_reads(phi, S3{});
      mfma_q(acc[0][0], fb0);
      bar();
      readB(buf + GG::slot_off(2), fb1);  // phase 1: (h0, hh1)
      end_reads(phi + 1, S0{});
      mfma_q(acc[0][1], fb1);
      bar();
      readA(buf + GG::slot_off(3));  // phase 2: (h1, hh1)
      end_reads(phi + 2, S1{});
      mfma_q(acc[1][1], fb1);
      bar();
      end_reads(phi + 3, S2{});  // phase 3: (h1, hh0) from registers
      mfma_q(acc[1][0], fb0);
      bar();
    }
    st_phi = phi - 1;
    st_cnt = 0;

    // epilogue: blocks (h, hh, i): row WM wr + HM h + 16 i + fr; columns WN wc + HN hh + 8 fq
    // + (0..7) from the block pair jb = 0, 1 (one 16-byte f16 store, two for f32)
    const int tm = T / tiles_n;
    const int m0 = tm * BM, n0 = (T - tm * tiles_n) * BN;
    constexpr int SPB = (EPI == EPI_F32_RESIDUAL || EPI == EPI_F32) ? 2 : 1;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int n = n0 + WN * wc + HN * hh + 8 * fq;
      float bn[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) bn[r] = sbias[n + r];
      // residual: the half's old C values in one batch of loads (rows clamped into the matrix)
      f32x4 cv[2][NI][2];
      if constexpr (EPI == EPI_F32_RESIDUAL) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const int mc = min(m0 + WM * wr + HM * h + 16 * i + fr, g.M - 1);
            const f32x4* p = (const f32x4*)((const float*)g.C + (size_t)mc * g.ldc + n);
            cv[h][i][0] = p[0];
            cv[h][i][1] = p[1];
          }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int mb = m0 + WM * wr + HM * h + 16 * i;  // wave-uniform block row
          const int m = mb + fr;
          if (mb < g.M) {  // uniform branch: a block with a valid row issues exactly
            st_cnt += SPB;  // SPB vector stores (counted for the vmcnt bookkeeping)
            if (m < g.M) {
              if constexpr (EPI == EPI_F32_RESIDUAL)
                gemm_store8_res(g, m, n, acc[h][hh][i][0], acc[h][hh][i][1], bn, cv[h][i][0], cv[h][i][1]);
              else
                gemm_store8<EPI>(g, m, n, acc[h][hh][i][0], acc[h][hh][i][1], bn);
            }
          }
        }
      }
    }
  }
  if (wr == 0) bar();  // same barrier count for both groups
}

// ---------------------------------------------------------------------------
// K3w (weight-stationary; the text towers' K <= 512 GEMMs with an f16 epilogue: q|k|v and fc1 of
// MiniLM-L6 and CLIP text at the config-5 batch, M = 16,000). The MLP / attention projections of
// modeling_bert.py:282-350 and modeling_clip.py:293-296,343-350 with K = 384 or 512 are too short
// for K3d's k-loop (six or eight 64-deep k-tiles per 256 x 256 tile: its fill and the epilogue set
// the time, 0.16-0.29 of the MFMA peak). Here a wave keeps its 16 NB weight columns over the
// whole K in the accumulator file for the whole launch (NB = 4, K = 512: 256 AGPRs), as K7 keeps
// its queries, and the activation rows stream through LDS in 64-row tiles by LDS-DMA, double
// buffered, one barrier per tile: per 32-deep k-step 4 NB MFMA 16x16x32 (the weight fragment as
// operand A, the activation fragment as operand B, one accumulator per output block, ascending k:
// K3's element order and K3's gemm_store4 epilogue, so rows are bit-identical to K3 / K3d). The
// previous tile's epilogue (bias, activation, f16 store) and the next tile's LDS-DMA pieces run
// in the MFMA gaps of the tile's first k-steps. Block b: panel p of 4 x 16 NB columns, row range
// r (tiles r, r + R, ...); where R % 8 == 0 the P panels of a row range share an XCD (blocks
// b = 8 s + x, s = r / 8 * P + p: an activation tile is fetched into one L2; speed only).
constexpr int WS_ROWS = 64, WS_WAVES = 4, WS_THREADS = 64 * WS_WAVES;

__device__ __forceinline__ void ws_mfma(f32x4& acc, const half8& w, const half8& a) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(a));
}
__device__ __forceinline__ void ws_mfma0(f32x4& acc, const half8& w, const half8& a) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "a"(w), "v"(a));
}

template <int EPI, int NB, int KT>
__global__ __launch_bounds__(WS_THREADS) void gemm_ws_kernel(GemmArgs g, int P, int R, int xcd_map) {
  constexpr int K = 32 * KT, ROW_BYTES = 2 * K, CPR = K / 8, TILE_BYTES = WS_ROWS * ROW_BYTES;
  constexpr int PW = TILE_BYTES / 1024 / WS_WAVES;  // 1 KiB LDS-DMA pieces per wave per tile
  constexpr int FRONT = 4;                          // pieces per k-step (k-steps 0 .. PW / 4 - 1)
  constexpr int NA = 5;                             // A-fragment ring
  constexpr int NFR = 4 * KT;                       // A fragments per tile: (kk, rb)
  constexpr int NBLK = 4 * NB;                      // output blocks per wave per tile
  constexpr int KDMA = PW / FRONT;                   // k-steps that issue the next tile's pieces
  constexpr int NST = 8;                             // output stores per wave per tile (8 rows each)
  constexpr int OUT_OFF = 2 * TILE_BYTES, OUT_WAVE = WS_ROWS * 128;  // per-wave 64 x 128-B output image
  static_assert(CPR % 16 == 0 && PW % FRONT == 0, "tile geometry");
  constexpr int KD0 = 3;                             // first k-step of the DMA pieces
  constexpr int WSLOTS = 4 * (KT - 2);               // output-block write slots: k-steps 2 .. KT - 1
  static_assert(NB >= 2 && NB <= 4 && KD0 + KDMA <= KT && NBLK <= WSLOTS, "slot plan");
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES + WS_WAVES * OUT_WAVE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, g4 = lane >> 4;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  int p, r;
  if (xcd_map) {
    const int s = (int)blockIdx.x >> 3;
    p = s % P;
    r = (s / P) * 8 + ((int)blockIdx.x & 7);
  } else {
    p = (int)blockIdx.x % P;
    r = (int)blockIdx.x / P;
  }
  const int mtiles = (g.M + WS_ROWS - 1) / WS_ROWS;
  const int my_tiles = r < mtiles ? (mtiles - 1 - r) / R + 1 : 0;
  if (my_tiles <= 0) return;  // whole workgroup, before any barrier
  const int n0 = (p * WS_WAVES + w) * 16 * NB;

  // LDS image of a tile: row j, 16-byte chunk c at position c ^ (j & 15) (conflict-free fragment
  // reads); piece (w PW + i) of a tile = 64 consecutive chunks of the image, one per lane
  auto stage_piece = [&](int buf, int tile, int i) {
    const int piece = w * PW + i;
    const int q = piece * 64 + lane;
    const int row = q / CPR, pos = q - row * CPR;
    const int c = pos ^ (row & 15);
    const int m = min(tile * WS_ROWS + row, g.M - 1);
    glds_x4(g.A + (size_t)m * g.lda + c * 8, lds_base + (uint32_t)(buf * TILE_BYTES + piece * 1024));
  };
  // the first tile's pieces go out first, then the bias, then the weights: the wait before the
  // first tile (below) covers the pieces and the bias only, and each weight fragment is waited
  // for at its first MFMA (the compiler counts the loads into AGPRs), so the weight panel lands
  // under the first tile's MFMAs instead of before them
#pragma unroll
  for (int i = 0; i < PW; ++i) stage_piece(0, r, i);
  // branch-free (a branch here made the compiler wait for every load in flight at its join):
  // without a bias the loads read the weights and the values are dropped
  const bool has_bias = g.bias != nullptr;
  float bias[NB][4];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) {
    const float* bp = has_bias ? g.bias + n0 + 16 * cb + 4 * g4 : (const float*)g.W;
    const f32x4 b4 = *(const f32x4*)bp;
#pragma unroll
    for (int q = 0; q < 4; ++q) bias[cb][q] = has_bias ? b4[q] : 0.0f;
  }

  // this wave's weight columns n0 + 16 cb + c16, all of K, in AGPRs for the launch
  half8 wf[KT][NB];
#pragma unroll
  for (int kk = 0; kk < KT; ++kk)
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
      wf[kk][cb] = *(const half8*)(g.W + (size_t)(n0 + 16 * cb + c16) * g.ldw + 32 * kk + 8 * g4);

  // A fragment (kk, rb): row 16 rb + c16, chunk 4 kk + g4 -> position (4 kk + g4) ^ c16
  const int offA0 = c16 * ROW_BYTES + 16 * (g4 ^ c16);
  half8 a[NA];
  auto read_a = [&](const char* tb, int n) {
    const int kk = n >> 2, rb = n & 3;
    a[n % NA] = *(const half8*)(tb + ((offA0 ^ ((kk & 3) << 6)) + (kk >> 2) * 256 + rb * 16 * ROW_BYTES));
  };

  f32x4 acc[2][4][NB];
  int m0_1 = 0, m0_2 = 0;  // first rows of tiles it - 1 (blocks written now) and it - 2 (rows stored now)
  // Epilogue through this wave's LDS output image (64 rows x 128 B; 8-byte unit u of row j at
  // u ^ 2 (j & 7): rows j and j + 8 of a ds_write_b64 lane group share a bank pair, 0.15 of the
  // kernel's LDS cycles; the conflict-free u ^ (j & 15) needs the odd rows' unit pairs swapped
  // back after the read and measured 2-4 % slower, profiles/r6s12_*): a block's four finished outputs (gemm_act of acc + bias: gemm_store4's
  // arithmetic) as one ds_write_b64, then whole 128-byte rows out by 16-byte global stores — one
  // store instruction = 8 rows x 128 B, 8 per tile, instead of 16 scattered 8-byte ones. During
  // tile it: k-steps 0-2 store tile it - 2's image (each row read a k-step before its store), the
  // next tile's pieces go out in k-steps 3 ..., and tile it - 1's blocks enter the image one per
  // few k-steps from k-step 2 on (its VALU spread over the MFMA gaps, not in one burst).
  char* const ow = smem + OUT_OFF + w * OUT_WAVE;
  auto epi_write = [&](auto y_c, int e) {
    constexpr int Y = decltype(y_c)::value;
    typedef _Float16 half4 __attribute__((ext_vector_type(4)));
    const int rb = e / NB, cb = e - (e / NB) * NB;
    const int j = 16 * rb + c16, u = 4 * cb + g4;
    const f32x4 v = acc[Y][rb][cb];
    half4 h;
#pragma unroll
    for (int q = 0; q < 4; ++q) h[q] = (_Float16)gemm_act<EPI>(v[q] + bias[cb][q]);
    *(half4*)(ow + j * 128 + 8 * (u ^ (2 * (j & 7)))) = h;
  };
  // rows 8 s .. 8 s + 7 of the image are read one k-step before their store (a read right before
  // its store made the wave wait for every LDS read in flight, the A-fragment ring included)
  half8 orow[4];
  auto epi_read = [&](int s) {
    const int j = 8 * s + (lane >> 3), q = lane & 7;
    orow[s & 3] = *(const half8*)(ow + j * 128 + 16 * (q ^ (j & 7)));
  };
  auto epi_store = [&](int s, int m0) {
    const int j = 8 * s + (lane >> 3), q = lane & 7;
    const int m = m0 + j;
    if (m < g.M && q < 2 * NB) *(half8*)((_Float16*)g.C + (size_t)m * g.ldc + n0 + 8 * q) = orow[s & 3];
  };

  auto tile_body = [&](auto x_c, int it) {
    constexpr int X = decltype(x_c)::value;
    constexpr int Y = 1 - X;
    const int tile = r + it * R;
    const bool has_next = it + 1 < my_tiles;
    const bool has_prev = it > 0, has_prev2 = it > 1;
    const char* tb = smem + X * TILE_BYTES;
#pragma unroll
    for (int n = 0; n < NA; ++n) read_a(tb, n);
    mrag::static_for<KT>([&](auto kk_c) {
      constexpr int kk = decltype(kk_c)::value;
      mrag::static_for<4 * NB>([&](auto j_c) {
        constexpr int j = decltype(j_c)::value;
        constexpr int rb = j / NB, cb = j % NB;
        constexpr int n = 4 * kk + rb;
        if constexpr (kk == 0)
          ws_mfma0(acc[X][rb][cb], wf[kk][cb], a[n % NA]);
        else
          ws_mfma(acc[X][rb][cb], wf[kk][cb], a[n % NA]);
        if constexpr (cb == NB - 1) {  // fragment n's last MFMA issued: read fragment n + NA
          if constexpr (n + NA < NFR) read_a(tb, n + NA);
        } else if constexpr (cb == 0) {  // tile it - 2's rows out, or the next tile's piece
          if constexpr (kk == 0) {
            if (has_prev2) epi_read(rb);
          } else if constexpr (kk == 1) {
            if (has_prev2) {
              epi_store(rb, m0_2);
              epi_read(4 + rb);
            }
          } else if constexpr (kk == 2) {
            if (has_prev2) epi_store(4 + rb, m0_2);
          } else if constexpr (kk >= KD0 && FRONT * (kk - KD0) + rb < PW) {
            if (has_next) stage_piece(Y, tile + R, FRONT * (kk - KD0) + rb);
          }
        } else if constexpr (cb == 1) {  // tile it - 1's output block e -> LDS (slot s = e WSLOTS / NBLK)
          if constexpr (kk >= 2) {
            constexpr int s = 4 * (kk - 2) + rb;
            constexpr int e = (s * NBLK + WSLOTS - 1) / WSLOTS;
            if constexpr (e < NBLK && e * WSLOTS / NBLK == s) {
              if (has_prev) epi_write(std::integral_constant<int, Y>{}, e);
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    // the stores went out in k-steps 1-2, before the pieces (k-steps 3 ...): this lands both
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    m0_2 = m0_1;
    m0_1 = tile * WS_ROWS;
    __syncthreads();
  };

  // the first tile's pieces and the bias (issued before the KT NB weight loads; the field holds
  // at most 63, which then also waits for the first weight loads)
  vmcnt_wait_c<(KT * NB < 63 ? KT * NB : 63)>();
  __syncthreads();
  // the first tile outside the loop: inside it the compiler waits for each weight fragment just
  // before its first MFMA; a loop using them would have all of them waited for at its entry
  tile_body(std::integral_constant<int, 0>{}, 0);
  for (int it = 1; it < my_tiles; it += 2) {
    tile_body(std::integral_constant<int, 1>{}, it);
    if (it + 1 < my_tiles) tile_body(std::integral_constant<int, 0>{}, it + 1);
  }
  // the image holds the second-to-last tile's rows (written during the last tile): out with them
  if (my_tiles > 1) {
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      epi_read(s);
      epi_store(s, m0_2);
    }
  }
  // the last tile's blocks: its MFMAs were the last instructions issued, so wait out their
  // results (MFMA -> VALU distance; the compiler does not see through the inline asm)
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
  if (my_tiles & 1) {
#pragma unroll
    for (int e = 0; e < NBLK; ++e) {
      asm volatile("" : "+v"(acc[0][e / NB][e % NB]));
      epi_write(std::integral_constant<int, 0>{}, e);
    }
  } else {
#pragma unroll
    for (int e = 0; e < NBLK; ++e) {
      asm volatile("" : "+v"(acc[1][e / NB][e % NB]));
      epi_write(std::integral_constant<int, 1>{}, e);
    }
  }
#pragma unroll
  for (int s = 0; s < NST; ++s) {
    epi_read(s);
    epi_store(s, m0_1);
  }
}

// ---------------------------------------------------------------------------
// K2: LayerNorm over rows of D <= 1024 (one wave per row, two-pass mean/var in f32).
// Optional row gather (pooling), f32 and/or f16 outputs (in-place f32 allowed).
__global__ __launch_bounds__(256) void layernorm_kernel(LayerNormArgs a) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.rows) return;
  const int src = a.gather ? a.gather[r] : r;
  const float* x = a.x + (size_t)src * a.ldx;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int d = lane + 64 * j;
    v[j] = d < a.D ? x[d] : 0.f;
    s += v[j];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  const float mean = s / (float)a.D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int d = lane + 64 * j;
    const float t = d < a.D ? v[j] - mean : 0.f;
    q += t * t;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
  const float rstd = rsqrtf(q / (float)a.D + a.eps);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int d = lane + 64 * j;
    if (d < a.D) {
      const float y = (v[j] - mean) * rstd * a.gamma[d] + a.beta[d];
      if (a.y32) a.y32[(size_t)r * a.D + d] = y;
      if (a.y16) a.y16[(size_t)r * a.D + d] = (_Float16)y;
    }
  }
}

// K2, vectorised (D % 4 == 0, 16-byte aligned rows: every encoder here): one wave per row,
// lane l owns the float4 chunks l, l + 64, ... (16-byte loads, 16-byte f32 / 8-byte f16
// stores); two-pass mean / variance in f32 from registers: one HBM pass over the row. (A
// single butterfly merging per-lane (count, mean, M2) pairs measured slower: 16.2 vs 12.5 us
// per ViT LayerNorm — three shuffles and a division per round.)
// gamma / beta chunks of this lane, loaded before the row's reductions (off their latency path)
__device__ __forceinline__ void ln_params4(int lane, int D, const float* gamma, const float* beta, f32x4 (&g4)[4],
                                           f32x4 (&b4)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    g4[j] = c < (D >> 2) ? ((const f32x4*)gamma)[c] : f32x4{};
    b4[j] = c < (D >> 2) ? ((const f32x4*)beta)[c] : f32x4{};
  }
}

__device__ __forceinline__ void ln_row4p(f32x4 (&v)[4], int lane, int D, float eps, const f32x4 (&g4)[4],
                                         const f32x4 (&b4)[4], float* y32, _Float16* y16) {
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  const int nc = D >> 2;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);  // v = 0 past the row
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  const float mean = s / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (lane + 64 * j < nc) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float d = v[j][t] - mean;
        q += d * d;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
  const float rstd = rsqrtf(q / (float)D + eps);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    if (c < nc) {
      f32x4 y;
#pragma unroll
      for (int t = 0; t < 4; ++t) y[t] = (v[j][t] - mean) * rstd * g4[j][t] + b4[j][t];
      if (y32) ((f32x4*)y32)[c] = y;
      if (y16) {
        half4 h;
#pragma unroll
        for (int t = 0; t < 4; ++t) h[t] = (_Float16)y[t];
        ((half4*)y16)[c] = h;
      }
    }
  }
}

__device__ __forceinline__ void ln_row4(f32x4 (&v)[4], int lane, int D, float eps, const float* gamma,
                                        const float* beta, float* y32, _Float16* y16) {
  f32x4 g4[4], b4[4];
  ln_params4(lane, D, gamma, beta, g4, b4);
  ln_row4p(v, lane, D, eps, g4, b4, y32, y16);
}

// One wave per row: the row's loads and the gamma / beta chunks are issued before the first
// reduction (two rows per wave measured slower: 14.3 vs 12.3 us per ViT LayerNorm).
__global__ __launch_bounds__(256) void layernorm4_kernel(LayerNormArgs a) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.rows) return;
  const int src = a.gather ? a.gather[r] : r;
  const f32x4* x = (const f32x4*)(a.x + (size_t)src * a.ldx);
  f32x4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = lane + 64 * j < (a.D >> 2) ? x[lane + 64 * j] : f32x4{};
  f32x4 g4[4], b4[4];
  ln_params4(lane, a.D, a.gamma, a.beta, g4, b4);
  ln_row4p(v, lane, a.D, a.eps, g4, b4, a.y32 ? a.y32 + (size_t)r * a.D : nullptr,
           a.y16 ? a.y16 + (size_t)r * a.D : nullptr);
}

// K2 streaming form (the same arithmetic, bit-identical to layernorm4_kernel): a persistent grid
// of LN_WG_PER_CU workgroups per CU; a wave walks rows w, w + W, ... (W = the grid's waves),
// loads its gamma / beta chunks once and issues the next row's loads before this row's
// reductions, so each wave keeps a row in flight while it reduces the previous one (one row per
// wave left every wave waiting on its own loads: ViT LayerNorm 13.6 -> 11.7 us; 2 and 8
// workgroups per CU measured 13.4 / 12.6 us).
constexpr int LN_WG_PER_CU = 4;
// Every load is unconditional (the prefetch of the last row re-loads it; chunks past the row load
// the row's last chunk and are zeroed after the wait) and the gather form is its own instance:
// with conditional loads the compiler merged the branch joins' counters and waited for ALL loads
// (`vmcnt(0)`, the prefetch included) before each row's reductions, so nothing overlapped.
template <bool GATHER>
__global__ __launch_bounds__(256) void layernorm_stream_kernel(LayerNormArgs a) {
  const int lane = threadIdx.x & 63;
  const int nw = (int)gridDim.x * 4;
  int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.rows) return;
  const int nc = a.D >> 2;
  f32x4 g4[4], b4[4];
  ln_params4(lane, a.D, a.gamma, a.beta, g4, b4);
  auto load = [&](int row, f32x4(&v)[4]) {
    const int src = GATHER ? a.gather[row] : row;
    const f32x4* x = (const f32x4*)(a.x + (size_t)src * a.ldx);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = x[min(lane + 64 * j, nc - 1)];
  };
  f32x4 v[4], vn[4];
  load(r, v);
  for (; r < a.rows; r += nw) {
    load(min(r + nw, a.rows - 1), vn);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (lane + 64 * j >= nc) v[j] = f32x4{};  // ln_row4p: v = 0 past the row
    ln_row4p(v, lane, a.D, a.eps, g4, b4, a.y32 ? a.y32 + (size_t)r * a.D : nullptr,
             a.y16 ? a.y16 + (size_t)r * a.D : nullptr);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = vn[j];
  }
}

// ViT token assembly + pre_layrnorm in one pass (modeling_clip.py:212-217, :642):
// X[b*T + t] = LN((t == 0 ? cls : patch[b*(T-1) + t-1]) + pos[t])   (f32)
__global__ __launch_bounds__(256) void vit_embed_ln_kernel(const float* __restrict__ patch,
                                                           const float* __restrict__ cls,
                                                           const float* __restrict__ pos, const float* gamma,
                                                           const float* beta, float* __restrict__ X, int B, int T,
                                                           int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B * T) return;
  const int b = r / T, t = r - (r / T) * T;
  const f32x4* e = (const f32x4*)(t == 0 ? cls : patch + ((size_t)b * (T - 1) + t - 1) * D);
  const f32x4* p = (const f32x4*)(pos + (size_t)t * D);
  f32x4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    v[j] = f32x4{};
    if (c < (D >> 2)) {
      const f32x4 a = e[c], q = p[c];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[j][u] = a[u] + q[u];
    }
  }
  ln_row4(v, lane, D, eps, gamma, beta, X + (size_t)r * D, nullptr);
}

// ---------------------------------------------------------------------------
// K4 helpers: transposed 16-bit LDS reads (ds_read_b64_tr_b16) for the V^T operand.
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4_lds __attribute__((__vector_size__(8)));

__device__ __forceinline__ half4_t lds_read_tr16(const _Float16* p) {
  const fp16x4_lds v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((AS3 fp16x4_lds*)(p));
  return __builtin_bit_cast(half4_t, v);
}

// V image of a key block in LDS: row r (key) of DH halves, no padding, 16-byte chunk j stored at
// position j ^ v_swz(r). Bank-conflict free for both accesses (MI355X_MICROARCH.md LDS table):
// the staging ds_write_b128 (8 contiguous lanes = whole rows: a permutation of each row's chunks),
// and the transposed ds_read_b64_tr_b16 of O^T += V^T P^T, whose 32-lane group reads 8 rows x 2
// chunks — the swizzle spreads those 16 chunks over the 16 four-bank slots (DH = 64: rows r and
// r + 1 share a slot base, so r & 6 moves the chunk pair; DH = 32: rows r and r + 4 share one,
// so (r >> 1) & 2 does). The padded row strides of round 5 left 2-way conflicts on the reads
// (DH = 64) or on the writes (DH = 32).
template <int DH>
__device__ __forceinline__ int v_swz(int r) {
  return DH == 64 ? (r & 6) : ((r >> 1) & 2);
}
// half offset of (row r, half column col) in such an image (col within one chunk's 8 halves kept)
template <int DH>
__device__ __forceinline__ int v_off(int r, int col) {
  return r * DH + ((((col >> 3) ^ v_swz<DH>(r)) << 3) | (col & 7));
}

// K4 v3 (flash form, any L <= 512, head_dim 32 or 64): one wave per (sequence, head, 16-query
// block); key blocks of 16 with an online softmax, all on MFMA 16x16:
//   S^T = K . Q^T    (16x16x32, DH/32 k-steps): lane (c, g) = (l & 15, l >> 4) holds query
//                    16 qb + c and keys 16 kb + 4 g + r — the query's row max / sum are the lane's
//                    4 registers plus two xor shuffles (16, 32);
//   O^T += V^T . P^T (16x16x16, one per 16 dims): P^T is the S^T accumulator cast to f16 in place
//                    (B operand: keys 4 g .. 4 g + 3 of query c), V^T comes from the wave's LDS
//                    copy of the key block by ds_read_b64_tr_b16 (A operand: dim 16 db + c, the
//                    same 4 keys); O^T holds 4 consecutive dims of query c: one 8-byte store each.
// Key blocks whose keys are all masked (the padding of a shorter sequence in a longer batch)
// are skipped, and every other block is processed identically whatever the batch's length:
// a sequence's result does not depend on how its batch is padded, for every L. Work per
// (sequence, head) grows with its own length only, not with a 64-row pad.
template <int DH>
__global__ __launch_bounds__(256) void attention_flash16_kernel(AttentionArgs a) {
  constexpr int KS = DH / 32;               // 32-dim k-steps of S^T
  constexpr int DB = DH / 16;               // 16-dim blocks of O^T
  typedef _Float16 half4_v __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) _Float16 Vs[4][16 * DH];  // v_off layout
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int L = a.L, nqb = (L + 15) >> 4;
  const int item = blockIdx.x * 4 + w;
  if (item >= a.B * a.H * nqb) return;  // whole wave (the transposed reads need EXEC all ones)
  const int qb = item % nqb, bh = item / nqb;
  const int hd = bh % a.H, b = bh / a.H;
  const int D = a.H * DH;
  const size_t rs = (size_t)3 * D;
  const _Float16* base = a.qkv + (size_t)b * L * rs + hd * DH;
  const int qrow = 16 * qb + c;
  half8 qf[KS];
#pragma unroll
  for (int st = 0; st < KS; ++st)
    qf[st] = qrow < L ? *(const half8*)(base + (size_t)qrow * rs + 32 * st + 8 * g) : half8{};
  f32x4 o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) o[db] = f32x4{};
  float m = -INFINITY, l = 0.f;
  _Float16* vs = Vs[w];
  const int nkb = a.causal ? min((L + 15) >> 4, qb + 1) : (L + 15) >> 4;
  // a key block's operands (K fragments, this lane's V chunks, its 4 keys' mask flags) are loaded
  // together at its top (24.6 us per ViT layer vs 27.1 for a K -> MFMA -> V chain; two blocks
  // ahead measured 27.0: the extra VGPRs halve the occupancy)
  struct Blk {
    half8 kf[KS], vv[KS];
    bool kv[4];
  };
  auto load_blk = [&](int kb, Blk& x) {
    const int krow = 16 * kb + c;
#pragma unroll
    for (int st = 0; st < KS; ++st)
      x.kf[st] = krow < L ? *(const half8*)(base + (size_t)krow * rs + D + 32 * st + 8 * g) : half8{};
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const int idx = lane + 64 * t, key = idx / (DH / 8), ch = idx % (DH / 8);
      const int kr = 16 * kb + key;
      x.vv[t] = kr < L ? *(const half8*)(base + (size_t)kr * rs + 2 * D + 8 * ch) : half8{};
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * kb + 4 * g + r;
      bool ok = key < L;
      if (ok && a.mask) ok = a.mask[(size_t)b * L + key] != 0;
      if (a.causal) ok = ok && key <= qrow;
      x.kv[r] = ok;
    }
  };
  Blk cur;
  for (int kb = 0; kb < nkb; ++kb) {
    load_blk(kb, cur);
    bool any_ok = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) any_ok |= cur.kv[r];
    if (!__any(any_ok)) continue;  // wave-uniform: a fully masked key block
    f32x4 sacc = {};
#pragma unroll
    for (int st = 0; st < KS; ++st) sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(cur.kf[st], qf[st], sacc, 0, 0, 0);
    // V rows of the block -> this wave's LDS image (16 B per lane per row chunk)
    asm volatile("" ::: "memory");  // the previous block's transposed reads come first
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const int idx = lane + 64 * t, key = idx / (DH / 8), ch = idx % (DH / 8);
      *(half8*)(vs + v_off<DH>(key, 8 * ch)) = cur.vv[t];
    }
    float sv[4], bmax = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sv[r] = cur.kv[r] ? sacc[r] * a.scale : -INFINITY;
      bmax = fmaxf(bmax, sv[r]);
    }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32));
    const float mn = fmaxf(m, bmax);
    const float alpha = m == -INFINITY ? 0.f : __expf(m - mn);
    half4_v pf;
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pv = sv[r] == -INFINITY ? 0.f : __expf(sv[r] - mn);
      pf[r] = (_Float16)pv;
      ps += pv;
    }
    ps += __shfl_xor(ps, 16);
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      o[db] *= alpha;
      const half4_t vt = lds_read_tr16(vs + v_off<DH>(4 * g + (c >> 2), 16 * db + 4 * (c & 3)));
      o[db] = __builtin_amdgcn_mfma_f32_16x16x16f16(vt, pf, o[db], 0, 0, 0);
    }
  }
  if (qrow < L) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    _Float16* orow = a.out + ((size_t)b * L + qrow) * D + hd * DH + 4 * g;
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      const half4_t h = {(_Float16)(o[db][0] * inv), (_Float16)(o[db][1] * inv), (_Float16)(o[db][2] * inv),
                         (_Float16)(o[db][3] * inv)};
      *(half4_t*)(orow + 16 * db) = h;
    }
  }
}

// ---------------------------------------------------------------------------
// K1 (prologue): CLIP pixel normalisation fused into the patch im2col.
// Reference: CLIPImageProcessor rescale (u8 -> f64 * 1/255 -> f32) then (x - mean) / std
// in f32 (app/ml/embeddings.py:85; bit-exact formula verified in SURVEY.md §8a a2), then the
// Conv2d(3, 768, k=32, s=32) as a GEMM with K ordered (c, kh, kw) like the torch weight.
// img: [B][S][S][3] u8 (HWC, the decoded RGB image), out: [B*G*G][3*P*P] f16.
// K4 v3, one sequence per workgroup (33 <= L <= 64: the ViT's 50 tokens): the four waves are the
// sequence's (up to) four 16-query blocks of one head, and the head's K and V rows are staged into
// LDS ONCE by all 256 threads (one round trip) instead of each wave loading every key block in
// turn (four dependent global round trips per wave: 27.8 us per ViT layer, latency-bound). The
// per-wave arithmetic is attention_flash16_kernel's, operand for operand (K fragments and the
// transposed V reads come from the shared image), so the outputs are bit-identical to it.
template <int DH>
__global__ __launch_bounds__(256) void attention_seq64_kernel(AttentionArgs a) {
  constexpr int KS = DH / 32, DB = DH / 16;
  typedef _Float16 half4_v __attribute__((ext_vector_type(4)));
  // K image: rows of DH halves, 16-byte chunk j at j ^ ((r >> 1) & (DH / 8 - 1)) — the K-fragment
  // ds_read_b128 of 16 rows x one chunk column per lane quarter covers all 64 banks (the GEMMs'
  // swz_off rule); V image: v_off (as attention_flash16_kernel)
  __shared__ __attribute__((aligned(16))) _Float16 Ks[64 * DH];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[64 * DH];
  __shared__ int kok[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int L = a.L, nqb = (L + 15) >> 4;
  const int bh = blockIdx.x, hd = bh % a.H, b = bh / a.H;
  const int D = a.H * DH;
  const size_t rs = (size_t)3 * D;
  const _Float16* base = a.qkv + (size_t)b * L * rs + hd * DH;
  // stage: 64 key rows x DH of K and of V (zeros past L), 16 B per thread per step; every global
  // load (K, V, the mask flag, this wave's Q fragments) is issued before the first LDS store, so
  // a workgroup pays one memory round trip
  constexpr int CH = DH / 8;             // 16-byte chunks per row
  constexpr int NST = 64 * CH / 256;     // staging steps per thread
  static_assert(NST * 256 == 64 * CH, "64 rows of DH halves in whole 256-thread steps");
  half8 kv[NST], vv[NST];
  // (rows past L load row L - 1, unconditionally, and are zeroed at the store: a conditional load
  // made the compiler wait for it at the branch join)
#pragma unroll
  for (int t = 0; t < NST; ++t) {
    const int idx = threadIdx.x + 256 * t, key = min(idx / CH, L - 1), ch = idx % CH;
    kv[t] = *(const half8*)(base + (size_t)key * rs + D + 8 * ch);
    vv[t] = *(const half8*)(base + (size_t)key * rs + 2 * D + 8 * ch);
  }
  const int qb = w;
  const int qrow = 16 * qb + c;
  half8 qf[KS];
#pragma unroll
  for (int st = 0; st < KS; ++st) qf[st] = *(const half8*)(base + (size_t)min(qrow, L - 1) * rs + 32 * st + 8 * g);
  int ok = 0;
  if (threadIdx.x < 64) {
    const int key = threadIdx.x;
    ok = key < L && (!a.mask || a.mask[(size_t)b * L + key] != 0);
  }
  auto k_off = [&](int r, int ch) { return r * DH + 8 * (ch ^ ((r >> 1) & (CH - 1))); };
#pragma unroll
  for (int t = 0; t < NST; ++t) {
    const int idx = threadIdx.x + 256 * t, key = idx / CH, ch = idx % CH;
    *(half8*)(Ks + k_off(key, ch)) = key < L ? kv[t] : half8{};
    *(half8*)(Vs + v_off<DH>(key, 8 * ch)) = key < L ? vv[t] : half8{};
  }
  if (threadIdx.x < 64) kok[threadIdx.x] = ok;
  if (qrow >= L) {
#pragma unroll
    for (int st = 0; st < KS; ++st) qf[st] = half8{};
  }
  __syncthreads();
  if (qb >= nqb) return;  // whole wave, after the barrier
  f32x4 o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db) o[db] = f32x4{};
  float m = -INFINITY, l = 0.f;
  const int nkb = a.causal ? min(nqb, qb + 1) : nqb;
  for (int kb = 0; kb < nkb; ++kb) {
    bool kv[4], any_ok = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * kb + 4 * g + r;
      kv[r] = kok[key] != 0 && (!a.causal || key <= qrow);
      any_ok |= kv[r];
    }
    if (!__any(any_ok)) continue;  // wave-uniform: a fully masked key block
    f32x4 sacc = {};
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const half8 kf = *(const half8*)(Ks + k_off(16 * kb + c, 4 * st + g));
      sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[st], sacc, 0, 0, 0);
    }
    float sv[4], bmax = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sv[r] = kv[r] ? sacc[r] * a.scale : -INFINITY;
      bmax = fmaxf(bmax, sv[r]);
    }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32));
    const float mn = fmaxf(m, bmax);
    const float alpha = m == -INFINITY ? 0.f : __expf(m - mn);
    half4_v pf;
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pv = sv[r] == -INFINITY ? 0.f : __expf(sv[r] - mn);
      pf[r] = (_Float16)pv;
      ps += pv;
    }
    ps += __shfl_xor(ps, 16);
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      o[db] *= alpha;
      const half4_t vt = lds_read_tr16(Vs + v_off<DH>(16 * kb + 4 * g + (c >> 2), 16 * db + 4 * (c & 3)));
      o[db] = __builtin_amdgcn_mfma_f32_16x16x16f16(vt, pf, o[db], 0, 0, 0);
    }
  }
  if (qrow < L) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    _Float16* orow = a.out + ((size_t)b * L + qrow) * D + hd * DH + 4 * g;
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      const half4_t h = {(_Float16)(o[db][0] * inv), (_Float16)(o[db][1] * inv), (_Float16)(o[db][2] * inv),
                         (_Float16)(o[db][3] * inv)};
      *(half4_t*)(orow + 16 * db) = h;
    }
  }
}

__global__ void vit_im2col_kernel(const uint8_t* __restrict__ img, _Float16* __restrict__ out, int B, int S,
                                  int P) {
  const int G = S / P;
  const int K = 3 * P * P;
  const int64_t total8 = (int64_t)B * G * G * (K / 8);
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total8) return;
  const int64_t row = idx / (K / 8);
  const int k8 = (int)(idx - row * (K / 8)) * 8;
  const int c = k8 / (P * P), kh = (k8 / P) % P, kw0 = k8 % P;
  const int b = (int)(row / (G * G)), pidx = (int)(row % (G * G));
  const int py = pidx / G, px = pidx % G;
  const float mean = c == 0 ? 0.48145466f : (c == 1 ? 0.4578275f : 0.40821073f);
  const float stdv = c == 0 ? 0.26862954f : (c == 1 ? 0.26130258f : 0.27577711f);
  const uint8_t* src = img + (((size_t)b * S + (size_t)py * P + kh) * S + (size_t)px * P + kw0) * 3 + c;
  _Float16 v8[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const float x = (float)((double)src[t * 3] * (1.0 / 255.0));
    v8[t] = (_Float16)((x - mean) / stdv);
  }
  *(half8*)(out + row * K + k8) = *(half8*)v8;
}

// K1 for P = 32 (ViT-B/32), same arithmetic: one thread per (patch, kernel row kh). The 32
// pixels x 3 channels of one patch row are 96 contiguous bytes (six 16-byte loads); each
// channel's 32 values are 64 contiguous bytes of the output row (K ordered c, kh, kw): four
// 16-byte stores per channel. Needs S % 16 == 0 and a 16-byte aligned image base.
__global__ __launch_bounds__(256) void vit_im2col32_kernel(const uint8_t* __restrict__ img,
                                                           _Float16* __restrict__ out, int B, int S) {
  constexpr int P = 32, K = 3 * P * P;
  const int G = S / P;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * G * G * P) return;
  const int kh = (int)(idx % P);
  const int64_t row = idx / P;
  const int b = (int)(row / (G * G)), pidx = (int)(row % (G * G));
  const int py = pidx / G, px = pidx % G;
  const uint4* src = (const uint4*)(img + (((size_t)b * S + (size_t)py * P + kh) * S + (size_t)px * P) * 3);
  union {
    uint4 v[6];
    uint8_t u[96];
  } pix;
#pragma unroll
  for (int i = 0; i < 6; ++i) pix.v[i] = src[i];
  _Float16* dst = out + row * K + kh * P;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float mean = c == 0 ? 0.48145466f : (c == 1 ? 0.4578275f : 0.40821073f);
    const float stdv = c == 0 ? 0.26862954f : (c == 1 ? 0.26130258f : 0.27577711f);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      half8 v8;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float x = (float)((double)pix.u[3 * (8 * h + t) + c] * (1.0 / 255.0));
        v8[t] = (_Float16)((x - mean) / stdv);
      }
      *(half8*)(dst + c * P * P + 8 * h) = v8;
    }
  }
}

// Token embeddings: X[b*T+t] = tok[ids] + pos[t] (+ type0 for BERT)   (f32)
// one workgroup per token row (float4 over D): X[bt] = tok[id] + pos[t] (+ type row)
__global__ __launch_bounds__(128) void token_embed_kernel(const int32_t* __restrict__ ids, const float* __restrict__ tok,
                                                          const float* __restrict__ pos, const float* __restrict__ type_tab,
                                                          const int32_t* __restrict__ types, float* __restrict__ X, int B,
                                                          int T, int D, int vocab) {
  const int bt = blockIdx.x;
  const int t = bt % T;
  int id = ids[bt];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const f32x4* e = (const f32x4*)(tok + (size_t)id * D);
  const f32x4* p = (const f32x4*)(pos + (size_t)t * D);
  const f32x4* ty = type_tab ? (const f32x4*)(type_tab + (size_t)(types ? (types[bt] != 0) : 0) * D) : nullptr;
  f32x4* o = (f32x4*)(X + (size_t)bt * D);
  for (int c = threadIdx.x; c < (D >> 2); c += blockDim.x) {
    f32x4 v = e[c], q = p[c];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] += q[u];
    if (ty) {  // BERT type_vocab_size 2
      const f32x4 w = ty[c];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] += w[u];
    }
    o[c] = v;
  }
}

// CLIP text pooling row per sequence: first index of eos_id (eos_id >= 0) or argmax of
// the ids (legacy configs with eos_token_id == 2), modeling_clip.py:561-580.
__global__ void eos_rows_kernel(const int32_t* __restrict__ ids, int B, int T, int eos_id, int* __restrict__ rows) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int32_t* r = ids + (size_t)b * T;
  int best = 0;
  if (eos_id >= 0) {
    for (int t = 0; t < T; ++t)
      if (r[t] == eos_id) {
        best = t;
        break;
      }
  } else {
    int bv = r[0];
    for (int t = 1; t < T; ++t)
      if (r[t] > bv) {
        bv = r[t];
        best = t;
      }
  }
  rows[b] = b * T + best;
}

// Rows b*T (the CLS token of each image).
__global__ void cls_rows_kernel(int B, int T, int* __restrict__ rows) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) rows[b] = b * T;
}

// sentence-transformers mean pooling: sum_t(h*m) / clamp(sum_t m, 1e-9)
__global__ void mean_pool_kernel(const float* __restrict__ X, const int32_t* __restrict__ mask,
                                 float* __restrict__ out, int B, int T, int D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * D) return;
  const int b = (int)(idx / D), d = (int)(idx % D);
  float s = 0.f, c = 0.f;
  for (int t = 0; t < T; ++t) {
    const float mm = mask ? (float)(mask[(size_t)b * T + t] != 0) : 1.f;
    s += X[((size_t)b * T + t) * D + d] * mm;
    c += mm;
  }
  out[idx] = s / fmaxf(c, 1e-9f);
}

// ---------------------------------------------------------------------------
// launchers
int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 256;
    return v;
  }();
  return n;
}

// K3 (128 x 128, two workgroups per CU) vs K3d (persistent 256 x 256, one per CU) by rounds:
// a K3 round (two tiles per CU) takes ~2/3 of a K3d round (one 4x larger tile) on the same K
// (measured at K = 512 / 2048, N = 512: 23.7 vs 35.4 us, 53.1 vs 75.5 us), so K3 wins where the
// 256 x 256 grid leaves CUs idle and the 128 x 128 one does not — the CLIP text tower at the
// config-5 batch (N = 512). Ties stay on K3d (ties to K3 measured slower on the overlapped
// config-5 leg). Both kernels accumulate every element in the same order.
bool k3_beats_k3d(const GemmArgs& g) {
  if (g.N % 256 != 0) return true;
  const long cus = std::max(8, num_cus() / 8 * 8);
  const long t256 = (long)((g.M + 255) / 256) * (g.N / 256), t128 = (long)((g.M + 127) / 128) * (g.N / 128);
  const long r_d = (t256 + cus - 1) / cus, r_3 = (t128 + 2 * cus - 1) / (2 * cus);
  return 2 * r_3 < 3 * r_d;  // K3 time ~ (2/3) r_3 < r_d
}

template <template <int> class KERN>
int launch_epi(int epi, dim3 grid, dim3 block, hipStream_t s, const GemmArgs& g) {
  switch (epi) {
    case EPI_F16: hipLaunchKernelGGL(KERN<EPI_F16>::fn, grid, block, 0, s, g); break;
    case EPI_F16_QUICK_GELU: hipLaunchKernelGGL(KERN<EPI_F16_QUICK_GELU>::fn, grid, block, 0, s, g); break;
    case EPI_F16_GELU_ERF: hipLaunchKernelGGL(KERN<EPI_F16_GELU_ERF>::fn, grid, block, 0, s, g); break;
    case EPI_F32_RESIDUAL: hipLaunchKernelGGL(KERN<EPI_F32_RESIDUAL>::fn, grid, block, 0, s, g); break;
    case EPI_F32: hipLaunchKernelGGL(KERN<EPI_F32>::fn, grid, block, 0, s, g); break;
    default: return mrag::fail(MRAG_ERR_ARG, "gemm: bad epilogue %d", epi);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}
template <int EPI>
struct K3dKern {
  static constexpr auto fn = gemm_8p_kernel<EPI>;
};
template <int EPI>
struct K3Kern {
  static constexpr auto fn = gemm_nt_kernel<EPI>;
};
template <int MB>
struct K3sKern {
  template <int EPI>
  struct Kern {
    static constexpr auto fn = gemm_skinny_kernel<EPI, MB>;
  };
};

// K3w's shapes: an f16 epilogue, K = 384 or 512 (the weight columns of a wave fit the accumulator
// file), N a multiple of 256 (NB = 4) or 192 (NB = 3), enough rows for every CU
bool gemm_ws_fits(const GemmArgs& g, int epi) {
  const bool f16 = epi == EPI_F16 || epi == EPI_F16_QUICK_GELU || epi == EPI_F16_GELU_ERF;
  return f16 && (g.K == 384 || g.K == 512) && (g.N % 256 == 0 || g.N % 192 == 0) && g.M >= 4096;
}
// The automatic rule takes K3w wherever it fits. Alone, per GEMM (profiles/r6s7_probe.jsonl,
// M = 16,000): CLIP-text q|k|v 37.6 us against 41.6 on K3d, MiniLM q|k|v 26.9 against 31.7 on K3,
// CLIP-text fc1 47.5 against 47.5 on K3d, MiniLM fc1 (erf) 42.2 against 46.3 on K3d (38.0 on K3);
// in the config-5 leg, four steps in flight, two interleaved rounds on one box
// (profiles/r6s9_fusion_ab.jsonl): 249.6k / 250.4k q/s against 248.6k / 248.4k with K3w on the
// q|k|v GEMMs only and 241.0k / 246.7k before K3w.
bool gemm_ws_auto(const GemmArgs& g, int epi) { return gemm_ws_fits(g, epi); }

template <int NB, int KT>
int launch_ws(const GemmArgs& g, int epi, hipStream_t s) {
  const int P = g.N / (64 * NB);
  const int cus = std::max(8, num_cus());
  int R = std::max(1, cus / P);
  int xcd_map = 0;
  if (R >= 8 && (R / 8 * 8) * 10 >= R * 9) {  // an XCD-aligned row split costing <= 10 % of the CUs
    R = R / 8 * 8;
    xcd_map = 1;
  }
  const dim3 grid((unsigned)(P * R)), block(WS_THREADS);
  switch (epi) {
    case EPI_F16: hipLaunchKernelGGL((gemm_ws_kernel<EPI_F16, NB, KT>), grid, block, 0, s, g, P, R, xcd_map); break;
    case EPI_F16_QUICK_GELU:
      hipLaunchKernelGGL((gemm_ws_kernel<EPI_F16_QUICK_GELU, NB, KT>), grid, block, 0, s, g, P, R, xcd_map);
      break;
    case EPI_F16_GELU_ERF:
      hipLaunchKernelGGL((gemm_ws_kernel<EPI_F16_GELU_ERF, NB, KT>), grid, block, 0, s, g, P, R, xcd_map);
      break;
    default: return mrag::fail(MRAG_ERR_ARG, "gemm K3w: epilogue %d unsupported", epi);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_gemm_ws(const GemmArgs& g, int epi, hipStream_t s) {
  MRAG_REQUIRE(gemm_ws_fits(g, epi), "gemm K3w: shape M=%d N=%d K=%d epilogue %d unsupported", g.M, g.N, g.K, epi);
  // K = 384 takes NB = 3 wherever N allows it: MiniLM fc1 (N = 1536, both fit) 43.1-43.2 -> 39.5-40.9
  // us alone, eight panels on all 256 CUs instead of six on 240; at K = 512 (CLIP-text q|k|v, also
  // both) NB = 3 measured no faster (profiles/r6s38_k3w_nb3_ab.jsonl)
  const bool nb4 = g.N % 256 == 0 && !(g.K == 384 && g.N % 192 == 0);
  if (g.K == 512) return nb4 ? launch_ws<4, 16>(g, epi, s) : launch_ws<3, 16>(g, epi, s);
  return nb4 ? launch_ws<4, 12>(g, epi, s) : launch_ws<3, 12>(g, epi, s);
}

int launch_gemm(const GemmArgs& g, int epi, hipStream_t s, int kernel) {
  if (g.M <= 0) return MRAG_OK;
  MRAG_REQUIRE(g.N % GN == 0 && g.K % GK == 0, "gemm: N=%d must be a multiple of %d and K=%d of %d", g.N, GN, g.K,
               GK);
  MRAG_REQUIRE(g.lda % 8 == 0 && g.ldw % 8 == 0 && g.ldc % 4 == 0, "gemm: lda/ldw must be multiples of 8, ldc of 4");
  MRAG_REQUIRE(((uintptr_t)g.bias & 15) == 0 && ((uintptr_t)g.C & 15) == 0, "gemm: bias and C must be 16-byte aligned");
  if (kernel == GEMM_K3W || (kernel == GEMM_AUTO && gemm_ws_auto(g, epi))) return launch_gemm_ws(g, epi, s);
  if (kernel == GEMM_K3D) {
    MRAG_REQUIRE(g.M >= 1024 && g.N <= G8_BIAS_MAX && g.N % 256 == 0, "gemm K3d: shape M=%d N=%d unsupported", g.M,
                 g.N);
    const int ntiles = ((g.M + G8Geom::BM - 1) / G8Geom::BM) * (g.N / G8Geom::BN);
    const int nb = std::min((ntiles + 7) / 8 * 8, std::max(8, num_cus() / 8 * 8));
    return launch_epi<K3dKern>(epi, dim3((unsigned)nb), dim3(G8_THREADS), s, g);
  }
  if (kernel == GEMM_K3S) {
    MRAG_REQUIRE(g.M <= 64, "gemm K3s: M=%d > 64", g.M);
  }
  if (kernel == GEMM_AUTO && g.M >= 1024 && g.N <= G8_BIAS_MAX && g.N % 256 == 0 && !k3_beats_k3d(g)) {
    const int ntiles = ((g.M + G8Geom::BM - 1) / G8Geom::BM) * (g.N / G8Geom::BN);
    const int nb = std::min((ntiles + 7) / 8 * 8, std::max(8, num_cus() / 8 * 8));
    return launch_epi<K3dKern>(epi, dim3((unsigned)nb), dim3(G8_THREADS), s, g);
  }
  if ((kernel == GEMM_AUTO && g.M <= 64) || kernel == GEMM_K3S) {
    const dim3 grid((unsigned)(g.N / 16));
    switch ((g.M + 15) / 16) {
      case 1: return launch_epi<K3sKern<1>::Kern>(epi, grid, dim3(64), s, g);
      case 2: return launch_epi<K3sKern<2>::Kern>(epi, grid, dim3(64), s, g);
      case 3: return launch_epi<K3sKern<3>::Kern>(epi, grid, dim3(64), s, g);
      default: return launch_epi<K3sKern<4>::Kern>(epi, grid, dim3(64), s, g);
    }
  }
  const dim3 grid((unsigned)(((g.M + GM - 1) / GM) * (g.N / GN)));
  return launch_epi<K3Kern>(epi, grid, dim3(GTHREADS), s, g);
}

int launch_layernorm(const LayerNormArgs& a, hipStream_t s) {
  if (a.rows <= 0) return MRAG_OK;
  MRAG_REQUIRE(a.D > 0 && a.D <= 1024, "layernorm: D=%d unsupported", a.D);
  const bool vec4 = a.D % 4 == 0 && a.ldx % 4 == 0 && ((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.gamma & 15) == 0 &&
                    ((uintptr_t)a.beta & 15) == 0 && ((uintptr_t)a.y32 & 15) == 0 && ((uintptr_t)a.y16 & 7) == 0;
  // in place through a gather, two output rows could read one input row another wave overwrites
  const bool alias = a.gather && a.y32 == a.x;
  if (vec4 && !alias) {
    const int nb = std::min((a.rows + 3) / 4, num_cus() * LN_WG_PER_CU);
    if (a.gather)
      hipLaunchKernelGGL(layernorm_stream_kernel<true>, dim3((unsigned)nb), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(layernorm_stream_kernel<false>, dim3((unsigned)nb), dim3(256), 0, s, a);
  } else if (vec4)
    hipLaunchKernelGGL(layernorm4_kernel, dim3((unsigned)((a.rows + 3) / 4)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)((a.rows + 3) / 4)), dim3(256), 0, s, a);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_vit_embed_ln(const float* patch, const float* cls, const float* pos, const float* gamma, const float* beta,
                        float* X, int B, int T, int D, float eps, hipStream_t s) {
  if (B * T == 0) return MRAG_OK;
  MRAG_REQUIRE(D % 4 == 0 && D <= 1024, "vit_embed_ln: D=%d unsupported", D);
  hipLaunchKernelGGL(vit_embed_ln_kernel, dim3((unsigned)((B * T + 3) / 4)), dim3(256), 0, s, patch, cls, pos, gamma,
                     beta, X, B, T, D, eps);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_attention(const AttentionArgs& a, int dh, hipStream_t s) {
  if (a.B <= 0) return MRAG_OK;
  MRAG_REQUIRE(a.L >= 1 && a.L <= 512, "attention: L=%d unsupported (1..512)", a.L);
  MRAG_REQUIRE(dh == 64 || dh == 32, "attention: head_dim %d unsupported (32, 64)", dh);
  const int64_t items = (int64_t)a.B * a.H * ((a.L + 15) / 16);
  MRAG_REQUIRE(items < (1ll << 33), "attention: batch too large");
  if (a.L > 32 && a.L <= 64) {  // one workgroup per (sequence, head): the ViT's 50 tokens
    hipLaunchKernelGGL(dh == 64 ? attention_seq64_kernel<64> : attention_seq64_kernel<32>,
                       dim3((unsigned)((int64_t)a.B * a.H)), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(dh == 64 ? attention_flash16_kernel<64> : attention_flash16_kernel<32>,
                       dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, a);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_vit_im2col(const uint8_t* img, _Float16* out, int B, int S, int P, hipStream_t s) {
  const int64_t total8 = (int64_t)B * (S / P) * (S / P) * (3 * P * P / 8);
  if (total8 == 0) return MRAG_OK;
  if (P == 32 && S % 16 == 0 && ((uintptr_t)img & 15) == 0) {
    const int64_t n = (int64_t)B * (S / P) * (S / P) * P;
    hipLaunchKernelGGL(vit_im2col32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, img, out, B, S);
    MRAG_CHECK_LAUNCH();
    return MRAG_OK;
  }
  hipLaunchKernelGGL(vit_im2col_kernel, dim3((unsigned)((total8 + 255) / 256)), dim3(256), 0, s, img, out, B, S, P);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_token_embed(const int32_t* ids, const float* tok, const float* pos, const float* type_tab,
                       const int32_t* types, float* X, int B, int T, int D, int vocab, hipStream_t s) {
  const int64_t n = (int64_t)B * T;
  if (n == 0 || D == 0) return MRAG_OK;
  MRAG_REQUIRE(D % 4 == 0 && n < (1ll << 31), "token_embed: D=%d must be a multiple of 4", D);
  hipLaunchKernelGGL(token_embed_kernel, dim3((unsigned)n), dim3(128), 0, s, ids, tok, pos, type_tab, types, X, B, T,
                     D, vocab);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

// Sequence-classification head (BertForSequenceClassification): logits[b][j] =
// sum_d tanh(pooled[b][d]) * Wc[j][d] + bc[j], pooled = the pooler dense output (f32, bias
// included). One wave per (row, label); f32 throughout.
__global__ __launch_bounds__(256) void cls_head_kernel(const float* __restrict__ pooled, const float* __restrict__ Wc,
                                                       const float* __restrict__ bc, float* __restrict__ out, int B,
                                                       int D, int NL) {
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wv >= B * NL) return;
  const int b = wv / NL, j = wv - (wv / NL) * NL;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64) acc = fmaf(tanhf(pooled[(size_t)b * D + d]), Wc[(size_t)j * D + d], acc);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) out[(size_t)b * NL + j] = acc + bc[j];
}

int launch_cls_head(const float* pooled, const float* Wc, const float* bc, float* out, int B, int D, int NL,
                    hipStream_t s) {
  if (B * NL == 0) return MRAG_OK;
  hipLaunchKernelGGL(cls_head_kernel, dim3((unsigned)((B * NL + 3) / 4)), dim3(256), 0, s, pooled, Wc, bc, out, B, D,
                     NL);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_eos_rows(const int32_t* ids, int B, int T, int eos_id, int* rows, hipStream_t s) {
  if (B == 0) return MRAG_OK;
  hipLaunchKernelGGL(eos_rows_kernel, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, s, ids, B, T, eos_id, rows);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

// dst[b] = src[rows[b]] for row_bytes-byte rows (row_bytes % 16 == 0): the pooled rows of a
// CLIP tower's last layer (cls / eos) gathered into a compact batch
__global__ __launch_bounds__(256) void gather_rows_kernel(const char* __restrict__ src, char* __restrict__ dst,
                                                           const int* __restrict__ rows, int B, int row_bytes) {
  const int chunks = row_bytes >> 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * chunks) return;
  const int b = (int)(i / chunks), c = (int)(i - (int64_t)b * chunks);
  ((f32x4*)(dst + (size_t)b * row_bytes))[c] = ((const f32x4*)(src + (size_t)rows[b] * row_bytes))[c];
}

int launch_gather_rows(const void* src, void* dst, const int* rows, int B, int row_bytes, hipStream_t s) {
  if (B <= 0) return MRAG_OK;
  MRAG_REQUIRE(row_bytes % 16 == 0, "gather_rows: row bytes %d not a multiple of 16", row_bytes);
  const int64_t n = (int64_t)B * (row_bytes / 16);
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const char*)src,
                     (char*)dst, rows, B, row_bytes);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_cls_rows(int B, int T, int* rows, hipStream_t s) {
  if (B == 0) return MRAG_OK;
  hipLaunchKernelGGL(cls_rows_kernel, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, s, B, T, rows);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_mean_pool(const float* X, const int32_t* mask, float* out, int B, int T, int D, hipStream_t s) {
  const int64_t n = (int64_t)B * D;
  if (n == 0) return MRAG_OK;
  hipLaunchKernelGGL(mean_pool_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, X, mask, out, B, T, D);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

}  // namespace mrag_enc
