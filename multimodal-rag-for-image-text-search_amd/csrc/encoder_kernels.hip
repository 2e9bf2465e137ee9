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
#include <map>
#include <mutex>

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
  // panel are fetched into ONE XCD's L2 instead of being dealt over tiles_n XCDs (speed only;
  // env MRAG_K3_REMAP=0 keeps the plain order for A/B timing)
  const int T = g.k3_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
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

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + 16 * j + 4 * fq;
    float bn[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bn[r] = g.bias ? g.bias[n + r] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * 64 + 16 * i + fr;
      if (m < g.M) gemm_store4<EPI>(g, m, n, acc[i][j], bn);
    }
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
constexpr int G8_THREADS = 512;
constexpr int G8_BUF = 65536;      // one K-tile: two A and two B half-tile slots
constexpr int G8_BIAS_MAX = 4096;  // bias floats staged in LDS

// Tile geometry. CFG 0: 256 x 256 tiles (waves of 128 x 64). CFG 1: 128 x 384 tiles (waves of
// 64 x 96) for N = 768 (out-proj, fc2 of ViT-B/32): 200 tiles instead of 150 on 256 CUs, one
// round of 3/4-size tiles. Same per-element accumulation order and epilogue in both.
template <int CFG>
struct G8Geom {
  static constexpr int BM = CFG == 0 ? 256 : 128, BN = CFG == 0 ? 256 : 384;
  static constexpr int WM = BM / 2, WN = BN / 4;  // wave tile (2 x 4 waves)
  static constexpr int HM = WM / 2, HN = WN / 2;  // one phase's quadrant
  static constexpr int NI = HM / 16, NJ = HN / 16;
  static constexpr int SA = BM / 2 * 128, SB = BN / 2 * 128;  // A / B half-tile slot bytes
  static constexpr int PA = BM / 128, PB = BN / 128;          // 1 KiB LDS-DMA pieces per wave per slot
  static constexpr int slot_off(int sl) { return sl == 0 ? 0 : sl == 1 ? SA : sl == 2 ? SA + SB : SA + 2 * SB; }
  static constexpr int pieces(int sl) { return (sl == 0 || sl == 3) ? PA : PB; }
  static_assert(2 * SA + 2 * SB == G8_BUF, "a K-tile is 64 KiB");
  static_assert(NJ == 2 || NJ == 3, "column permutation below");
};
// tile column (within a wave-column half) of B LDS row jj: lane group f of the 16 x 16 MFMA
// blocks owns consecutive columns — 8 for the block pair jb = 0, 1 (one 16-byte f16 store),
// 4 for a third block jb = 2 (one 8-byte store)
__device__ __forceinline__ int g8_colperm(int jj) {
  const int jb = jj >> 4, f = (jj >> 2) & 3, r = jj & 3;
  return jb < 2 ? 8 * f + 4 * jb + r : 32 + 4 * f + r;
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

// ABL (timing experiments only, wrong results): 1 = no LDS-DMA in the loop, 2 = no
// fragment ds_reads in the loop, 3 = both, 4 = no ping-pong stagger, 5 = LDS-DMA from the
// first two K-tiles only (L2-hot), 7 = no epilogue stores
//
// SK = 1: stream-K. The tiles of an XCD (the same contiguous range as above) are laid out as
// one sequence of K-tile iterations (tile-major) and cut into nbx equal contiguous ranges, one
// per workgroup of that XCD, so every CU gets the same number of MFMA K-steps however the tile
// count divides by 256 (ViT fc2 / out-proj: 150 tiles; fc1: 600). A range is a list of
// segments (tile, k-tiles [kb, ke)); even workgroups walk their range forward, odd ones
// backward, so the two pieces of a tile cut between workgroups s and s + 1 are computed at the
// same time (both at the start or both at the end of their ranges). A piece of a cut tile
// stores its raw accumulators to its slot (`sc1` 16-byte stores, each wave drains them, a
// barrier), one lane adds to the tile's arrival counter (agent-scope atomic), and the
// workgroup whose add comes last sums every piece IN K ORDER (p0 + p1 (+ p2), own piece from
// registers, the others by `sc1` loads), resets the counter and runs the normal epilogue:
// no workgroup ever waits for another (MI355X_MICROARCH.md, hand-off table row 1). The sum
// order depends only on the cut points, i.e. on (M, N, K, grid): a launch is deterministic,
// but a row's last bits can differ between batch sizes that cut differently (the launcher
// uses SK only from M >= 8192 rows, so smaller batches keep the one-accumulator order).
constexpr int SK_SLOT_BYTES = 256 * 256 * 4;  // one CFG-0 tile of f32 accumulators

template <int EPI, int ABL = 0, int CFG = 0, int SK = 0>
__global__ __launch_bounds__(G8_THREADS) void gemm_8p_kernel(GemmArgs g) {
  using GG = G8Geom<CFG>;
  constexpr int BM = GG::BM, BN = GG::BN, WM = GG::WM, WN = GG::WN, HM = GG::HM, HN = GG::HN;
  constexpr int NI = GG::NI, NJ = GG::NJ, PA = GG::PA, PB = GG::PB;
  static_assert(SK == 0 || (CFG == 0 && ABL == 0), "stream-K: 256 x 256 tiles only");
  constexpr int BIAS_BYTES = ABL == 8 ? 16 : G8_BIAS_MAX * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * G8_BUF + BIAS_BYTES + 16];
  float* sbias = (float*)(smem + 2 * G8_BUF);
  int* sflag = (int*)(smem + 2 * G8_BUF + BIAS_BYTES);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  // this workgroup's tiles: lo + s + k * nbx, k = 0 .. my_n - 1 (SK: see above)
  const int tiles_n = g.N / BN;
  const int ntiles = ((g.M + BM - 1) / BM) * tiles_n;
  const int xcd = blockIdx.x & 7, sidx = blockIdx.x >> 3;
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3;
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int cnt = q8 + (xcd < r8 ? 1 : 0);
  const int my_n = sidx < cnt ? (cnt - sidx + nbx - 1) / nbx : 0;
  const int ktiles = g.K / GK;
  const int64_t Ix = (int64_t)cnt * ktiles;  // SK: K-tile iterations of this XCD
  auto range_lo = [&](int s) { return (int64_t)s * Ix / nbx; };
  const int64_t it0 = SK ? range_lo(sidx) : 0, it1 = SK ? range_lo(sidx + 1) : 0;
  const int t_first = SK ? (int)(it0 / ktiles) : 0, t_last = SK ? (int)((it1 - 1) / ktiles) : 0;
  const bool fwd = (sidx & 1) == 0;
  const int nseg = SK ? (it1 > it0 ? t_last - t_first + 1 : 0) : my_n;
  if (nseg == 0) return;  // whole workgroup, before any barrier
  // segment i of this workgroup: tile T, k-tiles [kb, ke)
  auto seg = [&](int i, int& T, int& kb, int& ke) {
    if constexpr (SK) {
      const int t = fwd ? t_first + i : t_last - i;
      const int64_t base = (int64_t)t * ktiles;
      kb = (int)(it0 > base ? it0 - base : 0);
      ke = (int)(it1 - base < ktiles ? it1 - base : ktiles);
      T = lo + t;
    } else {
      T = lo + sidx + i * nbx;
      kb = 0;
      ke = ktiles;
    }
  };

  if constexpr (ABL != 8) {
    for (int i = threadIdx.x; i < g.N; i += G8_THREADS) sbias[i] = g.bias ? g.bias[i] : 0.f;
    __syncthreads();
  }

  const int KH = 4 * ktiles;                                // half-tiles per tile
  const int total = SK ? (int)(4 * (it1 - it0)) : my_n * KH;  // half-tiles of the whole stream

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
    const int k0 = (ABL == 5 ? (ld_kt & 1) : ld_kt) * GK;
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
        if constexpr (ABL == 2 || ABL == 3) asm volatile("" : "+v"(fa[i][kk]));
        else fa[i][kk] = *(const half8*)(slot + offA[i][kk]);
      }
  };
  auto readB = [&](const char* slot, half8 (&fb)[NJ][2]) {
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if constexpr (ABL == 2 || ABL == 3) asm volatile("" : "+v"(fb[jb][kk]));
        else fb[jb][kk] = *(const half8*)(slot + offB[jb][kk]);
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
    if (ABL != 1 && ABL != 3 && full) stage_slot(SL);
    const bool post = phi - st_phi <= 5;  // the last epilogue's stores are younger than L[phi + 2]
    if (__builtin_expect(full && !post, 1)) {
      vmcnt_wait(YSTEADY);
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
  // SK: the piece of local tile t held in `acc` (tile id T) is stored; returns true when this
  // workgroup's piece arrived last and `acc` now holds the whole tile's sum (see above)
  auto sk_piece = [&](int t, int T) -> bool {
    if (wr == 0) bar();  // group 0 waits for group 1's last phase: both groups aligned
    const __amdgpu_buffer_rsrc_t part = __builtin_amdgcn_make_buffer_rsrc(g.sk_part, 0, 0x7fffffff, 0x00020000);
    const uint32_t tid16 = threadIdx.x * 16;
    {
      const uint32_t base = (uint32_t)(2 * blockIdx.x + (t == t_first ? 0 : 1)) * SK_SLOT_BYTES + tid16;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int jb = 0; jb < NJ; ++jb) {
              const int r = ((h * 2 + hh) * NI + i) * NJ + jb;
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[h][hh][i][jb]), part,
                                                     base + r * (G8_THREADS * 16), 0, 16 /* sc1 */);
            }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's piece has left the CU
    bar();
    if (threadIdx.x == 0)
      *sflag = __hip_atomic_fetch_add(g.sk_cnt + T, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int arrived = *sflag;
    // the pieces of tile t: workgroups s_first .. s_last of this XCD, ascending s = ascending k
    const int64_t tb = (int64_t)t * ktiles;
    const int s_first = (int)(((tb + 1) * nbx - 1) / Ix), s_last = (int)(((tb + ktiles) * nbx - 1) / Ix);
    int np = 0;
    for (int s = s_first; s <= s_last; ++s) np += range_lo(s + 1) > range_lo(s) ? 1 : 0;
    if (arrived != np - 1) return false;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        f32x4 v[NI][NJ];
        bool first = true;
        for (int s = s_first; s <= s_last; ++s) {
          const int64_t a0 = range_lo(s), a1 = range_lo(s + 1);
          if (a1 <= a0) continue;
          if (s == sidx) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
              for (int jb = 0; jb < NJ; ++jb) v[i][jb] = first ? acc[h][hh][i][jb] : v[i][jb] + acc[h][hh][i][jb];
          } else {
            const uint32_t base =
                (uint32_t)(2 * (xcd + 8 * s) + (t == (int)(a0 / ktiles) ? 0 : 1)) * SK_SLOT_BYTES + tid16;
            f32x4 p[NI][NJ];
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
              for (int jb = 0; jb < NJ; ++jb) {
                const int r = ((h * 2 + hh) * NI + i) * NJ + jb;
                p[i][jb] = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(part, base + r * (G8_THREADS * 16), 0, 16 /* sc1 */));
              }
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
              for (int jb = 0; jb < NJ; ++jb) v[i][jb] = first ? p[i][jb] : v[i][jb] + p[i][jb];
          }
          first = false;
        }
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int jb = 0; jb < NJ; ++jb) acc[h][hh][i][jb] = v[i][jb];
      }
    if (threadIdx.x == 0) __hip_atomic_store(g.sk_cnt + T, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  };

  // waves 4..7 (one per SIMD beside a wave of 0..3) run one barrier behind waves 0..3
  if (ABL != 4 && wr == 1) bar();
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
    const bool split = SK && (kb != 0 || ke != ktiles);  // wave-uniform
    if (split && !sk_piece(T - lo, T)) {
      if (wr == 1) bar();  // restore the stagger (the workgroup's barrier counts stay equal)
      continue;
    }

    // epilogue: blocks (h, hh, i): row WM wr + HM h + 16 i + fr; columns WN wc + HN hh + 8 fq
    // + (0..7) from the block pair jb = 0, 1 (one 16-byte f16 store, two for f32) and, for
    // CFG 1, WN wc + HN hh + 32 + 4 fq + (0..3) from jb = 2 (one 8-byte f16 / 16-byte f32 store)
    const int tm = T / tiles_n;
    const int m0 = tm * BM, n0 = (T - tm * tiles_n) * BN;
    constexpr int SPB = ((EPI == EPI_F32_RESIDUAL || EPI == EPI_F32) ? 2 : 1) + (NJ == 3 ? 1 : 0);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int nb = n0 + WN * wc + HN * hh;
      const int n = nb + 8 * fq;
      float bn[8], bn4[4];
#pragma unroll
      for (int r = 0; r < 8; ++r) bn[r] = ABL == 8 ? 0.f : sbias[n + r];
      if constexpr (NJ == 3) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bn4[r] = ABL == 8 ? 0.f : sbias[nb + 32 + 4 * fq + r];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int mb = m0 + WM * wr + HM * h + 16 * i;  // wave-uniform block row
          const int m = mb + fr;
          if constexpr (ABL == 7) {
            asm volatile("" ::"v"(acc[h][hh][i][0]), "v"(acc[h][hh][i][1]), "v"(bn[0]));
          } else if (mb < g.M) {  // uniform branch: a block with a valid row issues exactly
            st_cnt += SPB;        // SPB vector stores (counted for the vmcnt bookkeeping)
            if (m < g.M) {
              gemm_store8<EPI>(g, m, n, acc[h][hh][i][0], acc[h][hh][i][1], bn);
              if constexpr (NJ == 3) gemm_store4<EPI>(g, m, nb + 32 + 4 * fq, acc[h][hh][i][NJ - 1], bn4);
            }
          }
        }
      }
    }
    if (split && wr == 1) bar();  // restore the stagger after a cut tile's epilogue
  }
  if (ABL != 4 && wr == 0) bar();  // same barrier count for both groups
}

// ---------------------------------------------------------------------------
// K3e (M >= 1024, N % 256 == 0, K % 64 == 0): persistent, one workgroup per CU, 256 x 256
// tiles, FOUR waves (2 x 2) of 128 x 128 — one wave per SIMD owning a quarter of the tile, so
// every fragment a wave reads from LDS feeds 8 MFMAs (K3d's 128 x 64 waves: 4 or 8) and the
// CU reads 128 KiB of fragments per 64 k instead of 192 KiB.
//  * accumulators: 8 x 8 blocks of 16 x 16 per wave = 256 f32 per lane, AGPR-resident (asm
//    MFMA operands);
//  * LDS: two 64-KiB K-tiles (A: 256 rows x 128 B, then B: 256 rows x 128 B), 16-byte chunk c
//    of row j at position c ^ ((j >> 1) & 7) (K3's conflict-free image). Rows of 128 B = 64 k
//    keep every LDS-DMA request a whole 128-byte line (rows of 64 B doubled the L2 requests:
//    notes/gemm_experiments.md);
//  * a K-tile is consumed in two 32-deep halves with one fragment set per half (R0, R1: 64
//    VGPRs each): half 0 of tile t runs on R0 while R1 is read from tile t; half 1 runs on R1
//    while R0 is read from tile t + 1. Tile t is fully read once half 0 ends, so the single
//    barrier per K-tile sits there: wait for K-tile t + 1 (own vmcnt), barrier, then the
//    LDS-DMA of K-tile t + 2 into tile t's buffer is spread over half 1's MFMAs. The load stream
//    runs across output tiles, so the epilogue overlaps the next tile's loads;
//  * waves 0, 1 stage the A half of every K-tile, waves 2, 3 the B half: 16 one-KiB pieces (8
//    rows of 128 B) per wave per K-tile through the SADDR form (lane part of the offset in a
//    VGPR, the piece's row offset and k in SGPRs);
//  * C^T blocks with the weight fragment as MFMA operand A and permuted weight rows, so a lane
//    stores 8 consecutive columns (gemm_store8) — the same per-element accumulation order
//    (32-deep chunks in ascending k, one accumulator) and epilogue as K3 / K3d, hence the same
//    bits whichever kernel a batch size selects.
constexpr int G4_THREADS = 256;
constexpr int G4_SLOT = 65536;  // one 64-deep K-tile: A 32 KiB + B 32 KiB

__device__ __forceinline__ void glds_x4_saddr(uint32_t voff, const void* sbase, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_addr)
      : "memory");
}

// weight LDS row j (0..127 within a wave column) -> its tile column: lane group f of block pair
// (2p, 2p + 1) owns the 8 consecutive columns 32 p + 8 f + 0..7. For j = 8 q + rr this splits
// into a piece part (uniform) and a lane part.
__device__ __forceinline__ constexpr int g4_colbase(int q) { return 32 * (q >> 2) + 16 * (q & 1) + 4 * ((q >> 1) & 1); }
__device__ __forceinline__ constexpr int g4_collane(int rr) { return 8 * (rr >> 2) + (rr & 3); }

template <int EPI>
__global__ __launch_bounds__(G4_THREADS) void gemm_4w_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * G4_SLOT + G8_BIAS_MAX * 4];
  float* sbias = (float*)(smem + 2 * G4_SLOT);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  // tiles: XCD x owns a contiguous range of tile ids (tm-major), round-robin over its workgroups
  const int tiles_n = g.N / 256;
  const int ntiles = ((g.M + 255) / 256) * tiles_n;
  const int xcd = blockIdx.x & 7, sidx = blockIdx.x >> 3;
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3;
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int cnt = q8 + (xcd < r8 ? 1 : 0);
  const int my_n = sidx < cnt ? (cnt - sidx + nbx - 1) / nbx : 0;
  if (my_n == 0) return;  // whole workgroup, before any barrier

  for (int i = threadIdx.x; i < g.N; i += G4_THREADS) sbias[i] = g.bias ? g.bias[i] : 0.f;

  const int ktiles = g.K / 64;
  const int total = my_n * ktiles;

  // loader: piece q (0..15) of this wave = LDS rows 8 (16 (w & 1) + q) + rr, rr = lane >> 3, of
  // the A half (waves 0, 1) or the B half (waves 2, 3); lane position lane & 7 holds source
  // chunk (lane & 7) ^ ((row >> 1) & 7) (row & 15 = 8 (q & 1) + rr)
  const bool loadsB = w >= 2;
  const int rr = lane >> 3;
  const uint32_t cb0 = (uint32_t)(((lane & 7) ^ (rr >> 1)) * 16);        // q even
  const uint32_t cb1 = (uint32_t)(((lane & 7) ^ (4 + (rr >> 1))) * 16);  // q odd
  const uint32_t ldb = (uint32_t)(loadsB ? g.ldw : g.lda) * 2u;          // row stride, bytes
  const uint32_t vlaneB = (uint32_t)g4_collane(rr) * ldb;
  const uint32_t lds_w = lds_base + (loadsB ? 32768u : 0u) + (uint32_t)(w & 1) * 16384u;
  int ld_kt = 0, ld_T = lo + sidx;
  int ld_m0 = 0, ld_n0 = 0;
  auto load_tile_origin = [&]() {
    const int tm = ld_T / tiles_n;
    ld_m0 = tm * 256;
    ld_n0 = (ld_T - tm * tiles_n) * 256;
  };
  load_tile_origin();
  // piece q of K-tile L[t]: A rows ld_m0 + 128 (w & 1) + 8 q + rr (clamped to M - 1), B rows
  // ld_n0 + 128 (w & 1) + g4_colbase(q) + g4_collane(rr)
  auto issue_piece = [&](int t, int q) {
    const uint32_t dst = lds_w + (uint32_t)(t & 1) * G4_SLOT + (uint32_t)q * 1024u;
    const uint32_t cb = (q & 1) ? cb1 : cb0;
    if (loadsB) {
      const char* sb = (const char*)(g.W + (size_t)(ld_n0 + 128 * (w & 1) + g4_colbase(q)) * g.ldw + ld_kt * 64);
      glds_x4_saddr(vlaneB + cb, sb, dst);
    } else {
      // rows past M re-read row M - 1: base row and lane row both clamped, so 0 <= row < M
      const int rbase = min(ld_m0 + 128 * (w & 1) + 8 * q, g.M - 1);
      const char* sb = (const char*)(g.A + (size_t)rbase * g.lda + ld_kt * 64);
      const uint32_t row = (uint32_t)min(rr, g.M - 1 - rbase);
      glds_x4_saddr(row * ldb + cb, sb, dst);
    }
  };
  auto advance_loader = [&]() {
    if (++ld_kt == ktiles) {
      ld_kt = 0;
      ld_T += nbx;
      if (ld_T < ntiles) load_tile_origin();
    }
  };

  // fragments: activation block i -> LDS A row 128 wr + 16 i + fr, weight block jb -> LDS B row
  // 128 wc + 16 jb + fr; half kk reads chunk 4 kk + fq; blocks 2 KiB apart
  int offA[2], offB[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    offA[kk] = swz_off(128 * wr + fr, 4 * kk + fq);
    offB[kk] = 32768 + swz_off(128 * wc + fr, 4 * kk + fq);
  }
  half8 fa[2][8], fb[2][8];  // [half][block]

  f32x4 acc[8][8];  // [activation block i][weight block jb], AGPR-resident (asm MFMA operand)
  constexpr int SPB = (EPI == EPI_F32_RESIDUAL || EPI == EPI_F32) ? 2 : 1;
  constexpr int ST_FULL = 32 * SPB;  // vector stores of a full tile's epilogue per wave
  constexpr int ST_WAIT = ST_FULL < 63 ? ST_FULL : 63;
  bool post = false;     // an epilogue ran since the last K-tile wait ...
  bool st_full = true;   // ... and issued ST_FULL stores (else fewer: partial tile)

  auto mfma_row = [&](int kk, int i) {
#pragma unroll
    for (int jb = 0; jb < 8; ++jb)
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[i][jb]) : "v"(fb[kk][jb]), "v"(fa[kk][i]));
  };

  // prologue: K-tiles 0, 1 in flight, K-tile 0 landed; R0 <- K-tile 0 half 0
#pragma unroll
  for (int q = 0; q < 16; ++q) issue_piece(0, q);
  advance_loader();
  if (total > 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) issue_piece(1, q);
    advance_loader();
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();  // also publishes sbias
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    fa[0][b] = *(const half8*)(smem + offA[0] + b * 2048);
    fb[0][b] = *(const half8*)(smem + offB[0] + b * 2048);
  }

  int t = 0;
  for (int tl = 0; tl < my_n; ++tl) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jb = 0; jb < 8; ++jb) acc[i][jb] = f32x4{};
    for (int kt = 0; kt < ktiles; ++kt, ++t) {
      const char* cur = (const char*)smem + (t & 1) * G4_SLOT;
      const char* nxt = (const char*)smem + ((t + 1) & 1) * G4_SLOT;
      // half 0 on R0; R1 <- this K-tile's half 1
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        mfma_row(0, i);
        fa[1][i] = *(const half8*)(cur + offA[1] + i * 2048);
        fb[1][i] = *(const half8*)(cur + offB[1] + i * 2048);
      }
      __builtin_amdgcn_s_setprio(0);
      // K-tile t + 1 landed (the only LDS-DMA in flight, plus the last epilogue's stores when
      // one ran since: they are younger; waiting for at most 63 outstanding is still enough);
      // every wave is done reading K-tile t
      if (__builtin_expect(!post, 1)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (st_full) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST_WAIT) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      post = false;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // half 1 on R1; R0 <- K-tile t + 1's half 0 (stale data past the stream's end, unused);
      // K-tile t + 2's LDS-DMA into this K-tile's buffer, two pieces per row block
      const bool more = t + 2 < total;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        mfma_row(1, i);
        fa[0][i] = *(const half8*)(nxt + offA[0] + i * 2048);
        fb[0][i] = *(const half8*)(nxt + offB[0] + i * 2048);
        if (more) {
          issue_piece(t + 2, 2 * i);
          issue_piece(t + 2, 2 * i + 1);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (more) advance_loader();
    }
    // the epilogue reads acc through VALU / accvgpr moves the hazard recognizer cannot relate to
    // the asm MFMAs: let the last ones retire first
    asm volatile("s_nop 15\n\ts_nop 3" ::: "memory");
    // epilogue: row m0 + 128 wr + 16 i + fr, columns n0 + 128 wc + 32 p + 8 fq + 0..7 from the
    // block pair (2p, 2p + 1)
    const int T = lo + sidx + tl * nbx;
    const int tm = T / tiles_n;
    const int m0 = tm * 256, n0 = (T - tm * tiles_n) * 256;
    post = true;
    st_full = m0 + 256 <= g.M;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = n0 + 128 * wc + 32 * p + 8 * fq;
      float bn[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) bn[r] = sbias[n + r];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + 128 * wr + 16 * i + fr;
        if (m < g.M) gemm_store8<EPI>(g, m, n, acc[i][2 * p], acc[i][2 * p + 1], bn);
      }
    }
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

// RPW rows per wave (consecutive): every row's loads and the gamma / beta chunks are issued
// before the first reduction, so a wave keeps RPW rows of loads in flight and a ViT / config-5
// LayerNorm fits the chip in one round of workgroups (RPW = 2: 12,800 rows -> 1,600
// workgroups) instead of 1.6 rounds with a tail. Per-row arithmetic is unchanged.
template <int RPW>
__global__ __launch_bounds__(256) void layernorm4_kernel(LayerNormArgs a) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (r0 >= a.rows) return;
  f32x4 v[RPW][4];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int r = r0 + rr < a.rows ? r0 + rr : r0;
    const int src = a.gather ? a.gather[r] : r;
    const f32x4* x = (const f32x4*)(a.x + (size_t)src * a.ldx);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[rr][j] = lane + 64 * j < (a.D >> 2) ? x[lane + 64 * j] : f32x4{};
  }
  f32x4 g4[4], b4[4];
  ln_params4(lane, a.D, a.gamma, a.beta, g4, b4);
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int r = r0 + rr;
    if (r < a.rows)
      ln_row4p(v[rr], lane, a.D, a.eps, g4, b4, a.y32 ? a.y32 + (size_t)r * a.D : nullptr,
               a.y16 ? a.y16 + (size_t)r * a.D : nullptr);
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
// K4: multi-head attention for sequences up to 512 (K and V of the head f32 in LDS:
// 2 L dh 4 bytes <= 160 KiB): one workgroup per (sequence, head), each thread takes query
// rows i, i + blockDim, ... with an online softmax over the keys (key padding mask,
// optional causal mask).
// qkv: [B*L][3*D] f16 (q | k | v, head h at columns h*DH), out: [B*L][D] f16.
template <int DH>
__global__ __launch_bounds__(256) void attention_kernel(AttentionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* Ks = sh;                       // [L][DH]
  float* Vs = sh + a.L * DH;            // [L][DH]
  int* valid = (int*)(sh + 2 * a.L * DH);  // [L]
  const int b = blockIdx.x / a.H, hd = blockIdx.x - (blockIdx.x / a.H) * a.H;
  const int D = a.H * DH;
  const size_t rs = (size_t)3 * D;
  const _Float16* base = a.qkv + (size_t)b * a.L * rs;
  for (int idx = threadIdx.x; idx < a.L * DH; idx += blockDim.x) {
    const int t = idx / DH, d = idx - (idx / DH) * DH;
    Ks[idx] = (float)base[t * rs + D + hd * DH + d];
    Vs[idx] = (float)base[t * rs + 2 * D + hd * DH + d];
  }
  for (int t = threadIdx.x; t < a.L; t += blockDim.x) valid[t] = a.mask ? (a.mask[b * a.L + t] != 0) : 1;
  __syncthreads();
  for (int i = threadIdx.x; i < a.L; i += blockDim.x) {
  float q[DH], o[DH];
  const _Float16* qr = base + i * rs + hd * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    q[d] = (float)qr[d] * a.scale;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const int jend = a.causal ? i + 1 : a.L;
  for (int j = 0; j < jend; ++j) {
    if (!valid[j]) continue;
    const float* kr = Ks + j * DH;
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) s = fmaf(q[d], kr[d], s);
    const float mn = fmaxf(m, s);
    const float alpha = __expf(m - mn);
    const float p = __expf(s - mn);
    l = l * alpha + p;
    const float* vr = Vs + j * DH;
#pragma unroll
    for (int d = 0; d < DH; ++d) o[d] = fmaf(p, vr[d], o[d] * alpha);
    m = mn;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  _Float16* orow = a.out + ((size_t)b * a.L + i) * D + hd * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) orow[d] = (_Float16)(o[d] * inv);
  }
}

// K4 (MFMA form) for L <= 64, head_dim 64 — the ViT-B/32 case (L = 50) and short text.
// One wave per (sequence, head), 4 heads per workgroup. Sequence padded to 64.
//   S^T = K . Q^T   (4 x 2x2 MFMA 32x32x16): lane owns query q = (l&31) + 32*qb, registers
//                   hold keys (reg&3) + 8(reg>>2) + 4(l>>5) + 32*kb, so the row softmax over
//                   keys is in-register plus one xor-32 shuffle (guide T12 "swapped QK^T").
//   O   = P . V     (4 x 2x2 MFMA): the P accumulator registers 8t..8t+7 of key block kb are
//                   the A fragment of k-step s = 2kb + t with the k order permuted
//                   (element j <-> key 16s + 8(j>>2) + 4(l>>5) + (j&3); guide §3
//                   "An accumulator tile as the next MFMA's operand"); V is gathered from
//                   LDS in that same order. P is normalised by its row sum before the cast.
__global__ __launch_bounds__(256) void attention_mfma64_kernel(AttentionArgs a) {
  constexpr int DH = 64;
  __shared__ __attribute__((aligned(16))) _Float16 Vs[4][64][DH];  // per-wave V tile (8 KiB)
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int hh = lane >> 5, r = lane & 31;
  const int pair = blockIdx.x * 4 + w;
  const bool active = pair < a.B * a.H;
  const int b = active ? pair / a.H : 0, hd = active ? pair - (pair / a.H) * a.H : 0;
  const int D = a.H * DH, L = a.L;
  const size_t rs = (size_t)3 * D;
  const _Float16* base = a.qkv + (size_t)b * L * rs;

  // V tile -> LDS (row per lane, zero rows >= L)
  {
    const int key = lane;
    half8* dst = (half8*)&Vs[w][key][0];
    if (active && key < L) {
      const half8* src = (const half8*)(base + (size_t)key * rs + 2 * D + hd * DH);
#pragma unroll
      for (int c = 0; c < 8; ++c) dst[c] = src[c];
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c) dst[c] = half8{};
    }
  }
  // K (A operand) and Q (B operand) fragments: row r + 32*blk, dims 16s + 8hh .. +7
  half8 kf[2][4], qf[2][4];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int row = r + 32 * blk;
    const bool ok = active && row < L;
    const _Float16* kr = base + (size_t)row * rs + D + hd * DH + 8 * hh;
    const _Float16* qr = base + (size_t)row * rs + hd * DH + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[blk][s] = ok ? *(const half8*)(kr + 16 * s) : half8{};
      qf[blk][s] = ok ? *(const half8*)(qr + 16 * s) : half8{};
    }
  }
  __syncthreads();
  if (!active) return;

  f32x16 st[2][2];  // [key block][query block]
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[kb][s], qf[qb][s], acc, 0, 0, 0);
      st[kb][qb] = acc;
    }

  // softmax over keys for the lane's two queries
  half8 pa[2][4];  // [query block][k-step]
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = r + 32 * qb;
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int key = (reg & 3) + 8 * (reg >> 2) + 4 * hh + 32 * kb;
        bool ok = key < L;
        if (a.mask) ok = ok && a.mask[(size_t)b * L + min(key, L - 1)] != 0;
        if (a.causal) ok = ok && key <= q;
        const float v = ok ? st[kb][qb][reg] * a.scale : -INFINITY;
        st[kb][qb][reg] = v;
        m = fmaxf(m, v);
      }
    m = fmaxf(m, __shfl_xor(m, 32));
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const float pv = m == -INFINITY ? 0.f : __expf(st[kb][qb][reg] - m);
        st[kb][qb][reg] = pv;
        l += pv;
      }
    l += __shfl_xor(l, 32);
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kb = s >> 1, t = s & 1;
      half8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (_Float16)(st[kb][qb][8 * t + j] * inv);
      pa[qb][s] = f;
    }
  }
  // V fragments in the permuted key order: element j <-> key 16s + 8(j>>2) + 4hh + (j&3)
  half8 vf[2][4];  // [dim block][k-step]
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = Vs[w][16 * s + 8 * (j >> 2) + 4 * hh + (j & 3)][r + 32 * db];
      vf[db][s] = f;
    }
  _Float16* orow = a.out + (size_t)b * L * D + hd * DH;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa[qb][s], vf[db][s], acc, 0, 0, 0);
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int q = (reg & 3) + 8 * (reg >> 2) + 4 * hh + 32 * qb;
        if (q < L) orow[(size_t)q * D + r + 32 * db] = (_Float16)acc[reg];
      }
    }
}

// K4 v2 (MFMA form, L <= 64, head_dim 64 or 32): as v1 up to the softmax, then
//   O^T = V^T . P^T: P^T is the S^T accumulator itself (registers 8t..8t+7 of key block kb
//                   are the B fragment of k-step 2kb + t, key order permuted: element j <->
//                   key 16s + 8(j>>2) + 4h + (j&3)); the V^T A fragments come from the row-major
//                   V image by ds_read_b64_tr_b16 in that same order (two per fragment, 16 in
//                   all; v1: 64 ds_read_u16).
//   The O^T block has the query on the lane and 4 consecutive dims per register group:
//   16 8-byte stores per lane (v1: 64 scattered 2-byte stores).
// No block barrier: each wave owns its V image, and a wave past the end returns whole (the
// transposed read needs EXEC all ones).
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4_lds __attribute__((__vector_size__(8)));

__device__ __forceinline__ half4_t lds_read_tr16(const _Float16* p) {
  const fp16x4_lds v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((AS3 fp16x4_lds*)(p));
  return __builtin_bit_cast(half4_t, v);
}

template <int DH>  // 64 (CLIP) or 32 (MiniLM)
__global__ __launch_bounds__(256) void attention_mfma64t_kernel(AttentionArgs a) {
  constexpr int KS = DH / 16;  // 16-dim k-steps of S^T = K . Q^T
  constexpr int DB = DH / 32;  // 32-dim output blocks of O^T
  constexpr int LPR = DH / 8;  // lanes per V row (16 B each)
  constexpr int VROW = 96;     // 192-byte rows: the 4 rows of one transposed read hit disjoint banks
  __shared__ __attribute__((aligned(16))) _Float16 Vs[4][64 * VROW];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int hh = lane >> 5, r = lane & 31;
  const int pair = blockIdx.x * 4 + w;
  if (pair >= a.B * a.H) return;
  const int b = pair / a.H, hd = pair - (pair / a.H) * a.H;
  const int D = a.H * DH, L = a.L;
  const size_t rs = (size_t)3 * D;
  const _Float16* base = a.qkv + (size_t)b * L * rs;
  _Float16* vs = Vs[w];

  // V rows -> LDS: 8 lanes x 16 B per row, 8 rows per instruction, zero rows >= L
#pragma unroll
  for (int it = 0; it < LPR; ++it) {  // LPR lanes x 16 B per row, 64 / LPR rows per instruction
    const int key = (64 / LPR) * it + lane / LPR, c = lane % LPR;
    half8 v = {};
    if (key < L) v = *(const half8*)(base + (size_t)key * rs + 2 * D + hd * DH + 8 * c);
    *(half8*)(vs + key * VROW + 8 * c) = v;
  }
  // K (A operand) and Q (B operand) fragments: row r + 32*blk, dims 16s + 8hh .. +7
  half8 kf[2][KS], qf[2][KS];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int row = r + 32 * blk;
    const bool ok = row < L;
    const _Float16* kr = base + (size_t)row * rs + D + hd * DH + 8 * hh;
    const _Float16* qr = base + (size_t)row * rs + hd * DH + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      kf[blk][s] = ok ? *(const half8*)(kr + 16 * s) : half8{};
      qf[blk][s] = ok ? *(const half8*)(qr + 16 * s) : half8{};
    }
  }
  f32x16 st[2][2];  // [key block][query block]
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[kb][s], qf[qb][s], acc, 0, 0, 0);
      st[kb][qb] = acc;
    }
  // softmax over keys for the lane's two queries (as v1); P^T fragments in permuted key order
  half8 pb[2][4];  // [query block][k-step]
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = r + 32 * qb;
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int key = (reg & 3) + 8 * (reg >> 2) + 4 * hh + 32 * kb;
        bool ok = key < L;
        if (a.mask) ok = ok && a.mask[(size_t)b * L + min(key, L - 1)] != 0;
        if (a.causal) ok = ok && key <= q;
        const float v = ok ? st[kb][qb][reg] * a.scale : -INFINITY;
        st[kb][qb][reg] = v;
        m = fmaxf(m, v);
      }
    m = fmaxf(m, __shfl_xor(m, 32));
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const float pv = m == -INFINITY ? 0.f : __expf(st[kb][qb][reg] - m);
        st[kb][qb][reg] = pv;
        l += pv;
      }
    l += __shfl_xor(l, 32);
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kb = s >> 1, t = s & 1;
      half8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (_Float16)(st[kb][qb][8 * t + j] * inv);
      pb[qb][s] = f;
    }
  }
  // V^T fragments: 16-lane group g reads rows (keys) r0 .. r0 + 3, columns (dims) c0 + 4p .. + 3
  // (lane 4q + p of the group supplies row q); lane i of the group receives dim c0 + i
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  half8 vf[DB][4];  // [dim block][k-step]
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const _Float16* pa = vs + (16 * s + 4 * hh + q4) * VROW + 32 * db + 16 * (g & 1) + 4 * p4;
      const half4_t lo = lds_read_tr16(pa), hi = lds_read_tr16(pa + 8 * VROW);
      vf[db][s] = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  _Float16* obase = a.out + (size_t)b * L * D + hd * DH;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = r + 32 * qb;
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[db][s], pb[qb][s], acc, 0, 0, 0);
      // lane: query q, dims 32 db + 8 g4 + 4 hh + (0..3)
      if (q < L) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const half4_t h = {(_Float16)acc[4 * g4], (_Float16)acc[4 * g4 + 1], (_Float16)acc[4 * g4 + 2],
                             (_Float16)acc[4 * g4 + 3]};
          *(half4_t*)(obase + (size_t)q * D + 32 * db + 8 * g4 + 4 * hh) = h;
        }
      }
    }
  }
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
template <int DH, int PF = 0>  // PF 0: a key block's operands at its top; 1: two blocks ahead (A/B)
__global__ __launch_bounds__(256) void attention_flash16_kernel(AttentionArgs a) {
  constexpr int KS = DH / 32;               // 32-dim k-steps of S^T
  constexpr int DB = DH / 16;               // 16-dim blocks of O^T
  constexpr int VROW = DH == 64 ? 96 : 48;  // LDS row stride (halves): a transposed read's 4 rows hit disjoint banks
  typedef _Float16 half4_v __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) _Float16 Vs[4][16 * VROW];
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
  // a key block's operands (K fragments, this lane's V chunks, its 4 keys' mask flags) are
  // loaded two blocks ahead, so the per-block chain is compute only after the first block's
  // load latency (it was K load -> MFMA -> V load -> LDS: two memory latencies per block)
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
  Blk cur, n1, n2;
  if (PF && nkb > 0) load_blk(0, n1);
  if (PF && nkb > 1) load_blk(1, n2);
  for (int kb = 0; kb < nkb; ++kb) {
    if constexpr (PF) {
      cur = n1;
      n1 = n2;
      if (kb + 2 < nkb) load_blk(kb + 2, n2);
    } else {
      load_blk(kb, cur);
    }
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
      *(half8*)(vs + key * VROW + 8 * ch) = cur.vv[t];
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
      const half4_t vt = lds_read_tr16(vs + (4 * g + (c >> 2)) * VROW + 16 * db + 4 * (c & 3));
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

// X[b*T + t] = (t == 0 ? cls : patch[b*(T-1) + t-1]) + pos[t]   (f32)
__global__ void vit_assemble_kernel(const float* __restrict__ patch, const float* __restrict__ cls,
                                    const float* __restrict__ pos, float* __restrict__ X, int B, int T, int D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * T * D) return;
  const int d = (int)(idx % D);
  const int64_t bt = idx / D;
  const int t = (int)(bt % T);
  const int64_t b = bt / T;
  const float e = t == 0 ? cls[d] : patch[(b * (T - 1) + t - 1) * D + d];
  X[idx] = e + pos[(size_t)t * D + d];
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
// env MRAG_GEMM_BIG (A/B timing): default -1 = K3d for M >= 1024 and N % 256 == 0, K3 otherwise;
// 0 = K3 only. MRAG_GEMM_ABL: K3d ablation builds (timing only, EPI_F16).
int gemm_big_mode() {
  static const int v = [] {
    const char* e = getenv("MRAG_GEMM_BIG");
    return e ? atoi(e) : -1;
  }();
  return v;
}

int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 256;
    return v;
  }();
  return n;
}

// K3d geometry: CFG 0 (256 x 256) unless env MRAG_G8_CFG=1 asks for CFG 1 (128 x 384) where
// N % 384 == 0. CFG 1 fills 200 instead of 150 CUs at N = 768 but measured no faster (fc2
// 97-99 us, out-proj 44 us either way; qkv 78 vs 59 us: notes/gemm_experiments.md), so the
// persistent 256 x 256 kernel stays the default; CFG 1 is kept for A/B timing and is covered by
// the parity tests (env-forced).
int g8_pick_cfg(const GemmArgs& g) {
  static const int force = [] {
    const char* e = getenv("MRAG_G8_CFG");
    return e ? atoi(e) : -1;
  }();
  if (force == 1 && g.N % 384 == 0) return 1;
  return g.N % 256 == 0 ? 0 : -1;
}

// K3 (128 x 128, two workgroups per CU) vs K3d (persistent 256 x 256, one per CU) by rounds:
// a K3 round (two tiles per CU) takes ~2/3 of a K3d round (one 4x larger tile) on the same K
// (measured at K = 512 / 2048, N = 512: 23.7 vs 35.4 us, 53.1 vs 75.5 us), so K3 wins where the
// 256 x 256 grid leaves CUs idle and the 128 x 128 one does not — the CLIP text tower at the
// config-5 batch (N = 512). Both kernels accumulate every element in the same order.
bool k3_beats_k3d(const GemmArgs& g) {
  if (g.N % 256 != 0) return true;
  const long cus = std::max(8, num_cus() / 8 * 8);
  const long t256 = (long)((g.M + 255) / 256) * (g.N / 256), t128 = (long)((g.M + 127) / 128) * (g.N / 128);
  const long r_d = (t256 + cus - 1) / cus, r_3 = (t128 + 2 * cus - 1) / (2 * cus);
  static const bool tie_k3 = [] {  // env MRAG_GEMM_TIE_K3=1: ties go to K3 (A/B timing)
    const char* e = getenv("MRAG_GEMM_TIE_K3");
    return e && atoi(e) == 1;
  }();
  return tie_k3 ? 2 * r_3 <= 3 * r_d : 2 * r_3 < 3 * r_d;  // K3 time ~ (2/3) r_3 < r_d; ties stay on K3d
}

// K3d stream-K (SK) policy: env MRAG_G8_SK = 0 (default) off, 1 where the estimate says it
// beats the data-parallel tile rounds, 2 wherever K3d runs (tests, A/B). Estimated in K-tile
// steps per CU: DP = ceil(tiles / CUs) * k-tiles; SK = tiles * k-tiles / CUs, +15 % and +2
// steps for the cut tiles' partial hand-off. Batches under 8192 rows keep the data-parallel
// order (a row computed alone and inside such a batch is bit-identical). Measured SLOWER on
// every ViT shape (fc2 106 -> 127 us, out-proj 46 -> 78, fc1 88 -> 109; CLIP 60.7k -> 46.8k
// img/s, one box): a cut 256 x 256 tile hands off 256 KiB of f32 partials each way, ~110 MB
// per out-proj launch against its 118 MB of operand fills (notes/gemm_experiments.md).
int g8_sk_mode() {
  static const int v = [] {
    const char* e = getenv("MRAG_G8_SK");
    return e ? atoi(e) : 0;
  }();
  return v;
}

bool g8_use_sk(const GemmArgs& g, int ntiles, int cus) {
  const int mode = g8_sk_mode();
  if (mode <= 0) return false;
  if (mode >= 2) return true;
  if (g.M < 8192) return false;
  const double kt = g.K / GK;
  const double dp = (double)((ntiles + cus - 1) / cus) * kt;
  const double sk = 1.15 * ntiles * kt / cus + 2.0;
  return sk < dp;
}

// Per-(device, stream) SK workspace: 2 partial slots per workgroup (grid <= CUs) and one
// arrival counter per tile, zeroed once (every launch leaves them zero). Launches on one
// stream are ordered, so they can share it; concurrent streams get their own.
struct SkWorkspace {
  float* part = nullptr;
  int* cnt = nullptr;
  int slots = 0, counters = 0;
};

int sk_workspace(hipStream_t s, int grid, int ntiles, GemmArgs& g) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, SkWorkspace> pool;
  int dev = 0;
  MRAG_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  SkWorkspace& w = pool[{dev, s}];
  if (w.slots < 2 * grid) {
    if (w.part) {
      MRAG_HIP(hipStreamSynchronize(s));
      MRAG_HIP(hipFree(w.part));
      w.part = nullptr;
      w.slots = 0;
    }
    MRAG_HIP(hipMalloc(&w.part, (size_t)2 * grid * SK_SLOT_BYTES));
    w.slots = 2 * grid;
  }
  if (w.counters < ntiles) {
    if (w.cnt) {
      MRAG_HIP(hipStreamSynchronize(s));
      MRAG_HIP(hipFree(w.cnt));
      w.cnt = nullptr;
      w.counters = 0;
    }
    const int n = std::max(ntiles, 4096);
    MRAG_HIP(hipMalloc(&w.cnt, (size_t)n * 4));
    MRAG_HIP(hipMemsetAsync(w.cnt, 0, (size_t)n * 4, s));
    w.counters = n;
  }
  g.sk_part = w.part;
  g.sk_cnt = w.cnt;
  return MRAG_OK;
}

template <int EPI>
int launch_gemm_8p_sk(const GemmArgs& g0, hipStream_t s) {
  const int ntiles = ((g0.M + 255) / 256) * (g0.N / 256);
  const int nb = std::max(8, num_cus() / 8 * 8);
  GemmArgs g = g0;
  if (int rc = sk_workspace(s, nb, ntiles, g)) return rc;
  static bool said = false;
  if (!said && getenv("MRAG_G8_VERBOSE")) {
    fprintf(stderr, "K3d stream-K: %d CUs, grid %d for %d tiles x %d k-tiles\n", num_cus(), nb, ntiles, g.K / GK);
    said = true;
  }
  hipLaunchKernelGGL((gemm_8p_kernel<EPI, 0, 0, 1>), dim3((unsigned)nb), dim3(G8_THREADS), 0, s, g);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

template <int CFG>
int launch_gemm_8p_cfg(const GemmArgs& g, int epi, hipStream_t s) {
  using GG = G8Geom<CFG>;
  const int ntiles = ((g.M + GG::BM - 1) / GG::BM) * (g.N / GG::BN);
  if (CFG == 0 && g8_use_sk(g, ntiles, std::max(8, num_cus() / 8 * 8))) {
    switch (epi) {
      case EPI_F16: return launch_gemm_8p_sk<EPI_F16>(g, s);
      case EPI_F16_QUICK_GELU: return launch_gemm_8p_sk<EPI_F16_QUICK_GELU>(g, s);
      case EPI_F16_GELU_ERF: return launch_gemm_8p_sk<EPI_F16_GELU_ERF>(g, s);
      case EPI_F32_RESIDUAL: return launch_gemm_8p_sk<EPI_F32_RESIDUAL>(g, s);
      case EPI_F32: return launch_gemm_8p_sk<EPI_F32>(g, s);
      default: return mrag::fail(MRAG_ERR_ARG, "gemm: bad epilogue %d", epi);
    }
  }
  int nb = std::min((ntiles + 7) / 8 * 8, std::max(8, num_cus() / 8 * 8));
  static const int grid_override = [] {
    const char* e = getenv("MRAG_G8_GRID");
    return e ? atoi(e) : 0;
  }();
  if (grid_override > 0) nb = std::min(nb, grid_override);
  static bool said = false;
  if (!said && getenv("MRAG_G8_VERBOSE")) {
    fprintf(stderr, "K3d cfg %d: %d CUs, grid %d for %d tiles\n", CFG, num_cus(), nb, ntiles);
    said = true;
  }
  const dim3 grid((unsigned)nb);
  static const int abl = [] {
    const char* e = getenv("MRAG_GEMM_ABL");
    return e ? atoi(e) : 0;
  }();
  if (CFG == 0 && abl != 0 && epi == EPI_F16) {
    switch (abl) {
      case 1: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 1>), grid, dim3(G8_THREADS), 0, s, g); break;
      case 2: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 2>), grid, dim3(G8_THREADS), 0, s, g); break;
      case 3: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 3>), grid, dim3(G8_THREADS), 0, s, g); break;
      case 5: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 5>), grid, dim3(G8_THREADS), 0, s, g); break;
      case 7: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 7>), grid, dim3(G8_THREADS), 0, s, g); break;
      case 8: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 8>), grid, dim3(G8_THREADS), 0, s, g); break;
      default: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 4>), grid, dim3(G8_THREADS), 0, s, g); break;
    }
    MRAG_CHECK_LAUNCH();
    return MRAG_OK;
  }
  switch (epi) {
    case EPI_F16: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16, 0, CFG>), grid, dim3(G8_THREADS), 0, s, g); break;
    case EPI_F16_QUICK_GELU:
      hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16_QUICK_GELU, 0, CFG>), grid, dim3(G8_THREADS), 0, s, g);
      break;
    case EPI_F16_GELU_ERF:
      hipLaunchKernelGGL((gemm_8p_kernel<EPI_F16_GELU_ERF, 0, CFG>), grid, dim3(G8_THREADS), 0, s, g);
      break;
    case EPI_F32_RESIDUAL:
      hipLaunchKernelGGL((gemm_8p_kernel<EPI_F32_RESIDUAL, 0, CFG>), grid, dim3(G8_THREADS), 0, s, g);
      break;
    case EPI_F32: hipLaunchKernelGGL((gemm_8p_kernel<EPI_F32, 0, CFG>), grid, dim3(G8_THREADS), 0, s, g); break;
    default: return mrag::fail(MRAG_ERR_ARG, "gemm: bad epilogue %d", epi);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

// K3e (4 waves of 128 x 128) instead of K3d where both apply: env MRAG_GEMM_4W=1 (A/B timing)
int gemm_4w_mode() {
  static const int v = [] {
    const char* e = getenv("MRAG_GEMM_4W");
    return e ? atoi(e) : 0;
  }();
  return v;
}

int launch_gemm_4w(const GemmArgs& g, int epi, hipStream_t s) {
  const int ntiles = ((g.M + 255) / 256) * (g.N / 256);
  const dim3 grid((unsigned)std::min((ntiles + 7) / 8 * 8, std::max(8, num_cus() / 8 * 8)));
  switch (epi) {
    case EPI_F16: hipLaunchKernelGGL(gemm_4w_kernel<EPI_F16>, grid, dim3(G4_THREADS), 0, s, g); break;
    case EPI_F16_QUICK_GELU: hipLaunchKernelGGL(gemm_4w_kernel<EPI_F16_QUICK_GELU>, grid, dim3(G4_THREADS), 0, s, g); break;
    case EPI_F16_GELU_ERF: hipLaunchKernelGGL(gemm_4w_kernel<EPI_F16_GELU_ERF>, grid, dim3(G4_THREADS), 0, s, g); break;
    case EPI_F32_RESIDUAL: hipLaunchKernelGGL(gemm_4w_kernel<EPI_F32_RESIDUAL>, grid, dim3(G4_THREADS), 0, s, g); break;
    case EPI_F32: hipLaunchKernelGGL(gemm_4w_kernel<EPI_F32>, grid, dim3(G4_THREADS), 0, s, g); break;
    default: return mrag::fail(MRAG_ERR_ARG, "gemm: bad epilogue %d", epi);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_gemm(const GemmArgs& g, int epi, hipStream_t s) {
  if (g.M <= 0) return MRAG_OK;
  MRAG_REQUIRE(g.N % GN == 0 && g.K % GK == 0, "gemm: N=%d must be a multiple of %d and K=%d of %d", g.N, GN, g.K,
               GK);
  MRAG_REQUIRE(g.lda % 8 == 0 && g.ldw % 8 == 0 && g.ldc % 4 == 0, "gemm: lda/ldw must be multiples of 8, ldc of 4");
  if (gemm_big_mode() != 0 && g.M >= 1024 && g.N <= G8_BIAS_MAX && !k3_beats_k3d(g)) {
    // K3e needs 32-bit byte offsets into A and W (SADDR LDS-DMA)
    if (gemm_4w_mode() == 1 && g.N % 256 == 0 && (long)g.M * g.lda * 2 < (1l << 31) &&
        (long)g.N * g.ldw * 2 < (1l << 31))
      return launch_gemm_4w(g, epi, s);
    const int cfg = g8_pick_cfg(g);
    if (cfg == 0) return launch_gemm_8p_cfg<0>(g, epi, s);
    if (cfg == 1) return launch_gemm_8p_cfg<1>(g, epi, s);
  }
  const dim3 grid((unsigned)(((g.M + GM - 1) / GM) * (g.N / GN)));
  static const int k3_remap = [] {
    const char* e = getenv("MRAG_K3_REMAP");
    return e ? atoi(e) : 1;
  }();
  GemmArgs g3 = g;
  g3.k3_remap = k3_remap;
  switch (epi) {
    case EPI_F16: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F16>, grid, dim3(GTHREADS), 0, s, g3); break;
    case EPI_F16_QUICK_GELU: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F16_QUICK_GELU>, grid, dim3(GTHREADS), 0, s, g3); break;
    case EPI_F16_GELU_ERF: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F16_GELU_ERF>, grid, dim3(GTHREADS), 0, s, g3); break;
    case EPI_F32_RESIDUAL: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F32_RESIDUAL>, grid, dim3(GTHREADS), 0, s, g3); break;
    case EPI_F32: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F32>, grid, dim3(GTHREADS), 0, s, g3); break;
    default: return mrag::fail(MRAG_ERR_ARG, "gemm: bad epilogue %d", epi);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_layernorm(const LayerNormArgs& a, hipStream_t s) {
  if (a.rows <= 0) return MRAG_OK;
  MRAG_REQUIRE(a.D > 0 && a.D <= 1024, "layernorm: D=%d unsupported", a.D);
  const bool vec4 = a.D % 4 == 0 && a.ldx % 4 == 0 && ((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.gamma & 15) == 0 &&
                    ((uintptr_t)a.beta & 15) == 0 && ((uintptr_t)a.y32 & 15) == 0 && ((uintptr_t)a.y16 & 7) == 0;
  static const int rpw = [] {  // env MRAG_LN_RPW = 2: two rows per wave (measured slower: 14.3 vs 12.3 us)
    const char* e = getenv("MRAG_LN_RPW");
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  if (vec4 && rpw == 2)
    hipLaunchKernelGGL(layernorm4_kernel<2>, dim3((unsigned)((a.rows + 7) / 8)), dim3(256), 0, s, a);
  else if (vec4)
    hipLaunchKernelGGL(layernorm4_kernel<1>, dim3((unsigned)((a.rows + 3) / 4)), dim3(256), 0, s, a);
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

// MRAG_ATTN_VALU=1 forces the VALU form everywhere (cross-check in tests).
bool force_valu_attention() {
  static const bool v = [] {
    const char* e = getenv("MRAG_ATTN_VALU");
    return e && atoi(e) == 1;
  }();
  return v;
}

bool mfma_attention_dh32() {
  static const bool v = [] {
    const char* e = getenv("MRAG_ATTN_DH32");
    return e && atoi(e) == 1;
  }();
  return v;
}

int launch_attention(const AttentionArgs& a, int dh, hipStream_t s) {
  if (a.B <= 0) return MRAG_OK;
  MRAG_REQUIRE(a.L >= 1 && a.L <= 512, "attention: L=%d unsupported (1..512)", a.L);
  const size_t shm = (size_t)2 * a.L * dh * 4 + (size_t)a.L * 4;
  MRAG_REQUIRE(shm <= 160 * 1024, "attention: L*dh too large for LDS");
  const int threads = std::min(256, (a.L + 63) / 64 * 64);
  const dim3 grid((unsigned)(a.B * a.H));
  // K/V of a head stay f32 in LDS; above 64 KiB the kernel must opt in (gfx950: 160 KiB/CU)
  static bool attr_set = false;
  if (!attr_set) {
    MRAG_HIP(hipFuncSetAttribute((const void*)attention_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024));
    MRAG_HIP(hipFuncSetAttribute((const void*)attention_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024));
    attr_set = true;
  }
  static const bool attn_v1 = [] {
    const char* e = getenv("MRAG_ATTN_V1");
    return e && atoi(e) == 1;
  }();
  static const bool legacy = [] {  // MRAG_ATTN_LEGACY=1: the round-1 dispatch (A/B timing)
    const char* e = getenv("MRAG_ATTN_LEGACY");
    return e && atoi(e) == 1;
  }();
  if ((dh == 64 || dh == 32) && !legacy && !force_valu_attention()) {
    const int64_t items = (int64_t)a.B * a.H * ((a.L + 15) / 16);
    MRAG_REQUIRE(items < (1ll << 33), "attention: batch too large");
    const dim3 g4((unsigned)((items + 3) / 4));
    // operands of a key block loaded together at its top (24.4 us per ViT layer vs 27.1 for the
    // round-1 K -> MFMA -> V chain); MRAG_ATTN_PREFETCH=1 loads them two blocks ahead instead,
    // which measured slower (27.0 us: 112 VGPRs halve the occupancy)
    static const bool no_prefetch = [] {
      const char* e = getenv("MRAG_ATTN_PREFETCH");
      return !(e && atoi(e) == 1);
    }();
    auto kern = dh == 64 ? (no_prefetch ? attention_flash16_kernel<64, 0> : attention_flash16_kernel<64, 1>)
                         : (no_prefetch ? attention_flash16_kernel<32, 0> : attention_flash16_kernel<32, 1>);
    hipLaunchKernelGGL(kern, g4, dim3(256), 0, s, a);
  } else if (dh == 64 && a.L <= 64 && !force_valu_attention() && !attn_v1) {
    hipLaunchKernelGGL(attention_mfma64t_kernel<64>, dim3((unsigned)((a.B * a.H + 3) / 4)), dim3(256), 0, s, a);
  } else if (dh == 32 && a.L <= 64 && mfma_attention_dh32()) {
    // opt-in (MRAG_ATTN_DH32=1): the BERT towers otherwise stay on the f32 VALU kernel for every
    // L, so a sequence's result does not depend on whether its batch pads past 64 tokens
    // (cross-encoder predict(pair) == predict(batch)[i] to 1e-6)
    hipLaunchKernelGGL(attention_mfma64t_kernel<32>, dim3((unsigned)((a.B * a.H + 3) / 4)), dim3(256), 0, s, a);
  } else if (dh == 64 && a.L <= 64 && !force_valu_attention()) {
    hipLaunchKernelGGL(attention_mfma64_kernel, dim3((unsigned)((a.B * a.H + 3) / 4)), dim3(256), 0, s, a);
  } else if (dh == 64) {
    hipLaunchKernelGGL(attention_kernel<64>, grid, dim3(threads), shm, s, a);
  } else if (dh == 32) {
    hipLaunchKernelGGL(attention_kernel<32>, grid, dim3(threads), shm, s, a);
  } else {
    return mrag::fail(MRAG_ERR_UNSUPPORTED, "attention: head_dim %d unsupported (32, 64)", dh);
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

int launch_vit_assemble(const float* patch, const float* cls, const float* pos, float* X, int B, int T, int D,
                        hipStream_t s) {
  const int64_t n = (int64_t)B * T * D;
  if (n == 0) return MRAG_OK;
  hipLaunchKernelGGL(vit_assemble_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, patch, cls, pos, X, B,
                     T, D);
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
