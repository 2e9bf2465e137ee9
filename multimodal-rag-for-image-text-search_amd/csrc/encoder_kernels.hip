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

// ---------------------------------------------------------------------------
// K3: C[m][n] (+)= act(sum_k A[m][k] W[n][k] + bias[n])   (the "NT" GEMM of nn.Linear)
// 128x128x64 block tile, 4 waves (2x2) of 64x64, MFMA 32x32x16 f16 -> f32.
// Operands staged to LDS by LDS-DMA, 128-byte rows with chunk c stored at position
// c ^ ((row >> 1) & 7) (source-address swizzle) so every ds_read_b128 fragment read is
// bank-conflict free; 2 stages, one barrier per 64-deep k-step.
template <int EPI>
__device__ __forceinline__ void gemm_store(const GemmArgs& g, int m, int n, float v) {
  const size_t o = (size_t)m * g.ldc + n;
  if constexpr (EPI == EPI_F16) {
    ((_Float16*)g.C)[o] = (_Float16)v;
  } else if constexpr (EPI == EPI_F16_QUICK_GELU) {
    // x * sigmoid(1.702 x) with hardware exp2 / rcp (~1 ulp each; the result is rounded
    // to fp16) instead of a full-precision divide
    v = v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.702f * 1.44269504088896341f * v));
    ((_Float16*)g.C)[o] = (_Float16)v;
  } else if constexpr (EPI == EPI_F16_GELU_ERF) {
    v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    ((_Float16*)g.C)[o] = (_Float16)v;
  } else if constexpr (EPI == EPI_F32_RESIDUAL) {
    ((float*)g.C)[o] += v;
  } else {
    ((float*)g.C)[o] = v;
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // blocks bid, bid+8, ... share an XCD; give each XCD a contiguous range of tile ids
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

constexpr int GM = 128, GN = 128, GK = 64;
constexpr int GTHREADS = 256;
constexpr int STAGE_BYTES = (GM + GN) * GK * 2;  // 32 KiB

template <int EPI>
__global__ __launch_bounds__(GTHREADS) void gemm_nt_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int h = lane >> 5, r32 = lane & 31;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  const int tiles_n = g.N / GN;
  // consecutive blocks walk N for a fixed M panel (the A panel stays L2-resident)
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - (blockIdx.x / tiles_n) * tiles_n;
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

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int sw = (r32 >> 1) & 7;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int ks = 0; ks < ksteps; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < ksteps) stage(cur ^ 1, (ks + 1) * GK);
    const char* At = (const char*)smem + cur * STAGE_BYTES;
    const char* Bt = At + GM * GK * 2;
    // read all 16 fragments of this 64-deep step first (64 VGPRs), then 16 MFMAs: the LDS
    // latency of later sub-steps hides under the earlier MFMAs
    half8 a[GK / 16][2], b[GK / 16][2];
#pragma unroll
    for (int kk = 0; kk < GK / 16; ++kk) {
      const int coff = (((2 * kk + h) ^ sw) * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i) a[kk][i] = *(const half8*)(At + (wr * 64 + i * 32 + r32) * 128 + coff);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[kk][j] = *(const half8*)(Bt + (wc * 64 + j * 32 + r32) * 128 + coff);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (hipcc would re-interleave them)
#pragma unroll
    for (int kk = 0; kk < GK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);  // MFMAs stay ahead of the stage wait + barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane owns column n of each 32x32 block and rows (reg&3)+8(reg>>2)+4h
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wc * 64 + j * 32 + r32;
    const float bn = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int m = m0 + wr * 64 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        // one epilogue for every GEMM kernel: a row's result must not depend on which
        // kernel the batch size selected
        if (m < g.M) gemm_store<EPI>(g, m, n, acc[i][j][reg] + bn);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K3b: the same GEMM for the big-M encoder batches (M >= 1024 rows: ViT at batch 256 is
// M = 12,800), 256 x BN block tile, 8 waves as 2 (M) x 4 (N) of 128 x BN/4, BK = 64.
// One workgroup per CU (128 KiB LDS at BN = 256): each A fragment read from LDS feeds
// BN/128 MFMAs and each B fragment four, half the LDS bytes per MFMA of K3.
// Pipeline per 64-deep k-step: the next k-step's tile is staged by LDS-DMA in pieces
// spread over the four 16-deep sub-steps (one job per MFMA cluster), the fragments of
// sub-step kk+1 are read while the MFMAs of kk run (two register sets), and one
// vmcnt(0) + barrier closes the k-step. Block ids are remapped so that the blocks of one
// A panel (same tm) run on the same XCD (bijective for any grid size).
constexpr int GB_BM = 256, GB_THREADS = 512;

template <int BN, int EPI, bool EARLY = true>
__global__ __launch_bounds__(GB_THREADS) void gemm_big_kernel(GemmArgs g) {
  constexpr int WN = BN / 4;                   // wave tile 128 x WN
  constexpr int TM = 4, TN = WN / 32;          // 32x32 blocks per wave
  constexpr int A_BYTES = GB_BM * GK * 2;      // 32 KiB
  constexpr int STAGE = (GB_BM + BN) * GK * 2;
  constexpr int PIECES = (GB_BM + BN) / 8;     // 1 KiB = 8 rows x 128 B
  constexpr int PPW = PIECES / 8;              // per wave per k-step
  static_assert(PIECES % 8 == 0 && PPW <= 8, "pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int h = lane >> 5, r32 = lane & 31;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  const int tiles_n = g.N / BN;
  const int nwg = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tm = t / tiles_n, tn = t - (t / tiles_n) * tiles_n;
  const int m0 = tm * GB_BM, n0 = tn * BN;
  const int ksteps = g.K / GK;

  // piece P of a stage: rows 8(P mod ...) .. +8 of A (P < 32) or of W; lane -> row rr, chunk pos
  auto stage_piece = [&](int buf, int k0, int i) {
    const int P = w * PPW + i;
    const int rr = lane >> 3, pos = lane & 7;
    const _Float16* src;
    int row;
    if (P < GB_BM / 8) {
      row = 8 * P + rr;
      const int c = pos ^ ((row >> 1) & 7);
      src = g.A + (size_t)min(m0 + row, g.M - 1) * g.lda + k0 + c * 8;
    } else {
      row = 8 * (P - GB_BM / 8) + rr;
      const int c = pos ^ ((row >> 1) & 7);
      src = g.W + (size_t)(n0 + row) * g.ldw + k0 + c * 8;
    }
    glds_x4(src, lds_base + buf * STAGE + P * 1024);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const int sw = (r32 >> 1) & 7;
  // fragment offsets (bytes within a stage): A row wr*128 + 32i + r32, B row wc*WN + 32j + r32
  const int offA = (wr * 128 + r32) * 128;
  const int offB = A_BYTES + (wc * WN + r32) * 128;
  half8 fa[2][TM], fb[2][TN];
  auto read_frags = [&](int set, int buf, int kk) {
    const char* st = (const char*)smem + buf * STAGE;
    const int coff = ((2 * kk + h) ^ sw) * 16;
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[set][i] = *(const half8*)(st + offA + i * 32 * 128 + coff);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[set][j] = *(const half8*)(st + offB + j * 32 * 128 + coff);
  };

#pragma unroll
  for (int i = 0; i < PPW; ++i) stage_piece(0, 0, i);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int ks = 0; ks < ksteps; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < ksteps;
    read_frags(0, cur, 0);
#pragma unroll
    for (int kk = 0; kk < GK / 16; ++kk) {
      const int set = kk & 1;
      if (kk + 1 < GK / 16) read_frags(set ^ 1, cur, kk + 1);
      // next k-step's pieces: all at the first sub-step (EARLY: a full k-step of latency
      // cover before the closing vmcnt(0)), or spread over the four sub-steps
      if constexpr (EARLY) {
        if (kk == 0) {
#pragma unroll
          for (int i = 0; i < PPW; ++i)
            if (more) stage_piece(cur ^ 1, (ks + 1) * GK, i);
        }
      } else {
#pragma unroll
        for (int i = kk * PPW / 4; i < (kk + 1) * PPW / 4; ++i)
          if (more) stage_piece(cur ^ 1, (ks + 1) * GK, i);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[set][i], fb[set][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane owns column n of each 32x32 block and rows (reg&3)+8(reg>>2)+4h
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wc * WN + j * 32 + r32;
    const float bn = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int m = m0 + wr * 128 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (m < g.M) gemm_store<EPI>(g, m, n, acc[i][j][reg] + bn);
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
__global__ void token_embed_kernel(const int32_t* __restrict__ ids, const float* __restrict__ tok,
                                   const float* __restrict__ pos, const float* __restrict__ type_tab,
                                   const int32_t* __restrict__ types, float* __restrict__ X, int B, int T, int D,
                                   int vocab) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * T * D) return;
  const int d = (int)(idx % D);
  const int64_t bt = idx / D;
  const int t = (int)(bt % T);
  int id = ids[bt];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  float e = tok[(size_t)id * D + d] + pos[(size_t)t * D + d];
  if (type_tab) e += type_tab[(types ? (types[bt] != 0) : 0) * D + d];  // BERT type_vocab_size 2
  X[idx] = e;
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
// env MRAG_GEMM_BIG (A/B timing): default -1 = K3b (BN 256 when N % 256 == 0, else 128) from
// M >= 1024; 0 = K3 only; 256 / 128 = K3b at that tile width; 2 = K3b with the LDS-DMA spread
int gemm_big_mode() {
  static const int v = [] {
    const char* e = getenv("MRAG_GEMM_BIG");
    return e ? atoi(e) : -1;
  }();
  return v;
}

template <int BN, bool EARLY>
int launch_gemm_big(const GemmArgs& g, int epi, hipStream_t s) {
  const dim3 grid((unsigned)(((g.M + GB_BM - 1) / GB_BM) * (g.N / BN)));
  switch (epi) {
    case EPI_F16: hipLaunchKernelGGL((gemm_big_kernel<BN, EPI_F16, EARLY>), grid, dim3(GB_THREADS), 0, s, g); break;
    case EPI_F16_QUICK_GELU: hipLaunchKernelGGL((gemm_big_kernel<BN, EPI_F16_QUICK_GELU, EARLY>), grid, dim3(GB_THREADS), 0, s, g); break;
    case EPI_F16_GELU_ERF: hipLaunchKernelGGL((gemm_big_kernel<BN, EPI_F16_GELU_ERF, EARLY>), grid, dim3(GB_THREADS), 0, s, g); break;
    case EPI_F32_RESIDUAL: hipLaunchKernelGGL((gemm_big_kernel<BN, EPI_F32_RESIDUAL, EARLY>), grid, dim3(GB_THREADS), 0, s, g); break;
    case EPI_F32: hipLaunchKernelGGL((gemm_big_kernel<BN, EPI_F32, EARLY>), grid, dim3(GB_THREADS), 0, s, g); break;
    default: return mrag::fail(MRAG_ERR_ARG, "gemm: bad epilogue %d", epi);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_gemm(const GemmArgs& g, int epi, hipStream_t s) {
  if (g.M <= 0) return MRAG_OK;
  MRAG_REQUIRE(g.N % GN == 0 && g.K % GK == 0, "gemm: N=%d must be a multiple of %d and K=%d of %d", g.N, GN, g.K,
               GK);
  MRAG_REQUIRE(g.lda % 8 == 0 && g.ldw % 8 == 0, "gemm: lda/ldw must be multiples of 8");
  const int big = gemm_big_mode();
  if (g.M >= 1024 && big != 0) {
    if (big == 2) return g.N % 256 == 0 ? launch_gemm_big<256, false>(g, epi, s) : launch_gemm_big<128, false>(g, epi, s);
    if ((big == -1 || big == 256) && g.N % 256 == 0) return launch_gemm_big<256, true>(g, epi, s);
    if (big != 256) return launch_gemm_big<128, true>(g, epi, s);  // N % 128 == 0 (checked above)
  }
  const dim3 grid((unsigned)(((g.M + GM - 1) / GM) * (g.N / GN)));
  switch (epi) {
    case EPI_F16: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F16>, grid, dim3(GTHREADS), 0, s, g); break;
    case EPI_F16_QUICK_GELU: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F16_QUICK_GELU>, grid, dim3(GTHREADS), 0, s, g); break;
    case EPI_F16_GELU_ERF: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F16_GELU_ERF>, grid, dim3(GTHREADS), 0, s, g); break;
    case EPI_F32_RESIDUAL: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F32_RESIDUAL>, grid, dim3(GTHREADS), 0, s, g); break;
    case EPI_F32: hipLaunchKernelGGL(gemm_nt_kernel<EPI_F32>, grid, dim3(GTHREADS), 0, s, g); break;
    default: return mrag::fail(MRAG_ERR_ARG, "gemm: bad epilogue %d", epi);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

int launch_layernorm(const LayerNormArgs& a, hipStream_t s) {
  if (a.rows <= 0) return MRAG_OK;
  MRAG_REQUIRE(a.D > 0 && a.D <= 1024, "layernorm: D=%d unsupported", a.D);
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)((a.rows + 3) / 4)), dim3(256), 0, s, a);
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
  if (dh == 64 && a.L <= 64 && !force_valu_attention()) {
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
  const int64_t n = (int64_t)B * T * D;
  if (n == 0) return MRAG_OK;
  hipLaunchKernelGGL(token_embed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ids, tok, pos, type_tab,
                     types, X, B, T, D, vocab);
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
