// knn.hip — K7/K8/K10/K11: exact flat cosine top-k over a device-resident corpus.
//
// Replaces the lancedb flat cosine scan behind app/storage/lancedb_store.py:103-123
// (`table.search(v).where("user_id == ...").metric("cosine").limit(max(k,1))`) and
// the per-row upsert at :87-101. Semantics are pinned in DESIGN.md §3:
//   score(q, x) = q.x / (|q| |x|) in f64 on the f32 vectors as given (0 on a zero
//   norm), label prefilter, order (score desc, row asc), at most k rows.
//
// Pipeline per search (all on one HIP stream):
//   prep   : queries f32 -> q32 (padded), |q| (f64), q16 = fp16(q/|q|)
//   K7 scan: MFMA fp16 Q.Dt over the fp16 scan copy of the corpus; every lane keeps
//            a running top-KL of the rows it sees; one list per (query, split)
//   K8     : per query, union of the split lists -> M best by approximate score ->
//            exact f64 rescoring against the f32 master rows -> certificate:
//            every row outside the candidate set has approx <= T, approx is within
//            EPS of exact, so if exact_k > T + EPS the top-k is proven exact
//   K7c    : (only for uncertified queries) threshold-collect scan: every row with
//            approx >= exact_k - EPS is collected — a superset of the true top-k
//   K10    : exact f64 rescoring of the collected rows + ordered selection
// The result is therefore exact for any data (ties and duplicates included), and
// the common case costs one fp16 MFMA pass plus a small gather.
//
// HBM layout per index (rows padded to DP = dim rounded up to 128):
//   x16    [cap][DP] fp16   normalised scan copy   (streamed by K7, 1 KiB rows at 512-d)
//   x32    [cap][DP] f32    master rows as given   (gathered by K8/K10 only)
//   xn     [cap]     f64    |x|
//   labels [cap]     int32  user label, MRAG_LABEL_DELETED for tombstones / padding
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <shared_mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "common.h"
#include "knn_generic.h"

#define AS1 __attribute__((address_space(1)))
#define AS3 __attribute__((address_space(3)))

namespace {

constexpr int TILE_ROWS = 64;
constexpr int SCAN_WAVES = 8;
constexpr int SCAN_THREADS = SCAN_WAVES * 64;
constexpr int QPW = 32;                     // queries per wave (MFMA 32x32 N dim)
constexpr int QPG = SCAN_WAVES * QPW;       // queries per workgroup
constexpr int MAX_MERGE_ENTRIES = 4096;     // splits * KL cap (LDS sort in K8)
constexpr int MAX_K = 256;
constexpr int MERGE_THREADS = 256;
#ifndef MRAG_SAMPLE_STRIDE
#define MRAG_SAMPLE_STRIDE 16
#endif
constexpr int SAMPLE_STRIDE = MRAG_SAMPLE_STRIDE;  // K7 sample pre-pass: every 16th tile of a split (A/B builds: -D)

// |approx - exact| bound for the fp16 scan:
//   fp16 rounding of both unit vectors: (2u + u^2) * sum|q_i x_i| <= 9.77e-4 (u = 2^-11)
//   f32 accumulation over <= 512 terms :  512 * 2^-24          <= 3.05e-5
//   fp16 subnormal flush, f32 normalise:                        <= 4e-6
constexpr double EPS_F16 = 1.05e-3;

struct ScanParams {
  const _Float16* x16;
  const int32_t* labels;
  const _Float16* q16;
  int ntiles, qgroups, splits, Qp, label_filter;
  // top-k mode
  float* part_s;
  int32_t* part_i;
  // collect mode
  const int32_t* fail_list;
  const int32_t* fail_cnt;
  const float* thresh;
  int32_t* cand_cnt;
  int32_t* cand;
  int ccap;
  // shared per-query rejection threshold (ordered-uint f32, 0 == none), top-k mode
  uint32_t* theta;
  // sample pre-pass (v3 MODE 1): tiles split + i * splits * sample_stride, i < sample_tiles
  int sample_tiles, sample_stride;
  // v3: requested k (publishing rule) and per-(split, query) bound on every dropped row
  int k;
  float* part_tau;
};

template <int KL>
__device__ __forceinline__ void list_insert(float (&ls)[KL], int (&li)[KL], float s, int r) {
  float cs = s;
  int cr = r;
#pragma unroll
  for (int j = 0; j < KL; ++j) {
    const bool sw = cs > ls[j];
    const float ts = ls[j];
    const int tr = li[j];
    ls[j] = sw ? cs : ts;
    li[j] = sw ? cr : tr;
    cs = sw ? ts : cs;
    cr = sw ? tr : cr;
  }
}

// The same insertion without the dependent chain: every position compares s with its own
// old entry (c_j = s > ls[j], monotone in j for a descending list) and takes s, its left
// neighbour or itself, all from the OLD list. Identical result to list_insert (s equal to an
// entry goes after it; s <= ls[KL-1] leaves the list unchanged); 3·KL - 2 independent selects
// per array instead of a KL-deep compare/swap chain (K7's group-test fire path).
template <int KL>
__device__ __forceinline__ void list_insert_par(float (&ls)[KL], int (&li)[KL], float s, int r) {
  bool c[KL];
#pragma unroll
  for (int j = 0; j < KL; ++j) c[j] = s > ls[j];
  float ns[KL];
  int ni[KL];
  ns[0] = c[0] ? s : ls[0];
  ni[0] = c[0] ? r : li[0];
#pragma unroll
  for (int j = 1; j < KL; ++j) {
    ns[j] = c[j] ? (c[j - 1] ? ls[j - 1] : s) : ls[j];
    ni[j] = c[j] ? (c[j - 1] ? li[j - 1] : r) : li[j];
  }
#pragma unroll
  for (int j = 0; j < KL; ++j) {
    ls[j] = ns[j];
    li[j] = ni[j];
  }
}

// LDS-DMA through inline asm: hipcc cannot prove that ds_reads of the current tile
// do not alias the in-flight DMA into the other buffer and would otherwise put an
// `s_waitcnt vmcnt(0)` right behind every builtin global_load_lds (serialising load
// and compute). Completion is enforced by hand: `s_waitcnt vmcnt(0)` + barrier at
// the end of every tile, before the buffer is read.
__device__ __forceinline__ void glds_x4(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}
// SADDR form: wave-uniform 64-bit base in SGPRs + per-lane 32-bit offset (no 64-bit VALU)
__device__ __forceinline__ void glds_x4_saddr(uint32_t voff, const void* sbase, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_addr)
      : "memory");
}
__device__ __forceinline__ void glds_x1(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

__device__ __forceinline__ float max16(const f32x16& a) {
  float m0 = fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3]));
  float m1 = fmaxf(fmaxf(a[4], a[5]), fmaxf(a[6], a[7]));
  float m2 = fmaxf(fmaxf(a[8], a[9]), fmaxf(a[10], a[11]));
  float m3 = fmaxf(fmaxf(a[12], a[13]), fmaxf(a[14], a[15]));
  return fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
}

// Row validity of accumulator register `reg` of block `blk` for this lane: bit
// (blk*32 + 8*(reg>>2) + (reg&3)) of the lane-shifted tile mask.
__device__ __forceinline__ bool row_ok(uint64_t lane_mask, int blk, int reg) {
  return (lane_mask >> (blk * 32 + 8 * (reg >> 2) + (reg & 3))) & 1ull;
}

__device__ __forceinline__ float masked_max16(const f32x16& a, uint64_t lane_mask, int blk) {
  float m = -INFINITY;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) m = fmaxf(m, row_ok(lane_mask, blk, reg) ? a[reg] : -INFINITY);
  return m;
}

// K7 / K7c. One workgroup = 8 waves = 256 queries x one split of the corpus tiles
// (tiles split, split+S, split+2S, ...). Corpus tiles (64 rows) are double-buffered in
// LDS by LDS-DMA (16 B/lane, rows XOR-swizzled on the source address so the
// A-fragment ds_read_b128 is conflict-free); each wave keeps its 32 queries' B
// fragments (all of DP) in VGPRs for the whole launch. MFMA 32x32x16 f16 with the
// corpus rows as A (M) and the queries as B (N): lane l owns query l&31 and rows
// (r&3) + 8(r>>2) + 4(l>>5) of each 32-row block.
//
// Epilogue (top-k mode): the common case is branch-free — a per-tile row-validity
// mask from one ballot over the tile's labels, the max of each lane's 32 scores,
// and ONE wave-level test against the lane's rejection threshold; the per-row list
// insertion runs only when some lane of the wave has a score above its threshold.
template <int DP, int KL, bool COLLECT>
__global__ __launch_bounds__(SCAN_THREADS) void knn_scan_kernel(ScanParams p) {
  constexpr int KSTEPS = DP / 16;
  constexpr int ROW_BYTES = DP * 2;
  constexpr int TILE_BYTES = TILE_ROWS * ROW_BYTES;
  constexpr int CPR = DP / 8;  // 16-byte chunks per row
  constexpr int GLDS_PER_WAVE = TILE_BYTES / 1024 / SCAN_WAVES;
  static_assert(TILE_BYTES % (1024 * SCAN_WAVES) == 0, "tile must split into 1 KiB pieces");
  static_assert(CPR % 16 == 0, "swizzle needs rows of a multiple of 16 chunks");
  constexpr int LBL_OFF = 2 * TILE_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES + 2 * TILE_ROWS * 4];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const int r32 = lane & 31;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  // block -> (query group, split). Blocks b, b+8, b+16, ... share an XCD (observed
  // round-robin dispatch; speed only): the query groups of one split are placed in
  // that stride so a corpus tile is fetched from HBM once per XCD and hits L2 after.
  int qg, split;
  {
    const int b = blockIdx.x;
    if ((p.splits & 7) == 0) {
      const int xcd = b & 7, slot = b >> 3;
      qg = slot % p.qgroups;
      split = (slot / p.qgroups) * 8 + xcd;
    } else {
      qg = b % p.qgroups;
      split = b / p.qgroups;
    }
  }

  int nslots = p.Qp;
  if constexpr (COLLECT) {
    nslots = *p.fail_cnt;
    if (qg * QPG >= nslots) return;  // uniform: no uncertified queries in this group
  }
  const int slot = qg * QPG + w * QPW + r32;  // query slot of this lane
  const bool wave_active = (qg * QPG + w * QPW) < nslots;
  const bool lane_active = slot < nslots;
  int qrow = slot;
  if constexpr (COLLECT) qrow = lane_active ? p.fail_list[slot] : 0;

  half8 qf[KSTEPS];
  if (wave_active) {
    const _Float16* qr = p.q16 + (size_t)(lane_active ? qrow : 0) * DP + h * 8;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) qf[kk] = *(const half8*)(qr + kk * 16);
    // Retire the fragment loads here, visibly to the compiler: otherwise its waitcnt
    // scoreboard carries them into the tile loop as `vmcnt(31..0)` waits between the
    // MFMAs, the last of which drains the next tile's LDS-DMA prefetch.
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) asm volatile("" ::"v"(qf[kk]));
  }
  float thr_collect = INFINITY;
  if constexpr (COLLECT) {
    if (lane_active) thr_collect = p.thresh[qrow];
  }

  float ls[KL];
  int li[KL];
#pragma unroll
  for (int j = 0; j < KL; ++j) {
    ls[j] = -INFINITY;
    li[j] = -1;
  }

  const int my_tiles = (split < p.ntiles) ? (p.ntiles - 1 - split) / p.splits + 1 : 0;

  // Shared rejection threshold (top-k mode). Every list publishes its KL-th score
  // (once full) with an agent-scope atomic max; every lane rejects rows scoring <=
  // the published maximum. Any value ever published is the KL-th of a full list
  // whose final KL-th can only be larger, so rows rejected this way score <= tau in
  // K8's certificate and exactness is unaffected; staleness only costs speed. The
  // value is re-read (sc1, L1 bypass) once per tile and used one tile later, after
  // the barrier has retired the load, so it never drains the LDS-DMA prefetch.
  float theta_f = -INFINITY;
  uint32_t theta_next = 0;
  float published = -INFINITY;
  uint32_t* theta_q = nullptr;
  if constexpr (!COLLECT) theta_q = p.theta + (lane_active ? slot : 0);

  // per-lane LDS offsets of the 8 distinct (kk mod 8) A-fragment chunks
  int offA[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) offA[j] = r32 * ROW_BYTES + (((2 * j + h) ^ (r32 & 15)) * 16);

  auto stage = [&](int buf, int tile) {
    const char* gt = (const char*)p.x16 + (size_t)tile * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < GLDS_PER_WAVE; ++i) {
      const int piece = w * GLDS_PER_WAVE + i;
      const int P = piece * 64 + lane;
      const int row = P / CPR;
      const int pos = P - row * CPR;
      const int c = pos ^ (row & 15);
      glds_x4(gt + row * ROW_BYTES + c * 16, lds_base + buf * TILE_BYTES + piece * 1024);
    }
    if (w == 0) glds_x1(p.labels + (size_t)tile * TILE_ROWS + lane, lds_base + LBL_OFF + buf * TILE_ROWS * 4);
  };

  // Slow path: per-row insertion / collection for one 32-row block.
  auto rows_pass = [&](const f32x16& acc, uint64_t lane_mask, int blk, int tile) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const float s = row_ok(lane_mask, blk, reg) ? acc[reg] : -INFINITY;
      const int row = tile * TILE_ROWS + blk * 32 + 8 * (reg >> 2) + 4 * h + (reg & 3);
      if constexpr (COLLECT) {
        // row_ok explicitly: masked rows carry -inf, which a -inf threshold (fewer than
        // k candidates in K8) would otherwise accept — padding and other users' rows
        if (row_ok(lane_mask, blk, reg) && s >= thr_collect) {
          const int pos = atomicAdd(p.cand_cnt + slot, 1);
          if (pos < p.ccap) p.cand[(size_t)slot * p.ccap + pos] = row;
        }
      } else {
        if (s > fmaxf(ls[KL - 1], theta_f)) list_insert<KL>(ls, li, s, row);
      }
    }
  };

  if (my_tiles > 0) {
    stage(0, split);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int it = 0; it < my_tiles; ++it) {
      const int cur = it & 1;
      const int tile = split + it * p.splits;
      if constexpr (!COLLECT) {
        if (theta_next != 0) theta_f = fmaxf(theta_f, mrag_ord2f(theta_next));
        if (wave_active) theta_next = __hip_atomic_load(theta_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (it + 1 < my_tiles) stage(cur ^ 1, tile + p.splits);

      // row validity of this tile: one label per lane -> 64-bit ballot (uniform)
      const int lab = ((const int*)(smem + LBL_OFF + cur * TILE_ROWS * 4))[lane];
      const bool lab_ok = (p.label_filter == MRAG_LABEL_ANY) ? (lab >= 0) : (lab == p.label_filter);
      const uint64_t tile_mask = __ballot(lab_ok);
      const uint64_t lane_mask = tile_mask >> (4 * h);

      if (wave_active && tile_mask != 0) {
        const char* tb = smem + cur * TILE_BYTES;
        f32x16 acc0 = {}, acc1 = {};
#pragma unroll
        for (int kk = 0; kk < KSTEPS; ++kk) {
          const int o = offA[kk & 7] + (kk >> 3) * 256;
          const half8 a0 = *(const half8*)(tb + o);
          const half8 a1 = *(const half8*)(tb + o + 32 * ROW_BYTES);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, qf[kk], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, qf[kk], acc1, 0, 0, 0);
        }
        {
          float m;
          if (tile_mask == ~0ull) {
            m = fmaxf(max16(acc0), max16(acc1));
          } else {
            m = fmaxf(masked_max16(acc0, lane_mask, 0), masked_max16(acc1, lane_mask, 1));
          }
          float thr;
          if constexpr (COLLECT) {
            thr = thr_collect;
            if (__any(m >= thr)) {
              rows_pass(acc0, lane_mask, 0, tile);
              rows_pass(acc1, lane_mask, 1, tile);
            }
          } else {
            thr = fmaxf(ls[KL - 1], theta_f);
            if (__any(m > thr)) {
              rows_pass(acc0, lane_mask, 0, tile);
              rows_pass(acc1, lane_mask, 1, tile);
              if (li[KL - 1] >= 0 && ls[KL - 1] > published) {
                published = ls[KL - 1];
                __hip_atomic_fetch_max(theta_q, mrag_f2ord(published), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
              }
            }
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  if constexpr (!COLLECT) {
    // fold the partner half-wave's list (same query, other rows) into lanes 0..31
    float ps[KL];
    int pi[KL];
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      ps[j] = __shfl_xor(ls[j], 32);
      pi[j] = __shfl_xor(li[j], 32);
    }
    if (h == 0 && lane_active) {
#pragma unroll
      for (int j = 0; j < KL; ++j)
        if (ps[j] > ls[KL - 1]) list_insert<KL>(ls, li, ps[j], pi[j]);
      float* os = p.part_s + ((size_t)split * p.Qp + slot) * KL;
      int32_t* oi = p.part_i + ((size_t)split * p.Qp + slot) * KL;
#pragma unroll
      for (int j = 0; j < KL; ++j) {
        os[j] = ls[j];
        oi[j] = li[j];
      }
    }
  }
}

constexpr int SCAN2_WAVES = 4;
constexpr int SCAN2_THREADS = SCAN2_WAVES * 64;
constexpr int QPW2 = 64;  // two 32-query blocks per wave
static_assert(SCAN2_WAVES * QPW2 == QPG, "v3 keeps the query-group size of v1");

using mrag::static_for;
// ---------------------------------------------------------------------------
// K7 v3 (top-k mode): v2's pipeline on MFMA 16x16x32. At equal cycles per FLOP the chip holds
// a higher clock on the 16x16x32 shape than on 32x32x16 with operands re-read from LDS
// (MI355X_MICROARCH.md, DVFS give-back item 7: 1.12-1.14x FLOP/s).
//  * one workgroup = 4 waves (one per SIMD) = 256 queries x one split; a wave owns 64 queries
//    as four 16-query blocks qb whose B fragments (all of DP) stay in AGPRs;
//  * a 64-row tile is four 16-row blocks rb: per 32-dim k-step the wave issues 16 MFMAs; the
//    A fragment of block rb (ds_read_b128, conflict-free under the row swizzle) is re-read for
//    the next k-step in the gap right after its last MFMA (one register set, 16 VGPRs); one
//    LDS-DMA piece of the next tile per k-step;
//  * C block (rb, qb): lane l holds query 16 qb + (l & 15), rows 16 rb + 4 (l >> 4) + r. Each
//    lane keeps a list of KL3 = 6 per query (8 spills at 256 VGPRs); the four lanes of a query
//    fold into the v2 output layout (8 per (split, query)) at the end, and part_tau records
//    max(6th of every full lane list, 8th of the folded list): every row of the split that is not in the folded list
//    scores <= that by approximation, so K8's certificate stays exact;
//  * double-buffered accumulators: the 16 group tests of tile t-1 (one (qb, rb) block: max of
//    4, one wave-uniform branch) run in the MFMA gaps of tile t;
//  * the shared threshold is the sample pre-pass seed (MODE 1: maxima only); a lane list
//    publishes its 6th score only when k <= 6 (a 6th is then a valid bound on the k-th).
constexpr int KL3 = 6;

__device__ __forceinline__ void mfma16_ab(f32x4& acc, const half8& a, const half8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}
__device__ __forceinline__ void mfma16_ab0(f32x4& acc, const half8& a, const half8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
}
// MFMA -> VALU distance for the accumulators of one tile (covers the 8-pass worst case)
__device__ __forceinline__ void mfma16_guard(f32x4 (&acc)[4][4]) {
  asm volatile("s_nop 15\n\ts_nop 3"
               : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[0][2]), "+v"(acc[0][3]), "+v"(acc[1][0]),
                 "+v"(acc[1][1]), "+v"(acc[1][2]), "+v"(acc[1][3]), "+v"(acc[2][0]), "+v"(acc[2][1]),
                 "+v"(acc[2][2]), "+v"(acc[2][3]), "+v"(acc[3][0]), "+v"(acc[3][1]), "+v"(acc[3][2]),
                 "+v"(acc[3][3]));
}
__device__ __forceinline__ void mfma16_guard(f32x4 (&acc)[4][1]) {
  asm volatile("s_nop 15\n\ts_nop 3" : "+v"(acc[0][0]), "+v"(acc[1][0]), "+v"(acc[2][0]), "+v"(acc[3][0]));
}

// The next tile's LDS-DMA pieces go out FRONT = 4 per k-step, all in the first quarter of the
// tile, so the last piece has three quarters of the tile to land before the end-of-tile
// vmcnt(0) + barrier (1 or 2 per k-step measured slower: notes/knn_scan_experiments.md).
//
// MODE 1 = the sample pre-pass: the same MFMA pipeline over a strided 1/sample_stride of each
// split's tiles, keeping only each lane's running max per lane group (no lists, no inserts); the
// per-(split, query, lane group) maxima go to part_s for theta_init_kernel, which seeds the
// shared threshold with the k-th largest of them.
//
// QB = query blocks of 16 per wave: 4 (a workgroup holds 256 queries; the MFMA-bound batches)
// or 1 (64 queries: the small batches of the reference's own call pattern, one query per
// retrieve_text / retrieve_images, app/ml/retrieve.py:53,84). With one block a tile costs a
// quarter of the MFMAs, so the scan streams the corpus at the fill / HBM rate instead of
// padding a single query to 256 (K7s). Lists, thresholds, part_tau and outputs are the same.
//
// MFMA -> VALU distance: the masking below reads this tile's accumulators right after their
// MFMAs, so it alone pays the s_nop guard; the group tests read them a tile later, at least the
// rest of that k-step's MFMAs after the last write (r3 A/B: an unconditional guard cost 1%).
#ifdef MRAG_K7_STAMPS
// Diagnostic build only (make stamp -> lib/libmrag_k7stamp.so): per wave, summed shader-clock
// spans of each tile's segments, [wave][K7_NSTAMP]; no other code reads them.
constexpr int K7_NSTAMP = 8, K7_MAXWAVES = 1 << 16;
__device__ unsigned long long g_k7_stamps[K7_MAXWAVES * K7_NSTAMP];
#define K7_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define K7_STAMP(v)
#endif

template <int DP, int MODE = 0, int QB = 4>
__global__ __launch_bounds__(SCAN2_THREADS) void knn_scan3_kernel(ScanParams p) {
  constexpr int KSTEPS = DP / 32;
  constexpr int ROW_BYTES = DP * 2;
  constexpr int TILE_BYTES = TILE_ROWS * ROW_BYTES;
  constexpr int CPR = DP / 8;
  constexpr int GLDS_PER_WAVE = TILE_BYTES / 1024 / SCAN2_WAVES;
  static_assert(GLDS_PER_WAVE == KSTEPS, "one LDS-DMA piece per k-step");
  static_assert(CPR % 16 == 0, "swizzle needs rows of a multiple of 16 chunks");
  constexpr int FRONT = 4;
  constexpr int NGROUPS = 4 * QB;  // group g: query block g >> 2, row block g & 3
  constexpr int QPW3 = 16 * QB, QPG3 = SCAN2_WAVES * QPW3;  // queries per wave / workgroup
  constexpr int LBL_OFF = 2 * TILE_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES + 2 * TILE_ROWS * 4];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g4 = lane >> 4;
  const int c16 = lane & 15;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((AS3 char*)smem));

  int qg, split;  // same XCD-aware block mapping as v1 / v2
  {
    const int b = blockIdx.x;
    if ((p.splits & 7) == 0) {
      const int xcd = b & 7, sl = b >> 3;
      qg = sl % p.qgroups;
      split = (sl / p.qgroups) * 8 + xcd;
    } else {
      qg = b % p.qgroups;
      split = b / p.qgroups;
    }
  }
  // query slot of block qb is slot0 + 16 qb; Qp is a multiple of QPG3 so every slot exists
  const int slot0 = qg * QPG3 + w * QPW3 + c16;

  half8 qf[KSTEPS][QB];
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk)
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
      qf[kk][qb] = *(const half8*)(p.q16 + (size_t)(slot0 + 16 * qb) * DP + kk * 32 + g4 * 8);
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk)
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) asm volatile("" ::"a"(qf[kk][qb]));

  float ls[QB][KL3];
  int li[QB][KL3];
  float theta_f[QB], published[QB];
  float thr[QB];  // fmaxf(ls[qb][KL3 - 1], theta_f[qb]): the group test's threshold
  uint32_t theta_next[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
    for (int j = 0; j < KL3; ++j) {
      ls[qb][j] = -INFINITY;
      li[qb][j] = -1;
    }
    theta_f[qb] = -INFINITY;
    thr[qb] = -INFINITY;
    published[qb] = -INFINITY;
    theta_next[qb] = 0u;
  }
  uint32_t* const theta_q = p.theta + slot0;
  const bool may_publish = p.k <= KL3;
  // row validity in one compare: (unsigned)(label - lo) <= span (ANY: label >= 0; else equality)
  const int lab_lo = p.label_filter == MRAG_LABEL_ANY ? 0 : p.label_filter;
  const uint32_t lab_span = p.label_filter == MRAG_LABEL_ANY ? 0x7fffffffu : 0u;

  // A fragment of row 16 rb + c16, chunk 4 kk + g4, sits at chunk (4 kk + g4) ^ c16: byte
  // offset (offA0 ^ ((kk & 3) << 6)) + (kk >> 2) * 256 + rb * 16 * ROW_BYTES
  const int offA0_init = c16 * ROW_BYTES + 16 * (g4 ^ c16);

  f32x4 acc[2][4][QB];  // [buffer][row block][query block]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      acc[1][i][j] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      acc[0][i][j] = f32x4{};
    }

  int my_tiles = (split < p.ntiles) ? (p.ntiles - 1 - split) / p.splits + 1 : 0;
  int tstep = p.splits;
  if constexpr (MODE == 1) {
    my_tiles = min(my_tiles, p.sample_tiles);
    tstep = p.splits * p.sample_stride;
  }
  float smax[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) smax[qb] = -INFINITY;

  auto stage_piece = [&](int buf, int tile, int i, int lane_t) {
    const char* gt = (const char*)p.x16 + (size_t)tile * TILE_BYTES;
    const unsigned piece = w * GLDS_PER_WAVE + i;
    const unsigned P = piece * 64 + (unsigned)lane_t;
    const unsigned row = P / CPR;
    const unsigned pos = P - row * CPR;
    const unsigned c = pos ^ (row & 15);
    glds_x4(gt + row * ROW_BYTES + c * 16, lds_base + buf * TILE_BYTES + piece * 1024);
  };
  auto stage_labels = [&](int buf, int tile) {
    if (w == 0) glds_x1(p.labels + (size_t)tile * TILE_ROWS + lane, lds_base + LBL_OFF + buf * TILE_ROWS * 4);
  };

  int prow = 0;  // first row of the filtered tile + 4 g4
#ifdef MRAG_K7_STAMPS
  // [0] tile top -> end of the DMA k-steps, [1] -> last MFMA issued, [2] -> tail + vmcnt(0),
  // [3] -> after the barrier, [4] tiles
  unsigned long long st_sum[7] = {0, 0, 0, 0, 0, 0, 0}, st_mid = 0;
#endif
  auto epi_group = [&](auto g_c, auto y_c) {
    constexpr int G = decltype(g_c)::value;
    constexpr int Y = decltype(y_c)::value;
    constexpr int qb = G >> 2, rb = G & 3;
    f32x4& av = acc[Y][rb][qb];
    // two VALU ops for the group maximum: the accumulators come out of inline asm, so fmaxf
    // would first canonicalise each operand (v_max x, x); scores are never NaN
    float gm;
    asm("v_max3_f32 %0, %1, %2, %3\n\tv_max_f32 %0, %0, %4"
        : "=&v"(gm)
        : "v"(av[0]), "v"(av[1]), "v"(av[2]), "v"(av[3]));
    if constexpr (MODE == 1) {
      float sm = smax[qb];
      asm volatile("v_max_f32 %0, %0, %1" : "+v"(sm) : "v"(gm));
      smax[qb] = sm;
    } else {
      // unlikely: the fire path is laid out away from the k-step's MFMAs, so the common case falls
      // through (no taken branch per k-step) and the two-tile loop keeps ~10 KB of hot code
      if (__builtin_expect(__any(gm > thr[qb]), 0)) {
#ifdef MRAG_K7_STAMPS
        const unsigned long long fire_t0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sv = av[r];
          if (sv > fmaxf(ls[qb][KL3 - 1], theta_f[qb]))
            list_insert_par<KL3>(ls[qb], li[qb], sv, prow + 16 * rb + r);
        }
        if (may_publish && li[qb][KL3 - 1] >= 0 && ls[qb][KL3 - 1] > published[qb]) {
          published[qb] = ls[qb][KL3 - 1];
          __hip_atomic_fetch_max(theta_q + 16 * qb, mrag_f2ord(published[qb]), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        }
        thr[qb] = fmaxf(ls[qb][KL3 - 1], theta_f[qb]);
#ifdef MRAG_K7_STAMPS
        st_sum[5] += 1;
        st_sum[6] += __builtin_amdgcn_s_memtime() - fire_t0;
#endif
      }
    }
  };

  // A fragments: fragment n = 4 kk + rb sits in a[n % NA]. QB = 4 keeps five, so fragment
  // n + 5 is read as soon as fragment n's MFMAs are issued: 16 MFMAs before its first use
  // (four buffers would give 12, which LDS latency under the DMA writes can exceed)
  constexpr int NA = QB == 4 ? 5 : 4;
  half8 a[NA];
  const int offA0 = offA0_init;
  auto read_a = [&](const char* tb, int kk, int rb) {
    a[(4 * kk + rb) % NA] =
        *(const half8*)(tb + ((offA0 ^ ((kk & 3) << 6)) + (kk >> 2) * 256 + rb * 16 * ROW_BYTES));
  };

  uint32_t m0_keep = 0;
#ifdef MRAG_K7_STAMPS
  unsigned long long st_end[3] = {0, 0, 0};
#endif
  // End of a tile: m0 back (`wait_part` false, before the masking), then (`wait_part` true) this
  // wave's DMA of the next tile landed, the shared threshold refreshed and the barrier: every
  // wave's DMA landed, and the tile's buffer is free for the next tile's DMA. (Moving the wait
  // and barrier before the last row block's MFMAs, with the next tile's first fragments read
  // under them, measured no faster: profiles/r3_k7_tail_ab.log.)
  auto end_of_tile = [&](bool wait_part) {
    if (!wait_part) {
#ifdef MRAG_K7_STAMPS
      st_end[0] = __builtin_amdgcn_s_memtime();
#endif
      if constexpr (CPR == 64 && QB == 4) asm volatile("s_mov_b32 m0, %0" ::"s"(m0_keep));
    }
    if (wait_part) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (MODE == 0) {
        if (may_publish) {
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) {
            if (theta_next[qb] != 0) theta_f[qb] = fmaxf(theta_f[qb], mrag_ord2f(theta_next[qb]));
            thr[qb] = fmaxf(ls[qb][KL3 - 1], theta_f[qb]);
            asm volatile("" : "+v"(theta_f[qb]), "+v"(thr[qb]));
          }
        }
      }
#ifdef MRAG_K7_STAMPS
      st_end[1] = __builtin_amdgcn_s_memtime();
#endif
      __syncthreads();
#ifdef MRAG_K7_STAMPS
      st_end[2] = __builtin_amdgcn_s_memtime();
#endif
    }
  };

  auto tile_body = [&](auto x_c, int it) {
    constexpr int X = decltype(x_c)::value;
    constexpr int Y = 1 - X;
    K7_STAMP(st0);
    const int tile = split + it * tstep;
    const bool has_next = it + 1 < my_tiles;
    const int ntile = has_next ? tile + tstep : tile;
    const char* gw = (const char*)p.x16 + (size_t)ntile * TILE_BYTES + (size_t)w * GLDS_PER_WAVE * ROW_BYTES;
    uint32_t ldsw = lds_base + Y * TILE_BYTES + w * GLDS_PER_WAVE * 1024;
    asm volatile("" : "+s"(gw), "+s"(ldsw));
    // the shared threshold only moves when lanes publish (k <= KL3); otherwise the seed read
    // before the loop stays exact and no tile pays the reloads or their tail update
    if constexpr (MODE == 0) {
      if (may_publish) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
          theta_next[qb] = __hip_atomic_load(theta_q + 16 * qb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const char* tb = smem + X * TILE_BYTES;
    int lane_t = lane;
    uint32_t lane16 = lane * 16;
    asm volatile("" : "+v"(lane_t), "+v"(lane16));
    // DP = 512: m0 holds the piece's LDS address from gap 1 to the DMA in gap 2 (nothing the
    // compiler emits in this loop reads m0: ds_read_b128 / MFMA / VALU / SALU only); it is saved
    // once per tile and restored before the barrier
    uint32_t voff = 0;
    if constexpr (CPR == 64 && QB == 4) asm volatile("s_mov_b32 %0, m0" : "=s"(m0_keep));
#pragma unroll
    for (int n = 0; n < NA; ++n) read_a(tb, n >> 2, n & 3);
    stage_labels(Y, ntile);
    // QB = 4: the tile's row-validity mask is built in the MFMA gaps (label read at k-step KLAB,
    // ballot one k-step later; buffer X's labels are not rewritten before the end-of-tile barrier),
    // so the tile tail holds only a wave-uniform test of it
    constexpr int KLAB = KSTEPS / 2 - 1;
    int lab_v = 0;
    uint64_t tile_mask = ~0ull;
    if constexpr (QB == 1) {
      // K7s (fill-bound): every piece of the next tile at the top of the tile, so the DMA has the
      // whole tile to land; per k-step the four row blocks' MFMAs, each followed by its next
      // fragment read; the previous tile's four group tests in the first k-step's gaps
#pragma unroll
      for (int i = 0; i < GLDS_PER_WAVE; ++i) stage_piece(Y, ntile, i, lane_t);
      static_for<KSTEPS>([&](auto kk_c) {
        constexpr int kk = decltype(kk_c)::value;
        static_for<4>([&](auto rb_c) {
          constexpr int rb = decltype(rb_c)::value;
          if constexpr (kk == 0)
            mfma16_ab0(acc[X][rb][0], a[(4 * kk + rb) % NA], qf[kk][0]);
          else
            mfma16_ab(acc[X][rb][0], a[(4 * kk + rb) % NA], qf[kk][0]);
          if constexpr (kk + 1 < KSTEPS) read_a(tb, kk + 1, rb);
          if constexpr (kk == 0) epi_group(std::integral_constant<int, rb>{}, std::integral_constant<int, Y>{});
          __builtin_amdgcn_sched_barrier(0);
        });
      });
    } else static_for<KSTEPS>([&](auto kk_c) {
      constexpr int kk = decltype(kk_c)::value;
      constexpr int g0 = (kk * NGROUPS + KSTEPS - 1) / KSTEPS;        // this k-step's groups:
      constexpr int g1 = ((kk + 1) * NGROUPS + KSTEPS - 1) / KSTEPS;  // [g0, g1), at most 4
      static_for<16>([&](auto j_c) {
        constexpr int j = decltype(j_c)::value;
        constexpr int rb = j >> 2, qb = j & 3;
        constexpr int n = 4 * kk + rb;  // this MFMA's A fragment
        if constexpr (kk == 0)
          mfma16_ab0(acc[X][rb][qb], a[n % NA], qf[kk][qb]);
        else
          mfma16_ab(acc[X][rb][qb], a[n % NA], qf[kk][qb]);
        // one job per MFMA gap
        if constexpr ((j & 3) == 3) {  // after the last MFMA of fragment n: fragment n + NA
          if constexpr (n + NA < 4 * KSTEPS) read_a(tb, (n + NA) >> 2, (n + NA) & 3);
        } else if constexpr ((j & 3) == 1) {  // piece FRONT kk + (j >> 2): m0 + source offset
          constexpr int pc = FRONT * kk + (j >> 2);
          if constexpr (CPR == 64 && (j >> 2) < FRONT && pc < GLDS_PER_WAVE) {
            voff = (lane16 ^ (uint32_t)(pc << 4)) + (uint32_t)(pc * 1024);
            asm volatile("s_mov_b32 m0, %1" : "+v"(voff) : "s"(ldsw + pc * 1024));
          }
          static_assert(KLAB * FRONT >= GLDS_PER_WAVE, "label slots must follow the DMA k-steps");
          if constexpr (kk == KLAB && j == 1) lab_v = ((const int*)(smem + LBL_OFF + X * TILE_ROWS * 4))[lane];
          if constexpr (kk == KLAB + 1 && j == 1) tile_mask = __ballot((uint32_t)(lab_v - lab_lo) <= lab_span);
        } else if constexpr ((j & 3) == 2) {  // ... and its DMA
          constexpr int pc = FRONT * kk + (j >> 2);
          if constexpr ((j >> 2) < FRONT && pc < GLDS_PER_WAVE) {
            if constexpr (CPR == 64)
              asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(gw) : "memory");
            else
              stage_piece(Y, ntile, pc, lane_t);
          }
        } else if constexpr ((j & 3) == 0) {
          if constexpr (g0 + (j >> 2) < g1)
            epi_group(std::integral_constant<int, g0 + (j >> 2)>{}, std::integral_constant<int, Y>{});
        }
#ifdef MRAG_K7_STAMPS
        if constexpr (kk == (GLDS_PER_WAVE + FRONT - 1) / FRONT - 1 && j == 15) st_mid = __builtin_amdgcn_s_memtime();
#endif
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    end_of_tile(false);
    if constexpr (QB == 1) {
      // K7s: the tile's labels, read after its MFMAs (a read at the top would wait for its LDS
      // round trip before the first MFMA; buffer X is not rewritten before the barrier)
      lab_v = ((const int*)(smem + LBL_OFF + X * TILE_ROWS * 4))[lane];
      tile_mask = __ballot((uint32_t)(lab_v - lab_lo) <= lab_span);
    }
    if (tile_mask != ~0ull) {
      mfma16_guard(acc[X]);
      const uint64_t lm = tile_mask >> (4 * g4);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = (lm >> (16 * rb + r)) & 1ull;
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) acc[X][rb][qb][r] = ok ? acc[X][rb][qb][r] : -INFINITY;
        }
    }
    prow = tile * TILE_ROWS + 4 * g4;
    end_of_tile(true);
#ifdef MRAG_K7_STAMPS
    if constexpr (QB == 4) {
      st_sum[0] += st_mid - st0;
      st_sum[1] += st_end[0] - st_mid;
    } else {
      st_sum[1] += st_end[0] - st0;
    }
    st_sum[2] += st_end[1] - st_end[0];
    st_sum[3] += st_end[2] - st_end[1];
    st_sum[4] += 1;
#endif
  };

  if constexpr (MODE == 0) {
    if (!may_publish) {  // the seed, read once (see the per-tile reloads in tile_body)
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        const uint32_t t0 = __hip_atomic_load(theta_q + 16 * qb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t0 != 0) theta_f[qb] = mrag_ord2f(t0);
        thr[qb] = theta_f[qb];
      }
    }
  }
  if (my_tiles > 0) {
#pragma unroll
    for (int i = 0; i < GLDS_PER_WAVE; ++i) stage_piece(0, split, i, lane);
    stage_labels(0, split);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int it = 0; it < my_tiles; it += 2) {
      tile_body(std::integral_constant<int, 0>{}, it);
      if (it + 1 < my_tiles) tile_body(std::integral_constant<int, 1>{}, it + 1);
    }
    if (my_tiles & 1) {
      static_for<NGROUPS>([&](auto g_c) { epi_group(g_c, std::integral_constant<int, 0>{}); });
    } else {
      static_for<NGROUPS>([&](auto g_c) { epi_group(g_c, std::integral_constant<int, 1>{}); });
    }
  }
#ifdef MRAG_K7_STAMPS
  if constexpr (MODE == 0) {
    const int wid = blockIdx.x * SCAN2_WAVES + w;
    if (lane == 0 && wid < K7_MAXWAVES)
      for (int i = 0; i < 7; ++i) g_k7_stamps[(size_t)wid * K7_NSTAMP + i] = st_sum[i];
  }
#endif

  if constexpr (MODE == 1) {
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      // four maxima per (split, query) over disjoint rows: lane group g4 = 0..3 (theta_init
      // takes the k-th largest of all splits' values: a valid lower bound, tighter than two)
      p.part_s[((size_t)split * p.Qp + slot0 + 16 * qb) * 4 + g4] = smax[qb];
    }
    return;
  }
  // fold the four lanes of each query (lanes c16 + 16 g) into one 8-list on g4 == 0
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    float fs[8];
    int fi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      fs[j] = j < KL3 ? ls[qb][j] : -INFINITY;
      fi[j] = j < KL3 ? li[qb][j] : -1;
    }
    float tau = li[qb][KL3 - 1] >= 0 ? ls[qb][KL3 - 1] : -INFINITY;
#pragma unroll
    for (int o = 16; o < 64; o += 16) {
#pragma unroll
      for (int j = 0; j < KL3; ++j) {
        const float ps = __shfl_xor(ls[qb][j], o);
        const int pi = __shfl_xor(li[qb][j], o);
        if (pi >= 0 && ps > fs[7]) list_insert<8>(fs, fi, ps, pi);
      }
      const int plast = __shfl_xor(li[qb][KL3 - 1], o);
      const float pl = __shfl_xor(ls[qb][KL3 - 1], o);
      if (plast >= 0) tau = fmaxf(tau, pl);
    }
    if (g4 == 0) {
      const int slot = slot0 + 16 * qb;
      float* os = p.part_s + ((size_t)split * p.Qp + slot) * 8;
      int32_t* oi = p.part_i + ((size_t)split * p.Qp + slot) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        os[j] = fs[j];
        oi[j] = fi[j];
      }
      if (fi[7] >= 0) tau = fmaxf(tau, fs[7]);
      p.part_tau[(size_t)split * p.Qp + slot] = tau;
    }
  }
}

// Seed of the shared threshold from the sample pre-pass: per query, the k-th largest of the
// 4*splits sample maxima (maxima of disjoint row sets, so k distinct rows score at least
// that), lowered by a margin of 2.5 EPS so that a seed equal to the k-th best approximate
// score cannot cost the certificate (K8 includes the final threshold in T). One wave per
// query; k rounds of wave arg-max extraction.
constexpr float THETA_SEED_MARGIN = (float)(2.5 * EPS_F16);
__global__ __launch_bounds__(64) void theta_init_kernel(const float* __restrict__ smax, int nvals, int Qp, int k,
                                                        uint32_t* __restrict__ theta) {
  constexpr int PER_LANE = 16;  // nvals = 4 * splits <= 4 * 256
  const int q = blockIdx.x, lane = threadIdx.x;
  float v[PER_LANE];
  // lane l takes splits l, l + 64, ... whole (one 16-byte load of the split's four maxima): the
  // (split, query) groups are 4 Qp floats apart, so per-value loads touched a line each; the
  // k-th largest does not depend on which lane holds a value
  const int splits = nvals / 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int sp = lane + 64 * t;
    const f32x4 x = sp < splits ? *(const f32x4*)(smax + ((size_t)sp * Qp + q) * 4)
                                : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int u = 0; u < 4; ++u) v[4 * t + u] = x[u];
  }
  float kth = -INFINITY;
  for (int r = 0; r < k; ++r) {
    float best = -INFINITY;
    int bt = 0;
#pragma unroll
    for (int t = 0; t < PER_LANE; ++t)
      if (v[t] > best) {
        best = v[t];
        bt = t;
      }
    float wbest = best;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wbest = fmaxf(wbest, __shfl_xor(wbest, off));
    if (wbest == -INFINITY) {
      kth = -INFINITY;
      break;
    }
    // remove exactly one occurrence: the lowest lane holding the maximum
    const uint64_t holders = __ballot(best == wbest);
    if (lane == (int)__builtin_ctzll(holders)) {
#pragma unroll
      for (int t = 0; t < PER_LANE; ++t)
        if (t == bt) v[t] = -INFINITY;
    }
    kth = wbest;
  }
  if (lane == 0) theta[q] = (kth == -INFINITY) ? 0u : mrag_f2ord(kth - THETA_SEED_MARGIN);
}

// ---------------------------------------------------------------------------
// Exact rescoring: mrag_knn::exact_cosine16 (knn_generic.h), shared with K7g.
using mrag_knn::exact_cosine16;

struct MergeParams {
  const float* part_s;
  const int32_t* part_i;
  int splits, KL, Qp, nq, k, M, R, Mp;
  const float* q32;
  const double* qn;
  const float* x32;
  const double* xn;
  int D, DP;
  float* out_s;
  double* out_s64;
  int64_t* out_r;
  int64_t row_offset;
  float* thresh;
  int32_t* fail_list;
  int32_t* fail_cnt;
  int32_t* host_fail;  // coherent pinned host word set to 1 by a failing query (null: none)
  const uint32_t* theta;  // final shared threshold (rows at or below it were never listed)
  const float* part_tau;  // v3: [splits][Qp] bound on the rows each split list dropped (or null)
};

__device__ __forceinline__ float f32_round_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}

// Wave-level bitonic network on E = 64 P keys held P per lane (element e = 64 p + lane),
// ascending. Stages with stride >= 64 swap registers within a lane, the others exchange with
// lane ^ stride. (Network checked against a host emulation for P = 1, 2.)
template <int P>
__device__ __forceinline__ void wave_sort_keys(uint64_t (&k)[P], int lane) {
  constexpr int E = 64 * P;
#pragma unroll
  for (int size = 2; size <= E; size <<= 1) {
#pragma unroll
    for (int st = size >> 1; st > 0; st >>= 1) {
      if (st >= 64) {  // P == 2, st == 64: element p = 0 is the lower one; size = 128 is ascending
        if constexpr (P == 2) {
          const uint64_t a = k[0], b = k[1];
          k[0] = a < b ? a : b;
          k[1] = a < b ? b : a;
        }
      } else {
#pragma unroll
        for (int pp = 0; pp < P; ++pp) {
          const int e = 64 * pp + lane;
          const bool asc = (e & size) == 0, lower = (lane & st) == 0;
          const uint64_t o = __shfl_xor((unsigned long long)k[pp], st);
          const uint64_t lo = k[pp] < o ? k[pp] : o, hi = k[pp] < o ? o : k[pp];
          k[pp] = (lower == asc) ? lo : hi;
        }
      }
    }
  }
}
// run <- the E smallest of run and b (both ascending), ascending: min(run[e], b[E-1-e]) is
// bitonic, then one ascending half-cleaner cascade
template <int P>
__device__ __forceinline__ void wave_merge_lowest(uint64_t (&run)[P], const uint64_t (&b)[P], int lane) {
#pragma unroll
  for (int pp = 0; pp < P; ++pp) {
    const uint64_t rb = __shfl((unsigned long long)b[P - 1 - pp], 63 - lane);
    run[pp] = run[pp] < rb ? run[pp] : rb;
  }
#pragma unroll
  for (int st = 32 * P; st > 0; st >>= 1) {
    if (st >= 64) {
      if constexpr (P == 2) {
        const uint64_t a = run[0], c = run[1];
        run[0] = a < c ? a : c;
        run[1] = a < c ? c : a;
      }
    } else {
#pragma unroll
      for (int pp = 0; pp < P; ++pp) {
        const uint64_t o = __shfl_xor((unsigned long long)run[pp], st);
        const bool lower = (lane & st) == 0;
        run[pp] = lower ? (run[pp] < o ? run[pp] : o) : (run[pp] < o ? o : run[pp]);
      }
    }
  }
}

#ifdef MRAG_K7_STAMPS
// Diagnostic build only: K8 phase times (s_memtime of wave 0) per workgroup, [block][8]
constexpr int K8_NSTAMP = 8, K8_MAXBLK = 4096;
__device__ unsigned long long g_k8_stamps[K8_MAXBLK * K8_NSTAMP];
#define K8_STAMP(i) k8t[i] = __builtin_amdgcn_s_memtime()
#else
#define K8_STAMP(i)
#endif
// K8: merge split lists, rescore exactly, certify. One workgroup per query.
// SEL = 0: bitonic sort of all S KL keys in LDS. SEL = P > 0 (when M + 1 <= 64 P): only the
// 64 P best keys are kept — every wave folds its share of the lists, 64 P keys at a time, into
// a running top-64P in registers (wave-level bitonic, no barriers), then wave 0 merges the four.
template <int SEL>
__global__ __launch_bounds__(MERGE_THREADS) void knn_merge_kernel(MergeParams p) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  uint64_t* keys = (uint64_t*)dsm;                                  // [R]
  double* ex = (double*)(dsm + (size_t)p.R * 8);                    // [Mp]
  int32_t* er = (int32_t*)(dsm + (size_t)p.R * 8 + (size_t)p.Mp * 8);  // [Mp]
  float* qs = (float*)(dsm + (size_t)p.R * 8 + (size_t)p.Mp * 12);     // [DP]
  float* red_f = (float*)(dsm + (size_t)p.R * 8 + (size_t)p.Mp * 12 + (size_t)p.DP * 4);  // [4]
  int* red_i = (int*)(red_f + MERGE_THREADS / 64);                                       // [4]

  const int q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef MRAG_K7_STAMPS
  unsigned long long k8t[K8_NSTAMP] = {};
#endif
  K8_STAMP(0);

  float tau = -INFINITY;
  int valid = 0;
  const int ntot = p.splits * p.KL;
  // candidate e of the union: the row and score are read together and unconditionally (a
  // clamped slot past the union), so a chunk costs one memory round trip and the next chunk's
  // reads can be in flight during this one's sort; invalid -> ~0 (sorts last)
  struct Raw {
    int r;
    float s;
  };
  auto load_raw = [&](int e) -> Raw {
    const int ec = e < ntot ? e : 0;
    const int sp = ec / p.KL, j = ec - sp * p.KL;
    const size_t o = ((size_t)sp * p.Qp + q) * p.KL + j;
    return Raw{p.part_i[o], p.part_s[o]};
  };
  auto make_key = [&](int e, Raw v) -> uint64_t {
    if (e >= ntot || v.r < 0) return ~0ull;
    ++valid;
    if (e % p.KL == p.KL - 1) tau = fmaxf(tau, v.s);
    return ((uint64_t)(~mrag_f2ord(v.s)) << 32) | (uint32_t)v.r;
  };
  auto load_key = [&](int e) -> uint64_t { return make_key(e, load_raw(e)); };
  // the splits' drop bounds and the query row first: their reads overlap the key fold
  if (p.part_tau)
    for (int sp = tid; sp < p.splits; sp += MERGE_THREADS) tau = fmaxf(tau, p.part_tau[(size_t)sp * p.Qp + q]);
  for (int d = tid; d < p.DP; d += MERGE_THREADS) qs[d] = p.q32[(size_t)q * p.DP + d];
  if constexpr (SEL == 0) {
    for (int e = tid; e < p.R; e += MERGE_THREADS) keys[e] = load_key(e);
  } else {
    constexpr int E = 64 * SEL;
    uint64_t run[SEL];
#pragma unroll
    for (int pp = 0; pp < SEL; ++pp) run[pp] = ~0ull;
    // software-pipelined: chunk c + 4's reads are issued before chunk c's sort (the reads, not
    // the sorts, bounded the fold: 42k -> 37k cycles for the eight chunks a wave folds in a
    // Q = 1 search; folding two chunks per step measured 35k there but slower at Q = 1000;
    // profiles/r3_k8_stamps_*.log)
    constexpr int NW = MERGE_THREADS / 64;
    Raw nx[SEL];
#pragma unroll
    for (int pp = 0; pp < SEL; ++pp) nx[pp] = load_raw(wave * E + 64 * pp + lane);
    for (int c = wave; c * E < ntot; c += NW) {  // wave-uniform
      uint64_t ch[SEL];
#pragma unroll
      for (int pp = 0; pp < SEL; ++pp) {
        ch[pp] = make_key(c * E + 64 * pp + lane, nx[pp]);
        nx[pp] = load_raw((c + NW) * E + 64 * pp + lane);
      }
      wave_sort_keys<SEL>(ch, lane);
      wave_merge_lowest<SEL>(run, ch, lane);
    }
#pragma unroll
    for (int pp = 0; pp < SEL; ++pp) keys[wave * E + 64 * pp + lane] = run[pp];
  }
  K8_STAMP(1);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    tau = fmaxf(tau, __shfl_xor(tau, off));
    valid += __shfl_xor(valid, off);
  }
  if (lane == 0) {
    red_f[wave] = tau;
    red_i[wave] = valid;
  }
  __syncthreads();
  tau = red_f[0];
  valid = red_i[0];
  for (int i = 1; i < MERGE_THREADS / 64; ++i) {
    tau = fmaxf(tau, red_f[i]);
    valid += red_i[i];
  }

  if constexpr (SEL == 0) {
    // bitonic sort of keys ascending == (approx desc, row asc)
    for (int size = 2; size <= p.R; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        __syncthreads();
        for (int i = tid; i < (p.R >> 1); i += MERGE_THREADS) {
          const int lo = 2 * i - (i & (stride - 1));
          const int hi = lo + stride;
          const bool asc = (lo & size) == 0;
          const uint64_t a = keys[lo], b = keys[hi];
          if ((a > b) == asc) {
            keys[lo] = b;
            keys[hi] = a;
          }
        }
      }
    }
  } else {  // wave 0 folds the other waves' top-E into its own; keys[0 .. E) = the E best
    constexpr int E = 64 * SEL;
    if (wave == 0) {
      uint64_t run[SEL], other[SEL];
#pragma unroll
      for (int pp = 0; pp < SEL; ++pp) run[pp] = keys[64 * pp + lane];
      for (int w2 = 1; w2 < MERGE_THREADS / 64; ++w2) {
#pragma unroll
        for (int pp = 0; pp < SEL; ++pp) other[pp] = keys[w2 * E + 64 * pp + lane];
        wave_merge_lowest<SEL>(run, other, lane);
      }
#pragma unroll
      for (int pp = 0; pp < SEL; ++pp) keys[64 * pp + lane] = run[pp];
    }
  }
  K8_STAMP(2);
  __syncthreads();
  K8_STAMP(3);

  const int M = min(p.M, valid);
  const float a_next = (valid > M) ? mrag_ord2f(~(uint32_t)(keys[M] >> 32)) : -INFINITY;
  // every row outside the candidate set scores <= T by approximation: rejected by a full
  // list (<= tau), by the shared threshold (<= theta; a seeded theta need not be any
  // list's KL-th, so it is bounded separately), or beyond the M-th candidate (<= a_next)
  float th = -INFINITY;
  if (p.theta && p.theta[q] != 0u) th = mrag_ord2f(p.theta[q]);
  const double T = (double)fmaxf(fmaxf(tau, a_next), th);
  const double qn = p.qn[q];

  {
    const int grp = tid >> 4, sub = tid & 15;
    for (int m0 = 0; m0 < p.Mp; m0 += MERGE_THREADS / 16) {
      const int m = m0 + grp;
      if (m < M) {
        const int r = (int)(uint32_t)(keys[m] & 0xffffffffu);
        const double s = exact_cosine16(qs, qn, p.x32, p.xn, r, p.D, p.DP, sub);
        if (sub == 0) {
          ex[m] = s;
          er[m] = r;
        }
      } else if (sub == 0 && m < p.Mp) {
        ex[m] = -INFINITY;
        er[m] = -1;
      }
    }
  }
  K8_STAMP(4);
  if (p.Mp <= 64) {
    // (ex, er) by (score desc, row asc), empty slots last: one wave's bitonic network in
    // registers (the block-wide network below pays a barrier per stage: 13.3k -> 7.0k cycles,
    // profiles/r3_k8_stamps_variants.log)
    __syncthreads();
    if (wave == 0) {
      double sv = lane < p.Mp ? ex[lane] : -INFINITY;
      int rv = lane < p.Mp ? er[lane] : -1;
#pragma unroll
      for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int st = size >> 1; st > 0; st >>= 1) {
          const double so = __shfl_xor(sv, st);
          const int ro = __shfl_xor(rv, st);
          const bool asc = (lane & size) == 0, lower = (lane & st) == 0;
          // the lower slot of an ascending pair keeps the one that ranks first
          if (mrag_before(so, ro, sv, rv) == (lower == asc)) {
            sv = so;
            rv = ro;
          }
        }
      }
      if (lane < p.Mp) {
        ex[lane] = sv;
        er[lane] = rv;
      }
    }
  }
  // bitonic sort of (ex, er) by (score desc, row asc); empty slots last
  for (int size = 2; size <= (p.Mp <= 64 ? 1 : p.Mp); size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = tid; i < (p.Mp >> 1); i += MERGE_THREADS) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const double sa = ex[lo], sb = ex[hi];
        const int ra = er[lo], rb = er[hi];
        // "ascending" in retrieval order == a ranks before b
        const bool b_first = mrag_before(sb, rb, sa, ra);
        if (b_first == asc) {
          ex[lo] = sb; er[lo] = rb;
          ex[hi] = sa; er[hi] = ra;
        }
      }
    }
  }
  __syncthreads();
  K8_STAMP(5);

  for (int j = tid; j < p.k; j += MERGE_THREADS) {
    const bool has = j < M;
    const double s = has ? ex[j] : -INFINITY;
    const size_t o = (size_t)q * p.k + j;
    p.out_s[o] = (float)s;
    if (p.out_s64) p.out_s64[o] = s;
    p.out_r[o] = has ? (int64_t)er[j] + p.row_offset : -1;
  }
  if (tid == 0) {
    bool cert;
    if (tau == -INFINITY && valid <= M) {
      cert = true;  // every matching row is in the union and was rescored
    } else {
      cert = (M >= p.k) && (ex[p.k - 1] > T + EPS_F16);
    }
    if (!cert) {
      p.thresh[q] = (M >= p.k) ? f32_round_down(ex[p.k - 1] - EPS_F16) : -INFINITY;
      const int s = atomicAdd(p.fail_cnt, 1);
      p.fail_list[s] = q;
      // the host reads this word after the stream completes and fetches the count only when
      // it is set (no device-to-host copy behind a search that certifies every query)
      if (p.host_fail) __hip_atomic_store(p.host_fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
#ifdef MRAG_K7_STAMPS
  K8_STAMP(6);
  if (tid == 0 && q < K8_MAXBLK)
    for (int i = 0; i < K8_NSTAMP; ++i) g_k8_stamps[(size_t)q * K8_NSTAMP + i] = k8t[i];
#endif
}

struct FinalParams {
  const int32_t* fail_list;
  const int32_t* fail_cnt;
  const int32_t* cand_cnt;
  const int32_t* cand;
  int ccap;
  double* scratch;  // [Qp][ccap]
  const float* q32;
  const double* qn;
  const float* x32;
  const double* xn;
  int D, DP, k;
  float* out_s;
  double* out_s64;
  int64_t* out_r;
  int64_t row_offset;
  int32_t* overflow;
};

// Block-wide "best after prev" selection step shared by K10 and K11.
__device__ void block_select_best(double& bs, int64_t& br) {
  __shared__ double rs[MERGE_THREADS / 64];
  __shared__ int64_t rr[MERGE_THREADS / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double os = __shfl_xor(bs, off);
    const int64_t orr = __shfl_xor(br, off);
    if (mrag_before(os, orr, bs, br)) {
      bs = os;
      br = orr;
    }
  }
  __syncthreads();
  if (lane == 0) {
    rs[wave] = bs;
    rr[wave] = br;
  }
  __syncthreads();
  bs = rs[0];
  br = rr[0];
  for (int i = 1; i < MERGE_THREADS / 64; ++i)
    if (mrag_before(rs[i], rr[i], bs, br)) {
      bs = rs[i];
      br = rr[i];
    }
}

// K10: exact top-k among the rows collected for an uncertified query.
__global__ __launch_bounds__(MERGE_THREADS) void knn_final_kernel(FinalParams p) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  float* qs = (float*)dsm;
  const int slot = blockIdx.x;
  if (slot >= *p.fail_cnt) return;
  const int q = p.fail_list[slot];
  const int n = p.cand_cnt[slot];
  if (n > p.ccap) {
    if (threadIdx.x == 0) atomicOr(p.overflow, 1);
    return;
  }
  const int tid = threadIdx.x;
  for (int d = tid; d < p.DP; d += MERGE_THREADS) qs[d] = p.q32[(size_t)q * p.DP + d];
  __syncthreads();
  const double qn = p.qn[q];
  double* sc = p.scratch + (size_t)slot * p.ccap;
  const int32_t* cr = p.cand + (size_t)slot * p.ccap;
  for (int m = tid >> 4; m < n; m += MERGE_THREADS / 16) {
    const double s = exact_cosine16(qs, qn, p.x32, p.xn, cr[m], p.D, p.DP, tid & 15);
    if ((tid & 15) == 0) sc[m] = s;
  }
  __syncthreads();
  double ps = INFINITY;
  int64_t pr = -1;  // sentinel "before everything"
  for (int j = 0; j < p.k; ++j) {
    double bs = -INFINITY;
    int64_t br = -1;
    for (int m = tid; m < n; m += MERGE_THREADS) {
      const double s = sc[m];
      const int64_t r = cr[m];
      const bool after_prev = (pr < 0) ? true : mrag_before(ps, pr, s, r);
      if (after_prev && mrag_before(s, r, bs, br)) {
        bs = s;
        br = r;
      }
    }
    block_select_best(bs, br);
    if (tid == 0) {
      const size_t o = (size_t)q * p.k + j;
      p.out_s[o] = (float)bs;
      if (p.out_s64) p.out_s64[o] = bs;
      p.out_r[o] = br >= 0 ? br + p.row_offset : -1;
    }
    ps = bs;
    pr = br;
    if (br < 0) {
      // no more rows: fill the rest
      for (int jj = j + 1 + tid; jj < p.k; jj += MERGE_THREADS) {
        const size_t o = (size_t)q * p.k + jj;
        p.out_s[o] = -INFINITY;
        if (p.out_s64) p.out_s64[o] = -INFINITY;
        p.out_r[o] = -1;
      }
      break;
    }
  }
}

// K11: merge nlists per-shard top-k lists per query (row-sharded search).
__global__ __launch_bounds__(MERGE_THREADS) void topk_merge_kernel(const double* __restrict__ s64,
                                                                   const int64_t* __restrict__ rows,
                                                                   int nlists, int64_t nq, int k,
                                                                   float* out_s, double* out_s64,
                                                                   int64_t* out_r) {
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x;
  const int n = nlists * k;
  double ps = INFINITY;
  int64_t pr = -1;
  for (int j = 0; j < k; ++j) {
    double bs = -INFINITY;
    int64_t br = -1;
    for (int m = tid; m < n; m += MERGE_THREADS) {
      const int l = m / k, jj = m - l * k;
      const size_t o = ((size_t)l * nq + q) * k + jj;
      const double s = s64[o];
      const int64_t r = rows[o];
      if (r < 0) continue;
      const bool after_prev = (pr < 0) ? true : mrag_before(ps, pr, s, r);
      if (after_prev && mrag_before(s, r, bs, br)) {
        bs = s;
        br = r;
      }
    }
    block_select_best(bs, br);
    if (tid == 0) {
      const size_t o = (size_t)q * k + j;
      out_s[o] = br >= 0 ? (float)bs : -INFINITY;
      if (out_s64) out_s64[o] = br >= 0 ? bs : -INFINITY;
      out_r[o] = br;
    }
    if (br >= 0) {
      ps = bs;
      pr = br;
    }
  }
}

// Row preparation: in f32 [nin][D] -> x32 [nout][DP] (zero padded), |x| f64,
// x16 = fp16(x/|x|). One wave per row.
// Per-search scratch cleared by the query prep (instead of three memset launches): the
// certificate counters, the per-slot collect counts and the shared thresholds.
struct PrepClear {
  int32_t* counters;  // [4] or null
  int32_t* cand_cnt;  // [nout] or null
  uint32_t* theta;    // [nout] or null
};

__global__ __launch_bounds__(256) void prep_rows_kernel(const float* __restrict__ in, int64_t nin,
                                                        int D, int DP, int64_t nout,
                                                        float* __restrict__ x32,
                                                        double* __restrict__ xn,
                                                        _Float16* __restrict__ x16, PrepClear clr) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (clr.counters && blockIdx.x == 0 && threadIdx.x < 4) clr.counters[threadIdx.x] = 0;
  if (row >= nout) return;
  if (lane == 0) {
    if (clr.cand_cnt) clr.cand_cnt[row] = 0;
    if (clr.theta) clr.theta[row] = 0u;
  }
  float v[8];
  double ss = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int d = lane + 64 * j;
    v[j] = (row < nin && d < D) ? in[row * D + d] : 0.0f;
    ss = fma((double)v[j], (double)v[j], ss);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
  const double nrm = sqrt(ss);
  const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int d = lane + 64 * j;
    if (d < DP) {
      x32[row * DP + d] = v[j];
      x16[row * DP + d] = (_Float16)(float)((double)v[j] * inv);
    }
  }
  if (lane == 0) xn[row] = nrm;
}

// Row preparation for DP > 512 (K7g widths): same outputs, two passes over the input row.
__global__ __launch_bounds__(256) void prep_rows_wide_kernel(const float* __restrict__ in, int64_t nin, int D, int DP,
                                                             int64_t nout, float* __restrict__ x32,
                                                             double* __restrict__ xn, _Float16* __restrict__ x16) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nout) return;
  const bool live = row < nin;
  double ss = 0.0;
  for (int d = lane; d < D; d += 64) {
    const float v = live ? in[row * D + d] : 0.0f;
    ss = fma((double)v, (double)v, ss);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
  const double nrm = sqrt(ss);
  const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
  for (int d = lane; d < DP; d += 64) {
    const float v = (live && d < D) ? in[row * D + d] : 0.0f;
    x32[row * DP + d] = v;
    x16[row * DP + d] = (_Float16)(float)((double)v * inv);
  }
  if (lane == 0) xn[row] = nrm;
}

int launch_prep(const float* in, int64_t nin, int D, int DP, int64_t nout, float* x32, double* xn, _Float16* x16,
                hipStream_t s, PrepClear clr = PrepClear{}) {
  if (nout <= 0) return MRAG_OK;
  if (DP <= 512)
    hipLaunchKernelGGL(prep_rows_kernel, dim3((unsigned)((nout + 3) / 4)), dim3(256), 0, s, in, nin, D, DP, nout,
                       x32, xn, x16, clr);
  else
    hipLaunchKernelGGL(prep_rows_wide_kernel, dim3((unsigned)((nout + 3) / 4)), dim3(256), 0, s, in, nin, D, DP,
                       nout, x32, xn, x16);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

__global__ void fill_i32_kernel(int32_t* p, int64_t n, int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void scatter_label_kernel(int32_t* labels, const int64_t* rows, int64_t n, int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) labels[rows[i]] = v;
}

__global__ void fill_empty_kernel(float* s, double* s64, int64_t* r, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    s[i] = -INFINITY;
    if (s64) s64[i] = -INFINITY;
    r[i] = -1;
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

int ensure(DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return MRAG_OK;
  if (b.p) {
    MRAG_HIP(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  const size_t want = std::max<size_t>(bytes, 256);
  MRAG_HIP(hipMalloc(&b.p, want));
  b.bytes = want;
  return MRAG_OK;
}

void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

typedef void (*scan_fn)(ScanParams);

template <int DP>
scan_fn pick_scan(int KL, bool collect) {
  if (collect) return knn_scan_kernel<DP, 8, true>;
  // Deeper lists keep 2*KL more VGPRs live next to the DP/4 query-fragment registers;
  // kl_for() caps KL where it would spill (the certificate stays exact either way).
  if constexpr (DP >= 512) {
    return knn_scan_kernel<DP, 8, false>;
  } else if constexpr (DP >= 256) {
    return KL <= 8 ? knn_scan_kernel<DP, 8, false> : knn_scan_kernel<DP, 16, false>;
  } else {
    return KL <= 8 ? knn_scan_kernel<DP, 8, false>
                   : (KL <= 16 ? knn_scan_kernel<DP, 16, false> : knn_scan_kernel<DP, 32, false>);
  }
}

// Per-lane list depth: >= k where registers allow (DP/4 VGPRs hold the query fragments).
int kl_for(int k, int DP) {
  if (k <= 8 || DP >= 512) return 8;
  if (k <= 16 || DP >= 256) return 16;
  return 32;
}

template <int MODE, int QB>
scan_fn get_scan3m(int DP) {
  switch (DP) {
    case 128: return knn_scan3_kernel<128, MODE, QB>;
    case 256: return knn_scan3_kernel<256, MODE, QB>;
    case 384: return knn_scan3_kernel<384, MODE, QB>;
    case 512: return knn_scan3_kernel<512, MODE, QB>;
    default: return nullptr;
  }
}
// the sample pre-pass (MODE 1) exists for the 256-query groups only (K7s runs without it)
scan_fn get_scan3(int DP, bool sample, int qb) {
  if (qb == 1) return sample ? nullptr : get_scan3m<0, 1>(DP);
  return sample ? get_scan3m<1, 4>(DP) : get_scan3m<0, 4>(DP);
}

// Query blocks per wave of the v3 scan for a batch: 1 (K7s, 64 queries per workgroup) while the
// batch fits one small group, else 4 (256 per workgroup).
int scan3_qb(int64_t nq) { return nq <= 64 ? 1 : 4; }

// Sample pre-pass stride for k: the main scan's fires grow with the rows above the seed, about
// k x stride, so k > 16 samples every 4th tile (512k x 512, k = 50: search 0.824 -> 0.736 ms,
// scan 0.659 -> 0.501; stride 8: 0.748; notes/knn_scan_experiments.md).
int sample_stride_for(int k) { return k > 16 ? 4 : SAMPLE_STRIDE; }

scan_fn get_scan(int DP, int KL, bool collect) {
  switch (DP) {
    case 128: return pick_scan<128>(KL, collect);
    case 256: return pick_scan<256>(KL, collect);
    case 384: return pick_scan<384>(KL, collect);
    case 512: return pick_scan<512>(KL, collect);
    default: return nullptr;
  }
}

int64_t next_pow2(int64_t x) {
  int64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

// Per-search buffers. A search takes a free context from its index's pool (a new one when all
// are in use), so several host threads can search one index at once, each on its own stream,
// while the corpus buffers stay shared and read-only (adds / deletes take the index lock
// exclusively). Two searches in flight let one search's K8 / certificate / host round trip run
// beside the other's scan (bench.py runs the kNN leg that way on one GPU).
struct SearchCtx {
  DevBuf qin, q32, qn, q16, part_s, part_i, thresh, fail_list, counters, cand_cnt, cand, scratch;
  DevBuf out_s, out_s64, out_r, theta, part_tau;
  int32_t* host_counters = nullptr;  // pinned [2]: fail_cnt, overflow
  int32_t* host_fail = nullptr;      // coherent pinned [4]: [0] = some query failed K8's certificate
  hipEvent_t done = nullptr;         // end of the search's device work (waited by spinning)
  hipEvent_t null_ev = nullptr;      // device inputs on the NULL stream: the search waits for it
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // scan timing (mrag_knn_profile)
  mrag_knn::Workspace gws[8];               // K7g buffers
};

struct mrag_knn_index {
  std::mutex mu;             // serialises mutations (add / set_labels / destroy) and profile toggles
  std::shared_mutex rw;      // searches shared, mutations exclusive
  int device = 0;
  int D = 0, DP = 0;
  int64_t n = 0, cap = 0;
  DevBuf x16, x32, xn, labels;
  hipStream_t stream = nullptr;
  DevBuf stage_rows, stage_labels, rowlist;  // mutation staging
  std::mutex pool_mu;                        // guards the context pool and the stats below
  std::vector<SearchCtx*> ctx_all, ctx_free;
  int64_t last_uncertified = 0, last_retries = 0;
  // diagnostics of the last search (mrag_debug_knn_last_collect): its context (buffers stay valid
  // until that context's next search) and the grid it used
  SearchCtx* last_ctx = nullptr;
  int32_t last_info[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // S, Qp, cgroups, Sc, ccap, uncertified, overflow, KL
  // optional scan timing (mrag_knn_profile)
  bool profile = false;
  double scan_ms = 0.0;
  int64_t scan_launches = 0;
};

namespace {

// Block until everything enqueued on s so far has run: an event recorded behind it, polled.
// The search's answer depends on the certificate counters it reads back, so a search returns
// only once its device work is done; polling wakes the host within a microsecond or two of the
// last kernel, where a stream synchronize could leave the GPU idle for tens of microseconds
// between back-to-back searches.
int wait_stream(SearchCtx* c, hipStream_t s) {
  MRAG_HIP(hipEventRecord(c->done, s));
  hipError_t e;
  while ((e = hipEventQuery(c->done)) == hipErrorNotReady) {
  }
  if (e != hipSuccess) return mrag::fail(MRAG_ERR_HIP, "search: %s", hipGetErrorString(e));
  return MRAG_OK;
}

void ctx_free_all(SearchCtx* c) {
  for (DevBuf* b : {&c->qin, &c->q32, &c->qn, &c->q16, &c->part_s, &c->part_i, &c->thresh, &c->fail_list,
                    &c->counters, &c->cand_cnt, &c->cand, &c->scratch, &c->out_s, &c->out_s64, &c->out_r,
                    &c->theta, &c->part_tau})
    release(*b);
  mrag_knn::release(c->gws);
  if (c->host_counters) (void)hipHostFree(c->host_counters);
  if (c->host_fail) (void)hipHostFree(c->host_fail);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->null_ev) (void)hipEventDestroy(c->null_ev);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  delete c;
}

// A free search context of ix (created on first need); returned by ctx_put.
int ctx_get(mrag_knn_index* ix, SearchCtx** out) {
  {
    std::lock_guard<std::mutex> lk(ix->pool_mu);
    if (!ix->ctx_free.empty()) {
      *out = ix->ctx_free.back();
      ix->ctx_free.pop_back();
      return MRAG_OK;
    }
  }
  auto* c = new SearchCtx();
  hipError_t e = hipHostMalloc((void**)&c->host_counters, 16, hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->host_fail, 16, hipHostMallocCoherent);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->null_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e != hipSuccess) {
    ctx_free_all(c);
    return mrag::fail(MRAG_ERR_HIP, "search context: %s", hipGetErrorString(e));
  }
  std::lock_guard<std::mutex> lk(ix->pool_mu);
  ix->ctx_all.push_back(c);
  *out = c;
  return MRAG_OK;
}

struct CtxLease {
  mrag_knn_index* ix;
  SearchCtx* c;
  ~CtxLease() {
    std::lock_guard<std::mutex> lk(ix->pool_mu);
    ix->ctx_free.push_back(c);
  }
};

int grow(mrag_knn_index* ix, int64_t need) {
  if (need <= ix->cap) return MRAG_OK;
  int64_t ncap = std::max<int64_t>({(int64_t)TILE_ROWS, ix->cap * 2, need});
  ncap = (ncap + 767) / 768 * 768;  // a multiple of the 64- and 48-row scan tiles and of K7g's 128-column GEMM tile
  DevBuf nx16, nx32, nxn, nlab;
  if (int rc = ensure(nx16, (size_t)ncap * ix->DP * 2)) return rc;
  if (int rc = ensure(nx32, (size_t)ncap * ix->DP * 4)) return rc;
  if (int rc = ensure(nxn, (size_t)ncap * 8)) return rc;
  if (int rc = ensure(nlab, (size_t)ncap * 4)) return rc;
  hipStream_t s = ix->stream;
  MRAG_HIP(hipMemsetAsync(nx16.p, 0, (size_t)ncap * ix->DP * 2, s));
  MRAG_HIP(hipMemsetAsync(nx32.p, 0, (size_t)ncap * ix->DP * 4, s));
  MRAG_HIP(hipMemsetAsync(nxn.p, 0, (size_t)ncap * 8, s));
  hipLaunchKernelGGL(fill_i32_kernel, dim3((unsigned)((ncap + 255) / 256)), dim3(256), 0, s,
                     (int32_t*)nlab.p, ncap, (int32_t)MRAG_LABEL_DELETED);
  MRAG_CHECK_LAUNCH();
  if (ix->n > 0) {
    MRAG_HIP(hipMemcpyAsync(nx16.p, ix->x16.p, (size_t)ix->n * ix->DP * 2, hipMemcpyDeviceToDevice, s));
    MRAG_HIP(hipMemcpyAsync(nx32.p, ix->x32.p, (size_t)ix->n * ix->DP * 4, hipMemcpyDeviceToDevice, s));
    MRAG_HIP(hipMemcpyAsync(nxn.p, ix->xn.p, (size_t)ix->n * 8, hipMemcpyDeviceToDevice, s));
    MRAG_HIP(hipMemcpyAsync(nlab.p, ix->labels.p, (size_t)ix->n * 4, hipMemcpyDeviceToDevice, s));
  }
  MRAG_HIP(hipStreamSynchronize(s));
  release(ix->x16);
  release(ix->x32);
  release(ix->xn);
  release(ix->labels);
  ix->x16 = nx16;
  ix->x32 = nx32;
  ix->xn = nxn;
  ix->labels = nlab;
  ix->cap = ncap;
  return MRAG_OK;
}

}  // namespace

extern "C" {
#ifdef MRAG_K7_STAMPS
// diagnostic build only: copy the per-wave K7 segment sums of the last scan (n <= 2^16 * 8)
// K8 phase stamps of the last merge: [block][8] s_memtime values (see knn_merge_kernel)
__attribute__((visibility("default"))) int mrag_debug_k8_stamps(unsigned long long* out, int n) {
  if (n > K8_MAXBLK * K8_NSTAMP) n = K8_MAXBLK * K8_NSTAMP;
  MRAG_HIP(hipDeviceSynchronize());
  MRAG_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k8_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost));
  return MRAG_OK;
}
__attribute__((visibility("default"))) int mrag_debug_k7_stamps(unsigned long long* out, int n) {
  if (n > K7_MAXWAVES * K7_NSTAMP) n = K7_MAXWAVES * K7_NSTAMP;
  MRAG_HIP(hipDeviceSynchronize());
  MRAG_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k7_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost));
  void* sym = nullptr;  // cleared for the next scan (waves it does not launch stay zero)
  MRAG_HIP(hipGetSymbolAddress(&sym, HIP_SYMBOL(g_k7_stamps)));
  MRAG_HIP(hipMemset(sym, 0, sizeof(g_k7_stamps)));
  MRAG_HIP(hipDeviceSynchronize());
  return MRAG_OK;
}
#endif

int mrag_knn_create(int32_t dim, int32_t device, mrag_knn_index** out) {
  MRAG_REQUIRE(out != nullptr, "out is NULL");
  *out = nullptr;
  MRAG_REQUIRE(dim >= 1 && dim <= mrag_knn::GENERIC_MAX_DIM, "dim %d unsupported (1..%d)", dim,
               mrag_knn::GENERIC_MAX_DIM);
  int ndev = 0;
  MRAG_HIP(hipGetDeviceCount(&ndev));
  MRAG_REQUIRE(device >= 0 && device < ndev, "device %d out of range (%d devices)", device, ndev);
  mrag::DeviceGuard g(device);
  auto* ix = new mrag_knn_index();
  ix->device = device;
  ix->D = dim;
  ix->DP = (dim + 127) / 128 * 128;
  hipError_t e = hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete ix;
    return mrag::fail(MRAG_ERR_HIP, "stream/pinned alloc: %s", hipGetErrorString(e));
  }
  *out = ix;
  return MRAG_OK;
}

int mrag_knn_destroy(mrag_knn_index* ix) {
  if (!ix) return MRAG_OK;
  {
    mrag::DeviceGuard g(ix->device);
    (void)hipStreamSynchronize(ix->stream);
    std::unique_lock<std::shared_mutex> wl(ix->rw);  // no search in flight
    for (DevBuf* b : {&ix->x16, &ix->x32, &ix->xn, &ix->labels, &ix->stage_rows, &ix->stage_labels, &ix->rowlist})
      release(*b);
    for (SearchCtx* c : ix->ctx_all) ctx_free_all(c);
    ix->ctx_all.clear();
    ix->ctx_free.clear();
    if (ix->stream) (void)hipStreamDestroy(ix->stream);
  }
  delete ix;
  return MRAG_OK;
}

int mrag_knn_size(const mrag_knn_index* ix, int64_t* n) {
  MRAG_REQUIRE(ix != nullptr && n != nullptr, "NULL argument");
  *n = ix->n;
  return MRAG_OK;
}

int mrag_knn_last_stats(const mrag_knn_index* ix, int64_t* uncertified, int64_t* retries) {
  MRAG_REQUIRE(ix != nullptr, "NULL index");
  std::lock_guard<std::mutex> lk(const_cast<mrag_knn_index*>(ix)->pool_mu);
  if (uncertified) *uncertified = ix->last_uncertified;
  if (retries) *retries = ix->last_retries;
  return MRAG_OK;
}

int mrag_knn_profile(mrag_knn_index* ix, int32_t enable, double* scan_ms_total, int64_t* scan_launches) {
  MRAG_REQUIRE(ix != nullptr, "NULL index");
  std::lock_guard<std::mutex> lk(ix->pool_mu);
  if (enable == 1) {
    ix->profile = true;
    ix->scan_ms = 0.0;
    ix->scan_launches = 0;
  } else if (enable == 0) {
    ix->profile = false;
  }
  if (scan_ms_total) *scan_ms_total = ix->scan_ms;
  if (scan_launches) *scan_launches = ix->scan_launches;
  return MRAG_OK;
}

int mrag_knn_add(mrag_knn_index* ix, const float* rows, const int32_t* labels, int64_t nrows,
                 int32_t ptr_kind, int64_t* first_row) {
  MRAG_REQUIRE(ix != nullptr, "NULL index");
  MRAG_REQUIRE(nrows >= 0, "negative row count");
  MRAG_REQUIRE(ptr_kind == MRAG_PTR_HOST || ptr_kind == MRAG_PTR_DEVICE, "bad ptr_kind %d", ptr_kind);
  std::lock_guard<std::mutex> lk(ix->mu);
  std::unique_lock<std::shared_mutex> wl(ix->rw);
  mrag::DeviceGuard g(ix->device);
  if (first_row) *first_row = ix->n;
  if (nrows == 0) return MRAG_OK;
  MRAG_REQUIRE(rows != nullptr && labels != nullptr, "NULL rows/labels");
  MRAG_REQUIRE(ix->n + nrows < (int64_t)1 << 31, "index would exceed 2^31 rows per shard");
  if (int rc = grow(ix, ix->n + nrows)) return rc;
  hipStream_t s = ix->stream;
  const float* src = rows;
  const int32_t* lsrc = labels;
  if (ptr_kind == MRAG_PTR_DEVICE) MRAG_HIP(hipStreamSynchronize(nullptr));  // inputs queued on the null stream
  if (ptr_kind == MRAG_PTR_HOST) {
    if (int rc = ensure(ix->stage_rows, (size_t)nrows * ix->D * 4)) return rc;
    if (int rc = ensure(ix->stage_labels, (size_t)nrows * 4)) return rc;
    MRAG_HIP(hipMemcpyAsync(ix->stage_rows.p, rows, (size_t)nrows * ix->D * 4, hipMemcpyHostToDevice, s));
    MRAG_HIP(hipMemcpyAsync(ix->stage_labels.p, labels, (size_t)nrows * 4, hipMemcpyHostToDevice, s));
    src = (const float*)ix->stage_rows.p;
    lsrc = (const int32_t*)ix->stage_labels.p;
  }
  const int64_t n0 = ix->n;
  if (int rc = launch_prep(src, nrows, ix->D, ix->DP, nrows, (float*)ix->x32.p + n0 * ix->DP, (double*)ix->xn.p + n0,
                           (_Float16*)ix->x16.p + n0 * ix->DP, s))
    return rc;
  MRAG_HIP(hipMemcpyAsync((int32_t*)ix->labels.p + n0, lsrc, (size_t)nrows * 4, hipMemcpyDeviceToDevice, s));
  MRAG_HIP(hipStreamSynchronize(s));
  ix->n += nrows;
  return MRAG_OK;
}

int mrag_knn_set_labels(mrag_knn_index* ix, const int64_t* rows, int64_t n, int32_t label) {
  MRAG_REQUIRE(ix != nullptr, "NULL index");
  MRAG_REQUIRE(n >= 0, "negative count");
  MRAG_REQUIRE(label >= 0 || label == MRAG_LABEL_DELETED, "label %d invalid", label);
  std::lock_guard<std::mutex> lk(ix->mu);
  std::unique_lock<std::shared_mutex> wl(ix->rw);
  mrag::DeviceGuard g(ix->device);
  if (n == 0) return MRAG_OK;
  MRAG_REQUIRE(rows != nullptr, "NULL rows");
  for (int64_t i = 0; i < n; ++i)
    MRAG_REQUIRE(rows[i] >= 0 && rows[i] < ix->n, "row %lld out of range [0,%lld)", (long long)rows[i],
                 (long long)ix->n);
  if (int rc = ensure(ix->rowlist, (size_t)n * 8)) return rc;
  MRAG_HIP(hipMemcpyAsync(ix->rowlist.p, rows, (size_t)n * 8, hipMemcpyHostToDevice, ix->stream));
  hipLaunchKernelGGL(scatter_label_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ix->stream,
                     (int32_t*)ix->labels.p, (const int64_t*)ix->rowlist.p, n, label);
  MRAG_CHECK_LAUNCH();
  MRAG_HIP(hipStreamSynchronize(ix->stream));
  return MRAG_OK;
}

int mrag_knn_search(mrag_knn_index* ix, const float* queries, int64_t nq, int32_t k,
                    int32_t label_filter, int64_t row_offset, float* out_scores, double* out_scores64,
                    int64_t* out_rows, int32_t ptr_kind, void* stream_arg) {
  MRAG_REQUIRE(ix != nullptr, "NULL index");
  MRAG_REQUIRE(nq >= 0, "negative query count");
  MRAG_REQUIRE(k >= 1 && k <= mrag_knn::GENERIC_MAX_K, "k=%d unsupported (1..%d)", k, mrag_knn::GENERIC_MAX_K);
  MRAG_REQUIRE(label_filter >= MRAG_LABEL_ANY, "label filter %d invalid", label_filter);
  MRAG_REQUIRE(ptr_kind == MRAG_PTR_HOST || ptr_kind == MRAG_PTR_DEVICE, "bad ptr_kind %d", ptr_kind);
  MRAG_REQUIRE(nq < (1 << 24), "too many queries in one call");
  std::shared_lock<std::shared_mutex> rl(ix->rw);
  mrag::DeviceGuard g(ix->device);
  if (nq == 0) return MRAG_OK;
  SearchCtx* c = nullptr;
  if (int rc = ctx_get(ix, &c)) return rc;
  CtxLease lease{ix, c};
  bool profile;
  {
    std::lock_guard<std::mutex> lk(ix->pool_mu);
    profile = ix->profile;
  }
  MRAG_REQUIRE(queries && out_scores && out_rows, "NULL query/output pointer");
  hipStream_t s = stream_arg ? (hipStream_t)stream_arg : ix->stream;
  const bool host = ptr_kind == MRAG_PTR_HOST;
  if (!host && !stream_arg)
    if (int rc = mrag::wait_null_stream(c->null_ev, s)) return rc;
  // destroyed before the lease and the shared lock: an error after the first launch drains s
  // before the context returns to the pool and mutations may free the corpus buffers
  mrag::StreamDrain drain(s);
  const int D = ix->D, DP = ix->DP;
  const int64_t nout = nq * k;

  // output destinations (device)
  float* os = out_scores;
  double* os64 = out_scores64;
  int64_t* orr = out_rows;
  if (host) {
    if (int rc = ensure(c->out_s, nout * 4)) return rc;
    if (int rc = ensure(c->out_r, nout * 8)) return rc;
    os = (float*)c->out_s.p;
    orr = (int64_t*)c->out_r.p;
    if (out_scores64) {
      if (int rc = ensure(c->out_s64, nout * 8)) return rc;
      os64 = (double*)c->out_s64.p;
    }
  }
  int64_t uncertified = 0, retries = 0;
  int32_t info[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  auto generic_args = [&]() {
    mrag_knn::GenericSearch ga{};
    ga.x16 = (const _Float16*)ix->x16.p;
    ga.x32 = (const float*)ix->x32.p;
    ga.xn = (const double*)ix->xn.p;
    ga.labels = (const int32_t*)ix->labels.p;
    ga.n = ix->n;
    ga.D = D;
    ga.DP = DP;
    ga.q16 = (const _Float16*)c->q16.p;
    ga.q32 = (const float*)c->q32.p;
    ga.qn = (const double*)c->qn.p;
    ga.nq = (int)nq;
    ga.k = k;
    ga.label_filter = label_filter;
    ga.row_offset = row_offset;
    ga.out_s = os;
    ga.out_s64 = os64;
    ga.out_r = orr;
    return ga;
  };

  if (ix->n == 0) {
    hipLaunchKernelGGL(fill_empty_kernel, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, s, os, os64,
                       orr, nout);
    MRAG_CHECK_LAUNCH();
  } else if (DP > 512 || k > MAX_K) {
    // K7g (knn_generic.hip): widths and depths the fused scan does not instantiate
    const float* qsrc = queries;
    if (host) {
      if (int rc = ensure(c->qin, (size_t)nq * D * 4)) return rc;
      MRAG_HIP(hipMemcpyAsync(c->qin.p, queries, (size_t)nq * D * 4, hipMemcpyHostToDevice, s));
      qsrc = (const float*)c->qin.p;
    }
    if (int rc = ensure(c->q32, (size_t)nq * DP * 4)) return rc;
    if (int rc = ensure(c->qn, (size_t)nq * 8)) return rc;
    if (int rc = ensure(c->q16, (size_t)nq * DP * 2)) return rc;
    if (int rc = launch_prep(qsrc, nq, D, DP, nq, (float*)c->q32.p, (double*)c->qn.p, (_Float16*)c->q16.p, s))
      return rc;
    if (int rc = mrag_knn::search_generic(generic_args(), c->gws, s, nullptr)) return rc;
  } else {
    // v3 (MFMA 16x16x32, 64 queries per wave, per-lane lists of 6 folded to 8 per split) unless
    // k is deep enough to want longer per-lane lists (v1). For 32 < k <= 64 the union of the S
    // split lists still holds S * 8 >= k + 32 candidates at the batch sizes that matter, and the
    // certificate sends any query whose top-k a list could not hold to the collect pass.
    const bool use_v3 = k <= 64;
    const int qb = use_v3 ? scan3_qb(nq) : 4;
    const int qpg = use_v3 ? 64 * qb : QPG;  // queries per scan workgroup
    // query slots: v3 reads every slot of its query group (no lane guard), so pad to a whole
    // group; padding rows are zero (prep) and never reach the output
    const int64_t qpad = use_v3 ? qpg : QPW;
    const int64_t Qp = (nq + qpad - 1) / qpad * qpad;
    const int qgroups = (int)((Qp + qpg - 1) / qpg);
    const int ntiles = (int)((ix->n + TILE_ROWS - 1) / TILE_ROWS);
    const int KL = use_v3 ? 8 : kl_for(k, DP);
    int S = std::max(1, 256 / qgroups);
    S = std::min(S, ntiles);
    S = std::min(S, MAX_MERGE_ENTRIES / KL);
    if (S >= 8) S &= ~7;
    const int M = std::min<int>(k + 32, S * KL);
    const int R = (int)next_pow2((int64_t)S * KL);
    const int Mp = (int)next_pow2(std::max(M, 2));
    info[0] = S;
    info[1] = (int32_t)Qp;
    info[7] = KL;

    const float* qsrc = queries;
    if (host) {
      if (int rc = ensure(c->qin, (size_t)nq * D * 4)) return rc;
      MRAG_HIP(hipMemcpyAsync(c->qin.p, queries, (size_t)nq * D * 4, hipMemcpyHostToDevice, s));
      qsrc = (const float*)c->qin.p;
    }
    if (int rc = ensure(c->q32, (size_t)Qp * DP * 4)) return rc;
    if (int rc = ensure(c->qn, (size_t)Qp * 8)) return rc;
    if (int rc = ensure(c->q16, (size_t)Qp * DP * 2)) return rc;
    if (int rc = ensure(c->part_s, (size_t)S * Qp * KL * 4)) return rc;
    if (int rc = ensure(c->part_i, (size_t)S * Qp * KL * 4)) return rc;
    if (int rc = ensure(c->thresh, (size_t)Qp * 4)) return rc;
    if (int rc = ensure(c->fail_list, (size_t)Qp * 4)) return rc;
    if (int rc = ensure(c->counters, 16)) return rc;
    if (int rc = ensure(c->cand_cnt, (size_t)Qp * 4)) return rc;
    if (int rc = ensure(c->theta, (size_t)Qp * 4)) return rc;
    if (use_v3)
      if (int rc = ensure(c->part_tau, (size_t)S * Qp * 4)) return rc;

    if (int rc = launch_prep(qsrc, nq, D, DP, Qp, (float*)c->q32.p, (double*)c->qn.p, (_Float16*)c->q16.p, s,
                             PrepClear{(int32_t*)c->counters.p, (int32_t*)c->cand_cnt.p, (uint32_t*)c->theta.p}))
      return rc;

    ScanParams sp{};
    sp.theta = (uint32_t*)c->theta.p;

    sp.x16 = (const _Float16*)ix->x16.p;
    sp.labels = (const int32_t*)ix->labels.p;
    sp.q16 = (const _Float16*)c->q16.p;
    sp.ntiles = ntiles;
    sp.qgroups = qgroups;
    sp.splits = S;
    sp.Qp = (int)Qp;
    sp.label_filter = label_filter;
    sp.part_s = (float*)c->part_s.p;
    sp.part_i = (int32_t*)c->part_i.p;
    sp.fail_list = (const int32_t*)c->fail_list.p;
    sp.fail_cnt = (const int32_t*)c->counters.p;
    sp.thresh = (const float*)c->thresh.p;
    sp.cand_cnt = (int32_t*)c->cand_cnt.p;
    sp.k = k;
    sp.part_tau = use_v3 ? (float*)c->part_tau.p : nullptr;

    const scan_fn scan = use_v3 ? get_scan3(DP, false, qb) : get_scan(DP, KL, false);
    const scan_fn collect = get_scan(DP, 8, true);
    if (!scan || !collect) return mrag::fail(MRAG_ERR_UNSUPPORTED, "no scan kernel for DP=%d", DP);
    const dim3 sgrid((unsigned)(qgroups * S));
    // Sample pre-pass (v3, when every split has >= 4 * SAMPLE_STRIDE tiles): seeds the shared
    // threshold near the k-th best so the main scan's list insertions stay rare. Four maxima per
    // (split, query), one per lane group (merging them in pairs, the round-1 seed, measured 0.2 %
    // slower in the main scan); stride 16 (32: +5 %, 64: +14 %, none: +70 % scan time). K7s
    // (qb == 1) streams at the HBM rate, where the pre-pass costs more than the inserts it saves
    // (Q = 1: 0.270 -> 0.247 ms without it, notes/knn_scan_experiments.md).
    const int min_tiles = ntiles / S;
    const int stride = sample_stride_for(k);
    if (use_v3 && qb == 4 && min_tiles >= 4 * stride) {
      sp.sample_stride = stride;
      sp.sample_tiles = min_tiles / stride;
      hipLaunchKernelGGL(get_scan3(DP, true, qb), sgrid, dim3(SCAN2_THREADS), 0, s, sp);
      MRAG_CHECK_LAUNCH();
      hipLaunchKernelGGL(theta_init_kernel, dim3((unsigned)nq), dim3(64), 0, s, (const float*)sp.part_s, 4 * S,
                         (int)Qp, k, sp.theta);
      MRAG_CHECK_LAUNCH();
    }
    if (profile) MRAG_HIP(hipEventRecord(c->ev0, s));
    hipLaunchKernelGGL(scan, sgrid, dim3(use_v3 ? SCAN2_THREADS : SCAN_THREADS), 0, s, sp);
    MRAG_CHECK_LAUNCH();
    if (profile) MRAG_HIP(hipEventRecord(c->ev1, s));

    MergeParams mp{};
    mp.part_s = sp.part_s;
    mp.part_i = sp.part_i;
    mp.splits = S;
    mp.KL = KL;
    mp.Qp = (int)Qp;
    mp.nq = (int)nq;
    mp.k = k;
    mp.M = M;
    mp.R = R;
    mp.Mp = Mp;
    mp.q32 = (const float*)c->q32.p;
    mp.qn = (const double*)c->qn.p;
    mp.x32 = (const float*)ix->x32.p;
    mp.xn = (const double*)ix->xn.p;
    mp.D = D;
    mp.DP = DP;
    mp.out_s = os;
    mp.out_s64 = os64;
    mp.out_r = orr;
    mp.row_offset = row_offset;
    mp.thresh = (float*)c->thresh.p;
    mp.fail_list = (int32_t*)c->fail_list.p;
    mp.fail_cnt = (int32_t*)c->counters.p;
    mp.theta = (const uint32_t*)c->theta.p;
    mp.part_tau = sp.part_tau;
    mp.host_fail = c->host_fail;
    __atomic_store_n(c->host_fail, 0, __ATOMIC_RELAXED);  // this context's previous search has completed
    // K8 key selection: the best M + 1 keys (the M candidates and the first one left out) by
    // the register top-64P fold when they fit, else the full bitonic sort (40.6 -> 36.5 us per
    // 1000-query search for the fold)
    const int sel = M + 1 <= 64 ? 1 : (M + 1 <= 128 ? 2 : 0);
    mp.R = sel ? std::max(R, 4 * 64 * sel) : R;  // the fold parks four waves' top-64P in keys[]
    const size_t msh = (size_t)mp.R * 8 + (size_t)Mp * 12 + (size_t)DP * 4 + 64;
    auto merge = sel == 1 ? knn_merge_kernel<1> : sel == 2 ? knn_merge_kernel<2> : knn_merge_kernel<0>;
    hipLaunchKernelGGL(merge, dim3((unsigned)nq), dim3(MERGE_THREADS), msh, s, mp);
    MRAG_CHECK_LAUNCH();

    // The failure count after K8: a failing query also raises the context's coherent host word,
    // so the common search (every query certified) ends with the stream wait alone and the count
    // is copied back only when the word is set (the 8-byte copy was a 4.4 us kernel per search);
    // the common search launches nothing more; otherwise K7c's grid is sized to the failing queries alone, with
    // more splits than the main scan (one failing query over the main scan's 64 splits is one
    // 8-wave workgroup per split, latency-bound on its own LDS-DMA round trips: 0.3 ms over
    // 512k rows, notes/knn_scan_experiments.md)
    if (int rc = wait_stream(c, s)) return rc;
    if (__atomic_load_n(c->host_fail, __ATOMIC_ACQUIRE)) {
      MRAG_HIP(hipMemcpyAsync(c->host_counters, c->counters.p, 8, hipMemcpyDeviceToHost, s));
      if (int rc = wait_stream(c, s)) return rc;
    } else {
      c->host_counters[0] = 0;
    }
    if (profile) {
      float ms = 0.f;
      MRAG_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
      std::lock_guard<std::mutex> lk(ix->pool_mu);
      ix->scan_ms += ms;
      ix->scan_launches++;
    }
    uncertified = c->host_counters[0];
    if (uncertified > 0) {
      // per-slot collect capacity of this search (K7c/K10 for the uncertified queries): at
      // most 4096 rows and 64M slots in all; a query that collects more (a run of more than
      // ccap near-duplicates within eps of its k-th score) sends the batch to K7g below,
      // whose per-query storage is sized from a histogram — nothing grows across searches
      const int ccap = (int)std::max<int64_t>(256, std::min<int64_t>(4096, ((int64_t)64 << 20) / Qp));
      if (int rc = ensure(c->cand, (size_t)Qp * ccap * 4)) return rc;
      if (int rc = ensure(c->scratch, (size_t)Qp * ccap * 8)) return rc;
      sp.cand = (int32_t*)c->cand.p;
      sp.ccap = ccap;
      // K7c: QPG failing queries per workgroup, about 1024 workgroups in all
      const int cgroups = (int)((uncertified + QPG - 1) / QPG);
      int Sc = std::max(S, 1024 / cgroups);
      Sc = std::min(Sc, ntiles);
      if (Sc >= 8) Sc &= ~7;
      sp.qgroups = cgroups;
      sp.splits = Sc;
      info[2] = cgroups;
      info[3] = Sc;
      info[4] = ccap;
      info[5] = (int32_t)uncertified;
      hipLaunchKernelGGL(collect, dim3((unsigned)(cgroups * Sc)), dim3(SCAN_THREADS), 0, s, sp);
      MRAG_CHECK_LAUNCH();
      FinalParams fp{};
      fp.fail_list = sp.fail_list;
      fp.fail_cnt = sp.fail_cnt;
      fp.cand_cnt = sp.cand_cnt;
      fp.cand = sp.cand;
      fp.ccap = ccap;
      fp.scratch = (double*)c->scratch.p;
      fp.q32 = mp.q32;
      fp.qn = mp.qn;
      fp.x32 = mp.x32;
      fp.xn = mp.xn;
      fp.D = D;
      fp.DP = DP;
      fp.k = k;
      fp.out_s = os;
      fp.out_s64 = os64;
      fp.out_r = orr;
      fp.row_offset = row_offset;
      fp.overflow = (int32_t*)c->counters.p + 1;
      hipLaunchKernelGGL(knn_final_kernel, dim3((unsigned)uncertified), dim3(MERGE_THREADS), (size_t)DP * 4, s, fp);
      MRAG_CHECK_LAUNCH();
      MRAG_HIP(hipMemcpyAsync(c->host_counters, c->counters.p, 8, hipMemcpyDeviceToHost, s));
      if (int rc = wait_stream(c, s)) return rc;
      info[6] = c->host_counters[1];
      if (c->host_counters[1] != 0) {
        retries = 1;
        if (int rc = mrag_knn::search_generic(generic_args(), c->gws, s, nullptr)) return rc;
      }
    }
  }

  if (host) {
    MRAG_HIP(hipMemcpyAsync(out_scores, os, nout * 4, hipMemcpyDeviceToHost, s));
    MRAG_HIP(hipMemcpyAsync(out_rows, orr, nout * 8, hipMemcpyDeviceToHost, s));
    if (out_scores64) MRAG_HIP(hipMemcpyAsync(out_scores64, os64, nout * 8, hipMemcpyDeviceToHost, s));
  }
  if (int rc = wait_stream(c, s)) return rc;
  drain.armed = false;
  std::lock_guard<std::mutex> lk(ix->pool_mu);
  ix->last_uncertified = uncertified;
  ix->last_retries = retries;
  ix->last_ctx = c;
  std::copy(info, info + 8, ix->last_info);
  return MRAG_OK;
}

#ifdef MRAG_K7_STAMPS
// Diagnostic build only (make stamp; not in mrag.h, not in the shipped libmrag.so): the
// collect-pass bookkeeping of the index's last search, for scripts/knn_collect_diag.py. Valid
// only while no other search runs on the index: it reads the last search's context buffers.
// info[8] = S, Qp, cgroups, Sc, ccap, uncertified, overflow flag, KL; fail_list / cand_cnt get
// the first `uncertified` slots, thresh the first `nthresh` queries (any pointer may be NULL).
__attribute__((visibility("default"))) int mrag_debug_knn_last_collect(mrag_knn_index* ix, int32_t* info,
                                                                       int32_t* fail_list, int32_t* cand_cnt,
                                                                       float* thresh, int64_t nthresh) {
  MRAG_REQUIRE(ix != nullptr && info != nullptr, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->pool_mu);
  std::copy(ix->last_info, ix->last_info + 8, info);
  SearchCtx* c = ix->last_ctx;
  if (!c) return MRAG_OK;
  mrag::DeviceGuard g(ix->device);
  const int64_t unc = ix->last_info[5];
  MRAG_HIP(hipDeviceSynchronize());
  if (fail_list && unc > 0) MRAG_HIP(hipMemcpy(fail_list, c->fail_list.p, unc * 4, hipMemcpyDeviceToHost));
  if (cand_cnt && unc > 0) MRAG_HIP(hipMemcpy(cand_cnt, c->cand_cnt.p, unc * 4, hipMemcpyDeviceToHost));
  if (thresh && nthresh > 0 && (size_t)nthresh * 4 <= c->thresh.bytes)
    MRAG_HIP(hipMemcpy(thresh, c->thresh.p, nthresh * 4, hipMemcpyDeviceToHost));
  return MRAG_OK;
}
#endif

int mrag_topk_merge(const double* scores64, const int64_t* rows, int32_t nlists, int64_t nq, int32_t k,
                    float* out_scores, double* out_scores64, int64_t* out_rows, void* stream) {
  MRAG_REQUIRE(nlists >= 1 && nq >= 0 && k >= 1 && k <= mrag_knn::GENERIC_MAX_K, "bad shape nlists=%d nq=%lld k=%d", nlists,
               (long long)nq, k);
  if (nq == 0) return MRAG_OK;
  MRAG_REQUIRE(scores64 && rows && out_scores && out_rows, "NULL pointer");
  MRAG_REQUIRE(nq < (1ll << 31), "too many queries");
  hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)nq), dim3(MERGE_THREADS), 0, (hipStream_t)stream,
                     scores64, rows, nlists, nq, k, out_scores, out_scores64, out_rows);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}

}  // extern "C"
