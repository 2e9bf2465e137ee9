// knn_generic.hip — K7g: exact flat cosine top-k for any width up to 4096 and any k up to
// 65536 (the configurations the fused K7/K8 scan does not instantiate; knn_generic.h).
//
// Per block of queries (all on the search stream):
//   pass 1, per corpus chunk: approx scores S[q][row] = fp16(q^) . fp16(x^) on MFMA (the
//          encoder GEMM, f32 accumulate) -> per-query 2048-bin histogram of the scores of the
//          rows the label filter admits (LDS histogram per workgroup, flushed with atomics);
//   K7g-t: per query, the highest bin b0 whose cumulative count from the top reaches k:
//          >= k rows have approx >= L(b0) - w, so the k-th exact score e_k >= L(b0) - w - eps
//          and every row of the exact top-k has approx >= L(b0) - w - 2 eps =: thr. The
//          histogram also bounds how many rows reach thr: that sizes the query's candidate
//          slice exactly (prefix sum on the host), so no global capacity can overflow;
//   pass 2, per corpus chunk (per sub-range of queries whose candidates fit the budget):
//          the same GEMM -> collect every admitted row with approx >= thr;
//   K7g-f: exact f64 rescoring of the candidates (mrag_knn::exact_cosine16, the same
//          arithmetic as K8/K10) and ordered selection (score desc, row asc): bitonic sort in
//          LDS up to 2048 candidates, k rounds of block arg-max beyond.
// Exact by construction for every input (duplicates and ties included): the candidate set
// is a superset of the exact top-k.
#include <algorithm>
#include <vector>

#include "encoder_kernels.h"
#include "knn_generic.h"

namespace mrag_knn {

namespace {

constexpr int HIST_BINS = 2048;
constexpr float HIST_LO = -1.0625f;  // scores of unit vectors (plus eps) lie in [-1.0625, 1.0625)
constexpr float HIST_SPAN = 2.125f;
constexpr int GF_THREADS = 256;
constexpr int GF_SORT_MAX = 2048;  // LDS sort capacity (12 B each; + the query row, <= 40 KiB)
constexpr size_t SCORE_BUDGET = (size_t)512 << 20;  // bytes of S per chunk
constexpr int64_t CAND_BUDGET = (int64_t)96 << 20;   // candidates per collect sub-range (12 B each)
constexpr int QBLOCK = 8192;                          // queries per histogram block

__device__ __forceinline__ int hist_bin(float s) {
  const float t = (fminf(fmaxf(s, HIST_LO), -HIST_LO) - HIST_LO) * (HIST_BINS / HIST_SPAN);
  return min(HIST_BINS - 1, max(0, (int)t));
}

__device__ __forceinline__ bool label_ok(int32_t lab, int32_t filter) {
  return filter == MRAG_LABEL_ANY ? lab >= 0 : lab == filter;
}

// One workgroup = one query row of S x one slice of the chunk's columns.
__global__ __launch_bounds__(256) void score_hist_kernel(const float* __restrict__ S, int ncols,
                                                         const int32_t* __restrict__ labels, int32_t filter,
                                                         uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[HIST_BINS];
  for (int i = threadIdx.x; i < HIST_BINS; i += 256) h[i] = 0;
  __syncthreads();
  const int qi = blockIdx.x;
  const float* srow = S + (size_t)qi * ncols;
  const int per = ((ncols + gridDim.y - 1) / gridDim.y + 3) & ~3;
  const int c0 = blockIdx.y * per, c1 = min(ncols, c0 + per);
  for (int c = c0 + 4 * (int)threadIdx.x; c < c1; c += 1024) {
    const f32x4 v = *(const f32x4*)(srow + c);
    const int4 lab = *(const int4*)(labels + c);
    if (label_ok(lab.x, filter)) atomicAdd(&h[hist_bin(v[0])], 1u);
    if (label_ok(lab.y, filter)) atomicAdd(&h[hist_bin(v[1])], 1u);
    if (label_ok(lab.z, filter)) atomicAdd(&h[hist_bin(v[2])], 1u);
    if (label_ok(lab.w, filter)) atomicAdd(&h[hist_bin(v[3])], 1u);
  }
  __syncthreads();
  uint32_t* hq = hist + (size_t)qi * HIST_BINS;
  for (int i = threadIdx.x; i < HIST_BINS; i += 256)
    if (h[i]) atomicAdd(hq + i, h[i]);
}

// One wave per query: lane l owns the 32 bins [BINS - 32 (l + 1), BINS - 32 l) (lane 0 the top).
__global__ __launch_bounds__(64) void hist_threshold_kernel(const uint32_t* __restrict__ hist, int k, float eps2w,
                                                            float* __restrict__ thr, int32_t* __restrict__ bound) {
  constexpr int PER = HIST_BINS / 64;
  const int qi = blockIdx.x, lane = threadIdx.x;
  const uint32_t* hq = hist + (size_t)qi * HIST_BINS + (HIST_BINS - PER * (lane + 1));
  uint32_t v[PER];
  uint64_t mine = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = hq[j];
    mine += v[j];
  }
  uint64_t incl = mine;  // inclusive prefix from the top (lane 0 first)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  const uint64_t total = __shfl(incl, 63);
  float t_q = -INFINITY;
  int bthr = 0;
  if (total > (uint64_t)k) {
    const uint64_t reach = __ballot(incl >= (uint64_t)k);
    const int l0 = __builtin_ctzll(reach);
    int b0 = 0;
    if (lane == l0) {
      uint64_t c = incl - mine;
      for (int j = PER - 1; j >= 0; --j) {  // bins from the top of this lane's range down
        c += v[j];
        if (c >= (uint64_t)k) {
          b0 = HIST_BINS - PER * (lane + 1) + j;
          break;
        }
      }
    }
    b0 = __shfl(b0, l0);
    const double lb = (double)HIST_LO + (double)b0 * ((double)HIST_SPAN / HIST_BINS);
    float f = (float)(lb - (double)eps2w);
    if ((double)f > lb - (double)eps2w) f = nextafterf(f, -INFINITY);
    t_q = f;
    bthr = max(0, hist_bin(t_q) - 1);
  }
  // rows with approx >= t_q sit in bins >= bin(t_q) >= bthr: their count bounds the collect
  uint64_t cnt = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (HIST_BINS - PER * (lane + 1) + j >= bthr) cnt += v[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) {
    thr[qi] = t_q;
    bound[qi] = (int32_t)min<uint64_t>(cnt, 0x7fffffffull);
  }
}

__global__ __launch_bounds__(256) void score_collect_kernel(const float* __restrict__ S, int ncols, int64_t row0,
                                                            const int32_t* __restrict__ labels, int32_t filter,
                                                            const float* __restrict__ thr,
                                                            const int64_t* __restrict__ off,
                                                            int32_t* __restrict__ cnt, int32_t* __restrict__ cand) {
  const int qi = blockIdx.x;
  const float t = thr[qi];
  const float* srow = S + (size_t)qi * ncols;
  const int per = ((ncols + gridDim.y - 1) / gridDim.y + 3) & ~3;
  const int c0 = blockIdx.y * per, c1 = min(ncols, c0 + per);
  const int64_t base = off[qi];
  const int cap = (int)(off[qi + 1] - base);
  for (int c = c0 + 4 * (int)threadIdx.x; c < c1; c += 1024) {
    const f32x4 v = *(const f32x4*)(srow + c);
    const int4 lab = *(const int4*)(labels + c);
    const int32_t lv[4] = {lab.x, lab.y, lab.z, lab.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (label_ok(lv[j], filter) && v[j] >= t) {
        const int pos = atomicAdd(cnt + qi, 1);
        if (pos < cap) cand[base + pos] = (int32_t)(row0 + c + j);  // pos < cap always (histogram bound)
      }
    }
  }
}

struct FinalParams {
  const int64_t* off;
  const int32_t* cnt;
  const int32_t* cand;
  double* scratch;
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

__device__ void block_best(double& bs, int64_t& br) {
  __shared__ double rs[GF_THREADS / 64];
  __shared__ int64_t rr[GF_THREADS / 64];
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
  for (int i = 1; i < GF_THREADS / 64; ++i)
    if (mrag_before(rs[i], rr[i], bs, br)) {
      bs = rs[i];
      br = rr[i];
    }
}

__device__ __forceinline__ void put(const FinalParams& p, size_t o, double s, int64_t r) {
  p.out_s[o] = r >= 0 ? (float)s : -INFINITY;
  if (p.out_s64) p.out_s64[o] = r >= 0 ? s : -INFINITY;
  p.out_r[o] = r >= 0 ? r + p.row_offset : -1;
}

// K7g-f: one workgroup per query of the sub-range (outputs at row qi of the block's outputs).
__global__ __launch_bounds__(GF_THREADS) void generic_final_kernel(FinalParams p) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  float* qs = (float*)dsm;                                   // [DP]
  double* ss = (double*)(dsm + (size_t)p.DP * 4);            // [GF_SORT_MAX]
  int32_t* sr = (int32_t*)(ss + GF_SORT_MAX);                // [GF_SORT_MAX]
  const int qi = blockIdx.x, tid = threadIdx.x;
  const int64_t base = p.off[qi];
  int n = p.cnt[qi];
  const int cap = (int)(p.off[qi + 1] - base);
  if (n > cap) {  // cannot happen (histogram bound); reported, never silent
    if (tid == 0) atomicOr(p.overflow, 1);
    n = cap;
  }
  for (int d = tid; d < p.DP; d += GF_THREADS) qs[d] = p.q32[(size_t)qi * p.DP + d];
  __syncthreads();
  const double qn = p.qn[qi];
  const int32_t* cr = p.cand + base;
  double* sc = p.scratch + base;
  const size_t obase = (size_t)qi * p.k;
  if (n <= GF_SORT_MAX) {
    int P = 1;
    while (P < n) P <<= 1;
    for (int m = tid >> 4; m < P; m += GF_THREADS / 16) {
      if (m < n) {
        const double s = exact_cosine16(qs, qn, p.x32, p.xn, cr[m], p.D, p.DP, tid & 15);
        if ((tid & 15) == 0) {
          ss[m] = s;
          sr[m] = cr[m];
        }
      } else if ((tid & 15) == 0) {
        ss[m] = -INFINITY;
        sr[m] = -1;
      }
    }
    for (int size = 2; size <= P; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        __syncthreads();
        for (int i = tid; i < (P >> 1); i += GF_THREADS) {
          const int lo = 2 * i - (i & (stride - 1));
          const int hi = lo + stride;
          const bool asc = (lo & size) == 0;
          const double sa = ss[lo], sb = ss[hi];
          const int ra = sr[lo], rb = sr[hi];
          if (mrag_before(sb, rb, sa, ra) == asc) {
            ss[lo] = sb; sr[lo] = rb;
            ss[hi] = sa; sr[hi] = ra;
          }
        }
      }
    }
    __syncthreads();
    for (int j = tid; j < p.k; j += GF_THREADS) put(p, obase + j, j < n ? ss[j] : -INFINITY, j < n ? sr[j] : -1);
    return;
  }
  for (int m = tid >> 4; m < n; m += GF_THREADS / 16) {
    const double s = exact_cosine16(qs, qn, p.x32, p.xn, cr[m], p.D, p.DP, tid & 15);
    if ((tid & 15) == 0) sc[m] = s;
  }
  __syncthreads();
  double ps = INFINITY;
  int64_t pr = -1;
  for (int j = 0; j < p.k; ++j) {
    double bs = -INFINITY;
    int64_t br = -1;
    for (int m = tid; m < n; m += GF_THREADS) {
      const double s = sc[m];
      const int64_t r = cr[m];
      if ((pr < 0 || mrag_before(ps, pr, s, r)) && mrag_before(s, r, bs, br)) {
        bs = s;
        br = r;
      }
    }
    block_best(bs, br);
    if (tid == 0) put(p, obase + j, bs, br);
    if (br < 0) {
      for (int jj = j + 1 + tid; jj < p.k; jj += GF_THREADS) put(p, obase + jj, -INFINITY, -1);
      break;
    }
    ps = bs;
    pr = br;
  }
}

int ensure(Workspace& b, size_t bytes) {
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

int gemm_scores(const GenericSearch& a, int q_lo, int mq, int64_t r0, int ncols, float* S, hipStream_t s) {
  mrag_enc::GemmArgs g{};
  g.A = a.q16 + (size_t)q_lo * a.DP;
  g.W = a.x16 + (size_t)r0 * a.DP;
  g.bias = nullptr;
  g.C = S;
  g.M = mq;
  g.N = ncols;
  g.K = a.DP;
  g.lda = a.DP;
  g.ldw = a.DP;
  g.ldc = ncols;
  return mrag_enc::launch_gemm(g, mrag_enc::EPI_F32, s);
}

}  // namespace

double eps_for_dim(int D) {
  const double u = std::ldexp(1.0, -11);
  const double e = (2.0 * u + u * u) + D * std::ldexp(1.0, -24) + 2.0 * std::sqrt((double)D) * std::ldexp(1.0, -25) +
                   4e-6;
  return std::max(1.05e-3, e * 1.02);
}

void release(Workspace (&ws)[8]) {
  for (auto& w : ws) {
    if (w.p) (void)hipFree(w.p);
    w.p = nullptr;
    w.bytes = 0;
  }
}

int search_generic(const GenericSearch& a, Workspace (&ws)[8], hipStream_t s, int64_t* n_candidates) {
  MRAG_REQUIRE(a.DP % 128 == 0 && a.DP <= GENERIC_MAX_DIM && a.D <= a.DP, "K7g: dim %d unsupported", a.D);
  MRAG_REQUIRE(a.k >= 1 && a.k <= GENERIC_MAX_K, "K7g: k=%d unsupported (1..%d)", a.k, GENERIC_MAX_K);
  if (n_candidates) *n_candidates = 0;
  if (a.nq == 0) return MRAG_OK;
  const double eps = eps_for_dim(a.D);
  const float eps2w = (float)(2.0 * eps + (double)HIST_SPAN / HIST_BINS);
  const int64_t ncols_total = (a.n + 127) / 128 * 128;  // the index's capacity is a multiple of 256
  const int lds_final = a.DP * 4 + GF_SORT_MAX * 12;
  for (int qb = 0; qb < a.nq; qb += QBLOCK) {
    const int mq = std::min(QBLOCK, a.nq - qb);
    const int64_t ch = std::max<int64_t>(
        128, std::min<int64_t>(ncols_total, (int64_t)(SCORE_BUDGET / ((size_t)mq * 4)) / 128 * 128));
    if (int rc = ensure(ws[0], (size_t)mq * ch * 4)) return rc;                 // S
    if (int rc = ensure(ws[1], (size_t)mq * HIST_BINS * 4)) return rc;          // hist
    if (int rc = ensure(ws[2], (size_t)mq * 4)) return rc;                      // thr
    if (int rc = ensure(ws[3], (size_t)mq * 4)) return rc;                      // bound
    if (int rc = ensure(ws[4], (size_t)(mq + 1) * 8)) return rc;                // off
    if (int rc = ensure(ws[5], (size_t)mq * 4 + 16)) return rc;                 // cnt (+ overflow word)
    float* S = (float*)ws[0].p;
    uint32_t* hist = (uint32_t*)ws[1].p;
    float* thr = (float*)ws[2].p;
    int32_t* bound = (int32_t*)ws[3].p;
    int64_t* off = (int64_t*)ws[4].p;
    int32_t* cnt = (int32_t*)ws[5].p;
    int32_t* overflow = cnt + mq;
    MRAG_HIP(hipMemsetAsync(hist, 0, (size_t)mq * HIST_BINS * 4, s));
    const int ysplit = std::max(1, std::min<int>((int)(ch / 4096), 64));
    for (int64_t r0 = 0; r0 < ncols_total; r0 += ch) {
      const int nc = (int)std::min<int64_t>(ch, ncols_total - r0);
      if (int rc = gemm_scores(a, qb, mq, r0, nc, S, s)) return rc;
      hipLaunchKernelGGL(score_hist_kernel, dim3((unsigned)mq, (unsigned)ysplit), dim3(256), 0, s, S, nc,
                         a.labels + r0, a.label_filter, hist);
      MRAG_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(hist_threshold_kernel, dim3((unsigned)mq), dim3(64), 0, s, hist, a.k, eps2w, thr, bound);
    MRAG_CHECK_LAUNCH();
    std::vector<int32_t> hb((size_t)mq);
    MRAG_HIP(hipMemcpyAsync(hb.data(), bound, (size_t)mq * 4, hipMemcpyDeviceToHost, s));
    MRAG_HIP(hipStreamSynchronize(s));
    // sub-ranges of queries whose candidate slices fit the budget (a larger single query alone)
    int lo = 0;
    while (lo < mq) {
      int hi = lo;
      int64_t tot = 0;
      while (hi < mq && (hi == lo || tot + hb[hi] <= CAND_BUDGET)) tot += hb[hi++];
      std::vector<int64_t> ho((size_t)(hi - lo + 1));
      ho[0] = 0;
      for (int i = lo; i < hi; ++i) ho[i - lo + 1] = ho[i - lo] + hb[i];
      if (n_candidates) *n_candidates += tot;
      if (int rc = ensure(ws[6], (size_t)std::max<int64_t>(tot, 1) * 4)) return rc;  // cand
      if (int rc = ensure(ws[7], (size_t)std::max<int64_t>(tot, 1) * 8)) return rc;  // scratch
      MRAG_HIP(hipMemcpyAsync(off, ho.data(), ho.size() * 8, hipMemcpyHostToDevice, s));
      MRAG_HIP(hipMemsetAsync(cnt, 0, (size_t)mq * 4 + 16, s));
      const int m = hi - lo;
      const int ch2 = (int)std::max<int64_t>(
          128, std::min<int64_t>(ncols_total, (int64_t)(SCORE_BUDGET / ((size_t)m * 4)) / 128 * 128));
      for (int64_t r0 = 0; r0 < ncols_total; r0 += ch2) {
        const int nc = (int)std::min<int64_t>(ch2, ncols_total - r0);
        if (int rc = gemm_scores(a, qb + lo, m, r0, nc, S, s)) return rc;
        const int ys = std::max(1, std::min<int>(nc / 4096, 64));
        hipLaunchKernelGGL(score_collect_kernel, dim3((unsigned)m, (unsigned)ys), dim3(256), 0, s, S, nc, r0,
                           a.labels + r0, a.label_filter, thr + lo, off, cnt, (int32_t*)ws[6].p);
        MRAG_CHECK_LAUNCH();
      }
      FinalParams fp{};
      fp.off = off;
      fp.cnt = cnt;
      fp.cand = (const int32_t*)ws[6].p;
      fp.scratch = (double*)ws[7].p;
      fp.q32 = a.q32 + (size_t)(qb + lo) * a.DP;
      fp.qn = a.qn + qb + lo;
      fp.x32 = a.x32;
      fp.xn = a.xn;
      fp.D = a.D;
      fp.DP = a.DP;
      fp.k = a.k;
      fp.out_s = a.out_s + (size_t)(qb + lo) * a.k;
      fp.out_s64 = a.out_s64 ? a.out_s64 + (size_t)(qb + lo) * a.k : nullptr;
      fp.out_r = a.out_r + (size_t)(qb + lo) * a.k;
      fp.row_offset = a.row_offset;
      fp.overflow = overflow;
      hipLaunchKernelGGL(generic_final_kernel, dim3((unsigned)m), dim3(GF_THREADS), lds_final, s, fp);
      MRAG_CHECK_LAUNCH();
      int32_t ovf = 0;
      MRAG_HIP(hipMemcpyAsync(&ovf, overflow, 4, hipMemcpyDeviceToHost, s));
      MRAG_HIP(hipStreamSynchronize(s));
      if (ovf) return mrag::fail(MRAG_ERR_STATE, "K7g: candidate bound violated (internal error)");
      lo = hi;
    }
  }
  return MRAG_OK;
}

}  // namespace mrag_knn
