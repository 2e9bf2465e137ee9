// l2norm.hip — K6: row L2-normalise, bit-identical to the reference's numpy call.
//
// Reference: app/ml/embeddings.py:46-49
//     norms = np.linalg.norm(embeddings, axis=1, keepdims=True)
//     norms[norms == 0] = 1.0
//     return embeddings / norms
// np.linalg.norm(axis=1) on f32 is sqrt(np.add.reduce(x*x, axis=1)); numpy's
// add.reduce over a contiguous row is its pairwise summation (blocks of <=128
// elements with 8 strided accumulators, halves split at n/2 rounded down to a
// multiple of 8). Reproducing that order (and f32 rounding of every product and
// partial sum, no FMA contraction) makes this kernel's output bit-identical to
// numpy's (checked by tests/test_knn_gpu.py::test_l2norm_bit_exact). Built with
// -ffp-contract=off: hipcc otherwise fuses x*x + r into v_fmac_f32.
//
// Work is tiny (B rows x 512 after an encoder batch), so one thread owns a row;
// the kernel is latency-bound by design and never on the critical path.
#include "common.h"

namespace {

#pragma clang fp contract(off)

// numpy pairwise_sum leaf (n <= 128).
__device__ float pw_leaf(const float* __restrict__ x, int n) {
  if (n < 8) {
    float r = -0.0f;
    for (int i = 0; i < n; ++i) r = __fadd_rn(r, __fmul_rn(x[i], x[i]));
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = __fmul_rn(x[j], x[j]);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], __fmul_rn(x[i + j], x[i + j]));
  }
  float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                        __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
  for (; i < n; ++i) res = __fadd_rn(res, __fmul_rn(x[i], x[i]));
  return res;
}

// Iterative form of numpy's recursive pairwise_sum (depth <= 24).
__device__ float pw_sumsq(const float* __restrict__ x, int n) {
  int off[24], len[24], st[24];
  float val[24];
  int fp = 0, vp = 0;
  off[0] = 0; len[0] = n; st[0] = 0;
  while (fp >= 0) {
    const int o = off[fp], m = len[fp];
    if (m <= 128) {
      val[vp++] = pw_leaf(x + o, m);
      --fp;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    if (st[fp] == 0) {
      st[fp] = 1;
      ++fp; off[fp] = o; len[fp] = n2; st[fp] = 0;
    } else if (st[fp] == 1) {
      st[fp] = 2;
      ++fp; off[fp] = o + n2; len[fp] = m - n2; st[fp] = 0;
    } else {
      const float b = val[--vp];
      const float a = val[--vp];
      val[vp++] = __fadd_rn(a, b);
      --fp;
    }
  }
  return val[0];
}

// numpy's recursion splits n > 128 at n2 = (n/2) - (n/2)%8, so for 128 < n <= 1024 the
// leaves are 2..8 blocks of 64..128 elements for n <= 968 (checked on the host for every n);
// n <= 128 is a single leaf.
struct Leaves {
  int n;
  int off[8], len[8];
};

__device__ void leaves_of(int off, int n, Leaves& L) {
  if (n <= 128) {
    L.off[L.n] = off;
    L.len[L.n] = n;
    ++L.n;
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  // depth <= 3 for n <= 1024: unrolled recursion through a tiny explicit stack
  int so[8], sn[8], sp = 0;
  so[sp] = off + n2; sn[sp++] = n - n2;
  so[sp] = off; sn[sp++] = n2;
  while (sp) {
    const int o = so[--sp], m = sn[sp];
    if (m <= 128) {
      L.off[L.n] = o;
      L.len[L.n] = m;
      ++L.n;
    } else {
      int h = m / 2;
      h -= h % 8;
      so[sp] = o + h; sn[sp++] = m - h;
      so[sp] = o; sn[sp++] = h;
    }
  }
}

// Tree combination of the leaf sums in numpy's order: (left + right) recursively.
__device__ float combine(const float* leaf, int off, int n, int& li) {
  if (n <= 128) return leaf[li++];
  int n2 = n / 2;
  n2 -= n2 % 8;
  const float a = combine(leaf, off, n2, li);
  const float b = combine(leaf, off + n2, n - n2, li);
  return __fadd_rn(a, b);
}

// Compile-time leaf table and combination tree for the encoder widths (no runtime recursion:
// the generic path below compiles to calls with a scratch stack).
struct LeafTab {
  int n;
  int off[8], len[8];
};
constexpr void leaves_rec(LeafTab& t, int off, int n) {
  if (n <= 128) {
    t.off[t.n] = off;
    t.len[t.n] = n;
    ++t.n;
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  leaves_rec(t, off, n2);
  leaves_rec(t, off + n2, n - n2);
}
constexpr LeafTab leaves_for(int dim) {
  LeafTab t{};
  leaves_rec(t, 0, dim);
  return t;
}
constexpr bool leaves_whole_octets(int dim) {  // every leaf a multiple of 8, >= 8 (no tails)
  const LeafTab t = leaves_for(dim);
  for (int i = 0; i < t.n; ++i)
    if (t.len[i] < 8 || t.len[i] % 8) return false;
  return true;
}
constexpr int leaf_at(const LeafTab& t, int off) {
  for (int i = 0; i < t.n; ++i)
    if (t.off[i] == off) return i;
  return -1;
}
template <int DIM, int OFF, int N>
__device__ __forceinline__ float combine_ct(const float (&lv)[8]) {
  if constexpr (N <= 128) {
    constexpr int i = leaf_at(leaves_for(DIM), OFF);
    static_assert(i >= 0, "leaf table");
    return lv[i];
  } else {
    constexpr int N2 = N / 2 - (N / 2) % 8;
    return __fadd_rn(combine_ct<DIM, OFF, N2>(lv), combine_ct<DIM, OFF + N2, N - N2>(lv));
  }
}

// One wave per row, DIM known at compile time (128 < DIM <= 1024, DIM % 8 == 0: every
// leaf is 64..128 elements, a multiple of 8). Lane 8 leaf + j owns accumulator j of leaf
// `leaf`; the leaf value ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) and the tree follow numpy.
template <int DIM>
__global__ __launch_bounds__(256) void l2norm_rows_ct_kernel(const float* x, float* y, int64_t rows) {
  constexpr LeafTab L = leaves_for(DIM);
  static_assert(L.n <= 8 && leaves_whole_octets(DIM), "<= 8 leaves, no leaf tails");
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * DIM;
  float* yr = y + r * DIM;
  const int leaf = lane >> 3, j = lane & 7;
  float acc = 0.f;
  int loff = 0, llen = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (q == leaf && q < L.n) {
      loff = L.off[q];
      llen = L.len[q];
    }
  if (llen) {
    const float* p = xr + loff;
    acc = __fmul_rn(p[j], p[j]);
    for (int i = j + 8; i < llen; i += 8) acc = __fadd_rn(acc, __fmul_rn(p[i], p[i]));
  }
  const int b = lane & ~7;
  float rr[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) rr[q] = __shfl(acc, b + q);
  const float lv0 = __fadd_rn(__fadd_rn(__fadd_rn(rr[0], rr[1]), __fadd_rn(rr[2], rr[3])),
                              __fadd_rn(__fadd_rn(rr[4], rr[5]), __fadd_rn(rr[6], rr[7])));
  float lv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) lv[q] = __shfl(lv0, 8 * q);
  const float ss = combine_ct<DIM, 0, DIM>(lv);
  float nrm = (float)sqrt((double)ss);  // correctly rounded f32 sqrt (see the generic kernel)
  if (nrm == 0.0f) nrm = 1.0f;
  for (int d = lane; d < DIM; d += 64) yr[d] = __fdiv_rn(xr[d], nrm);  // IEEE f32 division = numpy's
}

// One wave per row. Lane 8*leaf + j owns accumulator j of leaf `leaf` (numpy keeps 8
// strided accumulators per leaf); leaf and tree combinations follow numpy's order exactly.
__global__ __launch_bounds__(256) void l2norm_rows_wave_kernel(const float* x, float* y,  // may alias
                                                               int64_t rows, int dim) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * dim;
  float* yr = y + r * dim;
  Leaves L;
  L.n = 0;
  leaves_of(0, dim, L);
  const int leaf = lane >> 3, j = lane & 7;
  float acc = 0.f;
  if (leaf < L.n && L.len[leaf] >= 8) {
    const float* p = xr + L.off[leaf];
    const int full = L.len[leaf] - L.len[leaf] % 8;
    acc = __fmul_rn(p[j], p[j]);
    for (int i = j + 8; i < full; i += 8) acc = __fadd_rn(acc, __fmul_rn(p[i], p[i]));
  }
  // leaf value on lane 8*leaf: ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail in order
  const int b = lane & ~7;
  const float r0 = __shfl(acc, b + 0), r1 = __shfl(acc, b + 1), r2 = __shfl(acc, b + 2), r3 = __shfl(acc, b + 3);
  const float r4 = __shfl(acc, b + 4), r5 = __shfl(acc, b + 5), r6 = __shfl(acc, b + 6), r7 = __shfl(acc, b + 7);
  float lv = 0.f;
  if (j == 0 && leaf < L.n) {
    const float* p = xr + L.off[leaf];
    const int n = L.len[leaf];
    if (n < 8) {
      lv = -0.0f;
      for (int i = 0; i < n; ++i) lv = __fadd_rn(lv, __fmul_rn(p[i], p[i]));
    } else {
      lv = __fadd_rn(__fadd_rn(__fadd_rn(r0, r1), __fadd_rn(r2, r3)), __fadd_rn(__fadd_rn(r4, r5), __fadd_rn(r6, r7)));
      for (int i = n - n % 8; i < n; ++i) lv = __fadd_rn(lv, __fmul_rn(p[i], p[i]));
    }
  }
  float leafv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) leafv[q] = __shfl(lv, 8 * q);
  int li = 0;
  const float ss = combine(leafv, 0, dim, li);
  // v_sqrt_f32 is 1-ulp; sqrt and division are evaluated in f64 and rounded once
  // to f32, which is the correctly rounded f32 result (53 >= 2*24 + 2).
  float nrm = (float)sqrt((double)ss);
  if (nrm == 0.0f) nrm = 1.0f;
  for (int d = lane; d < dim; d += 64) yr[d] = (float)((double)xr[d] / (double)nrm);
}

__global__ void l2norm_rows_kernel(const float* x, float* y,  // may alias
                                   int64_t rows, int dim) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* xr = x + r * dim;
  float* yr = y + r * dim;
  float nrm = (float)sqrt((double)pw_sumsq(xr, dim));
  if (nrm == 0.0f) nrm = 1.0f;
  for (int d = 0; d < dim; ++d) yr[d] = (float)((double)xr[d] / (double)nrm);
}

}  // namespace

extern "C" int mrag_l2norm_rows(const float* x, float* y, int64_t rows, int32_t dim,
                                void* stream) {
  MRAG_REQUIRE(rows >= 0 && dim > 0, "bad shape rows=%lld dim=%d", (long long)rows, dim);
  MRAG_REQUIRE(dim <= (1 << 20), "dim %d too large", dim);
  if (rows == 0) return MRAG_OK;
  MRAG_REQUIRE(x != nullptr && y != nullptr, "NULL pointer");
  if (dim == 384 || dim == 512 || dim == 768) {  // the encoders' widths: compile-time tree
    const int64_t blocks = (rows + 3) / 4;
    MRAG_REQUIRE(blocks < (1ll << 31), "too many rows");
    auto k = dim == 384 ? l2norm_rows_ct_kernel<384> : dim == 512 ? l2norm_rows_ct_kernel<512> : l2norm_rows_ct_kernel<768>;
    hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, y, rows);
  } else if (dim <= 968) {  // wave per row: numpy splits dims <= 968 into <= 8 leaves of <= 128
    const int64_t blocks = (rows + 3) / 4;
    MRAG_REQUIRE(blocks < (1ll << 31), "too many rows");
    hipLaunchKernelGGL(l2norm_rows_wave_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, y,
                       rows, (int)dim);
  } else {  // thread per row, generic recursion
    const int threads = 64;
    const int64_t blocks = (rows + threads - 1) / threads;
    MRAG_REQUIRE(blocks < (1ll << 31), "too many rows");
    hipLaunchKernelGGL(l2norm_rows_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, x, y,
                       rows, (int)dim);
  }
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}
