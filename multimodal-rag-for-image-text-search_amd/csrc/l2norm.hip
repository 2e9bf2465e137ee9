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

__global__ void l2norm_rows_kernel(const float* x, float* y,  // may alias
                                   int64_t rows, int dim) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* xr = x + r * dim;
  float* yr = y + r * dim;
  // v_sqrt_f32 is 1-ulp; sqrt and division are evaluated in f64 and rounded once
  // to f32, which is the correctly rounded f32 result (53 >= 2*24 + 2).
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
  const int threads = 64;
  const int64_t blocks = (rows + threads - 1) / threads;
  MRAG_REQUIRE(blocks < (1ll << 31), "too many rows");
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3((unsigned)blocks), dim3(threads), 0,
                     (hipStream_t)stream, x, y, rows, (int)dim);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}
