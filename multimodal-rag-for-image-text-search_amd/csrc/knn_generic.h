// knn_generic.h — K7g: the exact flat-cosine search for configurations the fused scan
// (knn.hip K7/K8) does not instantiate: embedding widths above 512 (e.g. 768-d ViT-L/14 or
// MPNet, 1024-d, up to 4096) and k above 256. The reference accepts both
// (app/storage/lancedb_store.py:33-44 stores list<float32> of any length; :110,121 pass
// limit(max(top_k, 1)) straight through), so the drop-in must too.
#pragma once

#include "common.h"

namespace mrag_knn {

constexpr int GENERIC_MAX_DIM = 4096;
constexpr int GENERIC_MAX_K = 65536;

struct Workspace {
  void* p = nullptr;
  size_t bytes = 0;
};

struct GenericSearch {
  // corpus (the index's buffers): rows padded to DP, labels padded to a multiple of 256
  const _Float16* x16;
  const float* x32;
  const double* xn;
  const int32_t* labels;
  int64_t n;
  int D, DP;
  // prepared queries: q16 = fp16(q/|q|) [Qp][DP], q32 [Qp][DP], qn [Qp]
  const _Float16* q16;
  const float* q32;
  const double* qn;
  int nq;
  int k;
  int32_t label_filter;
  int64_t row_offset;
  // outputs (device) [nq][k]
  float* out_s;
  double* out_s64;  // may be null
  int64_t* out_r;
};

// |approx - exact| bound of an fp16-input, f32-accumulated dot product of two unit vectors
// of width D (DESIGN.md §3.3 generalised): fp16 rounding of both operands (2u + u^2,
// u = 2^-11), f32 accumulation (D * 2^-24), fp16 subnormal flush (2 sqrt(D) 2^-25), f32
// normalisation slack.
double eps_for_dim(int D);

// Exact rescoring helper shared by K8, K10 and K7g (one definition, so every path orders
// ties on bit-identical f64 scores): one aligned 16-lane group computes q.x in f64 — lane
// `sub` of the group accumulates the float4 chunks sub, sub + 16, ... in ascending order,
// then a fixed 4-step butterfly: deterministic — and returns the cosine on every lane of
// the group (0 when a norm is 0).
__device__ __forceinline__ double exact_cosine16(const float* qs, double qn, const float* __restrict__ x32,
                                                 const double* __restrict__ xn, int64_t row, int D, int DP, int sub) {
  const f32x4* xr = (const f32x4*)(x32 + (size_t)row * DP);
  const f32x4* q4 = (const f32x4*)qs;
  const int nc = (D + 3) >> 2;  // chunks; DP % 4 == 0, so the last chunk stays inside the row
  double acc = 0.0;
#pragma unroll 8
  for (int c = sub; c < nc; c += 16) {
    const f32x4 xv = xr[c], qv = q4[c];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (4 * c + t < D) acc = fma((double)qv[t], (double)xv[t], acc);
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  const double xnr = xn[row];
  return (qn > 0.0 && xnr > 0.0) ? acc / (qn * xnr) : 0.0;
}

// Two GEMM passes over the corpus (score histogram -> per-query collect threshold ->
// candidate collection -> exact f64 rescoring + ordered selection). Exact for every input;
// the per-query candidate storage is sized from the histogram (never by a global cap).
// `ws` holds 8 reusable device buffers; *n_candidates (optional) receives the total number
// of rows rescored exactly.
int search_generic(const GenericSearch& a, Workspace (&ws)[8], hipStream_t s, int64_t* n_candidates);

void release(Workspace (&ws)[8]);

}  // namespace mrag_knn
