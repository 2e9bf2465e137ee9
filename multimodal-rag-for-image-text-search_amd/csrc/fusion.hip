// fusion.hip — K12: the reference's z-score fusion of text and image hits, on the GPU,
// bit-identical to the host restatement (app.retrieval.fuse_scores) and therefore to
// app/ml/retrieve.py:158-195 (rerank off):
//
//   _format_results (app/storage/lancedb_store.py:125-139): score = 1.0 - float(f32(1 - s))
//   _z_scores: arr = np.array(scores, float32); mean = float(arr.mean()); std = float(arr.std())
//              std == 0 -> zeros; else (v - mean) / std in f64 on the f64 score v
//   _fuse_results: text items then image items, combined = their z, stable sort descending,
//              keep final_n.
//
// numpy's f32 reductions are reproduced exactly: add.reduce over a contiguous array is its
// pairwise summation (leaves of <= 128 elements with 8 strided accumulators, halves split at
// n/2 rounded down to a multiple of 8; the same order as K6, l2norm.hip); mean = sum / n and
// var = sum((x - mean)^2) / n with every product, difference and partial sum rounded to f32
// (no FMA contraction), std = correctly rounded f32 sqrt. One wave per query (see the kernel),
// which removes the host fusion (~5 ms per 1000 queries in numpy) from the config-5 step.
#include "common.h"

namespace {

#pragma clang fp contract(off)

// element i of a hit list as the reference's _z_scores sees it: f32 of the caller's f64 score
struct Hits {
  const float* s;
  __device__ double s64(int i) const { return 1.0 - (double)__fsub_rn(1.0f, s[i]); }
  __device__ float f32(int i) const { return (float)s64(i); }
};

struct SqDev {  // (x_i - mean)^2 in f32, numpy's _var order
  Hits h;
  float mean;
  __device__ float operator()(int i) const {
    const float d = __fsub_rn(h.f32(i), mean);
    return __fmul_rn(d, d);
  }
};

struct Plain {
  Hits h;
  __device__ float operator()(int i) const { return h.f32(i); }
};

template <class F>
__device__ float pw_leaf(const F& f, int o, int n) {
  if (n < 8) {
    float r = -0.0f;
    for (int i = 0; i < n; ++i) r = __fadd_rn(r, f(o + i));
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f(o + j);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], f(o + i + j));
  }
  float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                        __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
  for (; i < n; ++i) res = __fadd_rn(res, f(o + i));
  return res;
}

// numpy's recursive pairwise_sum, iteratively (depth <= 24)
template <class F>
__device__ float pw_sum(const F& f, int n) {
  int off[24], len[24], st[24];
  float val[24];
  int fp = 0, vp = 0;
  off[0] = 0;
  len[0] = n;
  st[0] = 0;
  while (fp >= 0) {
    const int o = off[fp], m = len[fp];
    if (m <= 128) {
      val[vp++] = pw_leaf(f, o, m);
      --fp;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    if (st[fp] == 0) {
      st[fp] = 1;
      ++fp;
      off[fp] = o;
      len[fp] = n2;
      st[fp] = 0;
    } else if (st[fp] == 1) {
      st[fp] = 2;
      ++fp;
      off[fp] = o + n2;
      len[fp] = m - n2;
      st[fp] = 0;
    } else {
      const float b = val[--vp];
      const float a = val[--vp];
      val[vp++] = __fadd_rn(a, b);
      --fp;
    }
  }
  return val[0];
}

// (mean, std) of the list's f32 values as numpy computes them; f32 division and sqrt are
// evaluated in f64 and rounded once (the correctly rounded f32 result: 53 >= 2 * 24 + 2)
__device__ void np_mean_std(const Hits& h, int n, double& mean, double& std) {
  const float m = (float)((double)pw_sum(Plain{h}, n) / (double)n);
  const float v = (float)((double)pw_sum(SqDev{h, m}, n) / (double)n);
  mean = (double)m;
  std = (double)(float)sqrt((double)v);
}

// One wave per query: lane 0 reproduces numpy's mean / std (serial pairwise order, a few
// hundred dependent adds), every lane computes the z of its items, and the stable top-final_n
// is final_n wave-wide (max z, min position) reductions — no per-thread scans of the list.
__global__ __launch_bounds__(256) void fuse_kernel(const float* __restrict__ ts, int kt, const float* __restrict__ is,
                                                   int ki, int64_t nq, int final_n, int64_t* __restrict__ pick,
                                                   double* __restrict__ combined) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;  // whole wave
  const Hits th{ts + q * kt}, ih{is + q * ki};
  int nt = 0, ni = 0;  // valid hits (finite scores) form the prefix of each list
  for (int b = 0; b < kt; b += 64) nt += __popcll(__ballot(b + lane < kt && isfinite(th.s[b + lane])));
  for (int b = 0; b < ki; b += 64) ni += __popcll(__ballot(b + lane < ki && isfinite(ih.s[b + lane])));
  double st[4] = {0, 0, 0, 0};  // text mean, std, image mean, std
  if (lane == 0) {
    if (nt) np_mean_std(th, nt, st[0], st[1]);
    if (ni) np_mean_std(ih, ni, st[2], st[3]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t bits = __shfl(__double_as_longlong(st[i]), 0);
    st[i] = __longlong_as_double(bits);
  }
  const int n = nt + ni;
  auto z = [&](int c) -> double {  // combined score of concatenated item c (c < nt + ni)
    if (c < nt) return st[1] == 0.0 ? 0.0 : (th.s64(c) - st[0]) / st[1];
    const int j = c - nt;
    return st[3] == 0.0 ? 0.0 : (ih.s64(j) - st[2]) / st[3];
  };
  // stable descending sort, first final_n: repeated "best after the previous pick" under
  // (combined desc, position asc); positions index the concatenated [text kt | image ki] list
  double pz = INFINITY;
  int pc = -1;
  for (int slot = 0; slot < final_n; ++slot) {
    double bz = -INFINITY;
    int bc = -1;
    for (int c = lane; c < n; c += 64) {
      const double zc = z(c);
      const bool after = pc < 0 || zc < pz || (zc == pz && c > pc);
      if (after && (bc < 0 || zc > bz)) {  // c ascends per lane: ties keep the first
        bz = zc;
        bc = c;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double oz = __longlong_as_double(__shfl_xor(__double_as_longlong(bz), off));
      const int oc = __shfl_xor(bc, off);
      if (oc >= 0 && (bc < 0 || oz > bz || (oz == bz && oc < bc))) {
        bz = oz;
        bc = oc;
      }
    }
    if (bc < 0) {  // fewer than final_n hits: the rest of the row is padding
      for (int r = slot + lane; r < final_n; r += 64) {
        pick[(size_t)q * final_n + r] = -1;
        combined[(size_t)q * final_n + r] = NAN;
      }
      break;
    }
    if (lane == 0) {
      pick[(size_t)q * final_n + slot] = bc < nt ? bc : kt + (bc - nt);
      combined[(size_t)q * final_n + slot] = bz;
    }
    pz = bz;
    pc = bc;
  }
}

}  // namespace

extern "C" int mrag_fuse_scores(const float* text_scores, int32_t kt, const float* image_scores, int32_t ki,
                                int64_t nq, int32_t final_n, int64_t* pick, double* combined, void* stream) {
  MRAG_REQUIRE(kt >= 0 && ki >= 0 && nq >= 0 && final_n >= 0, "bad shape kt=%d ki=%d nq=%lld final_n=%d", kt, ki,
               (long long)nq, final_n);
  if (nq == 0 || final_n == 0) return MRAG_OK;
  MRAG_REQUIRE(pick && combined && (kt == 0 || text_scores) && (ki == 0 || image_scores), "NULL pointer");
  MRAG_REQUIRE(nq < (1ll << 30), "too many queries");
  hipLaunchKernelGGL(fuse_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, (hipStream_t)stream, text_scores,
                     kt, image_scores, ki, nq, final_n, pick, combined);
  MRAG_CHECK_LAUNCH();
  return MRAG_OK;
}
