// blaslt.cpp — the encoders' plain GEMMs (bias, f32 residual accumulate, f32 out) on hipBLASLt,
// the vendor library, at the batch sizes where it is measured faster than the hand-written K3 /
// K3d (M >= 4096 rows; notes/gemm_experiments.md), for the CLIP image tower only (GemmArgs::lib_ok):
// the text towers keep the hand-written kernels everywhere, so a query's embedding — and with it
// retrieve_batch == retrieve() — does not depend on its batch. The image tower's fc1 (quick_gelu)
// runs as the library's swish: quick_gelu(z) = swish(1.702 z) / 1.702, so fc1 takes alpha = 1.702
// and a bias pre-scaled by 1.702, and fc2 takes alpha = 1 / 1.702 (encoder.hip clip_layer); the
// erf GELU (BERT) has no library form and stays on K3 / K3d.
//
// Row-major C[M][N] = A[M][K] . W[N][K]^T (+ bias[N]) (+ C for the residual) is the column-major
// product D (N x M, ld = ldc) = op_T(W: K x N, ld = ldw) . op_N(A: K x M, ld = lda), bias along D's
// rows. One plan (descriptors + the heuristic's first algorithm) per shape and epilogue, built
// once under a lock; one workspace per HIP stream (a stream-K algorithm keeps partial tiles
// there, so two streams never share one), sized to the largest plan that stream has run.
#include <hipblaslt/hipblaslt.h>

#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "encoder_kernels.h"

namespace mrag_enc {
namespace {

constexpr size_t WS_BYTES = 64ull << 20;

struct Plan {
  bool ok = false;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

struct State {
  std::mutex mu;
  bool init = false, usable = false;
  hipblasLtHandle_t h = nullptr;
  std::map<std::tuple<int, int, int, int, int, int, int, bool>, Plan> plans;
  struct Ws {
    void* p = nullptr;
    size_t bytes = 0;
  };
  std::map<hipStream_t, Ws> ws;
};
// one state per device: a hipBLASLt handle (and the algorithms it picks) belongs to the device
// that was current when it was created, and a process may drive several
State& st() {
  static std::mutex mu;
  static std::map<int, State> per_dev;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  return per_dev[dev];  // std::map nodes are stable
}

bool build_plan(State& S, const GemmArgs& g, int epi, Plan& p) {
  const bool f32 = epi == EPI_F32_RESIDUAL || epi == EPI_F32;
  const hipDataType dt = f32 ? HIP_R_32F : HIP_R_16F;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  const int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  if (epi == EPI_F16_SWISH_LIB) {
    const uint32_t e = g.bias ? HIPBLASLT_EPILOGUE_SWISH_BIAS_EXT : HIPBLASLT_EPILOGUE_SWISH_EXT;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  } else if (g.bias) {
    const uint32_t e = HIPBLASLT_EPILOGUE_BIAS;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  }
  if (g.bias) {
    const int32_t bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16F, g.K, g.N, g.ldw) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16F, g.K, g.M, g.lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, dt, g.N, g.M, g.ldc) != HIPBLAS_STATUS_SUCCESS)
    return false;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
  const uint64_t wsb = WS_BYTES;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t rc = hipblasLtMatmulAlgoGetHeuristic(S.h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (rc != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS) return false;
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  return p.ws <= WS_BYTES;
}

}  // namespace

// 0 = hand-written K3 / K3d only, 1 = hipBLASLt for the plain epilogues at M >= 4096 (default;
// MRAG_GEMM_BLASLT=0 in the environment, or mrag_gemm_set_library(0), selects 0)
std::atomic<int> g_mode{-1};
int blaslt_mode() {
  int m = g_mode.load(std::memory_order_relaxed);
  if (m < 0) {
    const char* e = std::getenv("MRAG_GEMM_BLASLT");
    int want = (e && std::atoi(e) == 0) ? 0 : 1;
    g_mode.compare_exchange_strong(m, want);
    m = g_mode.load(std::memory_order_relaxed);
  }
  return m;
}
int set_blaslt_mode(int mode) {
  const int prev = blaslt_mode();
  g_mode.store(mode ? 1 : 0);
  return prev;
}

bool blaslt_takes(int M) {
  // large-M calls only: small batches keep the hand-written kernels, and with them a row's result
  // independent of its batch size there
  return blaslt_mode() != 0 && M >= 4096;
}

bool blaslt_eligible(const GemmArgs& g, int epi) {
  if (!g.lib_ok || (epi != EPI_F16 && epi != EPI_F32_RESIDUAL && epi != EPI_F32 && epi != EPI_F16_SWISH_LIB))
    return false;
  return blaslt_takes(g.M);
}

// MRAG_OK, or MRAG_ERR_UNSUPPORTED when the library has no algorithm for the shape (the caller
// then runs K3 / K3d).
int launch_gemm_blaslt(const GemmArgs& g, int epi, hipStream_t s) {
  State& S = st();
  Plan* plan = nullptr;
  void* ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(S.mu);
    if (!S.init) {
      S.init = true;
      S.usable = hipblasLtCreate(&S.h) == HIPBLAS_STATUS_SUCCESS;
    }
    if (!S.usable) return MRAG_ERR_UNSUPPORTED;
    const auto key = std::make_tuple(epi, g.M, g.N, g.K, g.lda, g.ldw, g.ldc, g.bias != nullptr);
    auto it = S.plans.find(key);
    if (it == S.plans.end()) {
      Plan p;
      p.ok = build_plan(S, g, epi, p);
      it = S.plans.emplace(key, p).first;
    }
    if (!it->second.ok) return MRAG_ERR_UNSUPPORTED;
    plan = &it->second;
    if (plan->ws > 0) {
      State::Ws& w = S.ws[s];
      if (w.bytes < plan->ws) {  // grow: the stream's earlier calls may still be reading the old one
        if (w.p) {
          (void)hipStreamSynchronize(s);
          (void)hipFree(w.p);
          w.p = nullptr;
          w.bytes = 0;
        }
        if (hipMalloc(&w.p, plan->ws) != hipSuccess) {
          w.p = nullptr;
          return MRAG_ERR_UNSUPPORTED;
        }
        w.bytes = plan->ws;
      }
      ws = w.p;
    }
  }
  // the bias pointer is per call (a shape's plan serves every layer), so it is set on the shared
  // descriptor under the lock, right before the launch that reads it
  // D = act(alpha (W A) + beta C + bias): the bias is not scaled by alpha
  const float alpha = g.alpha != 0.f ? g.alpha : 1.f, beta = epi == EPI_F32_RESIDUAL ? 1.f : 0.f;
  std::lock_guard<std::mutex> lk(S.mu);
  if (g.bias)
    hipblasLtMatmulDescSetAttribute(plan->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &g.bias, sizeof(g.bias));
  const hipblasStatus_t rc = hipblasLtMatmul(S.h, plan->desc, &alpha, g.W, plan->la, g.A, plan->lb, &beta, g.C,
                                             plan->lc, g.C, plan->lc, &plan->algo, ws, plan->ws, s);
  if (rc != HIPBLAS_STATUS_SUCCESS) return mrag::fail(MRAG_ERR_HIP, "hipblasLtMatmul failed (%d)", (int)rc);
  return MRAG_OK;
}

}  // namespace mrag_enc
