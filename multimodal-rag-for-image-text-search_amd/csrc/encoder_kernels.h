// encoder_kernels.h — argument blocks and launchers of the encoder kernels (K1..K5).
#pragma once

#include "common.h"

namespace mrag_enc {

enum Epilogue {
  EPI_F16 = 0,             // C16 = acc + bias
  EPI_F16_QUICK_GELU = 1,  // C16 = quick_gelu(acc + bias)       (CLIP MLP fc1)
  EPI_F16_GELU_ERF = 2,    // C16 = gelu_erf(acc + bias)         (BERT intermediate)
  EPI_F32_RESIDUAL = 3,    // C32 += acc + bias                  (out-proj / fc2 into the residual)
  EPI_F32 = 4,             // C32 = acc + bias                   (patch embed, projections)
  // LayerNorm folding flags (encoder towers only; not reachable through mrag_gemm_nt):
  // a LayerNorm y = (x - mu) r gamma + beta feeding a GEMM is folded into it: W' = W diag(gamma),
  // bias' = bias + W beta, colsum[n] = sum_k W'[n][k]; the GEMM reads f16(x) (the raw residual
  // stream) and its epilogue applies acc' = r (acc - mu colsum[n]) before bias and activation.
  // mu, r come from per-row partials (sum, M2 = sum of squared deviations from the partial's
  // mean; merged by Chan's formula) that the residual GEMM producing x wrote in its own epilogue,
  // one per 64-column slab, so no LayerNorm pass runs in between.
  EPI_FOLD = 8,    // f16 epilogues: acc' = r (acc - mu colsum) from st_in
  EPI_STATS = 16,  // residual epilogue: also write c16 = f16(C) and st_out partials of C
  EPI_RESLN = 32,  // residual epilogue: the old C is first normalised, C = LN(C) + acc + bias
                   // (post-LN BERT: the residual branch carries the previous LayerNorm's output)
};
constexpr int epi_base(int e) { return e & 7; }

struct GemmArgs {
  const _Float16* A;  // [M][lda]
  const _Float16* W;  // [N][ldw]
  const float* bias;  // [N] or null
  void* C;            // [M][ldc] f16 or f32 per epilogue
  int M, N, K, lda, ldw, ldc;
  // LayerNorm folding (EPI_FOLD / EPI_STATS / EPI_RESLN), null / 0 otherwise
  const float2* st_in;  // [M][st_in_p] (sum, M2 about the partial's mean) of the normalised rows
  int st_in_p;
  int ln_d;             // LayerNorm width (the row length the partials cover)
  float ln_eps;
  const float* colsum;  // [N] EPI_FOLD
  const float* ln_g;    // [N] EPI_RESLN: gamma / beta of the LayerNorm applied to the old C
  const float* ln_b;
  _Float16* c16;        // [M][ldc] EPI_STATS
  float2* st_out;       // [M][N / 64] EPI_STATS
};

struct LayerNormArgs {
  const float* x;      // [*][ldx]
  const int* gather;   // optional: output row r reads input row gather[r]
  float* y32;          // optional [rows][D]
  _Float16* y16;       // optional [rows][D]
  const float* gamma;
  const float* beta;
  int rows, D, ldx;
  float eps;
};

struct AttentionArgs {
  const _Float16* qkv;   // [B*L][3*H*dh]
  _Float16* out;         // [B*L][H*dh]
  const int32_t* mask;   // [B][L] key padding mask (1 = keep) or null
  int B, L, H, causal;
  float scale;
};

int launch_gemm(const GemmArgs& g, int epi, hipStream_t s);
int launch_layernorm(const LayerNormArgs& a, hipStream_t s);
int launch_attention(const AttentionArgs& a, int dh, hipStream_t s);
int launch_vit_im2col(const uint8_t* img, _Float16* out, int B, int S, int P, hipStream_t s);
int launch_vit_embed_ln(const float* patch, const float* cls, const float* pos, const float* gamma, const float* beta,
                        float* X, _Float16* X16, float2* st, int B, int T, int D, float eps, hipStream_t s);
int launch_token_embed(const int32_t* ids, const float* tok, const float* pos, const float* type_tab,
                       const int32_t* types, float* X, _Float16* X16, float2* st, int B, int T, int D, int vocab,
                       hipStream_t s);
int launch_ln_fold_weight(const _Float16* W, const float* gamma, const float* beta, const float* bias, int N, int K,
                          _Float16* Wf, float* bf, float* cs, hipStream_t s);
int launch_cls_head(const float* pooled, const float* Wc, const float* bc, float* out, int B, int D, int NL,
                    hipStream_t s);
int launch_eos_rows(const int32_t* ids, int B, int T, int eos_id, int* rows, hipStream_t s);
int launch_cls_rows(int B, int T, int* rows, hipStream_t s);
int launch_gather_rows(const void* src, void* dst, const int* rows, int B, int row_bytes, hipStream_t s);
int launch_mean_pool(const float* X, const int32_t* mask, float* out, int B, int T, int D, hipStream_t s);

}  // namespace mrag_enc
