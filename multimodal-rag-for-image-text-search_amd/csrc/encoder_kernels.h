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
};

struct GemmArgs {
  const _Float16* A;  // [M][lda]
  const _Float16* W;  // [N][ldw]
  const float* bias;  // [N] or null
  void* C;            // [M][ldc] f16 or f32 per epilogue
  int M, N, K, lda, ldw, ldc;
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

// kernel: GEMM_AUTO (the rule in launch_gemm) or one kernel forced (A/B timing, bit-identity tests)
enum GemmKernel { GEMM_AUTO = 0, GEMM_K3 = 1, GEMM_K3D = 2, GEMM_K3S = 3, GEMM_K3W = 4 };
int launch_gemm(const GemmArgs& g, int epi, hipStream_t s, int kernel = GEMM_AUTO);
bool gemm_ws_fits(const GemmArgs& g, int epi);
int launch_layernorm(const LayerNormArgs& a, hipStream_t s);
int launch_attention(const AttentionArgs& a, int dh, hipStream_t s);
int launch_vit_im2col(const uint8_t* img, _Float16* out, int B, int S, int P, hipStream_t s);
int launch_vit_embed_ln(const float* patch, const float* cls, const float* pos, const float* gamma, const float* beta,
                        float* X, int B, int T, int D, float eps, hipStream_t s);
int launch_token_embed(const int32_t* ids, const float* tok, const float* pos, const float* type_tab,
                       const int32_t* types, float* X, int B, int T, int D, int vocab, hipStream_t s);
int launch_cls_head(const float* pooled, const float* Wc, const float* bc, float* out, int B, int D, int NL,
                    hipStream_t s);
int launch_eos_rows(const int32_t* ids, int B, int T, int eos_id, int* rows, hipStream_t s);
int launch_cls_rows(int B, int T, int* rows, hipStream_t s);
int launch_gather_rows(const void* src, void* dst, const int* rows, int B, int row_bytes, hipStream_t s);
int launch_mean_pool(const float* X, const int32_t* mask, float* out, int B, int T, int D, hipStream_t s);

}  // namespace mrag_enc
