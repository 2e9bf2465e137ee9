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
  EPI_F16_SWISH_LIB = 5,   // C16 = swish(alpha acc + bias), hipBLASLt only (image-tower fc1, blaslt.cpp)
};

struct GemmArgs {
  const _Float16* A;  // [M][lda]
  const _Float16* W;  // [N][ldw]
  const float* bias;  // [N] or null
  void* C;            // [M][ldc] f16 or f32 per epilogue
  int M, N, K, lda, ldw, ldc;
  int lib_ok;         // the call may run on hipBLASLt (plain epilogues, M >= 4096: blaslt.cpp)
  float alpha;        // C = alpha acc (+ ...): hipBLASLt only; 0 or 1 = none (K3 / K3d have none)
  // K3d stream-K workspace (set by the launcher): f32 partial tiles [2 * grid][256 * 256], an
  // arrival ticket per tile and a ready flag per partial slot (all zero between launches)
  float* sk_part;
  int* sk_cnt;
  int* sk_flag;
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
// plain epilogues (bias, residual, f32) on hipBLASLt where selected (blaslt.cpp)
bool blaslt_eligible(const GemmArgs& g, int epi);
bool blaslt_takes(int M);  // the library is selected and M is large enough (image tower)
int set_blaslt_mode(int mode);
int launch_gemm_blaslt(const GemmArgs& g, int epi, hipStream_t s);
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
