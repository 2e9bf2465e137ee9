// encoder.hip — native runner of the three encoders behind include/mrag.h:
//   MRAG_ENC_CLIP_VISION  CLIPModel.get_image_features  (app/ml/embeddings.py:84-91)
//   MRAG_ENC_CLIP_TEXT    CLIPModel.get_text_features   (app/ml/embeddings.py:101-105)
//   MRAG_ENC_BERT         SentenceTransformer(all-MiniLM-L6-v2).encode: BERT + mean pool
//                         (app/ml/embeddings.py:62-70)
//   MRAG_ENC_BERT_PAIR    CrossEncoder(ms-marco-MiniLM-L-6-v2).predict logits:
//                         BertForSequenceClassification (app/ml/retrieve.py:132-155)
// Parameters arrive under their Hugging Face state-dict names (f32 host arrays) and are
// packed once into device buffers: f16 GEMM weights with q|k|v fused into one [3D][D]
// matrix, f32 biases / LayerNorm params / embeddings. A forward is ~7 launches per layer
// on one HIP stream; activations live in a per-handle workspace sized for the largest
// batch seen.
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "encoder_kernels.h"

using namespace mrag_enc;

namespace {

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
};

int buf_ensure(Buf& b, size_t bytes) {
  if (b.p && b.bytes >= bytes) return MRAG_OK;
  if (b.p) MRAG_HIP(hipFree(b.p));
  b.p = nullptr;
  b.bytes = 0;
  MRAG_HIP(hipMalloc(&b.p, std::max<size_t>(bytes, 256)));
  b.bytes = std::max<size_t>(bytes, 256);
  return MRAG_OK;
}

void buf_free(Buf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

struct Layer {
  Buf wqkv, bqkv, wo, bo, w1, b1, w2, b2, ln1g, ln1b, ln2g, ln2b;
};

__global__ void f32_to_f16_kernel(const float* __restrict__ in, _Float16* __restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (_Float16)in[i];
}

}  // namespace

// One forward's activations. A large image batch runs as MRAG_IMG_LANES sub-batches ("lanes"),
// each on its own workspace and stream (see mrag_encoder_embed_images).
#ifndef MRAG_IMG_LANES
#define MRAG_IMG_LANES 2
#endif
#ifndef MRAG_IMG_LANE_MIN
#define MRAG_IMG_LANE_MIN 128
#endif
struct Work {
  Buf X, H16, QKV, ATT, F16, PATCH, IMG, IDS, MASK, TYPES, ROWS, POOL16, OUT, POOL32;
  Buf XG, AG, HG, FG;  // the pooled rows of a CLIP tower's last layer (clip_layer_pooled)
  int64_t ws_tokens = 0, ws_batch = 0;
};

struct mrag_encoder {
  std::mutex mu;
  mrag_encoder_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  std::vector<Layer> layers;
  // embeddings / heads
  Buf patch_w, cls, pos, pre_g, pre_b, post_g, post_b, proj_w;  // vision
  Buf tok, type0, emb_g, emb_b;                                  // text / bert (+pos); type0 = [2][D]
  Buf pool_w, pool_b, cls_w, cls_b;                              // bert pair: pooler + classifier
  std::map<std::string, bool> loaded;
  std::vector<std::string> expected;
  // workspace of a forward: w points at work[0], or at work[i] while image lane i is enqueued
  Work work[MRAG_IMG_LANES];
  Work* w = &work[0];
  // image lanes (mrag_encoder_embed_images): their streams (every lane on one of the handle's
  // own, made together), the fork event and one join event per lane
  hipStream_t lane_stream[MRAG_IMG_LANES] = {};
  hipEvent_t lane_ev[MRAG_IMG_LANES] = {};
  hipEvent_t lane_fork = nullptr;
  // Device-pointer calls return without a host sync (stream-ordered, like any kernel launch):
  // `done` marks the end of the last call's work on `last_stream`; a call on another stream
  // first waits for it (the workspace is shared), and a workspace reallocation first
  // drains it.
  hipEvent_t done = nullptr;
  hipStream_t last_stream = nullptr;
  hipEvent_t null_ev = nullptr;  // device inputs on the NULL stream: the call waits for it
  // Small host-pointer token batches (the reference's one query per retrieve call) replay a
  // captured hipGraph of the forward instead of ~90 individual launches; keyed by shape, valid
  // while the workspace buffers it baked in keep their addresses (`sig`).
  struct Graph {
    hipGraphExec_t exec = nullptr;
    std::vector<const void*> sig;
  };
  std::map<uint64_t, Graph> graphs;
};

namespace {

// Image handles of the process, for the lane decision of mrag_encoder_embed_images: a handle
// that is the only image handle on its device cannot have image calls of other handles beside
// its own. (Asking the runtime whether another handle's last call is still running — an event
// query per call — cost 4-5 % of the three-batches-in-flight rate even where it never split.)
std::mutex g_image_mu;
std::vector<mrag_encoder*> g_image_handles;

bool sole_image_handle(const mrag_encoder* e) {
  std::lock_guard<std::mutex> lk(g_image_mu);
  for (const mrag_encoder* h : g_image_handles)
    if (h != e && h->device == e->device) return false;
  return true;
}

// Upload n floats from host to a device buffer as f32 or f16.
int upload(Buf& b, const float* host, int64_t n, bool to_f16, hipStream_t s) {
  if (!to_f16) {
    if (int rc = buf_ensure(b, (size_t)n * 4)) return rc;
    MRAG_HIP(hipMemcpyAsync(b.p, host, (size_t)n * 4, hipMemcpyHostToDevice, s));
    return MRAG_OK;
  }
  if (int rc = buf_ensure(b, (size_t)n * 2)) return rc;
  void* tmp = nullptr;
  MRAG_HIP(hipMalloc(&tmp, (size_t)n * 4));
  hipError_t e = hipMemcpyAsync(tmp, host, (size_t)n * 4, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(f32_to_f16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float*)tmp,
                       (_Float16*)b.p, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(tmp);
  if (e != hipSuccess) return mrag::fail(MRAG_ERR_HIP, "upload: %s", hipGetErrorString(e));
  return MRAG_OK;
}

// Copy into a slice [off, off+n) of an f16 buffer of `total` elements (fused QKV).
int upload_slice_f16(Buf& b, int64_t total, int64_t off, const float* host, int64_t n, hipStream_t s) {
  if (!b.p) {
    if (int rc = buf_ensure(b, (size_t)total * 2)) return rc;
  }
  void* tmp = nullptr;
  MRAG_HIP(hipMalloc(&tmp, (size_t)n * 4));
  hipError_t e = hipMemcpyAsync(tmp, host, (size_t)n * 4, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(f32_to_f16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float*)tmp,
                       (_Float16*)b.p + off, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(tmp);
  if (e != hipSuccess) return mrag::fail(MRAG_ERR_HIP, "upload: %s", hipGetErrorString(e));
  return MRAG_OK;
}

int upload_slice_f32(Buf& b, int64_t total, int64_t off, const float* host, int64_t n, hipStream_t s) {
  if (!b.p) {
    if (int rc = buf_ensure(b, (size_t)total * 4)) return rc;
  }
  MRAG_HIP(hipMemcpyAsync((float*)b.p + off, host, (size_t)n * 4, hipMemcpyHostToDevice, s));
  MRAG_HIP(hipStreamSynchronize(s));
  return MRAG_OK;
}

bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }

// Expected state-dict names for a config (everything the forward reads).
std::vector<std::string> expected_names(const mrag_encoder_config& c) {
  std::vector<std::string> v;
  if (c.kind == MRAG_ENC_CLIP_VISION || c.kind == MRAG_ENC_CLIP_TEXT) {
    const std::string pre = c.kind == MRAG_ENC_CLIP_VISION ? "vision_model." : "text_model.";
    if (c.kind == MRAG_ENC_CLIP_VISION) {
      for (const char* n : {"embeddings.class_embedding", "embeddings.patch_embedding.weight",
                            "embeddings.position_embedding.weight", "pre_layrnorm.weight", "pre_layrnorm.bias",
                            "post_layernorm.weight", "post_layernorm.bias"})
        v.push_back(pre + n);
      v.push_back("visual_projection.weight");
    } else {
      for (const char* n : {"embeddings.token_embedding.weight", "embeddings.position_embedding.weight",
                            "final_layer_norm.weight", "final_layer_norm.bias"})
        v.push_back(pre + n);
      v.push_back("text_projection.weight");
    }
    for (int i = 0; i < c.layers; ++i) {
      const std::string l = pre + "encoder.layers." + std::to_string(i) + ".";
      for (const char* n : {"self_attn.q_proj.weight", "self_attn.q_proj.bias", "self_attn.k_proj.weight",
                            "self_attn.k_proj.bias", "self_attn.v_proj.weight", "self_attn.v_proj.bias",
                            "self_attn.out_proj.weight", "self_attn.out_proj.bias", "layer_norm1.weight",
                            "layer_norm1.bias", "layer_norm2.weight", "layer_norm2.bias", "mlp.fc1.weight",
                            "mlp.fc1.bias", "mlp.fc2.weight", "mlp.fc2.bias"})
        v.push_back(l + n);
    }
  } else {
    // BertModel names (sentence-transformers checkpoint) or "bert."-prefixed ones under
    // BertForSequenceClassification (the cross-encoder)
    const std::string pre = c.kind == MRAG_ENC_BERT_PAIR ? "bert." : "";
    for (const char* n : {"embeddings.word_embeddings.weight", "embeddings.position_embeddings.weight",
                          "embeddings.token_type_embeddings.weight", "embeddings.LayerNorm.weight",
                          "embeddings.LayerNorm.bias"})
      v.push_back(pre + n);
    if (c.kind == MRAG_ENC_BERT_PAIR)
      for (const char* n : {"bert.pooler.dense.weight", "bert.pooler.dense.bias", "classifier.weight", "classifier.bias"})
        v.push_back(n);
    for (int i = 0; i < c.layers; ++i) {
      const std::string l = pre + "encoder.layer." + std::to_string(i) + ".";
      for (const char* n : {"attention.self.query.weight", "attention.self.query.bias", "attention.self.key.weight",
                            "attention.self.key.bias", "attention.self.value.weight", "attention.self.value.bias",
                            "attention.output.dense.weight", "attention.output.dense.bias",
                            "attention.output.LayerNorm.weight", "attention.output.LayerNorm.bias",
                            "intermediate.dense.weight", "intermediate.dense.bias", "output.dense.weight",
                            "output.dense.bias", "output.LayerNorm.weight", "output.LayerNorm.bias"})
        v.push_back(l + n);
    }
  }
  return v;
}

int64_t expected_numel(const mrag_encoder_config& c, const std::string& name) {
  const int64_t D = c.hidden, I = c.intermediate;
  auto ends = [&](const char* suf) {
    const size_t n = strlen(suf);
    return name.size() >= n && name.compare(name.size() - n, n, suf) == 0;
  };
  if (ends("class_embedding")) return D;
  if (ends("pooler.dense.weight")) return D * D;
  if (ends("classifier.weight")) return (int64_t)c.proj_dim * D;
  if (ends("classifier.bias")) return c.proj_dim;
  if (ends("patch_embedding.weight")) return D * 3 * c.patch_size * c.patch_size;
  if (ends("embeddings.position_embedding.weight") || ends("position_embeddings.weight")) {
    if (c.kind == MRAG_ENC_CLIP_VISION) {
      const int64_t g = c.image_size / c.patch_size;
      return (g * g + 1) * D;
    }
    return (int64_t)c.max_positions * D;
  }
  if (ends("token_embedding.weight") || ends("word_embeddings.weight")) return (int64_t)c.vocab * D;
  if (ends("token_type_embeddings.weight")) return 2 * D;
  if (ends("visual_projection.weight") || ends("text_projection.weight")) return (int64_t)c.proj_dim * D;
  if (ends("fc1.weight") || ends("intermediate.dense.weight")) return I * D;
  if (ends("fc1.bias") || ends("intermediate.dense.bias")) return I;
  if (ends("fc2.weight") || (ends("output.dense.weight") && name.find("attention") == std::string::npos)) return D * I;
  if (ends(".weight") && (name.find("proj.weight") != std::string::npos || name.find("self.query") != std::string::npos ||
                          name.find("self.key") != std::string::npos || name.find("self.value") != std::string::npos ||
                          name.find("attention.output.dense") != std::string::npos))
    return D * D;
  return D;  // biases, LayerNorm params
}

int layer_index(const std::string& name, const std::string& marker) {
  const size_t p = name.find(marker);
  if (p == std::string::npos) return -1;
  return atoi(name.c_str() + p + marker.size());
}

int ensure_workspace(mrag_encoder* e, int B, int T) {
  const int64_t tokens = (int64_t)B * T;
  if (tokens <= e->w->ws_tokens && B <= e->w->ws_batch) return MRAG_OK;
  if (e->last_stream) MRAG_HIP(hipEventSynchronize(e->done));  // in-flight work still reads the old buffers
  const auto& c = e->cfg;
  const int64_t D = c.hidden, I = c.intermediate;
  // per-sequence buffers grow with B, per-token ones with B * T: either can grow alone (the
  // tokenisers pad to the longest sequence of a batch, so B can grow while B * T does not)
  if (B > e->w->ws_batch) {
    if (int rc = buf_ensure(e->w->XG, (size_t)B * D * 4)) return rc;  // pooled rows of the last CLIP layer
    if (int rc = buf_ensure(e->w->AG, (size_t)B * D * 2)) return rc;
    if (int rc = buf_ensure(e->w->HG, (size_t)B * D * 2)) return rc;
    if (int rc = buf_ensure(e->w->FG, (size_t)B * I * 2)) return rc;
    if (int rc = buf_ensure(e->w->ROWS, (size_t)B * 4 + 256)) return rc;
    if (int rc = buf_ensure(e->w->POOL16, (size_t)B * D * 2)) return rc;
    if (c.kind == MRAG_ENC_BERT_PAIR)
      if (int rc = buf_ensure(e->w->POOL32, (size_t)B * D * 4)) return rc;
    e->w->ws_batch = B;
  }
  if (tokens <= e->w->ws_tokens) return MRAG_OK;
  if (int rc = buf_ensure(e->w->X, tokens * D * 4)) return rc;
  if (int rc = buf_ensure(e->w->H16, tokens * D * 2)) return rc;
  if (int rc = buf_ensure(e->w->QKV, tokens * 3 * D * 2)) return rc;
  if (int rc = buf_ensure(e->w->ATT, tokens * D * 2)) return rc;
  int64_t f16n = tokens * I;
  if (c.kind == MRAG_ENC_CLIP_VISION) f16n = std::max<int64_t>(f16n, tokens * 3 * c.patch_size * c.patch_size);
  if (int rc = buf_ensure(e->w->F16, f16n * 2)) return rc;
  if (c.kind == MRAG_ENC_CLIP_VISION) {
    if (int rc = buf_ensure(e->w->PATCH, tokens * D * 4)) return rc;
  }
  e->w->ws_tokens = tokens;
  return MRAG_OK;
}

// GEMM helper: C = A[M][K] . W[N][K]^T (+bias), epilogue
int gemm(const void* A, const void* W, const void* bias, void* C, int M, int N, int K, int ldc, int epi,
         hipStream_t s) {
  GemmArgs g{};
  g.A = (const _Float16*)A;
  g.W = (const _Float16*)W;
  g.bias = (const float*)bias;
  g.C = C;
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = K;
  g.ldw = K;
  g.ldc = ldc;
  return launch_gemm(g, epi, s);
}

int layernorm(const float* x, const int* gather, float* y32, _Float16* y16, const Buf& g, const Buf& b, int rows,
              int D, float eps, hipStream_t s) {
  LayerNormArgs a{};
  a.x = x;
  a.gather = gather;
  a.y32 = y32;
  a.y16 = y16;
  a.gamma = (const float*)g.p;
  a.beta = (const float*)b.p;
  a.rows = rows;
  a.D = D;
  a.ldx = D;
  a.eps = eps;
  return launch_layernorm(a, s);
}

// Pre-LN transformer layer (CLIP): X += attn(LN1(X)); X += mlp(LN2(X)).
int clip_layer(mrag_encoder* e, const Layer& L, int B, int T, const int32_t* mask, int causal, hipStream_t s) {
  const auto& c = e->cfg;
  const int D = c.hidden, I = c.intermediate, M = B * T;
  float* X = (float*)e->w->X.p;
  _Float16* H = (_Float16*)e->w->H16.p;
  if (int rc = layernorm(X, nullptr, nullptr, H, L.ln1g, L.ln1b, M, D, c.ln_eps, s)) return rc;
  if (int rc = gemm(H, L.wqkv.p, L.bqkv.p, e->w->QKV.p, M, 3 * D, D, 3 * D, EPI_F16, s)) return rc;
  AttentionArgs a{};
  a.qkv = (const _Float16*)e->w->QKV.p;
  a.out = (_Float16*)e->w->ATT.p;
  a.mask = mask;
  a.B = B;
  a.L = T;
  a.H = c.heads;
  a.causal = causal;
  a.scale = 1.0f / sqrtf((float)(D / c.heads));
  if (int rc = launch_attention(a, D / c.heads, s)) return rc;
  if (int rc = gemm(e->w->ATT.p, L.wo.p, L.bo.p, X, M, D, D, D, EPI_F32_RESIDUAL, s)) return rc;
  if (int rc = layernorm(X, nullptr, nullptr, H, L.ln2g, L.ln2b, M, D, c.ln_eps, s)) return rc;
  const int act = c.act == 0 ? EPI_F16_QUICK_GELU : EPI_F16_GELU_ERF;
  if (int rc = gemm(H, L.w1.p, L.b1.p, e->w->F16.p, M, I, D, I, act, s)) return rc;
  return gemm(e->w->F16.p, L.w2.p, L.b2.p, X, M, D, I, D, EPI_F32_RESIDUAL, s);
}

// The LAST pre-LN layer of a tower that pools one row per sequence (CLIP: the class token of
// an image, the EOS token of a text): every row's LN1 / q|k|v / attention as in clip_layer (the
// pooled row attends to all of them), then out-proj, LN2 and the MLP only on the B pooled rows
// `rows`, gathered into XG (f32 residual) / AG (attention output). A GEMM row, a LayerNorm row
// and the residual add depend only on that row (every hand-written GEMM kernel accumulates in
// one order whatever M selects it), so the pooled rows are bit-identical to the full layer's
// (A/B check against the full layer in scripts/enc_dump.py). ViT-B/32 at
// B = 256: the layer's out-proj / fc1 / fc2 run on 256 rows instead of 12,800.
int clip_layer_pooled(mrag_encoder* e, const Layer& L, int B, int T, const int32_t* mask, int causal, const int* rows,
                      hipStream_t s) {
  const auto& c = e->cfg;
  const int D = c.hidden, I = c.intermediate, M = B * T;
  float* X = (float*)e->w->X.p;
  _Float16* H = (_Float16*)e->w->H16.p;
  if (int rc = layernorm(X, nullptr, nullptr, H, L.ln1g, L.ln1b, M, D, c.ln_eps, s)) return rc;
  if (int rc = gemm(H, L.wqkv.p, L.bqkv.p, e->w->QKV.p, M, 3 * D, D, 3 * D, EPI_F16, s)) return rc;
  AttentionArgs a{};
  a.qkv = (const _Float16*)e->w->QKV.p;
  a.out = (_Float16*)e->w->ATT.p;
  a.mask = mask;
  a.B = B;
  a.L = T;
  a.H = c.heads;
  a.causal = causal;
  a.scale = 1.0f / sqrtf((float)(D / c.heads));
  if (int rc = launch_attention(a, D / c.heads, s)) return rc;
  if (int rc = launch_gather_rows(X, e->w->XG.p, rows, B, D * 4, s)) return rc;
  if (int rc = launch_gather_rows(e->w->ATT.p, e->w->AG.p, rows, B, D * 2, s)) return rc;
  float* XG = (float*)e->w->XG.p;
  if (int rc = gemm(e->w->AG.p, L.wo.p, L.bo.p, XG, B, D, D, D, EPI_F32_RESIDUAL, s)) return rc;
  if (int rc = layernorm(XG, nullptr, nullptr, (_Float16*)e->w->HG.p, L.ln2g, L.ln2b, B, D, c.ln_eps, s)) return rc;
  const int act = c.act == 0 ? EPI_F16_QUICK_GELU : EPI_F16_GELU_ERF;
  if (int rc = gemm(e->w->HG.p, L.w1.p, L.b1.p, e->w->FG.p, B, I, D, I, act, s)) return rc;
  return gemm(e->w->FG.p, L.w2.p, L.b2.p, XG, B, D, I, D, EPI_F32_RESIDUAL, s);
}

// Post-LN transformer layer (BERT): X = LN(X + attn(X)); X = LN(X + ffn(X)).
// Invariant on entry and exit: X (f32) and H16 == f16(X).
int bert_layer(mrag_encoder* e, const Layer& L, int B, int T, const int32_t* mask, hipStream_t s) {
  const auto& c = e->cfg;
  const int D = c.hidden, I = c.intermediate, M = B * T;
  float* X = (float*)e->w->X.p;
  _Float16* H = (_Float16*)e->w->H16.p;
  if (int rc = gemm(H, L.wqkv.p, L.bqkv.p, e->w->QKV.p, M, 3 * D, D, 3 * D, EPI_F16, s)) return rc;
  AttentionArgs a{};
  a.qkv = (const _Float16*)e->w->QKV.p;
  a.out = (_Float16*)e->w->ATT.p;
  a.mask = mask;
  a.B = B;
  a.L = T;
  a.H = c.heads;
  a.causal = 0;
  a.scale = 1.0f / sqrtf((float)(D / c.heads));
  if (int rc = launch_attention(a, D / c.heads, s)) return rc;
  if (int rc = gemm(e->w->ATT.p, L.wo.p, L.bo.p, X, M, D, D, D, EPI_F32_RESIDUAL, s)) return rc;
  if (int rc = layernorm(X, nullptr, X, H, L.ln1g, L.ln1b, M, D, c.ln_eps, s)) return rc;
  if (int rc = gemm(H, L.w1.p, L.b1.p, e->w->F16.p, M, I, D, I, EPI_F16_GELU_ERF, s)) return rc;
  if (int rc = gemm(e->w->F16.p, L.w2.p, L.b2.p, X, M, D, I, D, EPI_F32_RESIDUAL, s)) return rc;
  return layernorm(X, nullptr, X, H, L.ln2g, L.ln2b, M, D, c.ln_eps, s);
}

int check_ready(mrag_encoder* e) {
  for (const auto& n : e->expected)
    if (!e->loaded.count(n)) return mrag::fail(MRAG_ERR_STATE, "encoder parameter '%s' not set", n.c_str());
  return MRAG_OK;
}

}  // namespace

namespace {
// Run `forward` on s as a replay of its captured graph (captured on first use of this shape, or
// again when a buffer it baked in moved). The kernels and their order are exactly those of a
// direct call, so results are bit-identical to it (tests/test_encoders_gpu.py).
template <class F>
int run_graph(mrag_encoder* e, uint64_t key, std::vector<const void*> sig, hipStream_t s, F&& forward) {
  auto it = e->graphs.find(key);
  if (it != e->graphs.end() && it->second.sig != sig) {
    (void)hipGraphExecDestroy(it->second.exec);
    e->graphs.erase(it);
    it = e->graphs.end();
  }
  if (it == e->graphs.end()) {
    if (e->graphs.size() >= 128) {  // bounded cache: query lengths vary
      for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second.exec);
      e->graphs.clear();
    }
    hipGraph_t gr = nullptr;
    MRAG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const int rc = forward(s);
    const hipError_t ce = hipStreamEndCapture(s, &gr);
    if (rc != MRAG_OK) {
      if (gr) (void)hipGraphDestroy(gr);
      return rc;
    }
    if (ce != hipSuccess) return mrag::fail(MRAG_ERR_HIP, "graph capture: %s", hipGetErrorString(ce));
    hipGraphExec_t ex = nullptr;
    const hipError_t ie = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    if (ie != hipSuccess) return mrag::fail(MRAG_ERR_HIP, "graph instantiate: %s", hipGetErrorString(ie));
    it = e->graphs.emplace(key, mrag_encoder::Graph{ex, std::move(sig)}).first;
  }
  MRAG_HIP(hipGraphLaunch(it->second.exec, s));
  return MRAG_OK;
}

// The image tower on B images (device u8 HWC) into dst (device f32 [B][proj_dim]) on s, with
// the workspace e->w.
int image_forward(mrag_encoder* e, const uint8_t* img, int B, float* dst, int normalize, hipStream_t s) {
  const auto& c = e->cfg;
  const int S = c.image_size, P = c.patch_size, G = S / P, T = G * G + 1, D = c.hidden;
  const int Kp = 3 * P * P;
  float* X = (float*)e->w->X.p;
  if (int rc = launch_vit_im2col(img, (_Float16*)e->w->F16.p, B, S, P, s)) return rc;
  if (int rc = gemm(e->w->F16.p, e->patch_w.p, nullptr, e->w->PATCH.p, B * (T - 1), D, Kp, D, EPI_F32, s)) return rc;
  if (int rc = launch_vit_embed_ln((const float*)e->w->PATCH.p, (const float*)e->cls.p, (const float*)e->pos.p,
                                   (const float*)e->pre_g.p, (const float*)e->pre_b.p, X, B, T, D, c.ln_eps, s))
    return rc;
  if (int rc = launch_cls_rows(B, T, (int*)e->w->ROWS.p, s)) return rc;
  const bool prune = c.layers > 0;
  for (int i = 0; i < c.layers; ++i) {
    if (prune && i == c.layers - 1) {
      if (int rc = clip_layer_pooled(e, e->layers[i], B, T, nullptr, 0, (const int*)e->w->ROWS.p, s)) return rc;
    } else if (int rc = clip_layer(e, e->layers[i], B, T, nullptr, 0, s)) {
      return rc;
    }
  }
  if (int rc = layernorm(prune ? (const float*)e->w->XG.p : X, prune ? nullptr : (const int*)e->w->ROWS.p, nullptr,
                         (_Float16*)e->w->POOL16.p, e->post_g, e->post_b, B, D, c.ln_eps, s))
    return rc;
  if (int rc = gemm(e->w->POOL16.p, e->proj_w.p, nullptr, dst, B, c.proj_dim, D, c.proj_dim, EPI_F32, s)) return rc;
  if (normalize)
    if (int rc = mrag_l2norm_rows(dst, dst, B, c.proj_dim, s)) return rc;
  return MRAG_OK;
}

}  // namespace

extern "C" {

int mrag_encoder_create(const mrag_encoder_config* cfg, int32_t device, mrag_encoder** out) {
  MRAG_REQUIRE(cfg && out, "NULL argument");
  *out = nullptr;
  const auto& c = *cfg;
  MRAG_REQUIRE(c.kind == MRAG_ENC_CLIP_VISION || c.kind == MRAG_ENC_CLIP_TEXT || c.kind == MRAG_ENC_BERT ||
                   c.kind == MRAG_ENC_BERT_PAIR,
               "unknown encoder kind %d", c.kind);
  MRAG_REQUIRE(c.hidden > 0 && c.hidden % 128 == 0 && c.hidden <= 1024, "hidden %d unsupported (multiple of 128, <= 1024)",
               c.hidden);
  MRAG_REQUIRE(c.intermediate % 128 == 0 && c.intermediate > 0, "intermediate %d must be a multiple of 128",
               c.intermediate);
  MRAG_REQUIRE(c.heads > 0 && c.hidden % c.heads == 0 && (c.hidden / c.heads == 64 || c.hidden / c.heads == 32),
               "head_dim must be 32 or 64");
  MRAG_REQUIRE(c.layers >= 1 && c.layers <= 64, "layers %d", c.layers);
  MRAG_REQUIRE(c.act == 0 || c.act == 1, "act %d", c.act);
  if (c.kind == MRAG_ENC_CLIP_VISION || c.kind == MRAG_ENC_CLIP_TEXT)
    MRAG_REQUIRE(c.proj_dim % 128 == 0 && c.proj_dim > 0, "proj_dim must be a multiple of 128");
  if (c.kind == MRAG_ENC_BERT_PAIR) MRAG_REQUIRE(c.proj_dim >= 1 && c.proj_dim <= 64, "num_labels %d", c.proj_dim);
  if (c.kind == MRAG_ENC_CLIP_VISION)
    MRAG_REQUIRE(c.patch_size > 0 && c.image_size % c.patch_size == 0 && (3 * c.patch_size * c.patch_size) % 64 == 0 &&
                     c.patch_size % 8 == 0,
                 "image/patch size unsupported");
  int ndev = 0;
  MRAG_HIP(hipGetDeviceCount(&ndev));
  MRAG_REQUIRE(device >= 0 && device < ndev, "device %d out of range", device);
  mrag::DeviceGuard g(device);
  auto* e = new mrag_encoder();
  e->cfg = c;
  e->device = device;
  e->layers.resize(c.layers);
  e->expected = expected_names(c);
  hipError_t err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
  if (err == hipSuccess) err = hipEventCreateWithFlags(&e->done, hipEventDisableTiming);
  if (err == hipSuccess) err = hipEventCreateWithFlags(&e->null_ev, hipEventDisableTiming);
  if (err != hipSuccess) {
    delete e;
    return mrag::fail(MRAG_ERR_HIP, "stream: %s", hipGetErrorString(err));
  }
  if (c.kind == MRAG_ENC_CLIP_VISION) {
    std::lock_guard<std::mutex> lk(g_image_mu);
    g_image_handles.push_back(e);
  }
  *out = e;
  return MRAG_OK;
}

int mrag_encoder_destroy(mrag_encoder* e) {
  if (!e) return MRAG_OK;
  {
    std::lock_guard<std::mutex> lk(g_image_mu);
    g_image_handles.erase(std::remove(g_image_handles.begin(), g_image_handles.end(), e), g_image_handles.end());
  }
  {
    mrag::DeviceGuard g(e->device);
    (void)hipStreamSynchronize(e->stream);
    if (e->last_stream) (void)hipEventSynchronize(e->done);
    if (e->done) (void)hipEventDestroy(e->done);
    if (e->null_ev) (void)hipEventDestroy(e->null_ev);
    for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second.exec);
    e->graphs.clear();
    for (auto& L : e->layers)
      for (Buf* b : {&L.wqkv, &L.bqkv, &L.wo, &L.bo, &L.w1, &L.b1, &L.w2, &L.b2, &L.ln1g, &L.ln1b, &L.ln2g, &L.ln2b})
        buf_free(*b);
    for (Buf* b : {&e->patch_w, &e->cls, &e->pos, &e->pre_g, &e->pre_b, &e->post_g, &e->post_b, &e->proj_w, &e->tok,
                   &e->type0, &e->emb_g, &e->emb_b, &e->pool_w, &e->pool_b, &e->cls_w, &e->cls_b})
      buf_free(*b);
    for (Work& w : e->work)
      for (Buf* b : {&w.X, &w.H16, &w.QKV, &w.ATT, &w.F16, &w.PATCH, &w.IMG, &w.IDS, &w.MASK, &w.ROWS, &w.POOL16, &w.OUT,
                     &w.POOL32, &w.TYPES, &w.XG, &w.AG, &w.HG, &w.FG})
        buf_free(*b);
    for (int i = 0; i < MRAG_IMG_LANES; ++i) {
      if (e->lane_stream[i]) (void)hipStreamDestroy(e->lane_stream[i]);
      if (e->lane_ev[i]) (void)hipEventDestroy(e->lane_ev[i]);
    }
    if (e->lane_fork) (void)hipEventDestroy(e->lane_fork);
    (void)hipStreamDestroy(e->stream);
  }
  delete e;
  return MRAG_OK;
}

int mrag_encoder_set_param(mrag_encoder* e, const char* cname, const float* data, int64_t numel) {
  MRAG_REQUIRE(e && cname && data, "NULL argument");
  std::lock_guard<std::mutex> lk(e->mu);
  mrag::DeviceGuard g(e->device);
  if (e->last_stream) MRAG_HIP(hipEventSynchronize(e->done));  // a forward may still read the weights
  for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second.exec);  // recaptured on next use
  e->graphs.clear();
  const std::string name(cname);
  const auto& c = e->cfg;
  bool known = false;
  for (const auto& n : e->expected)
    if (n == name) known = true;
  MRAG_REQUIRE(known, "unexpected parameter '%s' for this encoder", cname);
  const int64_t want = expected_numel(c, name);
  MRAG_REQUIRE(numel == want, "parameter '%s': %lld elements, expected %lld", cname, (long long)numel, (long long)want);
  hipStream_t s = e->stream;
  const int64_t D = c.hidden;
  auto ends = [&](const char* suf) {
    const size_t n = strlen(suf);
    return name.size() >= n && name.compare(name.size() - n, n, suf) == 0;
  };
  int rc = MRAG_OK;
  const bool bert = c.kind == MRAG_ENC_BERT || c.kind == MRAG_ENC_BERT_PAIR;
  const int li = bert ? layer_index(name, "encoder.layer.") : layer_index(name, "encoder.layers.");
  if (li >= 0) {
    MRAG_REQUIRE(li < c.layers, "layer index %d out of range", li);
    Layer& L = e->layers[li];
    int qkv = -1;
    bool is_w = ends(".weight");
    if (name.find("q_proj") != std::string::npos || name.find("self.query") != std::string::npos) qkv = 0;
    if (name.find("k_proj") != std::string::npos || name.find("self.key") != std::string::npos) qkv = 1;
    if (name.find("v_proj") != std::string::npos || name.find("self.value") != std::string::npos) qkv = 2;
    if (qkv >= 0) {
      rc = is_w ? upload_slice_f16(L.wqkv, 3 * D * D, qkv * D * D, data, numel, s)
                : upload_slice_f32(L.bqkv, 3 * D, qkv * D, data, numel, s);
    } else if (name.find("out_proj") != std::string::npos || name.find("attention.output.dense") != std::string::npos) {
      rc = is_w ? upload(L.wo, data, numel, true, s) : upload(L.bo, data, numel, false, s);
    } else if (name.find("fc1") != std::string::npos || name.find("intermediate.dense") != std::string::npos) {
      rc = is_w ? upload(L.w1, data, numel, true, s) : upload(L.b1, data, numel, false, s);
    } else if (name.find("fc2") != std::string::npos || name.find("output.dense") != std::string::npos) {
      rc = is_w ? upload(L.w2, data, numel, true, s) : upload(L.b2, data, numel, false, s);
    } else if (name.find("layer_norm1") != std::string::npos ||
               name.find("attention.output.LayerNorm") != std::string::npos) {
      rc = is_w ? upload(L.ln1g, data, numel, false, s) : upload(L.ln1b, data, numel, false, s);
    } else if (name.find("layer_norm2") != std::string::npos || name.find("output.LayerNorm") != std::string::npos) {
      rc = is_w ? upload(L.ln2g, data, numel, false, s) : upload(L.ln2b, data, numel, false, s);
    } else {
      return mrag::fail(MRAG_ERR_ARG, "unhandled layer parameter '%s'", cname);
    }
  } else if (ends("class_embedding")) {
    rc = upload(e->cls, data, numel, false, s);
  } else if (ends("patch_embedding.weight")) {
    rc = upload(e->patch_w, data, numel, true, s);  // [D][3][P][P] == [D][K] row-major
  } else if (ends("position_embedding.weight") || ends("position_embeddings.weight")) {
    rc = upload(e->pos, data, numel, false, s);
  } else if (ends("token_embedding.weight") || ends("word_embeddings.weight")) {
    rc = upload(e->tok, data, numel, false, s);
  } else if (ends("token_type_embeddings.weight")) {
    rc = upload(e->type0, data, numel, false, s);  // [2][D]; single-text BERT reads row 0
  } else if (ends("pooler.dense.weight")) {
    rc = upload(e->pool_w, data, numel, true, s);
  } else if (ends("pooler.dense.bias")) {
    rc = upload(e->pool_b, data, numel, false, s);
  } else if (ends("classifier.weight")) {
    rc = upload(e->cls_w, data, numel, false, s);
  } else if (ends("classifier.bias")) {
    rc = upload(e->cls_b, data, numel, false, s);
  } else if (ends("pre_layrnorm.weight")) {
    rc = upload(e->pre_g, data, numel, false, s);
  } else if (ends("pre_layrnorm.bias")) {
    rc = upload(e->pre_b, data, numel, false, s);
  } else if (ends("post_layernorm.weight") || ends("final_layer_norm.weight")) {
    rc = upload(e->post_g, data, numel, false, s);
  } else if (ends("post_layernorm.bias") || ends("final_layer_norm.bias")) {
    rc = upload(e->post_b, data, numel, false, s);
  } else if (ends("embeddings.LayerNorm.weight")) {
    rc = upload(e->emb_g, data, numel, false, s);
  } else if (ends("embeddings.LayerNorm.bias")) {
    rc = upload(e->emb_b, data, numel, false, s);
  } else if (ends("visual_projection.weight") || ends("text_projection.weight")) {
    rc = upload(e->proj_w, data, numel, true, s);
  } else {
    return mrag::fail(MRAG_ERR_ARG, "unhandled parameter '%s'", cname);
  }
  if (rc) return rc;
  MRAG_HIP(hipStreamSynchronize(s));
  e->loaded[name] = true;
  return MRAG_OK;
}

int mrag_encoder_missing(const mrag_encoder* e, int64_t* count) {
  MRAG_REQUIRE(e && count, "NULL argument");
  int64_t n = 0;
  for (const auto& name : e->expected)
    if (!e->loaded.count(name)) ++n;
  *count = n;
  return MRAG_OK;
}

// Start of a forward on stream s: order it after the previous call if that ran elsewhere, and
// after the null stream's work when device inputs come without a caller stream.
int begin_call(mrag_encoder* e, hipStream_t s, int32_t ptr_kind, void* stream_arg) {
  if (e->last_stream && e->last_stream != s) MRAG_HIP(hipStreamWaitEvent(s, e->done, 0));
  if (ptr_kind == MRAG_PTR_DEVICE && stream_arg == nullptr)
    if (int rc = mrag::wait_null_stream(e->null_ev, s)) return rc;
  return MRAG_OK;
}

// End of a forward: host pointers, or no caller stream (NULL = the handle's own stream, which
// the caller cannot order on), are complete on return; device pointers on a caller stream are
// stream-ordered (no host sync).
int end_call(mrag_encoder* e, hipStream_t s, int32_t ptr_kind, void* stream_arg) {
  MRAG_HIP(hipEventRecord(e->done, s));
  e->last_stream = s;
  if (ptr_kind == MRAG_PTR_HOST || stream_arg == nullptr) MRAG_HIP(hipStreamSynchronize(s));
  return MRAG_OK;
}

int mrag_encoder_embed_images(mrag_encoder* e, const uint8_t* images, int32_t batch, float* out, int32_t normalize,
                              int32_t ptr_kind, void* stream_arg) {
  MRAG_REQUIRE(e != nullptr, "NULL encoder");
  MRAG_REQUIRE(e->cfg.kind == MRAG_ENC_CLIP_VISION, "not an image encoder");
  MRAG_REQUIRE(batch >= 0, "negative batch");
  MRAG_REQUIRE(ptr_kind == MRAG_PTR_HOST || ptr_kind == MRAG_PTR_DEVICE, "bad ptr_kind");
  std::lock_guard<std::mutex> lk(e->mu);
  mrag::DeviceGuard g(e->device);
  if (int rc = check_ready(e)) return rc;
  if (batch == 0) return MRAG_OK;
  MRAG_REQUIRE(images && out, "NULL images/out");
  hipStream_t s = stream_arg ? (hipStream_t)stream_arg : e->stream;
  if (int rc = begin_call(e, s, ptr_kind, stream_arg)) return rc;
  mrag::StreamDrain drain(s);  // an error return after a launch drains s (workspace reuse)
  const auto& c = e->cfg;
  const int S = c.image_size, P = c.patch_size, G = S / P, T = G * G + 1, B = batch;
  // A lone batch of >= MRAG_IMG_LANE_MIN images runs as MRAG_IMG_LANES sub-batches ("lanes"),
  // each on its own workspace and stream, forked from and joined back into s: one batch's GEMM
  // rounds that leave CUs idle (the N = 768 grids: 150 tiles on 256 CUs) and its latency-bound
  // attention / LayerNorm then overlap with the other lane's kernels, as separate calls in flight
  // do (one batch at a time: 67.1k -> 73.5k img/s). Only the process's sole image handle on the
  // device splits: with several handles (the drop-in's pool grows one per concurrent caller) the
  // calls already share the GPU, and splitting them too measured 86.1k -> 75.1k img/s with three
  // batches in flight (profiles/r5s7_lanes_ab.jsonl). Every row depends only on its image (the
  // batch-consistency tests), so the result is bit-identical either way.
  int lanes = (MRAG_IMG_LANES > 1 && B >= MRAG_IMG_LANE_MIN && sole_image_handle(e)) ? MRAG_IMG_LANES : 1;
  // the lanes' streams and events are created on first use, all lanes' streams together: a
  // handle that never runs alone holds no extra stream. Every lane runs on one of these, none on
  // the caller's stream s: HIP puts the process's streams on GPU_MAX_HW_QUEUES hardware queues
  // (4 by default), and a lane on s shared a queue with the other lane's stream whenever s had
  // been made at another time (53k instead of 74k img/s one batch at a time,
  // profiles/r6s26_r6s27_hw_queues.txt); streams made one after the other take different queues.
  if (lanes > 1) {
    for (int i = 0; i < lanes; ++i)
      if (!e->lane_stream[i]) MRAG_HIP(hipStreamCreateWithFlags(&e->lane_stream[i], hipStreamNonBlocking));
    for (int i = 0; i < lanes; ++i)
      if (!e->lane_ev[i]) MRAG_HIP(hipEventCreateWithFlags(&e->lane_ev[i], hipEventDisableTiming));
    if (!e->lane_fork) MRAG_HIP(hipEventCreateWithFlags(&e->lane_fork, hipEventDisableTiming));
  }
  struct ResetWork {  // e->w back to work[0] on every return
    mrag_encoder* e;
    ~ResetWork() { e->w = &e->work[0]; }
  } reset{e};
  struct DrainLanes {  // an error return drains the lanes too
    mrag_encoder* e;
    int n;
    bool armed = true;
    ~DrainLanes() {
      if (armed && n > 1)
        for (int i = 0; i < n; ++i) (void)hipStreamSynchronize(e->lane_stream[i]);
    }
  } drain_lanes{e, lanes};
  e->w = &e->work[0];
  const uint8_t* img = images;
  if (ptr_kind == MRAG_PTR_HOST) {
    if (int rc = buf_ensure(e->w->IMG, (size_t)B * S * S * 3)) return rc;
    MRAG_HIP(hipMemcpyAsync(e->w->IMG.p, images, (size_t)B * S * S * 3, hipMemcpyHostToDevice, s));
    img = (const uint8_t*)e->w->IMG.p;
  }
  float* dst = out;
  if (ptr_kind == MRAG_PTR_HOST) {
    if (int rc = buf_ensure(e->w->OUT, (size_t)B * c.proj_dim * 4)) return rc;
    dst = (float*)e->w->OUT.p;
  }
  if (lanes > 1) MRAG_HIP(hipEventRecord(e->lane_fork, s));  // fork
  int b0 = 0;
  for (int i = 0; i < lanes; ++i) {
    const int nb = B / lanes + (i < B % lanes ? 1 : 0);
    hipStream_t ls = lanes > 1 ? e->lane_stream[i] : s;
    if (lanes > 1) MRAG_HIP(hipStreamWaitEvent(ls, e->lane_fork, 0));
    e->w = &e->work[i];
    if (int rc = ensure_workspace(e, nb, T)) return rc;
    if (int rc = image_forward(e, img + (size_t)b0 * S * S * 3, nb, dst + (size_t)b0 * c.proj_dim, normalize, ls))
      return rc;
    b0 += nb;
  }
  for (int i = 0; i < lanes && lanes > 1; ++i) {  // join
    MRAG_HIP(hipEventRecord(e->lane_ev[i], e->lane_stream[i]));
    MRAG_HIP(hipStreamWaitEvent(s, e->lane_ev[i], 0));
  }
  if (ptr_kind == MRAG_PTR_HOST)
    MRAG_HIP(hipMemcpyAsync(out, dst, (size_t)B * c.proj_dim * 4, hipMemcpyDeviceToHost, s));
  drain.armed = false;
  drain_lanes.armed = false;
  return end_call(e, s, ptr_kind, stream_arg);
}

int mrag_encoder_embed_tokens(mrag_encoder* e, const int32_t* ids, const int32_t* mask, int32_t batch, int32_t seq,
                              float* out, int32_t normalize, int32_t ptr_kind, void* stream_arg) {
  MRAG_REQUIRE(e != nullptr, "NULL encoder");
  MRAG_REQUIRE(e->cfg.kind == MRAG_ENC_CLIP_TEXT || e->cfg.kind == MRAG_ENC_BERT, "not a text encoder");
  MRAG_REQUIRE(batch >= 0 && seq >= 1, "bad shape batch=%d seq=%d", batch, seq);
  MRAG_REQUIRE(seq <= e->cfg.max_positions && seq <= 256, "seq %d exceeds max positions (%d) or 256", seq,
               e->cfg.max_positions);
  MRAG_REQUIRE(ptr_kind == MRAG_PTR_HOST || ptr_kind == MRAG_PTR_DEVICE, "bad ptr_kind");
  std::lock_guard<std::mutex> lk(e->mu);
  mrag::DeviceGuard g(e->device);
  if (int rc = check_ready(e)) return rc;
  if (batch == 0) return MRAG_OK;
  MRAG_REQUIRE(ids && out, "NULL ids/out");
  hipStream_t s = stream_arg ? (hipStream_t)stream_arg : e->stream;
  if (int rc = begin_call(e, s, ptr_kind, stream_arg)) return rc;
  mrag::StreamDrain drain(s);  // an error return after a launch drains s (workspace reuse)
  const auto& c = e->cfg;
  const int B = batch, T = seq, D = c.hidden;
  if (int rc = ensure_workspace(e, B, T)) return rc;
  const int32_t* dids = ids;
  const int32_t* dmask = mask;
  if (ptr_kind == MRAG_PTR_HOST) {
    if (int rc = buf_ensure(e->w->IDS, (size_t)B * T * 4)) return rc;
    MRAG_HIP(hipMemcpyAsync(e->w->IDS.p, ids, (size_t)B * T * 4, hipMemcpyHostToDevice, s));
    dids = (const int32_t*)e->w->IDS.p;
    if (mask) {
      if (int rc = buf_ensure(e->w->MASK, (size_t)B * T * 4)) return rc;
      MRAG_HIP(hipMemcpyAsync(e->w->MASK.p, mask, (size_t)B * T * 4, hipMemcpyHostToDevice, s));
      dmask = (const int32_t*)e->w->MASK.p;
    }
  }
  float* X = (float*)e->w->X.p;
  _Float16* H = (_Float16*)e->w->H16.p;
  const int outD = c.kind == MRAG_ENC_BERT ? D : c.proj_dim;
  float* dst = out;
  if (ptr_kind == MRAG_PTR_HOST) {
    if (int rc = buf_ensure(e->w->OUT, (size_t)B * outD * 4)) return rc;
    dst = (float*)e->w->OUT.p;
  }
  auto forward = [&](hipStream_t s) -> int {
    if (c.kind == MRAG_ENC_CLIP_TEXT) {
      if (int rc = launch_token_embed(dids, (const float*)e->tok.p, (const float*)e->pos.p, nullptr, nullptr, X, B, T,
                                      D, c.vocab, s))
        return rc;
      if (int rc = launch_eos_rows(dids, B, T, c.eos_token_id, (int*)e->w->ROWS.p, s)) return rc;
      const bool prune = c.layers > 0;
      for (int i = 0; i < c.layers; ++i) {
        if (prune && i == c.layers - 1) {
          if (int rc = clip_layer_pooled(e, e->layers[i], B, T, dmask, 1, (const int*)e->w->ROWS.p, s)) return rc;
        } else if (int rc = clip_layer(e, e->layers[i], B, T, dmask, 1, s)) {
          return rc;
        }
      }
      if (int rc = layernorm(prune ? (const float*)e->w->XG.p : X, prune ? nullptr : (const int*)e->w->ROWS.p, nullptr,
                             (_Float16*)e->w->POOL16.p, e->post_g, e->post_b, B, D, c.ln_eps, s))
        return rc;
      if (int rc = gemm(e->w->POOL16.p, e->proj_w.p, nullptr, dst, B, c.proj_dim, D, c.proj_dim, EPI_F32, s)) return rc;
    } else {
      if (int rc = launch_token_embed(dids, (const float*)e->tok.p, (const float*)e->pos.p, (const float*)e->type0.p,
                                      nullptr, X, B, T, D, c.vocab, s))
        return rc;
      if (int rc = layernorm(X, nullptr, X, H, e->emb_g, e->emb_b, B * T, D, c.ln_eps, s)) return rc;
      for (int i = 0; i < c.layers; ++i)
        if (int rc = bert_layer(e, e->layers[i], B, T, dmask, s)) return rc;
      if (int rc = launch_mean_pool(X, dmask, dst, B, T, D, s)) return rc;
    }
    if (normalize)
      if (int rc = mrag_l2norm_rows(dst, dst, B, outD, s)) return rc;
    return MRAG_OK;
  };
  // host-pointer calls of up to 2048 tokens (every input and output then lives in this handle's
  // workspace, at addresses the graph can bake in): graph replay; otherwise direct launches
  if (ptr_kind == MRAG_PTR_HOST && (int64_t)B * T <= 2048) {
    const uint64_t key = ((uint64_t)B << 32) | ((uint64_t)T << 2) | (dmask ? 2u : 0u) | (normalize ? 1u : 0u);
    std::vector<const void*> sig = {e->w->X.p,  e->w->H16.p, e->w->QKV.p, e->w->ATT.p,    e->w->F16.p, e->w->XG.p, e->w->AG.p,
                                    e->w->HG.p, e->w->FG.p,  e->w->ROWS.p, e->w->POOL16.p, e->w->IDS.p, e->w->MASK.p, e->w->OUT.p};
    if (int rc = run_graph(e, key, std::move(sig), s, forward)) return rc;
  } else if (int rc = forward(s)) {
    return rc;
  }
  if (ptr_kind == MRAG_PTR_HOST) MRAG_HIP(hipMemcpyAsync(out, dst, (size_t)B * outD * 4, hipMemcpyDeviceToHost, s));
  drain.armed = false;
  return end_call(e, s, ptr_kind, stream_arg);
}

int mrag_encoder_score_pairs(mrag_encoder* e, const int32_t* ids, const int32_t* type_ids, const int32_t* mask,
                             int32_t batch, int32_t seq, float* out, int32_t ptr_kind, void* stream_arg) {
  MRAG_REQUIRE(e != nullptr, "NULL encoder");
  MRAG_REQUIRE(e->cfg.kind == MRAG_ENC_BERT_PAIR, "not a cross-encoder (MRAG_ENC_BERT_PAIR)");
  MRAG_REQUIRE(batch >= 0 && seq >= 1, "bad shape batch=%d seq=%d", batch, seq);
  MRAG_REQUIRE(seq <= e->cfg.max_positions && seq <= 512, "seq %d exceeds max positions (%d) or 512", seq,
               e->cfg.max_positions);
  MRAG_REQUIRE(ptr_kind == MRAG_PTR_HOST || ptr_kind == MRAG_PTR_DEVICE, "bad ptr_kind");
  std::lock_guard<std::mutex> lk(e->mu);
  mrag::DeviceGuard g(e->device);
  if (int rc = check_ready(e)) return rc;
  if (batch == 0) return MRAG_OK;
  MRAG_REQUIRE(ids && out, "NULL ids/out");
  hipStream_t s = stream_arg ? (hipStream_t)stream_arg : e->stream;
  if (int rc = begin_call(e, s, ptr_kind, stream_arg)) return rc;
  mrag::StreamDrain drain(s);  // an error return after a launch drains s (workspace reuse)
  const auto& c = e->cfg;
  const int B = batch, T = seq, D = c.hidden, NL = c.proj_dim;
  if (int rc = ensure_workspace(e, B, T)) return rc;
  const int32_t* dids = ids;
  const int32_t* dmask = mask;
  const int32_t* dtypes = type_ids;
  if (ptr_kind == MRAG_PTR_HOST) {
    if (int rc = buf_ensure(e->w->IDS, (size_t)B * T * 4)) return rc;
    MRAG_HIP(hipMemcpyAsync(e->w->IDS.p, ids, (size_t)B * T * 4, hipMemcpyHostToDevice, s));
    dids = (const int32_t*)e->w->IDS.p;
    if (mask) {
      if (int rc = buf_ensure(e->w->MASK, (size_t)B * T * 4)) return rc;
      MRAG_HIP(hipMemcpyAsync(e->w->MASK.p, mask, (size_t)B * T * 4, hipMemcpyHostToDevice, s));
      dmask = (const int32_t*)e->w->MASK.p;
    }
    if (type_ids) {
      if (int rc = buf_ensure(e->w->TYPES, (size_t)B * T * 4)) return rc;
      MRAG_HIP(hipMemcpyAsync(e->w->TYPES.p, type_ids, (size_t)B * T * 4, hipMemcpyHostToDevice, s));
      dtypes = (const int32_t*)e->w->TYPES.p;
    }
  }
  float* X = (float*)e->w->X.p;
  _Float16* H = (_Float16*)e->w->H16.p;
  if (int rc = launch_token_embed(dids, (const float*)e->tok.p, (const float*)e->pos.p, (const float*)e->type0.p, dtypes,
                                  X, B, T, D, c.vocab, s))
    return rc;
  if (int rc = layernorm(X, nullptr, X, H, e->emb_g, e->emb_b, B * T, D, c.ln_eps, s)) return rc;
  for (int i = 0; i < c.layers; ++i)
    if (int rc = bert_layer(e, e->layers[i], B, T, dmask, s)) return rc;
  // pooler: dense over the [CLS] rows (token 0 of each sequence: A rows strided by T*D)
  GemmArgs pg{};
  pg.A = H;
  pg.W = (const _Float16*)e->pool_w.p;
  pg.bias = (const float*)e->pool_b.p;
  pg.C = e->w->POOL32.p;
  pg.M = B;
  pg.N = D;
  pg.K = D;
  pg.lda = T * D;
  pg.ldw = D;
  pg.ldc = D;
  if (int rc = launch_gemm(pg, EPI_F32, s)) return rc;
  float* dst = out;
  if (ptr_kind == MRAG_PTR_HOST) {
    if (int rc = buf_ensure(e->w->OUT, (size_t)B * NL * 4)) return rc;
    dst = (float*)e->w->OUT.p;
  }
  if (int rc = launch_cls_head((const float*)e->w->POOL32.p, (const float*)e->cls_w.p, (const float*)e->cls_b.p, dst, B, D,
                               NL, s))
    return rc;
  if (ptr_kind == MRAG_PTR_HOST) MRAG_HIP(hipMemcpyAsync(out, dst, (size_t)B * NL * 4, hipMemcpyDeviceToHost, s));
  drain.armed = false;
  return end_call(e, s, ptr_kind, stream_arg);
}

int mrag_gemm_nt(const void* A, const void* W, const float* bias, void* C, int32_t M, int32_t N, int32_t K,
                 int32_t epilogue, void* stream) {
  MRAG_REQUIRE(A && W && C, "NULL pointer");
  MRAG_REQUIRE(M >= 0 && N > 0 && K > 0, "bad shape");
  return gemm(A, W, bias, C, M, N, K, N, epilogue, (hipStream_t)stream);
}

int mrag_gemm_nt_kernel(const void* A, const void* W, const float* bias, void* C, int32_t M, int32_t N, int32_t K,
                        int32_t epilogue, int32_t kernel, void* stream) {
  MRAG_REQUIRE(A && W && C, "NULL pointer");
  MRAG_REQUIRE(M >= 0 && N > 0 && K > 0, "bad shape");
  MRAG_REQUIRE(kernel >= GEMM_AUTO && kernel <= GEMM_K3W, "bad kernel %d", kernel);
  GemmArgs g{};
  g.A = (const _Float16*)A;
  g.W = (const _Float16*)W;
  g.bias = bias;
  g.C = C;
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = K;
  g.ldw = K;
  g.ldc = N;
  return launch_gemm(g, epilogue, (hipStream_t)stream, kernel);
}

}  // extern "C"
