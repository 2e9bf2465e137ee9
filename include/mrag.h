/*
 * mrag.h — C ABI of the MI355X embed-and-retrieve engine (libmrag.so, gfx950).
 *
 * This is the drop-in boundary for the reference's hot path. The reference
 * (Sabarna07-tech/Multimodal-RAG-for-Image-Text-Search) is pure Python; its
 * numerics sit behind two FFI-like seams that this library replaces:
 *
 *   - lancedb (Rust) flat cosine scan + top-k, reached from
 *       app/storage/lancedb_store.py:103-123  (search_text / search_image)
 *       app/storage/lancedb_store.py:87-101   (upsert_text_vectors / upsert_image_vectors)
 *       app/storage/lancedb_store.py:63-69    (LanceDBStore._normalize)
 *   - torch/transformers encoder forwards, reached from
 *       app/ml/embeddings.py:46-49            (_normalize)
 *       app/ml/embeddings.py:62-70            (SentenceTransformer.encode, MiniLM-L6)
 *       app/ml/embeddings.py:84-91            (CLIP get_image_features, ViT-B/32)
 *       app/ml/embeddings.py:101-105          (CLIP get_text_features)
 *
 * Conventions:
 *   - every entry point returns int status, 0 == MRAG_OK; on failure the
 *     thread-local message is available from mrag_last_error();
 *   - plain pointers and sizes only; `ptr_kind` says whether data pointers are
 *     host (MRAG_PTR_HOST) or device (MRAG_PTR_DEVICE) memory;
 *   - `stream` is a hipStream_t passed as void* (NULL = the handle's stream);
 *     device-pointer inputs with stream == NULL are read after the work already
 *     queued on the legacy NULL stream (an event on stream 0 orders the handle's
 *     stream behind it), so data a caller produced with default-stream kernels or
 *     copies is complete when the library reads it;
 *   - handles are opaque; calls on one handle are serialised by an internal
 *     mutex, so a handle may be used from any single thread at a time.
 */
#ifndef MRAG_H
#define MRAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define MRAG_OK 0
#define MRAG_ERR_ARG 1         /* bad argument (shape, pointer, k, dim, ...)      */
#define MRAG_ERR_HIP 2         /* a HIP runtime call failed                       */
#define MRAG_ERR_OOM 3         /* device allocation failed                        */
#define MRAG_ERR_STATE 4       /* handle in the wrong state                       */
#define MRAG_ERR_UNSUPPORTED 5 /* no kernel instance for this configuration       */

#define MRAG_PTR_HOST 0
#define MRAG_PTR_DEVICE 1

/* Row labels: the reference filters every search with `user_id == '<id>'`
 * (lancedb_store.py:108,119). The engine stores one int32 label per row (the
 * host maps user ids to labels). Label filter MRAG_LABEL_ANY matches every
 * live row; rows whose label is MRAG_LABEL_DELETED are tombstones (upsert's
 * per-row delete, lancedb_store.py:91-92) and never match. */
#define MRAG_LABEL_ANY (-1)
#define MRAG_LABEL_DELETED (-2)

const char* mrag_last_error(void);
const char* mrag_version(void);
int mrag_get_device_count(int32_t* count);

/* ---- K6: row L2-normalise ---------------------------------------------
 * Replaces app/ml/embeddings.py:46-49 `_normalize`:
 *   y[r,:] = x[r,:] / ||x[r,:]||  (zero rows copied unchanged)
 * computed in f32 with numpy's pairwise summation order for the row sum of
 * squares, so the result is bit-identical to the reference's numpy call.
 * x, y: device pointers [rows, dim] row-major f32 (y may alias x). */
int mrag_l2norm_rows(const float* x, float* y, int64_t rows, int32_t dim, void* stream);

/* ---- K7/K8: flat cosine index ------------------------------------------
 * Replaces the Lance table + `table.search(v).where(user_id).metric("cosine")
 * .limit(max(k,1))` chain (lancedb_store.py:103-123). One index = one table
 * (text_collection or image_collection, lancedb_store.py:30-31) or one shard
 * of it. Exact semantics: score = cos(q, x) = q.x / (|q| |x|) evaluated in
 * f64 on the f32 vectors as given (0 if either norm is 0), results ordered by
 * (score desc, row asc), label prefilter, at most k rows.
 * Limits: 1 <= dim <= 4096, 1 <= k <= 65536 (the reference has none: Lance stores
 * list<float32> of any length, :33-44, and passes limit(max(k,1)) through, :110,121).
 * dim <= 512 with k <= 256 runs the fused fp16 scan (K7/K8, knn.hip); wider rows and deeper
 * k run K7g (knn_generic.hip: MFMA score GEMM + histogram threshold + exact selection).
 * Both are exact. */
typedef struct mrag_knn_index mrag_knn_index;

int mrag_knn_create(int32_t dim, int32_t device, mrag_knn_index** out);
int mrag_knn_destroy(mrag_knn_index* index);

/* Append n rows (f32 [n, dim]) with their labels (int32 [n]); the new rows get
 * consecutive row ids starting at *first_row (the current size). */
int mrag_knn_add(mrag_knn_index* index, const float* rows, const int32_t* labels, int64_t n,
                 int32_t ptr_kind, int64_t* first_row);

/* Overwrite the label of rows[i] (host int64 [n]); MRAG_LABEL_DELETED deletes. */
int mrag_knn_set_labels(mrag_knn_index* index, const int64_t* rows, int64_t n, int32_t label);

/* Number of row ids handed out so far (live + deleted). */
int mrag_knn_size(const mrag_knn_index* index, int64_t* n);

/* Search nq queries (f32 [nq, dim]) for their k best rows among rows whose
 * label matches `label_filter`. out_scores f32 [nq, k], out_rows int64
 * [nq, k]; row ids are offset by `row_offset` (a shard's first global row).
 * Slots past the number of matching rows get score -inf and row -1.
 * out_scores64 (optional, may be NULL) receives the f64 scores used for the
 * ordering — the sharded merge needs them. All data pointers share ptr_kind.
 * Returns once the search's device work is done (it reads back its certificate).
 * Thread-safe: several host threads may search one index at once, each on its
 * own stream (every call takes its own search workspace from the index's pool;
 * add / set_labels wait for searches in flight and exclude new ones). */
int mrag_knn_search(mrag_knn_index* index, const float* queries, int64_t nq, int32_t k,
                    int32_t label_filter, int64_t row_offset, float* out_scores,
                    double* out_scores64, int64_t* out_rows, int32_t ptr_kind, void* stream);

/* Statistics of the last search on this handle: number of queries whose fp16
 * candidate pass could not be certified exact and went through the
 * threshold-collect pass, and how many collect retries overflowed. */
int mrag_knn_last_stats(const mrag_knn_index* index, int64_t* uncertified, int64_t* retries);

/* Kernel timing for roofline reporting: HIP events recorded on the search
 * stream around every K7 scan launch. enable = 1 resets and enables, 0
 * disables, -1 only reads. Outputs (optional): total scan milliseconds and the
 * number of timed launches since the last reset. */
int mrag_knn_profile(mrag_knn_index* index, int32_t enable, double* scan_ms_total,
                     int64_t* scan_launches);

/* ---- K11: merge per-shard top-k lists (row-sharded multi-GPU search) ----
 * Input: nlists lists per query laid out [nlists][nq][k] (f64 score, int64
 * global row; row -1 = empty), e.g. the result of an RCCL all-gather of every
 * rank's mrag_knn_search output. Output: the k best per query under
 * (score desc, row asc) — identical to a single-index search.
 * Device pointers. */
int mrag_topk_merge(const double* scores64, const int64_t* rows, int32_t nlists, int64_t nq,
                    int32_t k, float* out_scores, double* out_scores64, int64_t* out_rows,
                    void* stream);

/* ---- K12: z-score fusion of text and image hits ----------------------------
 * Replaces app/ml/retrieve.py:158-195 (_z_scores + _fuse_results, rerank off) for a batch
 * of queries, bit-identical to the reference's float32 numpy arithmetic: per query, the
 * text hit scores text_scores [nq][kt] and image hit scores image_scores [nq][ki] (f32 as
 * mrag_knn_search returns them, hits in score order, -inf for missing hits; each score is
 * taken through the store's 1 - f32(1 - s)), z-scored per list, concatenated text-first,
 * stably sorted by combined score descending. Outputs pick [nq][final_n] (index into the
 * concatenated [kt | ki] slots, -1 past the hits) and combined [nq][final_n] (f64 z, NaN
 * for -1). Device pointers; asynchronous on `stream`. */
int mrag_fuse_scores(const float* text_scores, int32_t kt, const float* image_scores, int32_t ki, int64_t nq,
                     int32_t final_n, int64_t* pick, double* combined, void* stream);

/* ---- K1..K5: encoders ----------------------------------------------------
 * One handle = one encoder tower on one device:
 *   MRAG_ENC_CLIP_VISION  replaces CLIPModel.get_image_features
 *                         (app/ml/embeddings.py:84-91, transformers modeling_clip.py:719-755)
 *   MRAG_ENC_CLIP_TEXT    replaces CLIPModel.get_text_features
 *                         (app/ml/embeddings.py:101-105, modeling_clip.py:683-717)
 *   MRAG_ENC_BERT         replaces SentenceTransformer(all-MiniLM-L6-v2).encode =
 *                         BertModel + mean pooling (app/ml/embeddings.py:62-68)
 *   MRAG_ENC_BERT_PAIR    replaces CrossEncoder(ms-marco-MiniLM-L-6-v2).predict =
 *                         BertForSequenceClassification on (query, passage) pairs
 *                         (app/ml/retrieve.py:29-38, 132-155; modeling_bert.py pooler +
 *                         classifier); parameters under their "bert." / "classifier." names
 * Parameters are set by Hugging Face state-dict name (f32 host arrays, e.g.
 * "vision_model.encoder.layers.0.self_attn.q_proj.weight"); compute is fp16 MFMA
 * GEMMs with f32 accumulation and an f32 residual stream. With normalize != 0 the
 * output rows go through K6 (the reference's numpy _normalize, bit-exact).
 * Host pointers (MRAG_PTR_HOST), or stream == NULL (the handle's own stream): the call
 * returns with `out` written. Device pointers on a caller stream: the work is enqueued on
 * `stream` and the call returns without waiting (stream-ordered; a later call on another
 * stream is ordered after it by the handle). */
#define MRAG_ENC_CLIP_VISION 1
#define MRAG_ENC_CLIP_TEXT 2
#define MRAG_ENC_BERT 3
#define MRAG_ENC_BERT_PAIR 4

typedef struct mrag_encoder_config {
  int32_t kind;           /* MRAG_ENC_*                                            */
  int32_t hidden;         /* 768 (ViT-B/32), 512 (CLIP text), 384 (MiniLM-L6)      */
  int32_t layers;         /* 12, 12, 6                                             */
  int32_t heads;          /* 12, 8, 12                                             */
  int32_t intermediate;   /* 3072, 2048, 1536                                      */
  int32_t max_positions;  /* text: 77 / 512; vision: unused                        */
  int32_t vocab;          /* text: 49408 / 30522                                   */
  int32_t proj_dim;       /* CLIP: 512; BERT: unused; BERT_PAIR: num_labels (1)    */
  int32_t image_size;     /* vision: 224                                           */
  int32_t patch_size;     /* vision: 32                                            */
  int32_t act;            /* 0 = quick_gelu (CLIP), 1 = gelu (erf, BERT)          */
  int32_t eos_token_id;   /* CLIP text pooling: first id == eos (>= 0) or argmax(ids) (-1) */
  float ln_eps;           /* 1e-5 (CLIP), 1e-12 (BERT)                             */
} mrag_encoder_config;

typedef struct mrag_encoder mrag_encoder;

int mrag_encoder_create(const mrag_encoder_config* cfg, int32_t device, mrag_encoder** out);
int mrag_encoder_destroy(mrag_encoder* enc);
int mrag_encoder_set_param(mrag_encoder* enc, const char* name, const float* data, int64_t numel);
/* Number of required parameters not set yet (forward fails with MRAG_ERR_STATE until 0). */
int mrag_encoder_missing(const mrag_encoder* enc, int64_t* count);

/* CLIP image tower: images u8 [batch][S][S][3] (decoded RGB, HWC, S = image_size,
 * already resized/cropped) -> out f32 [batch][proj_dim]. */
int mrag_encoder_embed_images(mrag_encoder* enc, const uint8_t* images, int32_t batch, float* out,
                              int32_t normalize, int32_t ptr_kind, void* stream);

/* Text towers: token ids / attention mask int32 [batch][seq] (mask may be NULL =
 * all ones) -> out f32 [batch][proj_dim] (CLIP text) or [batch][hidden] (BERT,
 * mean-pooled over the mask). */
int mrag_encoder_embed_tokens(mrag_encoder* enc, const int32_t* ids, const int32_t* mask, int32_t batch,
                              int32_t seq, float* out, int32_t normalize, int32_t ptr_kind, void* stream);

/* Cross-encoder (MRAG_ENC_BERT_PAIR): ids / token_type_ids / attention mask int32
 * [batch][seq] ("[CLS] a [SEP] b [SEP]", types 0 / 1; type_ids or mask may be NULL =
 * zeros / ones), seq <= max_positions (512) -> out f32 [batch][num_labels] logits
 * (before any activation). */
int mrag_encoder_score_pairs(mrag_encoder* enc, const int32_t* ids, const int32_t* type_ids, const int32_t* mask,
                             int32_t batch, int32_t seq, float* out, int32_t ptr_kind, void* stream);

/* K0: image resize (shortest edge -> size, bicubic) + centre crop, bit-exact to the
 * reference's preprocessing (CLIPImageProcessor -> PIL.Image.resize(BICUBIC) + center_crop,
 * app/ml/embeddings.py:84-85; host restatement app/encoders/preprocess.py:to_u8_224).
 * pixels: device u8 RGB HWC images, image i at byte offset offsets[i] with size
 * widths[i] x heights[i] (offsets/widths/heights are host arrays of n entries);
 * out: device u8 [n][size][size][3] (the input of mrag_encoder_embed_images).
 * Synchronous on `stream` (returns after the kernels finish). */
int mrag_image_resize_crop(const uint8_t* pixels, const int64_t* offsets, const int32_t* widths,
                           const int32_t* heights, int32_t n, int32_t size, uint8_t* out, void* stream);

/* K13: baseline JPEG decode on the GPU, byte-identical to Pillow's decode + convert("RGB")
 * (replaces the per-file Image.open(path).convert("RGB") of the reference's embed_images_batch,
 * app/ml/embeddings.py:82-89, for the JPEGs it supports).
 * mrag_jpeg_probe: host-only header parse of one file; returns 1 and the size when K13 decodes it
 * (baseline / extended sequential Huffman, 8-bit, 1 or 3 components, 4:4:4 / 4:2:2 / 4:2:0,
 * restart intervals), 0 when the caller must decode it on the host (progressive, arithmetic,
 * CMYK, RGB-coded, other sampling, tiny chroma), negative on bad arguments. */
int mrag_jpeg_probe(const uint8_t* data, int64_t size, int32_t* width, int32_t* height);
/* mrag_jpeg_decode: n files (host bytes, every one probed 1) decoded into device memory `out`,
 * file i as H x W x 3 u8 RGB at byte offset out_offsets[i] (host array) — the pixel layout
 * mrag_image_resize_crop takes. Synchronous on `stream`. */
int mrag_jpeg_decode(const uint8_t* const* files, const int64_t* sizes, int32_t n, uint8_t* out,
                     const int64_t* out_offsets, int32_t device, void* stream);

/* K14: PNG decode with the scanline reconstruction on the GPU, byte-identical to Pillow's decode +
 * convert("RGB") (the same reference call as K13, for the PNGs it supports: bit depth 8, grey /
 * grey + alpha / RGB / RGBA, not interlaced, width <= 8192).
 * mrag_png_probe: host-only chunk parse (CRC-32 checked) of one file; returns 1, the size and the
 * inflated byte count when K14 decodes it, 0 when the caller must decode it on the host (palette,
 * 16-bit, interlaced, bad CRC ...), negative on bad arguments.
 * mrag_png_inflate: host zlib inflate of the IDAT stream into `raw` (cap >= the probe's raw_bytes:
 * h scanlines of 1 filter byte + w x bpp bytes); *bpp = bytes per pixel (1, 2, 3, 4); returns 1,
 * 0 when the stream is corrupt or short (decode that file on the host), negative on bad arguments.
 * Thread-safe, no device work: call it from decode threads.
 * mrag_png_unfilter: n inflated images (host raws, dims = n x {w, h, bpp}) reconstructed and
 * converted into device memory `out`, image i as H x W x 3 u8 RGB at out_offsets[i] (host array).
 * Synchronous on `stream`. */
int mrag_png_probe(const uint8_t* data, int64_t size, int32_t* width, int32_t* height, int64_t* raw_bytes);
int mrag_png_inflate(const uint8_t* data, int64_t size, uint8_t* raw, int64_t cap, int32_t* bpp);
int mrag_png_unfilter(const uint8_t* const* raws, const int32_t* dims, int32_t n, uint8_t* out,
                      const int64_t* out_offsets, int32_t device, void* stream);

/* The host half of image ingest in one call (the per-file Image.open of the reference's
 * embed_images_batch, app/ml/embeddings.py:82-89): mrag_files_prepare reads n files on `threads`
 * host threads of its own and classifies each — kind 1: a JPEG K13 decodes, 2: a PNG K14
 * reconstructs (inflated here), 0: anything else (decode it with Pillow), -1: unreadable (open it
 * yourself to get the error); device_decode = 0 classifies every readable file as 0. A file of
 * more than max_pixels pixels (max(1, w) * max(1, h), Pillow's decompression-bomb count) is kind 0
 * too, so Pillow warns or raises DecompressionBombError for it as in the reference; pass Pillow's
 * Image.MAX_IMAGE_PIXELS, or max_pixels < 0 for no limit (MAX_IMAGE_PIXELS = None).
 * mrag_files_info: kind / width / height per file (arrays of n). mrag_files_bytes: a file's bytes
 * (valid until mrag_files_free). mrag_files_decode: K13 + K14 for the kind 1 / 2 files into
 * device memory `out`, file i as H x W x 3 u8 RGB at out_offsets[i] (host array of n; entries of
 * other kinds unused); synchronous on `stream`. */
typedef struct mrag_files mrag_files;
int mrag_files_prepare(const char* const* paths, int32_t n, int32_t threads, int32_t device_decode,
                       int64_t max_pixels, mrag_files** out);
int mrag_files_info(const mrag_files* files, int32_t* kind, int32_t* width, int32_t* height);
int mrag_files_bytes(const mrag_files* files, int32_t i, const uint8_t** data, int64_t* size);
int mrag_files_decode(const mrag_files* files, uint8_t* out, const int64_t* out_offsets, int32_t device, void* stream);
int mrag_files_free(mrag_files* files);
/* mrag_paths_exist: pathlib.Path(p).exists() for n paths at once (index_image_nodes' filter of
 * missing files, reference app/ml/index_build.py:114-118) on `threads` host threads: out[i] = 1
 * (stat succeeds; "" is Path("") = "."), 0 (missing: ENOENT / ENOTDIR / EBADF / ELOOP, the errors
 * Path.exists ignores), -1 (any other error: the caller asks Path.exists, which raises it). */
int mrag_paths_exist(const char* const* paths, int32_t n, int32_t threads, int32_t* out);

/* mrag_hash_tokenize: the offline stand-in tokeniser of app/encoders/tokenize.py (no local
 * vocabulary: the reference's sentence-transformers / CLIPProcessor tokenisers, app/ml/
 * embeddings.py:62-67 / :100-103, cannot load their hub vocabularies offline) for ASCII texts, on
 * `threads` host threads: the tokens of `\w+|[^\w\s]` over the lowercased text, each id = lo +
 * crc32(token) % (hi - lo), at most max_tokens per text, into ids[i * max_tokens ...];
 * counts[i] = the number written, or -1 when text i (texts[i], lens[i] bytes) holds a non-ASCII
 * byte (the caller tokenises it in Python: NFC and Unicode classes). */
int mrag_hash_tokenize(const char* const* texts, const int64_t* lens, int32_t n, int32_t lo, int32_t hi,
                       int32_t max_tokens, int32_t threads, int32_t* ids, int32_t* counts);

/* K3 building block: C[M][N] (op)= A[M][K] . W[N][K]^T + bias (device pointers;
 * A, W fp16 row-major; epilogue 0 f16 out, 1 f16 quick_gelu, 2 f16 gelu_erf,
 * 3 f32 C += , 4 f32 out). N % 128 == 0, K % 64 == 0; bias and C 16-byte aligned. */
int mrag_gemm_nt(const void* A, const void* W, const float* bias, void* C, int32_t M, int32_t N, int32_t K,
                 int32_t epilogue, void* stream);
/* The same with the kernel chosen: 0 the automatic rule, 1 K3 (128 x 128 tiles), 2 K3d (persistent
 * 256 x 256), 3 K3s (M <= 64), 4 K3w (weight-stationary: f16 epilogues, K 384 / 512, N % 192 == 0 or
 * N % 256 == 0, M >= 4096). Every kernel gives the same bytes (one accumulation order); this entry
 * exists for per-kernel timing and the bit-identity tests. */
int mrag_gemm_nt_kernel(const void* A, const void* W, const float* bias, void* C, int32_t M, int32_t N, int32_t K,
                        int32_t epilogue, int32_t kernel, void* stream);


#ifdef __cplusplus
}
#endif

#endif /* MRAG_H */
