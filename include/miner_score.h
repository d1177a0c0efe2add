/*
 * miner_score.h — C ABI of libminer_hip.so, the MI355X (gfx950) scoring path of MINER.
 *
 * The reference (MrRobot2211/miner @ 2024-08-07) has no FFI: its boundary is the Python
 * nn.Module contract of src/model/model.py. These entry points replace the tensor math of that
 * contract, one per reference interface, and are what a ctypes binding in the reference's
 * src/model/model.py would call (the binding is shown in INTEGRATION.md):
 *
 *   miner_pack_weights(...)
 *       one-time repack of the module parameters poly_attn.linear.weight, poly_attn.context_codes
 *       and target_aware_attn.linear.weight (model.py:155-157, :198) into the kernel layout.
 *   miner_score(..., score_type = WEIGHTED|MAX|MEAN)
 *       replaces Miner.forward after the news encoder, src/model/model.py:113-138
 *       (PolyAttention.forward :159-185 -> Cand·muiᵀ :127 -> aggregation :128-136, with
 *       TargetAwareAttention.forward :200-216 for 'weighted').
 *   miner_score(..., score_type = NONE)
 *       replaces PolyAttention.forward alone, src/model/model.py:159-185 (user_out required).
 *   miner_target_aware(...)
 *       replaces TargetAwareAttention.forward, src/model/model.py:200-216.
 *
 * Conventions (all entry points):
 *   - every pointer is caller-owned DEVICE memory, row-major and contiguous, 16-byte aligned;
 *     nothing is allocated inside, nothing synchronises: work is enqueued on `stream`
 *     (a hipStream_t; NULL = the default stream) and the call returns immediately;
 *   - `dtype` selects the element type of the activation AND weight tensors and the arithmetic:
 *     MINER_DTYPE_F32 = fp32 tensors, fp32-class products (the parity mode: within 1e-5 of the
 *     reference's fp32 path; see each entry point for the form, e.g. fp16 pairs on the fp16
 *     matrix cores for miner_score), MINER_DTYPE_F32_MFMA = the same fp32 tensors with every product on
 *     the fp32 MFMA (exact fp32 fma chains), MINER_DTYPE_BF16 = bf16 operands with fp32
 *     accumulation, the throughput mode. Masks are uint8 (0/1, torch.bool storage), offsets int32,
 *     bias/scores/user_out fp32;
 *   - return 0 on success, a negative MINER_E* code for invalid arguments (nothing launched), or a
 *     positive hipError_t from the launch. miner_strerror() names the code.
 *   - no global state beyond a cached device-attribute query: thread-safe per stream. The product
 *     library reads no environment variable; every kernel form is chosen by the arguments. Two
 *     timing-ablation switches of the diagnostic tools (MINER_NEWS_ABL: miner_score_news;
 *     MINER_FF_ABL: miner_fastformer_score) are read once per process, 0 when unset.
 */
#ifndef MINER_SCORE_H
#define MINER_SCORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MINER_ABI_VERSION 5

/* MINER_DTYPE_F16 is accepted by the full-corpus entry points of miner_corpus.h only (config 5).
 * MINER_DTYPE_F32_MFMA (fp32 tensors, every product on the fp32 MFMA) by miner_score,
 * miner_score_gather, miner_target_aware and the host queries of this header; MINER_DTYPE_F32_X6
 * (fp32 tensors, news_score32's products as bf16x6 on the bf16 matrix cores) by miner_score_news
 * and miner_news_supported (miner_news.h). */
enum miner_dtype {
  MINER_DTYPE_F32 = 0,
  MINER_DTYPE_BF16 = 1,
  MINER_DTYPE_F16 = 2,
  MINER_DTYPE_F32_MFMA = 3,
  MINER_DTYPE_F32_X6 = 4
};

/* src/model/model.py:128-136 ('weighted' = TargetAwareAttention). NONE = PolyAttention only. */
enum miner_score_type {
  MINER_SCORE_WEIGHTED = 0,
  MINER_SCORE_MAX = 1,
  MINER_SCORE_MEAN = 2,
  MINER_SCORE_NONE = 3
};

enum miner_error {
  MINER_OK = 0,
  MINER_EINVAL = -1,      /* null pointer, bad enum, non-positive size */
  MINER_ESHAPE = -2,      /* shape outside what this build supports (see miner_supported) */
  MINER_EALIGN = -3,      /* a pointer is not 16-byte aligned */
  MINER_ELDS = -4         /* the shape needs more LDS than one CU has */
};

/*
 * Weights, packed once per model (they are static during evaluation) into the kernel's tiled
 * layout: 32-row x 32-column tiles, rows in the order the MFMA accumulators want them, zero padded
 * (see DESIGN.md "Packed weights").  `packed` is caller-owned device memory of
 * miner_packed_weights_bytes() bytes, 16-byte aligned.
 *   w_poly        [Dc, d]  dtype  poly_attn.linear.weight          (model.py:155)
 *   context_codes [K, Dc]  dtype  poly_attn.context_codes          (model.py:156-157)
 *   w_target      [d, d]   dtype  target_aware_attn.linear.weight  (model.py:198); NULL when the
 *                                 model has no TargetAwareAttention (score_type max/mean)
 */
size_t miner_packed_weights_bytes(int dtype, int d, int Dc, int K);
int miner_pack_weights(void* stream, int dtype, const void* w_poly, const void* context_codes,
                       const void* w_target, int d, int Dc, int K, void* packed);

/*
 * TargetAwareAttention.linear.weight [d, d] alone (model.py:198), for miner_target_aware with
 * Dc = 0: the W2 part of the miner_pack_weights layout, miner_target_weights_bytes() bytes.
 */
size_t miner_target_weights_bytes(int dtype, int d);
int miner_pack_target_weights(void* stream, int dtype, const void* w_target, int d, void* packed);

/*
 * Score B impressions.
 * dtype MINER_DTYPE_F32 (the reference's precision): the W1·Eᵀ and W2·muiᵀ contractions run on
 * fp16 pairs (each fp32 operand x of a row with a power-of-two unit u carried as hi = f16(x/u),
 * lo = f16(x/u - hi); lo·hi + hi·lo + hi·hi on the fp16 matrix cores, fp32 accumulation, the units
 * applied exactly; error vs float64 within 1.5x the fp32 MFMA's), the rest on the fp32 MFMA. The
 * fp32 packed buffer carries pair copies of W1 and W2 and their row units for this; where the LDS
 * carve leaves room for two workgroups per CU (small shapes), W1·Eᵀ stays bf16x6 (three bf16 terms
 * per operand, six partial products). dtype MINER_DTYPE_F32_MFMA: every product on the fp32 MFMA
 * (exact fp32 fma chains; the Python layer passes it under MINER_DENSE_FP32=mfma32).
 *   history      [B, L, d]  dtype  clicked-news embeddings, left-padded (reader.py:369)
 *   his_mask     [B, L]     uint8  1 = real click, 0 = pad (entities.py:395)
 *   his_bias     [B, L]     fp32   optional category bias, already averaged over the candidates
 *                                  (model.py:113-122, :176); NULL = use_category_bias off
 *   candidates   [sum C_b, d] dtype candidate-news embeddings, impression-major
 *   cand_offsets [B + 1]    int32  optional CSR offsets of each impression's candidates;
 *                                  NULL = dense, C_b = C for every impression
 *   packed_weights          dtype  miner_pack_weights() output (w_target packed when
 *                                  score_type == WEIGHTED)
 *   scores       [sum C_b]  fp32   matching scores (model.py:138 second output); may be NULL
 *                                  only when score_type == NONE
 *   user_out     [B, K, d]  fp32   optional multi_user_interest (model.py:138 first output)
 */
int miner_score(void* stream, int dtype, int score_type,
                const void* history, const uint8_t* his_mask, const float* his_bias,
                const void* candidates, const int32_t* cand_offsets, const void* packed_weights,
                int B, int L, int C, int d, int Dc, int K,
                float* scores, float* user_out);

/*
 * miner_score with the news rows gathered by id from a device news-embedding table:
 *   news_table [n_news, d] dtype  the news encoder's output for every news item, computed once
 *                                 (the reference re-encodes each sample's news through
 *                                 Miner.forward, model.py:104-111, fed by reader.py:366-379 and
 *                                 entities.py:375-411)
 *   his_ids    [B, L]      int32  table rows of the (left-padded) history; the pad news is a row
 *   cand_ids   [sum C_b]   int32  table rows of the candidates (CSR by cand_offsets, or [B, C])
 * Everything else as miner_score. Ids outside [0, n_news) are clamped (never read out of bounds);
 * the Python wrapper validates them and raises.
 */
int miner_score_gather(void* stream, int dtype, int score_type, const void* news_table, int n_news,
                       const int32_t* his_ids, const uint8_t* his_mask, const float* his_bias,
                       const int32_t* cand_ids, const int32_t* cand_offsets, const void* packed_weights,
                       int B, int L, int C, int d, int Dc, int K, float* scores, float* user_out);

/*
 * TargetAwareAttention.forward (model.py:200-216) on its own:
 *   query [B, K, d] dtype (multi_user_interest), key [sum C_b, d] dtype (candidates),
 *   value [sum C_b, K] fp32 (matching scores Cand·muiᵀ), packed_weights with w_target packed
 *   (Dc = the context-code dim they were packed with, or 0 for a miner_pack_target_weights
 *   buffer) -> out [sum C_b] fp32.
 */
int miner_target_aware(void* stream, int dtype,
                       const void* query, const void* key, const float* value,
                       const int32_t* cand_offsets, const void* packed_weights, int Dc,
                       int B, int C, int d, int K, float* out);

/* 0 if (dtype, L, d, Dc, K) is supported by this build, else the MINER_E* code miner_score
 * would return. Host-only, no device call. */
int miner_supported(int dtype, int L, int d, int Dc, int K);

/* LDS bytes one workgroup of miner_score uses for this shape (host-only). */
int miner_lds_bytes(int dtype, int score_type, int L, int d, int Dc);

const char* miner_strerror(int code);
int miner_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MINER_SCORE_H */
