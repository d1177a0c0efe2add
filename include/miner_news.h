/*
 * miner_news.h — C ABI of the news-side precompute path of libminer_hip.so (MI355X, gfx950):
 * SURVEY.md §8(f2) "news-table gather input mode + news-side precompute".
 *
 * The reference (MrRobot2211/miner @ 2024-08-07, src/model/model.py) scores an impression from the
 * news encoder's output for its history and candidates. Two of its per-impression products only
 * depend on ONE news item each, so over a news table they are computed once per news item instead
 * of once per (impression, history slot):
 *
 *   logits[n, k] = Σ_c tanh(W1 e_n)_c · Q[k, c]        PolyAttention.forward, model.py:171-174
 *   proj[n, :]   = W2 · e_n                             the linear of TargetAwareAttention,
 *                                                       model.py:212, before the GELU
 *
 * and by linearity mui_k · W2ᵀ = Σ_l A[k,l] · proj[his_l] (A = the attention weights of
 * model.py:181), so per impression only the contractions over the history (K×L×d: mui and the
 * TargetAwareAttention pre-activation) and over the candidates (C×d×K) remain:
 *
 *   miner_news_precompute(...)  per news row: logits (fp32) and proj (dtype). Replaces, for a whole
 *                               news table, model.py:171-174 and the W2 product of :212.
 *   miner_score_news(...)       per impression, from news ids: A = softmax over the history of the
 *                               gathered logits (+ category bias, masked slots = 1e-30, model.py:
 *                               176-181); mui = A·E (:182); X = gelu(A·proj) (= gelu(mui·W2ᵀ),
 *                               :212); M = Cand·muiᵀ (:127); the aggregation (:128-136, with
 *                               TargetAwareAttention :213-214 for 'weighted'). Replaces
 *                               Miner.forward after the news encoder, model.py:113-138.
 *
 * Conventions are those of miner_score.h (caller-owned 16-byte-aligned device memory, enqueued on
 * `stream`, 0 / negative MINER_E* / positive hipError_t). dtype MINER_DTYPE_F32 is the parity mode
 * (fp32 tensors, fp32-class products: within 1e-5 of the reference), MINER_DTYPE_BF16 the
 * throughput mode (bf16 operands, fp32 accumulation, logits always fp32).
 * Limits: L <= 64, K <= 32 with K % 4 == 0, d % 64 == 0 and d <= 1024, Dc <= 256, and at most
 * MINER_NEWS_MAX_CAND candidates per impression (dense C or every ragged C_b).
 */
#ifndef MINER_NEWS_H
#define MINER_NEWS_H

#include <stddef.h>
#include <stdint.h>

#include "miner_score.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MINER_NEWS_MAX_CAND 512

/*
 * Per-news precompute over a table.
 *   news_table     [n_news, d]  dtype  the news encoder's output (row 0 may be the pad news)
 *   packed_weights              dtype  miner_pack_weights() output (w_target needed for news_proj)
 *   news_logits    [n_news, K]  fp32   out
 *   news_proj      [n_news, d]  dtype  out, or NULL (score_type max / mean need no projection)
 * dtype MINER_DTYPE_F32: the W1 / W2 products on fp16 pairs (one power-of-two unit per table row
 * and per weight row, three f16 MFMAs per product: the operand form of the scoring kernels), within
 * 1.5x the fp32 MFMA's error against float64; MINER_DTYPE_F32_MFMA: every product on the fp32 MFMA
 * (exact fp32 fma chains; also the form at d = 1024 with Dc = 256, where the pair form's 128 bytes of
 * row units do not fit beside the 160 KiB carve). Both take the same fp32 packed weights.
 */
int miner_news_precompute(void* stream, int dtype, const void* news_table, int n_news,
                          const void* packed_weights, int d, int Dc, int K, float* news_logits,
                          void* news_proj);

/*
 * Score B impressions given as news ids (the reference's eval layout, reader.py:351-379).
 *   news_table [n_news, d] dtype, news_logits [n_news, K] fp32, news_proj [n_news, d] dtype (NULL
 *   unless score_type == WEIGHTED) — the table and its miner_news_precompute() outputs;
 *   his_ids [B, L] int32, his_mask [B, L] uint8, his_bias [B, L] fp32 or NULL,
 *   cand_ids [B, C] int32 (cand_offsets NULL) or [sum C_b] with cand_offsets [B + 1] int32;
 *   scores [sum C_b] fp32 (may be NULL only for score_type NONE);
 *   user_out [B, K, d] fp32 multi_user_interest, or NULL.
 * Ids are clamped to [0, n_news) on the device (never read out of bounds); the Python wrapper
 * validates them and raises.
 */
int miner_score_news(void* stream, int dtype, int score_type, const void* news_table,
                     const float* news_logits, const void* news_proj, int n_news,
                     const int32_t* his_ids, const uint8_t* his_mask, const float* his_bias,
                     const int32_t* cand_ids, const int32_t* cand_offsets, int B, int L, int C,
                     int d, int K, float* scores, float* user_out);

/*
 * fp32 scoring on the fp16 matrix cores (miner_amd/csrc/news_x2.hip; the bench headline since
 * round 3). Every fp32 operand x is carried as an exact-sum fp16 pair in a power-of-two scale s:
 * x·s = hi + lo, hi = fp16(x·s), lo = fp16(x·s - hi), |x·s - hi - lo| <= 2^-22·|x·s|; a product
 * a·b is lo_a·hi_b + hi_a·lo_b + hi_a·hi_b on v_mfma_f32_16x16x32_f16 (fp16 products are exact in
 * fp32; fp32 accumulation). The pair table takes 4 bytes per element, as fp32.
 *
 * miner_news_split_x2: src [n, d] fp32 -> dst [n, d] pairs: per row, per 64-column chunk, the 64
 *   hi then the 64 lo fp16 values (256 bytes) of x / u_r, with one power-of-two unit per row
 *   u_r = 2^(e_r - 14), max|row r| < 2^e_r, written to row_unit[r] (n floats, device memory).
 *   Apply it to the news table (the x2 table) and to miner_news_precompute's fp32 news_proj.
 *   d % 64 == 0, d <= 1024.
 * miner_score_news_x2: miner_score_news (fp32) from the pair tables: table_unit / proj_unit are
 *   the row units of the two splits (proj2 / proj_unit NULL unless score_type == WEIGHTED).
 *   Same limits, plus n_news·d·4 < 2^32 (32-bit row offsets). disagree_out [B] fp32 or NULL:
 *   the eval loss's per-impression disagreement term, mean over k != k' of cos(mui_k, mui_k') with
 *   the diagonal zeroed (src/loss.py:81, src/utils.py:9-29), formed in the kernel from the Gram
 *   matrix of mui (no mui is written unless user_out is given).
 *   Wide shapes (round 5): L up to MINER_NEWS_X2W_MAX_L and K up to MINER_NEWS_X2W_MAX_K (K % 4 ==
 *   0) are scored by the kernel's wide form (news_score_x2w: 32-column steps, history groups in four
 *   blocks of 32, four interest tiles); the reference limits neither (model.py:18-21, :159-185).
 *   news_logits then has K columns: miner_news_precompute takes K <= 32, so a caller computes the
 *   logits in 32-interest slices of Q (miner_pack_weights of each slice) and places them side by
 *   side. disagree_out must be NULL there (the eval loss then reads user_out).
 */
#define MINER_NEWS_X2W_MAX_L 128
#define MINER_NEWS_X2W_MAX_K 64
int miner_news_split_x2(void* stream, const float* src, int n, int d, void* dst, float* row_unit);
int miner_score_news_x2(void* stream, int score_type, const void* table2, const float* table_unit,
                        const float* news_logits, const void* proj2, const float* proj_unit,
                        int n_news, const int32_t* his_ids, const uint8_t* his_mask,
                        const float* his_bias, const int32_t* cand_ids, const int32_t* cand_offsets,
                        int B, int L, int C, int d, int K, float* scores, float* user_out,
                        float* disagree_out);

/* 0 if (dtype, L, d, Dc, K) is supported by the news path, else the MINER_E* code. Host-only. */
int miner_news_supported(int dtype, int L, int d, int Dc, int K);

#ifdef __cplusplus
}
#endif

#endif /* MINER_NEWS_H */
