/*
 * miner_wide.h — C ABI of the wide-shape scoring tail of libminer_hip.so (MI355X, gfx950).
 *
 * The reference (MrRobot2211/miner @ 2024-08-07) puts no limit on the number of interests
 * (Miner(num_context_codes=K), src/model/model.py:18-21, PolyAttention :141-157) or on the history
 * length (PolyAttention.forward :159-185 is shape-generic). The fused kernels of miner_score.h and
 * miner_news.h keep a whole impression on one CU and stop at K <= 32, L <= 64. Past that, an
 * impression is scored in two launches:
 *
 *   miner_encode_users (miner_corpus.h)   PolyAttention -> mui [B,K,d] and, for 'weighted',
 *                                         proj = gelu(mui · W2ᵀ) [B,K,d]     (model.py:159-185, :212)
 *                                         for L <= 256, K <= 64, Dc <= 256, d <= 768
 *   miner_score_wide (below)              M = Cand · muiᵀ (:127), the aggregation (:128-136) with
 *                                         TargetAwareAttention (:213-214) for 'weighted'
 *
 * and TargetAwareAttention.forward alone (:200-216) for K > 32 is miner_wide_proj (its projection,
 * :212) + miner_score_wide with the given value tensor.
 *
 * Conventions are those of miner_score.h: caller-owned 16-byte-aligned device memory, enqueued on
 * `stream`, returns 0 / a negative MINER_E* code / a positive hipError_t. dtype MINER_DTYPE_F32 is
 * the parity mode (exact fp32 fma chains on the fp32 matrix cores, libm exp / erf), MINER_DTYPE_BF16
 * and MINER_DTYPE_F16 use 16-bit operands with fp32 accumulation.
 */
#ifndef MINER_WIDE_H
#define MINER_WIDE_H

#include <stddef.h>
#include <stdint.h>

#include "miner_score.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MINER_WIDE_MAX_K 64

/*
 * Scores of B impressions from their users' interest vectors.
 *   user_mui  [B, K, d] dtype   multi_user_interest (unused when `value` is given)
 *   user_proj [B, K, d] dtype   gelu(mui · W2ᵀ) (score_type WEIGHTED only, else NULL)
 *   cand      candidate rows, dtype: [B, C, d] (cand_ids and cand_offsets NULL), [N, d] with
 *             cand_offsets [B + 1] int32 (ragged), or the news table [n_news, d] with cand_ids
 *             [B, C] / [N] int32 rows of it (clamped to [0, n_news) on the device)
 *   value     [B, C, K] / [N, K] fp32 or NULL: the matching scores M given by the caller
 *             (TargetAwareAttention alone, model.py:200-216; score_type WEIGHTED)
 *   scores    [B, C] / [N] fp32 out
 * Limits: K <= MINER_WIDE_MAX_K, d % 32 == 0 (16-bit: d % 64 == 0), any C.
 */
int miner_score_wide(void* stream, int dtype, int score_type, const void* user_mui, const void* user_proj,
                     const void* cand, const int32_t* cand_ids, int n_news, const int32_t* cand_offsets,
                     const float* value, int B, int C, int d, int K, float* scores);

/*
 * out[r, :] = gelu(x[r, :] · W2ᵀ) for r < R (TargetAwareAttention's projection, model.py:212;
 * torch.nn.functional.gelu, exact erf).  x [R, d], w_target [d, d] (nn.Linear layout: out x in),
 * out [R, d], all dtype.  d % 64 == 0.
 */
int miner_wide_proj(void* stream, int dtype, const void* x, const void* w_target, int R, int d, void* out);

/* 0 if (dtype, L, d, Dc, K) is scored by the wide path (miner_encode_users + miner_score_wide). */
int miner_wide_supported(int dtype, int L, int d, int Dc, int K);

#ifdef __cplusplus
}
#endif

#endif /* MINER_WIDE_H */
