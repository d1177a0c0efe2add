/*
 * miner_corpus.h — C ABI of the full-corpus ranking path of libminer_hip.so (MI355X, gfx950):
 * BASELINE config 5 ("1M users x 200k news, history=200, K=64, d=768, fp16"), SURVEY.md §7 step 6
 * and §8(d): every user against every news item of a table with the MINER click score, and a fused
 * top-k — the U x N score matrix is never materialised.
 *
 * The arithmetic is the reference's (MrRobot2211/miner, src/model/model.py), with the candidate set
 * of an impression replaced by the whole news table:
 *
 *   miner_encode_users(...)   per user: PolyAttention.forward (model.py:159-185) -> mui [K, d], and
 *                             for score_type 'weighted' the TargetAwareAttention projection
 *                             proj = gelu(mui · W2ᵀ) (model.py:212) [K, d].
 *   miner_rank_topk(...)      per (user, news n): M_k = mui_k · e_n (model.py:127) and
 *                             weighted: Σ_k softmax_k(proj_k · e_n) · M_k (model.py:213-214)
 *                             max / mean: max_k / mean_k M_k (model.py:128-131);
 *                             per user the topk best (score desc, news id asc on ties).
 *
 * Conventions are those of miner_score.h. dtype: MINER_DTYPE_F32 (exact fp32, parity mode),
 * MINER_DTYPE_BF16 or MINER_DTYPE_F16 (16-bit operands, fp32 accumulation and softmax).
 * Limits: L <= 256, K <= 64, Dc <= 256, d % 64 == 0 (fp32: d % 32 == 0), d <= 1024,
 * topk <= 256.
 */
#ifndef MINER_CORPUS_H
#define MINER_CORPUS_H

#include <stddef.h>
#include <stdint.h>

#include "miner_score.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MINER_CORPUS_MAX_L 256
#define MINER_CORPUS_MAX_K 64
#define MINER_CORPUS_MAX_TOPK 256

/* Weights of the user encoder (Dc and K up to 256 / 64), packed once per model:
 *   w_poly [Dc, d], context_codes [K, Dc], w_target [d, d] (NULL: no projection), all dtype. */
size_t miner_encoder_packed_bytes(int dtype, int d, int Dc, int K);
int miner_encoder_pack(void* stream, int dtype, const void* w_poly, const void* context_codes,
                       const void* w_target, int d, int Dc, int K, void* packed);

/*
 * Encode U users.
 *   history    [U, L, d] dtype (his_ids NULL), or the news table [n_news, d] with
 *   his_ids    [U, L] int32 rows of it (gather mode; clamped to [0, n_news) on the device)
 *   his_mask   [U, L] uint8, his_bias [U, L] fp32 or NULL (added to the logits, model.py:176)
 *   mui_f32    [U, K, d] fp32 out or NULL;  user_mui [U, K, d] dtype out (ranking operand);
 *   user_proj  [U, K, d] dtype out, gelu(mui · W2ᵀ), or NULL (the pack must hold w_target).
 */
int miner_encode_users(void* stream, int dtype, const void* history, const int32_t* his_ids, int n_news,
                       const uint8_t* his_mask, const float* his_bias, const void* packed, int U, int L,
                       int d, int Dc, int K, float* mui_f32, void* user_mui, void* user_proj);

/*
 * Rank every news item of `news` [N, d] for each of U users; top_scores [U, topk] fp32 and
 * top_ids [U, topk] int32, best first (rows past N: -inf / -1). score_type as miner_score.h
 * (WEIGHTED needs user_proj).
 */
int miner_rank_topk(void* stream, int dtype, int score_type, const void* user_mui, const void* user_proj,
                    const void* news, int U, int N, int d, int K, int topk, float* top_scores,
                    int32_t* top_ids);

/*
 * The same with a caller-owned device workspace of workspace_bytes bytes (16-byte aligned; NULL: the
 * form above). With a workspace of at least miner_rank_topk_workspace_bytes(U, topk) bytes, on a
 * 256-CU device, the split form runs: the news table is split in 8 slices whose per-user top-k
 * lists are merged by a second launch (8x the workgroups for small user batches), the users mapped
 * so that the CUs of one XCD share 8 users' rows in their L2. A smaller workspace is never written
 * (the unsplit form runs). Same results as miner_rank_topk, bit for bit.
 * miner_rank_topk_workspace_bytes returns 0 where the split form cannot run (not a 256-CU device,
 * invalid arguments). miner_rank_topk_split_recommended(U) is 1 where the split form is the faster
 * one (fewer than 256 two-user tiles: U <= 510), so a caller passes a workspace only then.
 */
size_t miner_rank_topk_workspace_bytes(int U, int topk);
int miner_rank_topk_split_recommended(int U);
int miner_rank_topk_ws(void* stream, int dtype, int score_type, const void* user_mui, const void* user_proj,
                       const void* news, int U, int N, int d, int K, int topk, float* top_scores,
                       int32_t* top_ids, void* workspace, size_t workspace_bytes);

#ifdef __cplusplus
}
#endif

#endif /* MINER_CORPUS_H */
