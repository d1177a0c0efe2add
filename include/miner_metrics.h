/*
 * miner_metrics.h — C ABI of the per-impression ranking metrics in libminer_hip.so (gfx950).
 *
 * Replaces the per-impression metric loop of the reference evaluator
 * (src/evaluation.py:36-84 BaseEvaluator.compute_scores with compute_mrr_score :177-192,
 * compute_dcg_score / compute_ndcg_score :195-231, is_hit :245-249 and sklearn's roc_auc_score for
 * group_auc :56-61), which the reference runs as a Python loop (~0.9 ms per impression). The
 * flattened global `auc` (:53-55) is not per-impression: miner_global_auc computes it on the device.
 *
 * Conventions as in miner_score.h: caller-owned device memory, asynchronous on `stream`.
 */
#ifndef MINER_METRICS_H
#define MINER_METRICS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MINER_METRICS_MAX_K 8

/*
 * Per-impression metrics of G impressions in CSR layout (impression g owns [offsets[g],
 * offsets[g+1]) of `scores` / `labels`, device memory), in one pass; `ks` is a HOST array of
 * nk <= MINER_METRICS_MAX_K cut-offs (the @k of ndcg@k / hit@k):
 *   out [G][2 + 2*nk] float64: group AUC (ties count 1/2; NaN when the impression has a single
 *                              class), MRR, nDCG@ks[0..nk), hit@ks[0..nk)
 *   mixed_ties [G] uint8 (may be NULL): 1 when two candidates with different labels share a score.
 * `scores` are what the reference ranks (the sigmoid probabilities of eval_batch,
 * evaluation.py:165), fp32. hit@k ranks ties in candidate order (Python's stable `sorted`, :247) and
 * group AUC averages ties, both exactly; MRR and nDCG follow `np.argsort(..)[::-1]` (:188, :208),
 * whose order among tied scores is numpy's — exact here unless mixed_ties[g] is set, in which case
 * the caller recomputes that impression's MRR/nDCG on the host with the reference functions.
 */
int miner_impression_metrics(void* stream, const float* scores, const uint8_t* labels,
                             const int32_t* offsets, int G, const int32_t* ks, int nk,
                             double* out, uint8_t* mixed_ties);

/*
 * The flattened global `auc` of the reference (src/evaluation.py:53-55: sklearn roc_auc_score over
 * every (label, probability) pair of the eval set), exactly, on the device: a radix sort of the
 * scores (rocPRIM), a reduce-by-key over runs of equal scores and an integer Mann-Whitney sum with
 * ties counted 1/2.  n (int64_t) <= 2^31 - 1 pairs, MINER_ESHAPE past it (the rocPRIM sort's
 * 32-bit sizes); `scores` fp32, `labels` uint8 0/1 (device memory);
 * `workspace` caller-owned device memory of at least miner_auc_workspace_bytes(n) bytes (about
 * 33 bytes per pair); `auc_out` one float64 in DEVICE memory, NaN when one class is absent
 * (sklearn raises there).
 */
size_t miner_auc_workspace_bytes(int64_t n);
int miner_global_auc(void* stream, const float* scores, const uint8_t* labels, int64_t n, void* workspace,
                     size_t workspace_bytes, double* auc_out);

#ifdef __cplusplus
}
#endif

#endif /* MINER_METRICS_H */
