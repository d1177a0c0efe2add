// miner_metrics.hip — per-impression ranking metrics on the GPU (gfx950), SURVEY.md §8 row f1.
//
// The reference computes group_auc / mrr / ndcg@k / hit@k in a Python loop over impressions
// (src/evaluation.py:36-84, :177-249; ~0.9 ms per impression). Here one wave scores one impression:
// each lane takes candidates i = lane, lane+64, ... and compares its score with every other
// candidate of the impression (O(C²) compares, C is tens to a few hundred), which yields exactly
//   rank_i  = #{j : s_j > s_i} + #{j < i : s_j == s_i}  (descending, ties in candidate order =
//             Python's stable sorted(..., reverse=True) of is_hit, evaluation.py:245-249)
//   auc     = Σ_{pos i} (#{neg j : s_j < s_i} + ½ #{neg j : s_j == s_i}) / (P·N)
//             (the Mann-Whitney form of sklearn's roc_auc_score, ties counted one half)
//   mrr     = Σ_{pos i} 1/(rank_i + 1) / P                      (evaluation.py:177-192)
//   ndcg@k  = Σ_{pos i, rank_i < k} 1/log2(rank_i + 2) / Σ_{t < min(P,k)} 1/log2(t + 2)
//             (binary gains 2^y - 1, evaluation.py:195-231)
//   hit@k   = [∃ pos i : rank_i < k]
// MRR and nDCG in the reference use np.argsort(..)[::-1], whose order among tied scores is numpy's;
// any order gives the same value unless a tie mixes labels, which is flagged for the host.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/miner_metrics.h"
#include "../../include/miner_score.h"

namespace {

struct Ks {
  int k[MINER_METRICS_MAX_K];
};

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void impression_metrics_kernel(const float* __restrict__ scores,
                                                                  const uint8_t* __restrict__ labels,
                                                                  const int32_t* __restrict__ offs, int G, Ks ks,
                                                                  int nk, double* __restrict__ out,
                                                                  uint8_t* __restrict__ mixed) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (g >= G) return;   // whole waves exit together (g is wave-uniform)
  const int base = offs[g], C = offs[g + 1] - base;
  const float* s = scores + base;
  const uint8_t* y = labels + base;

  double auc_num = 0.0, rr = 0.0, dcg[MINER_METRICS_MAX_K], pos = 0.0;
  int hit[MINER_METRICS_MAX_K];
#pragma unroll
  for (int t = 0; t < MINER_METRICS_MAX_K; ++t) { dcg[t] = 0.0; hit[t] = 0; }
  int mix = 0;
  for (int i = lane; i < C; i += 64) {
    const float si = s[i];
    const int yi = y[i] != 0;
    int gt = 0, eqb = 0, neg_lt = 0, neg_eq = 0, other_eq = 0;
    for (int j = 0; j < C; ++j) {
      const float sj = s[j];
      const int yj = y[j] != 0;
      gt += sj > si;
      const int eq = (sj == si) & (j != i);
      eqb += eq & (j < i);
      neg_lt += (!yj) & (sj < si);
      neg_eq += (!yj) & eq;
      other_eq |= eq & (yj != yi);
    }
    mix |= other_eq;
    if (yi) {
      const int rank = gt + eqb;
      pos += 1.0;
      auc_num += (double)neg_lt + 0.5 * (double)neg_eq;
      rr += 1.0 / (double)(rank + 1);
#pragma unroll
      for (int t = 0; t < MINER_METRICS_MAX_K; ++t) {
        if (t < nk && rank < ks.k[t]) {
          dcg[t] += 1.0 / log2((double)rank + 2.0);
          hit[t] = 1;
        }
      }
    }
  }
  auc_num = wave_sum(auc_num);
  rr = wave_sum(rr);
  pos = wave_sum(pos);
#pragma unroll
  for (int t = 0; t < MINER_METRICS_MAX_K; ++t) {
    dcg[t] = wave_sum(dcg[t]);
    hit[t] = wave_sum(hit[t]);
  }
  mix = wave_sum(mix);
  if (lane == 0) {
    const int stride = 2 + 2 * nk;
    double* o = out + (size_t)g * stride;
    const double P = pos, N = (double)C - pos;
    o[0] = (P > 0.0 && N > 0.0) ? auc_num / (P * N) : (double)NAN;
    o[1] = rr / P;   // 0/0 = NaN with no click, as the reference
    for (int t = 0; t < nk; ++t) {
      double idcg = 0.0;
      const int top = (int)P < ks.k[t] ? (int)P : ks.k[t];
      for (int r = 0; r < top; ++r) idcg += 1.0 / log2((double)r + 2.0);
      o[2 + t] = dcg[t] / idcg;
      o[2 + nk + t] = hit[t] ? 1.0 : 0.0;
    }
    if (mixed) mixed[g] = mix ? 1 : 0;
  }
}

}  // namespace

extern "C" int miner_impression_metrics(void* stream, const float* scores, const uint8_t* labels,
                                        const int32_t* offsets, int G, const int32_t* ks, int nk, double* out,
                                        uint8_t* mixed_ties) {
  if (G < 0 || nk < 0 || nk > MINER_METRICS_MAX_K) return MINER_EINVAL;
  if (G == 0) return MINER_OK;
  if (!scores || !labels || !offsets || !out || (nk > 0 && !ks)) return MINER_EINVAL;
  Ks k{};
  for (int t = 0; t < nk; ++t) {
    if (ks[t] <= 0) return MINER_EINVAL;
    k.k[t] = ks[t];
  }
  const int per_block = 4;   // one wave per impression
  hipLaunchKernelGGL(impression_metrics_kernel, dim3((G + per_block - 1) / per_block), dim3(64 * per_block), 0,
                     static_cast<hipStream_t>(stream), scores, labels, offsets, G, k, nk, out, mixed_ties);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}
