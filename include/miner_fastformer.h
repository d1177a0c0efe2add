/*
 * miner_fastformer.h — C ABI of the FastFormer user-encoder path of libminer_hip.so (MI355X,
 * gfx950): BASELINE config 4, SURVEY.md §8 row f3.
 *
 * Replaces, after the news encoder, the tensor math of the reference's FastFormer model
 * (MrRobot2211/miner, src/model/model.py):
 *
 *   miner_fastformer_pack(...)
 *       one-time repack of FastFormer.fast_attn (FastformerEncoder, model.py:482-545) parameters.
 *   miner_fastformer_score(...)
 *       FastFormer.forward after the news encoder, model.py:318-322:
 *         user = FastformerEncoder(history, his_mask)          (model.py:511-545, 2 x
 *                FastformerLayer :469-480 = FastAttention :458-467 (FastSelfAttention :373-455 +
 *                BertSelfOutput) + BertIntermediate + BertOutput, then AttentionPooling :345-371)
 *         scores[c] = candidates[c] · user                     (model.py:322)
 *   miner_fastformer_score_gather(...)
 *       the same with history / candidate rows taken by id from a device news-embedding table.
 *
 * Conventions are those of miner_score.h (device pointers, 16-byte aligned, enqueued on `stream`,
 * MINER_DTYPE_F32 = exact fp32 parity mode, MINER_DTYPE_BF16 = bf16 operands with fp32
 * accumulation; 0 / negative MINER_E* / positive hipError_t).  The hidden size is fixed at 256
 * (16 heads x 16, intermediate 256: the reference's BertConfig, model.py:245-266).
 */
#ifndef MINER_FASTFORMER_H
#define MINER_FASTFORMER_H

#include <stddef.h>
#include <stdint.h>

#include "miner_score.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MINER_FF_HIDDEN 256
#define MINER_FF_MAX_L 64          /* history positions per impression supported by the kernel */
/* floats in the flat parameter blob: FastformerEncoder.state_dict() values, flattened and
 * concatenated in state_dict order (encoders.0.* (20 tensors), encoders.1.*,
 * position_embeddings.weight, LayerNorm.{weight,bias}, poolers.0.att_fc1.{weight,bias},
 * poolers.0.att_fc2.{weight,bias}) */
#define MINER_FF_PARAM_FLOATS 940097

/*
 * params  [MINER_FF_PARAM_FLOATS] fp32 device blob (layout above) -> packed (device memory of
 * miner_fastformer_packed_bytes(dtype) bytes): the 13 hidden x hidden matrices and the two
 * 16 x hidden head projections per layer as 32x32 MFMA tiles in dtype, biases / LayerNorm
 * vectors / position embeddings kept in fp32.
 */
size_t miner_fastformer_packed_bytes(int dtype);
int miner_fastformer_pack(void* stream, int dtype, const float* params, void* packed);

/*
 * history      [B, L, 256]  dtype  clicked-news embeddings (left-padded, reader.py:369)
 * his_mask     [B, L]       uint8  1 = real click (entities.py:395); 0 -> additive -10000
 *                                  (model.py:519-521) and excluded from the pooling (:366)
 * candidates   [sum C_b, 256] dtype  candidate embeddings, impression-major
 * cand_offsets [B + 1]      int32  impression b owns candidates [off[b], off[b+1]); NULL = C each
 * scores       [sum C_b]    fp32   out (NULL: user vectors only)
 * user_out     [B, 256]     fp32   out, the pooled user vector (NULL: not written)
 * 1 <= L <= MINER_FF_MAX_L.
 */
int miner_fastformer_score(void* stream, int dtype, const void* history, const uint8_t* his_mask,
                           const void* candidates, const int32_t* cand_offsets, const void* packed,
                           int B, int L, int C, float* scores, float* user_out);

/* As miner_fastformer_score with history row (b, l) = news_table[his_ids[b, l]] and candidate i
 * = news_table[cand_ids[i]]; ids are clamped to [0, n_news) on the device (validate on the host). */
int miner_fastformer_score_gather(void* stream, int dtype, const void* news_table, int n_news,
                                  const int32_t* his_ids, const uint8_t* his_mask,
                                  const int32_t* cand_ids, const int32_t* cand_offsets,
                                  const void* packed, int B, int L, int C, float* scores,
                                  float* user_out);

/* LDS bytes one workgroup of the FastFormer kernel uses (dtype-dependent). */
int miner_fastformer_lds_bytes(int dtype);

#ifdef __cplusplus
}
#endif

#endif /* MINER_FASTFORMER_H */
