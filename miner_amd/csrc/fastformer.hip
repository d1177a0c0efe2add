// fastformer.hip — fused FastFormer user encoder + click predictor for MI355X (gfx950 / CDNA4):
// BASELINE config 4, SURVEY.md §8 row f3.  Reference: src/model/model.py:223-545 (FastFormer,
// AttentionPooling, FastSelfAttention, FastAttention, FastformerLayer, FastformerEncoder) with the
// HF BertSelfOutput / BertIntermediate / BertOutput blocks, eval mode (dropout = identity).
//
// One workgroup (8 waves) encodes one impression at a time (persistent over b = blockIdx.x,
// + gridDim.x, ...). The hidden size is 256 = 8 slabs of 32, and a history has L <= 64 rows =
// two 32-row tiles. Every hidden x hidden linear layer is computed transposed, Yᵀ = W · Xᵀ:
//   A operand = W, packed 32x32 tiles streamed from L2 (rows in pi order), wave w owning output
//               columns [32w, 32w+32) = heads 2w, 2w+1;
//   B operand = X, bf16/fp32 rows in an LDS image (16-byte chunk c of row m at c ^ (m & 15)).
// So lane (h, r) of wave w ends up holding Y[m = 32mt + r][n = 32w + 16h + e] in accumulator
// register e: a whole head's 16 features for one history row. Row-wise work (LayerNorm) meets
// across waves through a small LDS exchange; head-wise work (the additive attentions' pooled query
// / key, model.py:431-447) is register-local plus a 32-lane reduction; the residual stream x stays
// in fp32 registers for the whole impression.
//
// Per layer (model.py:409-459, :469-480; 11 barriers):
//   G12  mq = x·Wqᵀ + bq, mk = x·Wkᵀ + bk                      (one pass over the x image)
//   qfs  = (mq·Wqaᵀ + bqa)/4 + ext -> softmax over L per head   (per-wave MFMA partial over its
//        own slab, 8 partials summed through LDS)              (model.py:421-426)
//   pq   = Σ_l qw·mq (per head); mqk = mk ⊙ pq; qks, kw likewise; pk = Σ_l kw·mqk   (:427-447)
//   G3   t  = (pk ⊙ mq)·Wtᵀ + bt + mq                           (:448-455)
//   G4   a  = LN(t·Woᵀ + bo + x)                                (BertSelfOutput)
//   G5   h  = gelu(a·Wiᵀ + bi)                                  (BertIntermediate)
//   G6   x' = LN(h·Wo2ᵀ + bo2 + a)                              (BertOutput)
// then the pooler (model.py:361-368: alpha = exp(att_fc2(tanh(att_fc1 x))) · mask / (Σ + 1e-8),
// no max subtraction, as the reference) and scores[c] = cand[c] · user (model.py:322).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>

#include "../../include/miner_fastformer.h"
#include "cdna4_common.h"

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kH = MINER_FF_HIDDEN;     // hidden = intermediate = 256 (model.py:251-253)
constexpr int kHeads = 16;              // 16 heads x 16 (model.py:257)
constexpr int kNS = kH / 32;            // slabs per contraction
constexpr int kMaxL = MINER_FF_MAX_L;
constexpr int kLayers = 2;
constexpr int kMat = kH * kH;
constexpr float kLnEps = 1e-12f;        // layer_norm_eps (model.py:255)
#ifndef FF_PF
#define FF_PF 4            // register prefetch depth of the weight ring (bf16)
#endif
#ifndef FF_PF32
#define FF_PF32 1          // fp32 parity mode: 16 MFMAs per slab and matrix, one slab covers the latency
#endif
#ifndef FF_MQK_LDS
#define FF_MQK_LDS 0   // experiment (bf16): mq / mk in two bf16 LDS images instead of fp32 registers, the
                       // 29 vector slots read from L2 — the first step toward two impressions per CU
#endif
#ifndef FF_QFOLD
// experiment (bf16): query_att folded into the query layer, qfs = x·W_fᵀ + b_f with W_f = Wqa·Wq and
// b_f = Wqa·bq + bqa (model.py:416, :421: two linear maps in a row), packed in place of qa. Every
// wave forms the logits of its own two heads from the x image (32 v_mfma_f32_16x16x32_bf16) instead
// of a per-slab partial summed over the 8 waves through LDS: one barrier fewer per layer (8).
#define FF_QFOLD 0
#endif
template <class T> constexpr bool kQFold = FF_QFOLD && sizeof(T) == 2 && !FF_MQK_LDS;

// ---------------------------------------------------------------------------------------------
// flat parameter blob (floats): FastformerEncoder.state_dict() order
// ---------------------------------------------------------------------------------------------
namespace blob {
constexpr int q_w = 0, q_b = q_w + kMat, qa_w = q_b + kH, qa_b = qa_w + kHeads * kH, k_w = qa_b + kHeads,
              k_b = k_w + kMat, ka_w = k_b + kH, ka_b = ka_w + kHeads * kH, t_w = ka_b + kHeads, t_b = t_w + kMat,
              o_w = t_b + kH, o_b = o_w + kMat, ln1_w = o_b + kH, ln1_b = ln1_w + kH, i_w = ln1_b + kH,
              i_b = i_w + kMat, o2_w = i_b + kH, o2_b = o2_w + kMat, ln2_w = o2_b + kH, ln2_b = ln2_w + kH,
              layer = ln2_b + kH;
constexpr int pos = kLayers * layer, ln0_w = pos + kMat, ln0_b = ln0_w + kH, p1_w = ln0_b + kH, p1_b = p1_w + kMat,
              p2_w = p1_b + kH, p2_b = p2_w + kH, total = p2_b + 1;
static_assert(total == MINER_FF_PARAM_FLOATS, "blob layout");
}  // namespace blob

// ---------------------------------------------------------------------------------------------
// packed layout:  [13 big matrices, T | 4 head projections, T | 29 vector slots, fp32 | pos, fp32]
//   big matrix g (layer ly: 6ly + {q, k, t, o, i, o2}; 12 = att_fc1): 64 fragment-major 32x32
//     tiles, tile (nt, j) at (8nt + j)·1024 = rows 32nt + pi(rr), columns 32j + cc;
//   head projection 2ly + {qa, ka}: 8 tiles (one 32-row tile, rows pi(rr) >= 16 zero);
//   vector slot s: 256 floats (zero padded).
// ---------------------------------------------------------------------------------------------
constexpr int kBig = 13, kSmall = 4;
constexpr int kSmallElems = kNS * 1024;
constexpr size_t kTElems = (size_t)kBig * kMat + (size_t)kSmall * kSmallElems;
enum VecSlot { vLn0W = 0, vLn0B = 1, vLayer = 2, vP1B = 2 + 12 * kLayers, vP2W, vP2B, kVecSlots };
enum LayerVec { lvQB = 0, lvKB, lvQaB, lvKaB, lvTB, lvOB, lvLn1W, lvLn1B, lvIB, lvO2B, lvLn2W, lvLn2B };
enum BigMat { bmQ = 0, bmK, bmT, bmO, bmI, bmO2 };
constexpr int kFElems = kVecSlots * kH + kMat;   // fp32 section: vectors then pos
static_assert(kVecSlots == 29, "vector slots");

template <class T>
constexpr size_t packed_bytes_t() { return kTElems * sizeof(T) + (size_t)kFElems * 4; }

__host__ __device__ inline int big_src(int g) {
  if (g == 12) return blob::p1_w;
  const int ly = g / 6, m = g % 6;
  const int offs[6] = {blob::q_w, blob::k_w, blob::t_w, blob::o_w, blob::i_w, blob::o2_w};
  return ly * blob::layer + offs[m];
}
__host__ __device__ inline int vec_src(int s, int& len) {
  len = kH;
  switch (s) {
    case vLn0W: return blob::ln0_w;
    case vLn0B: return blob::ln0_b;
    case vP1B: return blob::p1_b;
    case vP2W: return blob::p2_w;
    case vP2B: len = 1; return blob::p2_b;
    default: break;
  }
  const int ly = (s - vLayer) / 12, v = (s - vLayer) % 12;
  const int offs[12] = {blob::q_b, blob::k_b, blob::qa_b, blob::ka_b, blob::t_b, blob::o_b,
                        blob::ln1_w, blob::ln1_b, blob::i_b, blob::o2_b, blob::ln2_w, blob::ln2_b};
  if (v == lvQaB || v == lvKaB) len = kHeads;
  return ly * blob::layer + offs[v];
}

template <class T>
__global__ void ff_pack_kernel(const float* __restrict__ src, T* __restrict__ outT) {
  float* outF = reinterpret_cast<float*>(outT + kTElems);
  const size_t n = kTElems + kFElems;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (i < kTElems) {
      float v = 0.f;
      int rr, cc;
      block_pos<T>((int)(i & 1023), rr, cc);
      if (i < (size_t)kBig * kMat) {
        const int g = (int)(i / kMat), tile = (int)((i % kMat) >> 10);
        const int row = (tile >> 3) * 32 + pi_row(rr), col = (tile & 7) * 32 + cc;
        v = src[big_src(g) + row * kH + col];
      } else {
        const size_t q = i - (size_t)kBig * kMat;
        const int s = (int)(q / kSmallElems), j = (int)((q % kSmallElems) >> 10);
        const int ly = s >> 1;
        const int base = ly * blob::layer + ((s & 1) ? blob::ka_w : blob::qa_w);
        const int row = pi_row(rr);
        if (kQFold<T> && !(s & 1)) {
          // W_f = Wqa·Wq row-major [16][256] in the first 4096 elements of the qa slot
          const int f = (int)(q % kSmallElems);
          if (f < kHeads * kH) {
            const int hd = f / kH, k = f % kH;
            const float* wqa = src + base + hd * kH;
            const float* wq = src + ly * blob::layer + blob::q_w + k;
            double acc = 0.0;
            for (int n = 0; n < kH; ++n) acc += (double)wqa[n] * (double)wq[(size_t)n * kH];
            v = (float)acc;
          }
        } else if (row < kHeads) {
          v = src[base + row * kH + 32 * j + cc];
        }
      }
      outT[i] = (T)v;
    } else {
      const size_t q = i - kTElems;
      float v;
      if (q < (size_t)kVecSlots * kH) {
        int len;
        const int slot = (int)(q / kH);
        const int off = vec_src(slot, len);
        const int e = (int)(q % kH);
        v = e < len ? src[off + e] : 0.f;
        if (kQFold<T> && slot >= vLayer && slot < vP1B && (slot - vLayer) % 12 == lvQaB && e < kHeads) {
          // b_f = Wqa·bq + bqa
          const int ly = (slot - vLayer) / 12;
          const float* wqa = src + ly * blob::layer + blob::qa_w + e * kH;
          const float* bq = src + ly * blob::layer + blob::q_b;
          double acc = (double)v;
          for (int n = 0; n < kH; ++n) acc += (double)wqa[n] * (double)bq[n];
          v = (float)acc;
        }
      } else {
        v = src[blob::pos + (q - (size_t)kVecSlots * kH)];
      }
      outF[q] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// kernel
// ---------------------------------------------------------------------------------------------
struct FfParams {
  const void* hist;          // dense: [B, L, 256]; gather: the news table [n_news, 256]
  const uint8_t* mask;       // [B, L]
  const void* cand;          // dense: [sum C_b, 256]; gather: the news table
  const int32_t* cand_off;   // [B + 1] or null (C per impression)
  const int32_t* his_ids;    // gather: [B, L]
  const int32_t* cand_ids;   // gather: [sum C_b]
  const void* wp;            // packed parameters
  float* scores;             // [sum C_b] or null
  float* user_out;           // [B, 256] or null
  int B, L, C, n_news;
  int abl;                   // experiment bits (MINER_FF_ABL): 1 = static priority for waves 4-7,
                             // 2 = history rows DMA'd with the default cache policy instead of nt
};

// LDS carve (bytes): two activation images | LN / pooler exchange | head softmax weights | user
#ifndef FF_IMG_PAD
#define FF_IMG_PAD 1   // activation images with 16-byte padded rows (addresses: a per-lane row base + immediates)
#endif
template <class T> constexpr int kRowB = kH * (int)sizeof(T);                  // bytes of one feature row
template <class T> constexpr int kRowP = kRowB<T> + (FF_IMG_PAD ? 16 : 0);    // row stride of an activation image
template <class T> constexpr int kImg = kMaxL * kRowP<T>;
constexpr int kRedBytes = 2 * kWaves * kMaxL * 8;      // per-row reduction partials (kRedRow floats per row)
constexpr int kSwBytes = kHeads * kMaxL * 4;           // [16 heads][64 rows] fp32
// bf16: the 29 parameter-vector slots (biases, LayerNorm gains) live in LDS too (29 KiB); the fp32
// parity mode has no room for them and reads them from L2
template <class T> constexpr int kVecLds = sizeof(T) == 2 ? kVecSlots * kH * 4 : 0;
template <class T> constexpr int kOffVec = 2 * kImg<T> + kRedBytes + kSwBytes + kH * 4;
template <class T> constexpr bool kMqkLds = FF_MQK_LDS && sizeof(T) == 2;
// kQFold: both layers' folded query weights [layer][16 heads][256] bf16 after the vector slots
constexpr int kFoldLds = kLayers * kHeads * kH * 2;
template <class T> constexpr int kOffFold = kOffVec<T> + (kMqkLds<T> ? 2 * kImg<T> : kVecLds<T>);
template <class T> constexpr int kLdsTotal = kOffFold<T> + (kQFold<T> ? kFoldLds : 0);
static_assert(kWaves * kHeads * kMaxL * 4 <= kImg<__bf16>, "head partials fit a free image");

// lane id from an opaque copy of threadIdx.x: per-lane addresses derived from it are recomputed in
// every stage instead of being hoisted out of the impression loop (and spilled)
__device__ __forceinline__ int fresh_lane() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t & 63;
}

// activation image row `row`, 16-byte chunk c: FF_IMG_PAD rows padded by 16 bytes (the 16 rows of a
// ds_read_b128 / ds_write_b128 lane group start 4 banks apart, so they hit 16 different bank
// groups, and the address is a per-lane row base plus a compile-time offset — no per-access VALU);
// else 512-byte rows with the chunk XOR-swizzled within its 256-byte group
template <class T>
__device__ __forceinline__ u32x4* img_chunk(char* img, int row, int c) {
  if constexpr (FF_IMG_PAD) return reinterpret_cast<u32x4*>(img + row * kRowP<T> + (c << 4));
  else return reinterpret_cast<u32x4*>(img + row * kRowB<T> + ((c ^ (row & 15)) << 4));
}
// the history rows as dma_history lands them: unpadded rows, chunk XOR-swizzled (an LDS-DMA
// instruction writes its 1 KiB linearly; the swizzle is applied on the source address)
template <class T>
__device__ __forceinline__ const u32x4* hist_chunk(const char* img, int row, int c) {
  return reinterpret_cast<const u32x4*>(img + row * kRowB<T> + ((c ^ (row & 15)) << 4));
}
// slab fragment (slab j, lane half h) of image row `row`, and its store
template <class T>
__device__ __forceinline__ void img_load(Frag<T>& f, char* img, int row, int j, int h) {
  const int c0 = (32 * j + 16 * h) * (int)sizeof(T) / 16;
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i) f.q[i] = *img_chunk<T>(img, row, c0 + i);
}
template <class T>
__device__ __forceinline__ void img_store(char* img, int row, int j, int h, const Frag<T>& f) {
  const int c0 = (32 * j + 16 * h) * (int)sizeof(T) / 16;
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i) *img_chunk<T>(img, row, c0 + i) = f.q[i];
}
// both row tiles of the wave's column tile -> image
template <class T>
__device__ __forceinline__ void tile_store(char* img, const f32x16 (&v)[2], int wave) {
  const int lane = fresh_lane();
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    Frag<T> f;
    acc_to_frag<T>(f, v[mt]);
    img_store<T>(img, 32 * mt + r, wave, h, f);
  }
}

// 16 consecutive fp32 (16-byte aligned) -> registers
__device__ __forceinline__ f32x16 load16(const float* p) {
  const float4* q = reinterpret_cast<const float4*>(p);
  f32x16 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 t = q[i];
    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
  }
  return v;
}
// 16 elements of T -> fp32
template <class T>
__device__ __forceinline__ f32x16 frag_f32(const Frag<T>& f) {
  f32x16 v;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const unsigned u = f.q[m >> 2][m & 3];
      v[2 * m] = __uint_as_float(u << 16);
      v[2 * m + 1] = __uint_as_float(u & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = __uint_as_float(f.q[e >> 2][e & 3]);
  }
  return v;
}

// cross-lane exchanges without the LDS pipe: v_permlane16_swap / v_permlane32_swap (gfx950) with
// the same register as both operands return (own, partner) in some order, so the sum / max of the
// pair is the combination with lane l ^ 16 (within each 32-lane half) / l ^ 32
__device__ __forceinline__ float xor16_sum(float x) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float xor16_max(float x) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float xor32_max(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
// sum over the 32 lanes of a lane half (every lane gets it); over all 64 lanes
// the DPP row reductions with bound_ctrl set: every pattern is a permutation within the row, so all
// source lanes are valid and it changes nothing, but it lets hipcc fold each v_mov_b32_dpp into the
// v_add / v_max that uses it (one VALU per step instead of two)
#ifndef FF_DPP_FOLD
#define FF_DPP_FOLD 1
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_b(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xf, 0xf, FF_DPP_FOLD != 0));
}
__device__ __forceinline__ float row_sum16(float x) {
  x += dpp_b<0xB1>(x);
  x += dpp_b<0x4E>(x);
  x += dpp_b<0x141>(x);
  return x + dpp_b<0x140>(x);
}
__device__ __forceinline__ float row_max16(float x) {
  x = fmaxf(x, dpp_b<0xB1>(x));
  x = fmaxf(x, dpp_b<0x4E>(x));
  x = fmaxf(x, dpp_b<0x141>(x));
  return fmaxf(x, dpp_b<0x140>(x));
}
__device__ __forceinline__ float half_sum(float x) { return xor16_sum(row_sum16(x)); }
__device__ __forceinline__ float wave_sum(float x) { return xor32_sum(half_sum(x)); }
__device__ __forceinline__ float wave_max(float x) { return xor32_max(xor16_max(row_max16(x))); }

template <class T> __device__ __forceinline__ float ff_exp(float x) {
  if constexpr (sizeof(T) == 2) return __expf(x); else return expf(x);
}
#ifndef FF_FAST_DIV
#define FF_FAST_DIV 1   // bf16: 1/x and 1/sqrt(x) by v_rcp_f32 / v_rsq_f32 (~1 ulp) instead of IEEE division (~10 VALU)
#endif
template <class T> __device__ __forceinline__ float ff_rcp(float x) {
  if constexpr (sizeof(T) == 2 && FF_FAST_DIV) return __builtin_amdgcn_rcpf(x); else return 1.0f / x;
}
template <class T> __device__ __forceinline__ float ff_rsqrt(float x) {
  if constexpr (sizeof(T) == 2 && FF_FAST_DIV) return __builtin_amdgcn_rsqf(x); else return 1.0f / sqrtf(x);
}
template <class T> __device__ __forceinline__ float ff_tanh(float x) {
  if constexpr (sizeof(T) == 2) return tanh_fast(x); else return tanhf(x);
}

// Weight rings: the first PF slabs of a GEMM's weight tiles are loaded by ring_load, normally
// before the epilogue and barrier that precede the GEMM, so the L2 latency hides behind them.
// (slabs in flight per matrix; a two-matrix GEMM issues twice the MFMAs per slab, so half the depth)
template <class T, int NMAT> constexpr int kPF = (sizeof(T) == 2 ? FF_PF : FF_PF32) / NMAT > 0 ? (sizeof(T) == 2 ? FF_PF : FF_PF32) / NMAT : 1;
template <class T, int NMAT> using Ring = Frag<T>[NMAT][kPF<T, NMAT>];


template <class T, int NMAT, int PF = kPF<T, NMAT>>
__device__ __forceinline__ void ring_load(Frag<T> (&ring)[NMAT][PF], const T* const (&W)[NMAT], int wave) {
  const int lane = fresh_lane();
#pragma unroll
  for (int m = 0; m < NMAT; ++m) {
#pragma unroll
    for (int s = 0; s < PF; ++s) frag_load_tile<T>(ring[m][s], W[m] + (size_t)(wave * kNS + s) * 1024, lane);
  }
}

// acc[m][mt] = (W_m · Xᵀ)[column tile `wave`, row tile mt] over the full 256 contraction, X the
// image `img`; W_m fragment-major packed (the wave's 8 tiles are contiguous), its first slabs
// already in `ring`. Every load is unconditional and the loop fully unrolled.
template <class T, int NMAT, int PF = kPF<T, NMAT>>
__device__ __forceinline__ void gemm_run(f32x16 (&acc)[NMAT][2], char* img, Frag<T> (&ring)[NMAT][PF],
                                         const T* const (&W)[NMAT], int wave) {
  const int lane = fresh_lane();
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int m = 0; m < NMAT; ++m) {
    acc[m][0] = zero16();
    acc[m][1] = zero16();
  }
  // B fragments double-buffered: slab j + 1's LDS reads are in flight during slab j's MFMAs
  Frag<T> xb[2][2];
  img_load<T>(xb[0][0], img, r, 0, h);
  img_load<T>(xb[0][1], img, 32 + r, 0, h);
#pragma unroll
  for (int j = 0; j < kNS; ++j) {
    if (j + 1 < kNS) {
      img_load<T>(xb[(j + 1) & 1][0], img, r, j + 1, h);
      img_load<T>(xb[(j + 1) & 1][1], img, 32 + r, j + 1, h);
    }
    const Frag<T>& x0 = xb[j & 1][0];
    const Frag<T>& x1 = xb[j & 1][1];
#pragma unroll
    for (int m = 0; m < NMAT; ++m) {
      mma_slab<T>(acc[m][0], ring[m][j % PF], x0);
      mma_slab<T>(acc[m][1], ring[m][j % PF], x1);
      // refill the slot just consumed (no register copies of the ring)
      if (j + PF < kNS) frag_load_tile<T>(ring[m][j % PF], W[m] + (size_t)(wave * kNS + j + PF) * 1024, lane);
    }
  }
}

// v += the wave's 16 entries of vector slot s (columns 32·wave + 16h + e)
__device__ __forceinline__ void add_vec(f32x16 (&v)[2], const float* vecs, int s, int wave, int h) {
  const f32x16 b = load16(vecs + s * kH + 32 * wave + 16 * h);
  v[0] += b;
  v[1] += b;
}

// the value lane l ^ 32 holds (v_permlane32_swap)
__device__ __forceinline__ float other_half(float x, int h) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(h ? sw[0] : sw[1]);
}

// LDS exchange rows of the per-row reductions: row m holds 8 (LayerNorm: float2 per wave) or 16
// (pooler: float per lane half) partials; rows padded to 80 bytes so a ds_read_b128 lane group hits
// 16 different bank quads
constexpr int kRedRow = 20;   // floats
static_assert(kMaxL * kRedRow * 4 <= kRedBytes, "reduction rows fit");

// LayerNorm over the 256 features of every row (torch layer_norm, biased variance, eps 1e-12).
// (mean, M2) of each lane's 16 features, combined exactly (Chan et al.) first with the other lane
// half in registers (the row's 32 features of this wave), then over the 8 waves through LDS:
// mean = Σ mean_g / G, M2 = Σ M2_g + n Σ (mean_g - mean)².
#ifndef FF_LN_PK
#define FF_LN_PK 1   // LayerNorm's per-element work on packed fp32 pairs (v_pk_add / v_pk_fma: half the VALU issue)
#endif
__device__ __forceinline__ f32x2 pair(const f32x16& v, int i) { return f32x2{v[2 * i], v[2 * i + 1]}; }

template <class T>
__device__ __forceinline__ void layer_norm(f32x16 (&v)[2], float* red, const float* vecs, int sw, int sb,
                                           int wave) {
  const int lane = fresh_lane();
  const int r = lane & 31, h = lane >> 5;
#if FF_LN_PK
  // the same statistics, combined in the same way; the sums over a lane's 16 features as pair trees
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x2 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = pair(v[mt], 2 * i) + pair(v[mt], 2 * i + 1);
    const f32x2 sp = (a[0] + a[1]) + (a[2] + a[3]);
    const float mean = (sp.x + sp.y) * (1.0f / 16.0f);
    const f32x2 mm = {mean, mean};
    f32x2 c0 = {0.f, 0.f}, c1 = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      const f32x2 d0 = pair(v[mt], i) - mm, d1 = pair(v[mt], i + 1) - mm;
      c0 = __builtin_elementwise_fma(d0, d0, c0);
      c1 = __builtin_elementwise_fma(d1, d1, c1);
    }
    const f32x2 cs = c0 + c1;
    const float m2 = cs.x + cs.y;
    const float om = other_half(mean, h), om2 = other_half(m2, h);
    const float dm = mean - om;
    if (h == 0)
      *reinterpret_cast<float2*>(red + (32 * mt + r) * kRedRow + 2 * wave) =
          make_float2(0.5f * (mean + om), m2 + om2 + 8.0f * dm * dm);
  }
  const f32x16 g = load16(vecs + sw * kH + 32 * wave + 16 * h);
  const f32x16 bb = load16(vecs + sb * kH + 32 * wave + 16 * h);
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const float4* row = reinterpret_cast<const float4*>(red + (32 * mt + r) * kRedRow);
    float4 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = row[i];
    // (mean_w, M2_w) pairs of the 8 waves: one pair sum gives (Σ mean_w, Σ M2_w)
    const f32x2 s01 = f32x2{q[0].x, q[0].y} + f32x2{q[0].z, q[0].w};
    const f32x2 s23 = f32x2{q[1].x, q[1].y} + f32x2{q[1].z, q[1].w};
    const f32x2 s45 = f32x2{q[2].x, q[2].y} + f32x2{q[2].z, q[2].w};
    const f32x2 s67 = f32x2{q[3].x, q[3].y} + f32x2{q[3].z, q[3].w};
    const f32x2 st = (s01 + s23) + (s45 + s67);
    const float mean = st.x * (1.0f / kWaves);
    const float mw[8] = {q[0].x, q[0].z, q[1].x, q[1].z, q[2].x, q[2].z, q[3].x, q[3].z};
    float dev = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const float dlt = mw[w] - mean;
      dev += dlt * dlt;
    }
    const float var = (st.y + 32.0f * dev) * (1.0f / (float)kH);
    const float rstd = ff_rsqrt<T>(var + kLnEps);
    const f32x2 rr = {rstd, rstd}, mm = {mean, mean};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x2 t = __builtin_elementwise_fma((pair(v[mt], i) - mm) * rr, pair(g, i), pair(bb, i));
      v[mt][2 * i] = t.x;
      v[mt][2 * i + 1] = t.y;
    }
  }
#else
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) s += v[mt][e];
    const float mean = s * (1.0f / 16.0f);
    float m2 = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float dlt = v[mt][e] - mean;
      m2 += dlt * dlt;
    }
    const float om = other_half(mean, h), om2 = other_half(m2, h);
    const float dm = mean - om;
    if (h == 0)
      *reinterpret_cast<float2*>(red + (32 * mt + r) * kRedRow + 2 * wave) =
          make_float2(0.5f * (mean + om), m2 + om2 + 8.0f * dm * dm);
  }
  const f32x16 g = load16(vecs + sw * kH + 32 * wave + 16 * h);
  const f32x16 bb = load16(vecs + sb * kH + 32 * wave + 16 * h);
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const float4* row = reinterpret_cast<const float4*>(red + (32 * mt + r) * kRedRow);
    float4 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = row[i];
    const float mw[8] = {q[0].x, q[0].z, q[1].x, q[1].z, q[2].x, q[2].z, q[3].x, q[3].z};
    const float m2w[8] = {q[0].y, q[0].w, q[1].y, q[1].w, q[2].y, q[2].w, q[3].y, q[3].w};
    float ms = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) ms += mw[w];
    const float mean = ms * (1.0f / kWaves);
    float m2 = 0.f, dev = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const float dlt = mw[w] - mean;
      m2 += m2w[w];
      dev += dlt * dlt;
    }
    const float var = (m2 + 32.0f * dev) * (1.0f / (float)kH);
    const float rstd = ff_rsqrt<T>(var + kLnEps);
#pragma unroll
    for (int e = 0; e < 16; ++e) v[mt][e] = (v[mt][e] - mean) * rstd * g[e] + bb[e];
  }
#endif
}

// per-wave partial of an additive-attention logit, (W_att · Xᵀ) over the wave's own slab:
// the accumulator X tile is the B operand directly; lanes of half 0 hold the 16 heads. Stored as
// [head][position][8 waves] (slot rotated by position >> 2: the 32 lanes of a ds_write_b32 hit 32
// banks) so a lane reads a position's 8 partials with two ds_read_b128.
__device__ __forceinline__ int part_slot(int hd, int m, int w) { return (hd * kMaxL + m) * kWaves + ((w + (m >> 2)) & 7); }

template <class T>
__device__ __forceinline__ void head_partial(float* part, const Frag<T>& a, const f32x16 (&x)[2], int wave) {
  const int lane = fresh_lane();
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    Frag<T> b;
    acc_to_frag<T>(b, x[mt]);
    f32x16 acc = zero16();
    mma_slab<T>(acc, a, b);
    if (h == 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) part[part_slot(e, 32 * mt + r, wave)] = acc[e];
    }
  }
}

// softmax over the history of heads 2·wave, 2·wave + 1 (lane = position):
// w = softmax((Σ_waves part + b) / 4 + ext)  (model.py:421-426 / :440-444)
template <class T>
__device__ __forceinline__ void head_softmax(const float* part, const float* batt, float* swt, float extl, int wave) {
  const int lane = fresh_lane();
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int hd = 2 * wave + hh;
    const float4* row = reinterpret_cast<const float4*>(part + (hd * kMaxL + lane) * kWaves);   // 8 slots
    const float4 a = row[0], b = row[1];
    float s = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
    s = (s + batt[hd]) / 4.0f + extl;          // extl = -inf past L (excluded)
    const float mx = wave_max(s);
    const float ex = ff_exp<T>(s - mx);
    const float sum = wave_sum(ex);
    swt[hd * kMaxL + lane] = sizeof(T) == 2 && FF_FAST_DIV ? ex * ff_rcp<T>(sum) : ex / sum;
  }
}

// kQFold: the query softmax of heads 2·wave, 2·wave + 1 straight from the x image (model.py:421-426),
// w = softmax((x·W_fᵀ + b_f) / 4 + ext). A = W_f rows: lane group g holds head 2·wave + (g & 1) in
// all four of its rows; B = x rows 16·pt + n (the image chunk 4s + g is exactly the B fragment);
// D register 0 of lane (n, g) = that head's logit at position 16·pt + n.
__device__ __forceinline__ void qfold_softmax(const char* fold, char* img, const float* bf, float* swt, float extl,
                                              int wave) {
  static_assert(kMaxL == 64, "four 16-position tiles");
  const int lane = fresh_lane();
  const int n = lane & 15, g = lane >> 4;
  const int hd = 2 * wave + (g & 1);
  f32x4 acc[4];
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) acc[pt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kNS; ++s) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(fold + hd * (kH * 2) + (4 * s + g) * 16);
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) acc[pt] = mfma16_bf16(a, *img_chunk<__bf16>(img, 16 * pt + n, 4 * s + g), acc[pt]);
  }
  const float b = bf[hd];
  float sc[4], mx = -INFINITY;
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    sc[pt] = (acc[pt][0] + b) / 4.0f + __shfl(extl, 16 * pt + n);   // ext of position 16·pt + n
    mx = fmaxf(mx, sc[pt]);
  }
  mx = row_max16(mx);
  float sum = 0.f;
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    sc[pt] = __expf(sc[pt] - mx);
    sum += sc[pt];
  }
  sum = row_sum16(sum);
  if (g < 2) {
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) swt[hd * kMaxL + 16 * pt + n] = sc[pt] / sum;
  }
}

// the wave's slab fragment of a head projection (qa / ka)
template <class T>
__device__ __forceinline__ void small_load(Frag<T>& a, const T* Watt, int wave) {
  frag_load_tile<T>(a, Watt + (size_t)wave * 1024, fresh_lane());
}

// out[e] = Σ_m w[head][m] · v[m][e], head = 2·wave + h (every lane of the half gets it)
__device__ __forceinline__ void head_pool(float (&out)[16], const f32x16 (&v)[2], const float* swt, int wave) {
  const int lane = fresh_lane();
  const int r = lane & 31, h = lane >> 5;
  const float a0 = swt[(2 * wave + h) * kMaxL + r], a1 = swt[(2 * wave + h) * kMaxL + 32 + r];
#pragma unroll
  for (int e = 0; e < 16; ++e) out[e] = half_sum(a0 * v[0][e] + a1 * v[1][e]);
}

// history image of impression bn: the LDS-DMA (untracked, see cdna4_common.h) writes each wave-
// instruction's 1 KiB linearly; the XOR swizzle is applied on the per-lane source address.
template <class T> constexpr int kCpr = kH * (int)sizeof(T) / 16;      // 16-byte chunks per row
template <class T> constexpr int kRowsPerDma = 64 / kCpr<T>;          // rows per DMA instruction
template <class T> constexpr int kDmaPerWave = kCpr<T> / kWaves;      // DMA instructions per wave
template <class T> constexpr int kHistIds = kDmaPerWave<T> * kRowsPerDma<T>;

// a wave-uniform int from global memory through the scalar cache (s_load, counted by lgkmcnt — a
// vector load here would be waited with vmcnt, behind every vector load in flight)
__device__ __forceinline__ int sload(const int32_t* q) {
  return *(const __attribute__((address_space(4))) int32_t*)(uintptr_t)q;
}

// rows (table ids, or dense row indices) of the history rows this wave's DMA instructions cover;
// wave-uniform (scalar loads), rows past L clamped to L - 1 (their values are never used)
template <class T, bool GATHER>
__device__ __forceinline__ void history_rows(const FfParams& p, int bn, int wave, int (&rows)[kHistIds<T>]) {
#pragma unroll
  for (int k = 0; k < kDmaPerWave<T>; ++k) {
#pragma unroll
    for (int j = 0; j < kRowsPerDma<T>; ++j) {
      const int m = min((wave + kWaves * k) * 64 / kCpr<T> + j, p.L - 1);
      int row;
      if constexpr (GATHER) row = min(max(sload(p.his_ids + (size_t)bn * p.L + m), 0), p.n_news - 1);
      else row = bn * p.L + m;
      rows[k * kRowsPerDma<T> + j] = __builtin_amdgcn_readfirstlane(row);   // keep it scalar
    }
  }
}
template <class T>
__device__ __forceinline__ void dma_history(const T* base, const int (&rows)[kHistIds<T>], char* img, int wave, bool rt) {
  const int lane = fresh_lane();
#pragma unroll
  for (int k = 0; k < kDmaPerWave<T>; ++k) {
    const int P = (wave + kWaves * k) * 64 + lane;
    const int m = P / kCpr<T>, pc = P % kCpr<T>;
    const int row = kRowsPerDma<T> == 2 ? ((lane >> 5) ? rows[2 * k + 1] : rows[2 * k]) : rows[k];
    const T* g = base + (size_t)row * kH + ((pc ^ (m & 15)) << 4) / (int)sizeof(T);
    const unsigned la = __builtin_amdgcn_readfirstlane(lds_offset(img + (wave + kWaves * k) * 1024));
    if (rt) dma_b128_rt(g, la);
    else dma_b128(g, la);
  }
}

// per-lane mask state of an impression: ext of position `lane` (model.py:519-521; -inf past L)
// and the pooling mask of rows r, 32 + r (model.py:366). Loaded raw (unconditional byte loads at
// clamped positions: a predicated load is waited with vmcnt(0)) one impression ahead, decoded at
// the start of the impression that uses it.
struct MaskRaw {
  unsigned ml, m0, m1;
};
struct MaskState {
  float extl;
  bool m0, m1;
};
__device__ __forceinline__ MaskRaw load_mask(const FfParams& p, int b) {
  const int lane = fresh_lane();
  const int r = lane & 31, L = p.L;
  const uint8_t* mrow = p.mask + (size_t)b * L;
  return MaskRaw{mrow[min(lane, L - 1)], mrow[min(r, L - 1)], mrow[min(32 + r, L - 1)]};
}
__device__ __forceinline__ MaskState decode_mask(const MaskRaw& m, int L) {
  const int lane = fresh_lane();
  const int r = lane & 31;
  MaskState s;
  s.extl = lane < L ? (m.ml ? 0.0f : -10000.0f) : -INFINITY;
  s.m0 = r < L && m.m0;
  s.m1 = 32 + r < L && m.m1;
  return s;
}

// candidate rows: 4 elements per lane (bf16: 8 bytes, fp32: 16 bytes)
template <class T> struct CandVec { typedef u32x4 type; };
template <> struct CandVec<__bf16> { typedef unsigned int type __attribute__((ext_vector_type(2))); };
constexpr int kCandPf = 8;          // candidates per wave prefetched before the pooler (C <= 64 in one round)

template <class T>
__device__ __forceinline__ float cand_dot(const typename CandVec<T>::type& w, const float4& u) {
  if constexpr (sizeof(T) == 2) {
    return __uint_as_float(w.x << 16) * u.x + __uint_as_float(w.x & 0xffff0000u) * u.y +
           __uint_as_float(w.y << 16) * u.z + __uint_as_float(w.y & 0xffff0000u) * u.w;
  } else {
    return __uint_as_float(w.x) * u.x + __uint_as_float(w.y) * u.y + __uint_as_float(w.z) * u.z +
           __uint_as_float(w.w) * u.w;
  }
}
template <bool GATHER>
__device__ __forceinline__ int cand_index(const FfParams& p, int cbase, int c) {
  if constexpr (GATHER) return min(max(sload(p.cand_ids + cbase + c), 0), p.n_news - 1);
  else return cbase + c;
}
template <class T, bool GATHER>
__device__ __forceinline__ const T* cand_row(const FfParams& p, int cbase, int c) {
  return static_cast<const T*>(p.cand) + (size_t)cand_index<GATHER>(p, cbase, c) * kH;
}

#ifdef MINER_STAMPS
// diagnostic build only: thread 0 of every workgroup sums the s_memtime cycles of each stage
__device__ unsigned long long g_ff_stage_cycles[16];
__device__ unsigned long long g_ff_imps;
#define FF_STAMP_DECL unsigned long long st_acc[16] = {0}; unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define FF_STAMP(i) do { if (threadIdx.x == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } } while (0)
#define FF_STAMP_FLUSH(n) do { if (threadIdx.x == 0) { for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&g_ff_stage_cycles[i_], st_acc[i_]); atomicAdd(&g_ff_imps, (unsigned long long)(n)); } } while (0)
#else
#define FF_STAMP_DECL
#define FF_STAMP(i) do {} while (0)
#define FF_STAMP_FLUSH(n) do {} while (0)
#endif

// Image use per impression (img0 / img1):
//   start      E rows (DMA'd during the previous impression) in img1 -> x = LN(E + pos) -> img0
//   layer ly   cur = the x image, oth = the other one:
//     qfs partials -> oth, qks partials -> cur (x is dead after G12), wv -> oth, t -> cur,
//     a -> oth, h -> cur, x' -> oth; swap
//   pooler     x in img0 (two swaps), img1 free: the next impression's E rows are DMA'd there
// Barriers per layer: qfs partials, qks partials, wv, t, LN1 stats, a, h, LN2 stats, x' (9). The
// head softmaxes need none: wave w owns heads 2w, 2w+1 and is the only reader of their weights.
// kQFold: no qfs partials (8 barriers), x stays in cur: qks partials -> oth, wv -> cur, t -> oth,
// a -> cur, h -> oth, x' -> cur, no swap (the pooler still finds x in img0).
template <class T, bool GATHER>
__global__ __launch_bounds__(kThreads) void ff_fused(FfParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* img0 = smem;
  char* img1 = smem + kImg<T>;
  float* red = reinterpret_cast<float*>(smem + 2 * kImg<T>);
  float* swt = reinterpret_cast<float*>(smem + 2 * kImg<T> + kRedBytes);
  float* userL = reinterpret_cast<float*>(smem + 2 * kImg<T> + kRedBytes + kSwBytes);
  const T* __restrict__ big = static_cast<const T*>(p.wp);
  const T* __restrict__ small = big + (size_t)kBig * kMat;
  const float* __restrict__ gvecs = reinterpret_cast<const float*>(big + kTElems);
  const float* __restrict__ pos = gvecs + kVecSlots * kH;
  constexpr bool kBf16 = sizeof(T) == 2;
  // parameter vectors: LDS copy (bf16) or L2 (fp32)
  const float* vecs = (kBf16 && !kMqkLds<T>) ? reinterpret_cast<const float*>(smem + kOffVec<T>) : gvecs;
  [[maybe_unused]] char* imgq = smem + kOffVec<T>;          // kMqkLds: mq, mk images
  [[maybe_unused]] char* imgk = smem + kOffVec<T> + kImg<T>;
  if constexpr (kBf16 && !kMqkLds<T>) {
    float4* dst = reinterpret_cast<float4*>(smem + kOffVec<T>);
    for (int i = threadIdx.x; i < kVecSlots * kH / 4; i += kThreads) dst[i] = reinterpret_cast<const float4*>(gvecs)[i];
  }
  [[maybe_unused]] const char* foldL = smem + kOffFold<T>;
  if constexpr (kQFold<T>) {     // W_f of both layers (the first 4096 elements of each qa slot) -> LDS
    u32x4* dst = reinterpret_cast<u32x4*>(smem + kOffFold<T>);
    constexpr int kPer = kHeads * kH * 2 / 16;
    for (int i = threadIdx.x; i < kLayers * kPer; i += kThreads)
      dst[i] = reinterpret_cast<const u32x4*>(small + (size_t)(2 * (i / kPer)) * kSmallElems)[i % kPer];
  }
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  const int L = p.L;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto tile_load = [&](char* img, f32x16 (&v)[2]) {         // this wave's column tile, both row tiles
    const int lane = fresh_lane();
    const int r = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      Frag<T> f;
      img_load<T>(f, img, 32 * mt + r, wave, hh);
      v[mt] = frag_f32<T>(f);
    }
  };
  if ((p.abl & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  FF_STAMP_DECL
  int n_done = 0;

  // position embeddings of this lane's rows: the same for every impression (model.py:524-527),
  // reloaded before each pooler so they are not held through the layers
  f32x16 posv[2];
  auto load_pos = [&]() {
    const int lane = fresh_lane();
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) posv[mt] = load16(pos + min(32 * mt + r, L - 1) * kH + 32 * wave + 16 * h);
  };
  load_pos();
  MaskRaw mraw{};
  if (blockIdx.x < p.B) {
    int rows[kHistIds<T>];
    history_rows<T, GATHER>(p, blockIdx.x, wave, rows);
    dma_history<T>(hist, rows, img1, wave, (p.abl & 2) != 0);
    mraw = load_mask(p, blockIdx.x);
  }

  for (int b = blockIdx.x; b < p.B; b += gridDim.x) {
    ++n_done;
    const int bn = b + gridDim.x;
    const bool has_next = bn < p.B;
    // scalar prefetches for later in this impression: candidate range, next impression's ids
    const int cbase = p.cand_off ? sload(p.cand_off + b) : b * p.C;
    const int Cb = p.cand_off ? sload(p.cand_off + b + 1) - cbase : p.C;
    int rows_next[kHistIds<T>];
    if (has_next) history_rows<T, GATHER>(p, bn, wave, rows_next);
    // the table rows of this wave's first kCandPf candidates
    int crow[kCandPf];
#pragma unroll
    for (int i = 0; i < kCandPf; ++i) crow[i] = cand_index<GATHER>(p, cbase, min(wave + kWaves * i, max(Cb - 1, 0)));
    const MaskState ms = decode_mask(mraw, L);

    // ---- x = LN(E + pos[0:L])  (model.py:524-531) ----
    if (n_done == 1) vm_wait_all();   // the first impression's history DMA (later ones: before the scores)
    __syncthreads();
    f32x16 x[2];
    Ring<T, 2> rq;
    Frag<T> sq, sk;
    {
      const int lane = fresh_lane();
      const int r = lane & 31, h = lane >> 5;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int m = 32 * mt + r;
        Frag<T> f;
        {
          const int c0 = 32 * wave * (int)sizeof(T) / 16 + 16 * h * (int)sizeof(T) / 16;
#pragma unroll
          for (int i = 0; i < kNQ<T>; ++i) f.q[i] = *hist_chunk<T>(img1, m, c0 + i);
        }
        const f32x16 e = frag_f32<T>(f);
#pragma unroll
        for (int i = 0; i < 16; ++i) x[mt][i] = m < L ? e[i] + posv[mt][i] : 0.0f;
      }
      const T* const W[2] = {big + bmQ * kMat, big + bmK * kMat};
      ring_load<T, 2>(rq, W, wave);
      if constexpr (!kQFold<T>) small_load<T>(sq, small, wave);
      small_load<T>(sk, small + kSmallElems, wave);
    }
    layer_norm<T>(x, red, vecs, vLn0W, vLn0B, wave);
    tile_store<T>(img0, x, wave);
    __syncthreads();
    FF_STAMP(0);

    char* cur = img0;
    char* oth = img1;
    // the pooler's att_fc1 slabs, loaded during the last layer's G6: all 8 (bf16), so the pooler
    // GEMM issues no load behind the HBM-latency DMA / candidate loads it runs beside
#ifndef FF_POOL_ALL
#define FF_POOL_ALL 1
#endif
    constexpr int kPoolPF = (kBf16 && FF_POOL_ALL) ? kNS : kPF<T, 1>;
    Frag<T> rp[1][kPoolPF];
#pragma unroll
    for (int ly = 0; ly < kLayers; ++ly) {
      const T* Wl = big + (size_t)ly * 6 * kMat;
      const int vb = vLayer + 12 * ly;
      const int h = fresh_lane() >> 5;
      // kQFold keeps x in `cur` for the whole layer: the buffers after the query softmax swap roles
      char* bA = kQFold<T> ? oth : cur;
      char* bB = kQFold<T> ? cur : oth;
      if constexpr (kQFold<T>)
        qfold_softmax(foldL + ly * (kHeads * kH * 2), cur, vecs + (vb + lvQaB) * kH, swt, ms.extl, wave);

      // G12: mixed query / key layers (model.py:416-417)
      f32x16 qk[2][2];
      {
        const T* const W[2] = {Wl + bmQ * kMat, Wl + bmK * kMat};
        gemm_run<T, 2>(qk, cur, rq, W, wave);
      }
      Ring<T, 1> r1;
      f32x16 mq[2] = {qk[0][0], qk[0][1]};
      f32x16 mk[2] = {qk[1][0], qk[1][1]};
      add_vec(mq, vecs, vb + lvQB, wave, h);
      add_vec(mk, vecs, vb + lvKB, wave, h);
      if constexpr (kMqkLds<T>) {        // only this wave reads its tiles back: no barrier
        tile_store<T>(imgq, mq, wave);
        tile_store<T>(imgk, mk, wave);
      }
      if (ly == 0) {
        // pin the ids' scalar loads (issued at the impression start; HBM latency) here, one GEMM
        // later: sunk to their uses they would sit in the lgkmcnt queue beside the LDS reads of
        // the pooler (scalar loads return out of order: every LDS wait there becomes lgkmcnt(0))
#pragma unroll
        for (int i = 0; i < kHistIds<T>; ++i) asm volatile("" : "+s"(rows_next[i]));
#pragma unroll
        for (int i = 0; i < kCandPf; ++i) asm volatile("" : "+s"(crow[i]));
      }
      FF_STAMP(1);

      // query attention -> pooled query (model.py:421-433); partials in oth
      if constexpr (!kQFold<T>) {
        if constexpr (kMqkLds<T>) tile_load(imgq, mq);
        head_partial<T>(reinterpret_cast<float*>(oth), sq, mq, wave);
        __syncthreads();
        FF_STAMP(2);
        head_softmax<T>(reinterpret_cast<float*>(oth), vecs + (vb + lvQaB) * kH, swt, ms.extl, wave);
      }
      FF_STAMP(3);
      {
        float pq[16];
        if constexpr (kMqkLds<T>) tile_load(imgq, mq);
        head_pool(pq, mq, swt, wave);
        if constexpr (kMqkLds<T>) tile_load(imgk, mk);
#pragma unroll
        for (int e = 0; e < 16; ++e) {   // mixed_query_key_layer = mk ⊙ pooled query (:436)
          mk[0][e] *= pq[e];
          mk[1][e] *= pq[e];
        }
      }
      // key attention -> pooled key (model.py:439-447); partials in bA (cur: x is dead after G12)
      if constexpr (kMqkLds<T>) tile_store<T>(imgk, mk, wave);
      head_partial<T>(reinterpret_cast<float*>(bA), sk, mk, wave);
      __syncthreads();
      FF_STAMP(4);
      head_softmax<T>(reinterpret_cast<float*>(bA), vecs + (vb + lvKaB) * kH, swt, ms.extl, wave);
      FF_STAMP(5);
      {
        const T* const W[1] = {Wl + bmT * kMat};   // G3's first slabs, behind the pooled key and a barrier
        ring_load<T, 1>(r1, W, wave);
      }
      {
        float pk[16];
        if constexpr (kMqkLds<T>) {
          tile_load(imgk, mk);
          tile_load(imgq, mq);
        }
        head_pool(pk, mk, swt, wave);
        f32x16 wv[2];
#pragma unroll
        for (int e = 0; e < 16; ++e) {   // weighted_value = pooled key ⊙ query layer (:448)
          wv[0][e] = pk[e] * mq[0][e];
          wv[1][e] = pk[e] * mq[1][e];
        }
        tile_store<T>(bB, wv, wave);
      }
      __syncthreads();
      FF_STAMP(6);

      // G3: transform(weighted_value) + mixed query layer (model.py:452-453)
      f32x16 t[1][2];
      {
        const T* const W[1] = {Wl + bmT * kMat};
        gemm_run<T, 1>(t, bB, r1, W, wave);
        const T* const Wn[1] = {Wl + bmO * kMat};
        ring_load<T, 1>(r1, Wn, wave);
      }
      add_vec(t[0], vecs, vb + lvTB, wave, h);
      if constexpr (kMqkLds<T>) tile_load(imgq, mq);
      t[0][0] += mq[0];
      t[0][1] += mq[1];
      tile_store<T>(bA, t[0], wave);
      __syncthreads();
      FF_STAMP(7);

      // G4: BertSelfOutput — LayerNorm(dense(t) + x)
      {
        const T* const W[1] = {Wl + bmO * kMat};
        gemm_run<T, 1>(t, bA, r1, W, wave);
        const T* const Wn[1] = {Wl + bmI * kMat};
        ring_load<T, 1>(r1, Wn, wave);
      }
      add_vec(t[0], vecs, vb + lvOB, wave, h);
      x[0] += t[0][0];
      x[1] += t[0][1];
      layer_norm<T>(x, red, vecs, vb + lvLn1W, vb + lvLn1B, wave);   // x := a
      tile_store<T>(bB, x, wave);
      __syncthreads();
      FF_STAMP(8);

      // G5: BertIntermediate — gelu(dense(a))
      {
        const T* const W[1] = {Wl + bmI * kMat};
        gemm_run<T, 1>(t, bB, r1, W, wave);
        const T* const Wn[1] = {Wl + bmO2 * kMat};
        ring_load<T, 1>(r1, Wn, wave);
      }
      add_vec(t[0], vecs, vb + lvIB, wave, h);
      gelu_tile<T>(t[0][0]);
      gelu_tile<T>(t[0][1]);
      tile_store<T>(bA, t[0], wave);
      __syncthreads();
      FF_STAMP(9);

      // G6: BertOutput — LayerNorm(dense(h) + a)
      {
        const T* const W[1] = {Wl + bmO2 * kMat};
        gemm_run<T, 1>(t, bA, r1, W, wave);
        // next: the following layer's q / k, or the pooler's att_fc1 (first ring slot)
        if (ly + 1 < kLayers) {
          const T* const Wn[2] = {Wl + (6 + bmQ) * kMat, Wl + (6 + bmK) * kMat};
          ring_load<T, 2>(rq, Wn, wave);
          if constexpr (!kQFold<T>) small_load<T>(sq, small + (size_t)(2 * ly + 2) * kSmallElems, wave);
          small_load<T>(sk, small + (size_t)(2 * ly + 3) * kSmallElems, wave);
        } else {
          const T* const Wn[1] = {big + (size_t)12 * kMat};
          ring_load<T, 1, kPoolPF>(rp, Wn, wave);
        }
      }
      add_vec(t[0], vecs, vb + lvO2B, wave, h);
      x[0] += t[0][0];
      x[1] += t[0][1];
      layer_norm<T>(x, red, vecs, vb + lvLn2W, vb + lvLn2B, wave);
      tile_store<T>(bB, x, wave);
      __syncthreads();
      FF_STAMP(10);
      if constexpr (!kQFold<T>) { char* tmp = cur; cur = oth; oth = tmp; }
    }

    // ---- loads for later, short-latency ones first: vmcnt is in order, so anything issued after
    // the HBM-latency DMA / candidate loads waits for them ----
    load_pos();
    if (has_next) mraw = load_mask(p, bn);
    // next impression's history rows -> img1 (free until the next impression starts)
    if (has_next) dma_history<T>(hist, rows_next, img1, wave, (p.abl & 2) != 0);

    // candidate rows of this impression, in flight during the pooler
    typename CandVec<T>::type cv[kCandPf];
    if (p.scores) {
      const int lane = fresh_lane();
#pragma unroll
      for (int i = 0; i < kCandPf; ++i) {
        const T* cp = static_cast<const T*>(p.cand) + (Cb > 0 ? (size_t)crow[i] * kH : 0);
        cv[i] = *reinterpret_cast<const typename CandVec<T>::type*>(cp + 4 * lane);
      }
    }

    // ---- AttentionPooling (model.py:361-368) ----
    f32x16 e1[1][2];
    {
      const T* const W[1] = {big + (size_t)12 * kMat};
      gemm_run<T, 1, kPoolPF>(e1, cur, rp, W, wave);
    }
    {
      const int lane = fresh_lane();
      const int r = lane & 31, h = lane >> 5;
      add_vec(e1[0], vecs, vP1B, wave, h);
      FF_STAMP(11);
      const f32x16 w2 = load16(vecs + vP2W * kH + 32 * wave + 16 * h);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) s += ff_tanh<T>(e1[0][mt][e]) * w2[e];
        red[(32 * mt + r) * kRedRow + 2 * wave + h] = s;    // row m: 16 lane-half partials
      }
      const float bp2 = vecs[vP2B * kH];
      __syncthreads();
      float al[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const float4* row = reinterpret_cast<const float4*>(red + (32 * mt + r) * kRedRow);
        const float4 q0 = row[0], q1 = row[1], q2 = row[2], q3 = row[3];
        const float s = (((q0.x + q0.y) + (q0.z + q0.w)) + ((q1.x + q1.y) + (q1.z + q1.w))) +
                        (((q2.x + q2.y) + (q2.z + q2.w)) + ((q3.x + q3.y) + (q3.z + q3.w)));
        const float a = ff_exp<T>(s + bp2);
        al[mt] = (mt ? ms.m1 : ms.m0) ? a : 0.0f;
      }
      const float tot = half_sum(al[0] + al[1]) + 1e-8f;
      if constexpr (sizeof(T) == 2 && FF_FAST_DIV) {
        const float it = ff_rcp<T>(tot);
        al[0] *= it;
        al[1] *= it;
      } else {
        al[0] /= tot;
        al[1] /= tot;
      }
      f32x16 u;
#pragma unroll
      for (int e = 0; e < 16; ++e) u[e] = half_sum(al[0] * x[0][e] + al[1] * x[1][e]);
      if (r == 0) {
        float* ud = userL + 32 * wave + 16 * h;
#pragma unroll
        for (int e = 0; e < 16; ++e) ud[e] = u[e];
        if (p.user_out) {
          float* uo = p.user_out + (size_t)b * kH + 32 * wave + 16 * h;
#pragma unroll
          for (int e = 0; e < 16; ++e) uo[e] = u[e];
        }
      }
    }
    __syncthreads();
    FF_STAMP(12);

    // ---- scores = candidates · user (model.py:322) ----
    vm_wait_all();          // candidate rows, and the next impression's history DMA
    if (p.scores) {
      const int lane = fresh_lane();
      const float4 uv = reinterpret_cast<const float4*>(userL)[lane];
#pragma unroll
      for (int i = 0; i < kCandPf; ++i) {
        const int c = wave + kWaves * i;
        if (c < Cb) {
          const float s = wave_sum(cand_dot<T>(cv[i], uv));
          if (lane == 0) p.scores[cbase + c] = s;
        }
      }
      for (int c = wave + kWaves * kCandPf; c < Cb; c += kWaves) {
        const typename CandVec<T>::type w =
            *reinterpret_cast<const typename CandVec<T>::type*>(cand_row<T, GATHER>(p, cbase, c) + 4 * lane);
        const float s = wave_sum(cand_dot<T>(w, uv));
        if (lane == 0) p.scores[cbase + c] = s;
      }
    }
    FF_STAMP(13);
  }
  FF_STAMP_FLUSH(n_done);
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
inline bool aligned16(const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15u) == 0; }

int num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}

template <class T, bool GATHER>
int launch(void* stream, const FfParams& prm) {
  auto kern = ff_fused<T, GATHER>;
  const int lds = kLdsTotal<T>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return (int)e;
  int grid = num_cus();
  if (grid > prm.B) grid = prm.B;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

int run(void* stream, int dtype, const FfParams& prm_in) {
  FfParams prm = prm_in;
  // timing-ablation bits of the diagnostic tools (tools/ff_ab.py): read once per process
  static const int abl = [] { const char* e = getenv("MINER_FF_ABL"); return e ? atoi(e) : 0; }();
  prm.abl = abl;
  const bool gather = prm.his_ids != nullptr;
  if (dtype == MINER_DTYPE_BF16) return gather ? launch<__bf16, true>(stream, prm) : launch<__bf16, false>(stream, prm);
  return gather ? launch<float, true>(stream, prm) : launch<float, false>(stream, prm);
}

int check_common(int dtype, int B, int L, int C, const uint8_t* mask, const void* packed, const float* scores,
                 const float* user_out) {
  if (dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) return MINER_EINVAL;
  if (B < 0 || C < 0 || L <= 0) return MINER_EINVAL;
  if (L > kMaxL) return MINER_ESHAPE;
  if (!mask || !packed || (!scores && !user_out)) return MINER_EINVAL;
  if (!aligned16(packed)) return MINER_EALIGN;
  return MINER_OK;
}

}  // namespace

extern "C" {

size_t miner_fastformer_packed_bytes(int dtype) {
  if (dtype == MINER_DTYPE_BF16) return packed_bytes_t<__bf16>();
  if (dtype == MINER_DTYPE_F32) return packed_bytes_t<float>();
  return 0;
}

int miner_fastformer_pack(void* stream, int dtype, const float* params, void* packed) {
  if (dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) return MINER_EINVAL;
  if (!params || !packed) return MINER_EINVAL;
  if (!aligned16(packed)) return MINER_EALIGN;
  const int grid = 2048;
  if (dtype == MINER_DTYPE_BF16)
    hipLaunchKernelGGL(ff_pack_kernel<__bf16>, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), params,
                       static_cast<__bf16*>(packed));
  else
    hipLaunchKernelGGL(ff_pack_kernel<float>, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), params,
                       static_cast<float*>(packed));
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

int miner_fastformer_score(void* stream, int dtype, const void* history, const uint8_t* his_mask,
                           const void* candidates, const int32_t* cand_offsets, const void* packed, int B, int L,
                           int C, float* scores, float* user_out) {
  const int ck = check_common(dtype, B, L, C, his_mask, packed, scores, user_out);
  if (ck != MINER_OK) return ck;
  if (!history || (scores && !candidates)) return MINER_EINVAL;
  if (!aligned16(history) || !aligned16(candidates)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  FfParams prm{};
  prm.hist = history; prm.mask = his_mask; prm.cand = candidates; prm.cand_off = cand_offsets;
  prm.wp = packed; prm.scores = scores; prm.user_out = user_out;
  prm.B = B; prm.L = L; prm.C = C; prm.n_news = 0;
  return run(stream, dtype, prm);
}

int miner_fastformer_score_gather(void* stream, int dtype, const void* news_table, int n_news,
                                  const int32_t* his_ids, const uint8_t* his_mask, const int32_t* cand_ids,
                                  const int32_t* cand_offsets, const void* packed, int B, int L, int C,
                                  float* scores, float* user_out) {
  const int ck = check_common(dtype, B, L, C, his_mask, packed, scores, user_out);
  if (ck != MINER_OK) return ck;
  if (!news_table || !his_ids || n_news <= 0 || (scores && !cand_ids)) return MINER_EINVAL;
  if (!aligned16(news_table)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  FfParams prm{};
  prm.hist = news_table; prm.mask = his_mask; prm.cand = news_table; prm.cand_off = cand_offsets;
  prm.his_ids = his_ids; prm.cand_ids = cand_ids; prm.wp = packed; prm.scores = scores; prm.user_out = user_out;
  prm.B = B; prm.L = L; prm.C = C; prm.n_news = n_news;
  return run(stream, dtype, prm);
}

#ifdef MINER_STAMPS
// diagnostic build only: read (and reset) the per-stage cycle sums; out[0..15] cycles, out[16] impressions
int miner_ff_debug_stage_cycles(unsigned long long* out) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ff_stage_cycles), 16 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_ff_imps), sizeof(unsigned long long));
  unsigned long long z[16] = {0};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_ff_stage_cycles), z, 16 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_ff_imps), z, sizeof(unsigned long long));
  return (int)e;
}
#endif

int miner_fastformer_lds_bytes(int dtype) {
  if (dtype == MINER_DTYPE_BF16) return kLdsTotal<__bf16>;
  if (dtype == MINER_DTYPE_F32) return kLdsTotal<float>;
  return 0;
}

}  // extern "C"
