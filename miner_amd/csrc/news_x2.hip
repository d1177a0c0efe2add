// news_x2.hip — fp32 MINER scoring from news ids on the fp16 matrix cores (SURVEY.md §8 a1-a7 on
// the f2 news path), MI355X (gfx950 / CDNA4). The bench headline kernel since round 3.
//
// Why. The fp32 scoring kernel news_score32 (news.hip) runs its contractions on the fp32 MFMA:
// 64 FLOP/clk/SIMD, and it excludes the VALU of its SIMD, so the GELU and every other vector
// instruction add to the MFMA time (round-2 verdict: MFMA-bound at 0.56 of the fp32 peak). Here
// every fp32 operand x is carried as an exact-sum pair of fp16 values in a power-of-two scale s
// (per table row, or per interest for the attention weights and the user vectors),
//     x·s = hi + lo,  hi = fp16(x·s),  lo = fp16(x·s − hi)          (|x·s − hi − lo| ≤ 2⁻²²·|x·s|
//                                                                    while lo is a normal fp16)
// and a product a·b is the three partial products lo_a·hi_b + hi_a·lo_b + hi_a·hi_b on
// v_mfma_f32_16x16x32_f16 (every fp16 x fp16 product is exact in fp32, the accumulation is fp32;
// the dropped lo_a·lo_b is below 2⁻²²·|a·b|). The operand error is the fp32 rounding's order, far
// below the fp32 accumulation error of a 768-long dot product, which both forms share
// (tests/test_gpu_news.py measures both against float64). Three fp16 MFMAs (48 cycles) replace
// the 256 cycles of a 16x16x32 contraction on the fp32 MFMA, and they co-issue with the other
// wave's VALU. The pair planes of the news table and of its projection take 4 bytes per element,
// the same as fp32, so the gathered bytes do not grow.
//
// Kernels:
//   x2_split_rows  the pair planes with one power-of-two unit per ROW: row n holds x / u_n with
//                u_n = 2^(e_n - 14), max|row n| < 2^e_n (so every |x / u_n| < 2^14 < 65504); per
//                64-column chunk cc: [hi of the 64 columns | lo of the 64 columns], 256 B. A
//                per-row unit keeps each row's lo plane out of the fp16 subnormals however far its
//                magnitude is from the table's largest row (tests/test_gpu_news.py heavy-tailed
//                tables: rows 1e4x and 1e5x the median norm)
//   news_score_x2  per impression (one persistent workgroup of 8 waves per CU), from the ids:
//                A   = softmax_L(logits[his] + bias, masked slots = 1e-30)  (model.py:176-181)
//                mui = A·E[his]                                             (model.py:182)
//                X   = gelu(A·proj[his]) = gelu(mui·W2ᵀ)                    (model.py:212)
//                M   = Cand·muiᵀ,  Lg = Cand·Xᵀ                             (model.py:127, :213)
//                score = Σ_k softmax_k(Lg)·M | max_k M | mean_k M           (model.py:128-136, :214)
//
// Stream. The history rows of E and proj and the candidate rows stream in 64-column chunks (one
// 256-byte row piece per row: both planes) through two 48 KiB LDS slots [E[his] | proj[his] |
// Cand] (64 rows each), LDS-DMA by id one chunk ahead, one barrier per chunk; rows past L or past
// the candidate count are not fetched. Wave w = (path P = w >> 2, column half ch = (w >> 1) & 1,
// interest tile kt = w & 1), so each SIMD pairs a mui wave (P = 0) with an X wave (P = 1, the
// GELU). Per chunk and wave:
//   muiᵀ / Xᵀ [32 cols x 16 interests] = part[his]ᵀ·Aᵀ : 2 column tiles x 2 history blocks x 3
//       MFMAs; the history operand read transposed (ds_read_b64_tr_b16), Aᵀ in registers
//   M / Lg [16 cands x 16 interests] += Cand·muiᵀ / Xᵀ : 3 MFMAs per candidate tile, the two
//       accumulators of the first product ARE the B operand (lane (g, i) holds columns 4g..4g+3 of
//       both column tiles: contraction index 8g + e), split to fp16 pairs in registers
// At a pass end (<= 64 candidates) each wave publishes its partial M / Lg into its own LDS block;
// S7 (softmax over K, model.py:213-214) runs on the X waves at the next pass's first chunk.
// The per-impression ids, mask, bias and logit rows ride in small LDS "aux" blocks DMA'd one to
// four impressions ahead (as news.hip), so no load the compiler can see is waited on in the loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>
#include <type_traits>

#include "../../include/miner_news.h"
#include "cdna4_common.h"

namespace {

// Timing ablations only (tools/x2_ab.py builds; the product build never sets it; wrong scores):
// 2 no row DMAs, 4 no products, 8 no GELU, 16 no candidate MFMAs, 32 no history MFMAs. The
// measured-negative variants of rounds 4-5 (the per-impression work spread over the chunks, the
// 3-slot ring, S7 one chunk later, the dedupe on a mui wave, M0 left clobbered, two workgroups per
// CU) are not in this file: DESIGN §6i keeps their numbers.
#ifndef X2_ABL
#define X2_ABL 0
#endif

// (1024 / 2048: the mui / X waves skip the history softmax after the first impression, keeping the
// last A)
// (eval-loss form, GS: 64 no diagonal Gram tile, 128 no operand exchange / off-diagonal tile, 256 no
// per-chunk Gram work, 512 no per-impression D step)
constexpr int kNB = 2;                                // row-DMA blocks per wave per part
constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kMaxL = 64;
constexpr int kMaxK = 32;
constexpr int kMaxCand = MINER_NEWS_MAX_CAND;
constexpr int kCW = 64;                                // columns per chunk
constexpr int kRB = 256;                               // bytes per staged row piece (hi | lo)
constexpr int kPart = 64 * kRB;                        // 64 rows: E[his] | proj[his] | Cand
// the candidate part's 16-row tiles are kCTile apart (16 B of padding after each): the reads of
// tiles q and q + 1 from one base register are then neither a ds_read2_b64 (offsets <= 2040 B)
// nor a ds_read2st64_b64 (multiples of 512 B) pair, which hipcc would otherwise form and whose
// 16-lane groups bank by dword mod 32 — a 2-way conflict on these 16-row reads
// (MI355X_MICROARCH.md §LDS); ds_read_b64 banks mod 64 over 32 lanes: none
constexpr int kCTile = 16 * kRB + 16;
constexpr int kCPart = 4 * kCTile;
constexpr int kSlot = 2 * kPart + kCPart;
constexpr float kSA = 16384.0f;                        // scale of the attention weights (A <= 1)

// LDS carve (bytes): [ring x2 | F (pass partials) | logit blocks x2 | aux L1 x4 | aux L0 x8 | prep x2]
constexpr int kRingB = 2 * kSlot;                      // 98304
constexpr int kFB = 4 * 64 * 32 * 4;                   // F[P][ch] [c][k ^ swz] fp32
constexpr int kLogB = 64 * 128;                        // 64 history rows x K (<= 32) fp32
constexpr int kL1B = 4 * 64 * 3 + 4 * kMaxCand;        // his ids | mask words | bias | cand ids
constexpr int kL0B = 16;
constexpr int kPrepB = 2 * 64 * 4;                     // softmax (±multiplicity | add) per history group
constexpr int kOffF = kRingB;
constexpr int kOffLog = kOffF + kFB;
constexpr int kOffL1 = kOffLog + 2 * kLogB;
constexpr int kOffL0 = kOffL1 + 4 * kL1B;
constexpr int kOffPrep = kOffL0 + 8 * kL0B;
constexpr int kOffGram = kOffPrep + 3 * kPrepB;   // eval loss: one wave's Gram partial (3 16x16 tiles) + 32 norms
constexpr int kGramB = 3 * 256 * 4 + 32 * 4;
constexpr int kOffDup = kOffGram + kGramB;     // per L1 slot: U, the unique history rows of the impression
constexpr int kDupB = 16;
constexpr int kX2Lds = kOffDup + 4 * kDupB;
static_assert(kX2Lds <= 160 * 1024, "news_score_x2 LDS");

// The carve by field (the names the kernel reads through Cv::)
struct X2C {
  static constexpr int kPart = 64 * kRB;                 // 64 history rows of a part
  static constexpr int kSlot = 2 * kPart + 4 * kCTile;   // E[his] | proj[his] | 4 candidate tiles
  static constexpr int kRing = 2 * kSlot;
  static constexpr int kFBlk = 64 * 32;                  // floats of one F[P][ch] block
  static constexpr int kOffF = kRing;
  static constexpr int kLogB = 64 * 128;
  static constexpr int kOffLog = kOffF + 4 * kFBlk * 4;
  static constexpr int kL1Cand = 768;
  static constexpr int kL1B = 4 * 64 * 3 + 4 * kMaxCand;
  static constexpr int kOffL1 = kOffLog + 2 * kLogB;
  static constexpr int kOffL0 = kOffL1 + 4 * kL1B;
  static constexpr int kOffPrep = kOffL0 + 8 * kL0B;
  static constexpr int kOffGram = kOffPrep + 3 * kPrepB;
  static constexpr int kOffDup = kOffGram + kGramB;
  static constexpr int kLds = kOffDup + 4 * kDupB;
};
static_assert(X2C::kLds == kX2Lds, "x2 carve");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void raw_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ float x_both_max(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float x_both_sum(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
// all-reduce over the 4 16-lane rows (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float x_rows4_max(float x) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return x_both_max(fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1])));
}
__device__ __forceinline__ float x_rows4_sum(float x) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return x_both_sum(__uint_as_float(s[0]) + __uint_as_float(s[1]));
}

// one row DMA (saddr form: scalar base + 32-bit per-lane offset) into M0 = m, M0 saved / restored
__device__ __forceinline__ void x2_dma_row(uint32_t off, const char* base, unsigned m) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(t) : "v"(off), "s"(base), "s"(__builtin_amdgcn_readfirstlane(m)) : "memory");
}
__device__ __forceinline__ void x2_dma_b128(const void* g, unsigned lds) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(g), "s"(lds) : "memory");
}

// 16-byte chunk swizzle of a staged 256-byte row (16 chunks: hi plane 0..7, lo plane 8..15):
// chunk slot = chunk ^ x2swz(row) = chunk ^ ((row & 7) << 1 | (row >> 3) & 1): a bijection on rows
// 0..15, so the ds_read_b64 candidate operand (16 rows, one chunk, per 32-lane half) is
// conflict-free; the transposed history reads (8 consecutive rows 8n..8n+7 of a half, two adjacent
// chunks) see 8 distinct values of bits 1-3, so their 16 pieces land in 16 chunk slots.
__host__ __device__ inline int x2swz(int row) { return ((row & 7) << 1) | ((row >> 3) & 1); }

__device__ __forceinline__ f32x4 mfma_h(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// c += a·b at fp32 accuracy from fp16 pairs (smallest terms first)
__device__ __forceinline__ f32x4 mfma_x2(f32x4 c, const u32x4& ah, const u32x4& al, const u32x4& bh, const u32x4& bl) {
  c = mfma_h(al, bh, c);
  c = mfma_h(ah, bl, c);
  return mfma_h(ah, bh, c);
}
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16_h(unsigned a0, unsigned a1, unsigned b0, unsigned b1, f32x4 c) {
  typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, u32x2v{a0, a1}),
                                                __builtin_bit_cast(f16x4, u32x2v{b0, b1}), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16_x2(f32x4 c, const u32x4& a, const u32x4& b) {
  c = mfma16_h(a[2], a[3], b[0], b[1], c);
  c = mfma16_h(a[0], a[1], b[2], b[3], c);
  return mfma16_h(a[0], a[1], b[0], b[1], c);
}
// two fp32 values -> (hi, lo) fp16 pairs, packed. The residual is taken against the hi bits as
// packed: left to itself hipcc packs hi with v_cvt_pk_f16_f32 but recomputes the f32 value of hi
// with a separate v_cvt_f16_f32, and the two round some halfway cases differently (one fp16 ulp of
// hi lost in 4 of 480k attention weights at config 3; tools/x2_diag.py)
__device__ __forceinline__ void split2(float x0, float x1, unsigned& hi, unsigned& lo) {
  const f16x2 h = {(_Float16)x0, (_Float16)x1};
  unsigned hb = __builtin_bit_cast(unsigned, h);
  asm volatile("" : "+v"(hb));
  const f16x2 hh = __builtin_bit_cast(f16x2, hb);
  // x - hi (exact) with hi read as an f16 half of the packed register: v_fma_mix_f32, no separate
  // v_cvt_f32_f16 (bit-identical; -0.9 % on the x2 kernel)
  float r0, r1;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r0) : "v"(hb), "v"(x0));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1) : "v"(hb), "v"(x1));
  (void)hh;
  const f16x2 l = {(_Float16)r0, (_Float16)r1};
  hi = hb;
  lo = __builtin_bit_cast(unsigned, l);
}
// the attention weights w·e·c (w a small integer multiplicity, e = exp, c = κ·unit / Σ) -> (hi, lo)
// fp16 pairs with the residual taken from exact products (fma), so a group of m slots carries one
// rounding of its weight, not the three of w·(e·c) rounded step by step
__device__ __forceinline__ void split2w(float w0, float e0, float c0, float w1, float e1, float c1, unsigned& hi,
                                        unsigned& lo) {
  const float p0 = e0 * c0, p1 = e1 * c1;
  const float q0 = __builtin_fmaf(e0, c0, -p0), q1 = __builtin_fmaf(e1, c1, -p1);
  const f16x2 h = {(_Float16)(w0 * p0), (_Float16)(w1 * p1)};
  unsigned hb = __builtin_bit_cast(unsigned, h);
  asm volatile("" : "+v"(hb));
  const f16x2 hh = __builtin_bit_cast(f16x2, hb);
  const f16x2 l = {(_Float16)__builtin_fmaf(w0, q0, __builtin_fmaf(w0, p0, -(float)hh[0])),
                   (_Float16)__builtin_fmaf(w1, q1, __builtin_fmaf(w1, p1, -(float)hh[1]))};
  hi = hb;
  lo = __builtin_bit_cast(unsigned, l);
}
// 8 fp32 values -> hi / lo f16x8 operands
__device__ __forceinline__ void split8h(const float* x, u32x4& hi, u32x4& lo) {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    unsigned h, l;
    split2(x[2 * m], x[2 * m + 1], h, l);
    hi[m] = h;
    lo[m] = l;
  }
}
__device__ __forceinline__ uint2 lds_u64(const char* p) { return *reinterpret_cast<const uint2*>(p); }

// e^x for the softmaxes' x = s - max <= 0: 2^(x·log2 e) on v_exp_f32 with the product's rounding
// carried to first order (x·log2 e = yh + yl, yl from one fma and log2 e's low part; e^x =
// 2^yh·(1 + yl·ln 2)), a few ulp like libm expf in 6 VALU instead of ~14 (its range reduction and
// over/underflow selects); x is clamped at -104 (e^-104 underflows to 0 either way), so -inf gives 0
// and a NaN propagates
__device__ __forceinline__ float x2_exp(float x) {
  x = x < -104.0f ? -104.0f : x;                    // not fmaxf: a NaN logit stays NaN (torch softmax)
  const float yh = x * 1.4426950408889634f;
  const float yl = __builtin_fmaf(x, 1.925963033500011e-8f, __builtin_fmaf(x, 1.4426950408889634f, -yh));
  const float e = __builtin_amdgcn_exp2f(yh);
  return __builtin_fmaf(e, yl * 0.69314718055994531f, e);
}

__device__ __forceinline__ uint2 lds_tr(const char* p) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds_char*)p));
}

// ================================================================================================
// pair planes
// ================================================================================================
// the unit of a row from its max |x|: u = 2^(e - 14) with max|x| < 2^e, so the pair values x / u
// stay below 2^14 (< 65504); e clamped to [-110, 128] (1 / u representable); an all-zero row gets
// u = 2^-14, a non-finite max u = 1 (an infinite or NaN entry then stays one in its pair)
__device__ __forceinline__ int x2_row_exp(float m) {
  if (!(m > 0.f)) return 0;
  if (!isfinite(m)) return 14;
  int e;
  frexpf(m, &e);                                     // m = f·2^e, f in [0.5, 1)
  return min(max(e, -110), 128);
}

// one wave per row: dst row n = for each 64-column chunk, 64 hi then 64 lo fp16 of x / u_n (the x2
// layout); unit[n] = u_n. A per-row unit (not one per table) keeps every row's lo plane out of the
// fp16 subnormals when one row of the table is many orders of magnitude larger than the others
constexpr int kSplitMaxG = 2;                         // 8-column groups per lane: d <= 1024
__global__ __launch_bounds__(256) void x2_split_rows(const float* __restrict__ src, int N, int d,
                                                     unsigned short* __restrict__ dst, float* __restrict__ unit) {
  const int lane = threadIdx.x & 63;
  const int g8 = d >> 3;                             // groups of 8 columns per row
  for (int n = blockIdx.x * 4 + (threadIdx.x >> 6); n < N; n += gridDim.x * 4) {
    const float* row = src + (size_t)n * d;
    float4 v[kSplitMaxG][2];
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < kSplitMaxG; ++j) {
      const int gi = lane + 64 * j;
      if (gi < g8) {
        const float4* q = reinterpret_cast<const float4*>(row + 8 * gi);
        v[j][0] = q[0];
        v[j][1] = q[1];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[j][0].x), fabsf(v[j][0].y)), fmaxf(fabsf(v[j][0].z), fabsf(v[j][0].w))));
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[j][1].x), fabsf(v[j][1].y)), fmaxf(fabsf(v[j][1].z), fabsf(v[j][1].w))));
      }
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const int e = x2_row_exp(m);
    const float s = ldexpf(1.0f, 14 - e);
    if (lane == 0) unit[n] = ldexpf(1.0f, e - 14);
#pragma unroll
    for (int j = 0; j < kSplitMaxG; ++j) {
      const int gi = lane + 64 * j;
      if (gi < g8) {
        const float x[8] = {v[j][0].x * s, v[j][0].y * s, v[j][0].z * s, v[j][0].w * s,
                            v[j][1].x * s, v[j][1].y * s, v[j][1].z * s, v[j][1].w * s};
        u32x4 hi, lo;
        split8h(x, hi, lo);
        const int c0 = 8 * gi;
        unsigned short* o = dst + (size_t)n * (2 * d) + (c0 >> 6) * 128 + (c0 & 63);
        *reinterpret_cast<u32x4*>(o) = hi;
        *reinterpret_cast<u32x4*>(o + 64) = lo;
      }
    }
  }
}

// ================================================================================================
// per-impression scoring
// ================================================================================================
// diagnostic build only (-DMINER_STAMPS): per-wave stage cycles (lane 0 of each wave sums s_memtime
// deltas; read with miner_news_x2_debug_stage_cycles). The stamps wait for outstanding LDS reads.
#ifdef MINER_STAMPS
__device__ unsigned long long g_x2_stage[kWaves][8];
__device__ unsigned long long g_x2_items;
#define X2_STAMP_DECL unsigned long long st_acc[8] = {0}; unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define X2_STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } while (0)
#define X2_STAMP_FLUSH(n) do { if ((threadIdx.x & 63) == 0) { for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_x2_stage[threadIdx.x >> 6][i_], st_acc[i_]); if (threadIdx.x == 0) atomicAdd(&g_x2_items, (unsigned long long)(n)); } } while (0)
#else
#define X2_STAMP_DECL
#define X2_STAMP(i) do {} while (0)
#define X2_STAMP_FLUSH(n) do {} while (0)
#endif

struct X2Params {
  const void* table2;      // [n_news, d] pairs (x2 layout): row n holds x / unit_t[n]
  const float* logits;     // [n_news, K]
  const void* proj2;       // [n_news, d] pairs, row n = x / unit_p[n] (weighted only)
  const float* unit_t;     // [n_news] per-row units (powers of two, x2_split_rows)
  const float* unit_p;
  const int32_t* his_ids;
  const uint8_t* mask;
  const float* bias;
  const int32_t* cand_ids;
  const int32_t* cand_off;
  float* scores;
  float* mui_out;
  float* dis_out;          // [B] per-impression disagreement (the eval loss's Gram term), or null
  int n_news, B, L, C, d, K, score_type;
};

__device__ __forceinline__ int* l1_his(char* smem, int slot) { return reinterpret_cast<int*>(smem + X2C::kOffL1 + slot * X2C::kL1B); }
__device__ __forceinline__ uint32_t* l1_mask(char* smem, int slot) { return reinterpret_cast<uint32_t*>(smem + X2C::kOffL1 + slot * X2C::kL1B + 256); }
__device__ __forceinline__ float* l1_bias(char* smem, int slot) { return reinterpret_cast<float*>(smem + X2C::kOffL1 + slot * X2C::kL1B + 512); }
__device__ __forceinline__ int* l1_cand(char* smem, int slot) { return reinterpret_cast<int*>(smem + X2C::kOffL1 + slot * X2C::kL1B + X2C::kL1Cand); }
__device__ __forceinline__ int* l0_off(char* smem, int slot) { return reinterpret_cast<int*>(smem + X2C::kOffL0 + slot * kL0B); }
__device__ __forceinline__ int* dup_u(char* smem, int slot) { return reinterpret_cast<int*>(smem + X2C::kOffDup + slot * kDupB); }
__device__ __forceinline__ float* prep_blk(char* smem, int i) { return reinterpret_cast<float*>(smem + X2C::kOffPrep + (i % 3) * kPrepB); }

// NCH: 64-column chunks per row (0: d / 64 at run time). SHP 2: the MIND shape (history L = 50,
// K = 32 interests) compile-time, no category bias and no mui output (plain scoring: the bench, the
// eval without the eval loss); SHP 0: run-time L, K. LOSS: also the eval loss's per-impression
// disagreement D = mean_{k != k'} cos(mui_k, mui_k') (loss.py:81, utils.py:9-29) from the Gram matrix
// mui·muiᵀ, accumulated per chunk by the mui waves of interest tile 0: they run the history product
// for both interest tiles (the transposed E reads are shared) and add the 3 Gram tiles of their 32
// columns; at the pass end wave 2 hands its tiles to wave 0 through LDS, which forms D at the next
// chunk (no mui is written).
template <int ST, bool RAGGED, int NCH, int SHP, bool LOSS = false>
__global__ __launch_bounds__(kThreads) void news_score_x2(X2Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool WEIGHTED = ST == MINER_SCORE_WEIGHTED;
  constexpr bool WITH_CAND = ST != MINER_SCORE_NONE;
  const int G = gridDim.x;
  const int n_i = (p.B - (int)blockIdx.x + G - 1) / G;      // impressions of this workgroup
  const int L = SHP == 2 ? 50 : p.L;
  const int KK = SHP == 2 ? 32 : p.K;
  const int d = NCH > 0 ? NCH * kCW : p.d;
  const int nchunk = NCH > 0 ? NCH : d / kCW;
  const float* const bias = SHP == 2 ? nullptr : p.bias;
  float* const mui_out = SHP == 2 ? nullptr : p.mui_out;
  float* const dis_out = LOSS ? p.dis_out : nullptr;
  using Cv = X2C;
  constexpr int kDedupeWave = 7;                       // an X wave (they wait at the barriers)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P = wave >> 2, ch = (wave >> 1) & 1, kt = wave & 1;
  const bool k_live = 16 * kt < KK;
  const bool path_live = P == 0 || WEIGHTED;
  // The eval loss's Gram. GS (the MIND shape: L = 50, 4 or 12 chunks): spread over the four mui
  // waves — each adds its own diagonal 16x16 tile over its 32 columns from the operand of its
  // candidate product (no extra split); the off-diagonal tile is split by column tile: the wave of
  // interest tile kt adds G_{kt,1-kt} over columns [16 kt, +16) of its column half, with the other
  // wave's operand of those columns through LDS one chunk later (rows 56..63 of part ch of that
  // chunk's ring slot: no DMA writes them at L <= 52, and the history products read zero rows in
  // their place, trH3). Otherwise (run-time shapes) waves 0 and 2 run the history product for both
  // interest tiles and add all three tiles of their 32 columns.
  constexpr bool GS = LOSS && SHP == 2;
  static_assert(!GS || (NCH >= 3 && WEIGHTED), "the spread Gram: chunk counts >= 3, 'weighted' scoring");
  const bool gram_w = LOSS && P == 0 && (GS || kt == 0);
  const char* tabB = static_cast<const char*>(p.table2);
  const char* prjB = WEIGHTED ? static_cast<const char*>(p.proj2) : tabB;
  const unsigned sbase = __builtin_amdgcn_readfirstlane(lds_offset(smem));
  // Scales. Pair-plane row u holds part_u / unit_u; the history product's B operand is
  // κ_k·A_ku·unit_u (κ_k a power of two per interest, softmax_inwave), so it accumulates
  // acc_k = κ_k·(A·part)_k. Per lane (its interest k): the accumulator -> split operand factor
  // (mui path 2^-14: |κ_k·mui_k| < 2^28; X path 1/κ_k, the GELU's input), the X path's factor after
  // the GELU (κ_k·2^-14), the pass-end factor of the M / Lg partials (2^14 / κ_k, leaving only the
  // candidate's unit for S7) and 1 / κ_k for the mui output. Set per impression.
  float kap = kSA;                         // κ_k of this lane's interest (the wave's path), per impression
  float uc_pend_r = 1.0f;                  // S7 lane's candidate unit (X waves), loaded a chunk ahead

  auto imp_b = [&](int i) { return (int)blockIdx.x + i * G; };
  auto cands = [&](int i, int& off, int& cnt) {
    if constexpr (!WITH_CAND) { off = 0; cnt = 0; return; }
    if constexpr (RAGGED) {
      const int* o = l0_off(smem, i & 7);
      off = __builtin_amdgcn_readfirstlane(o[0]);
      cnt = __builtin_amdgcn_readfirstlane(o[1]) - off;
    } else {
      off = imp_b(i) * p.C;
      cnt = p.C;
    }
    cnt = min(max(cnt, 0), kMaxCand);
  };
  // ---- aux DMA jobs (after a barrier): L0 CSR offsets -> L1 ids / mask / bias -> L2 logit rows ----
  auto issue_L0 = [&](int i) {
    if (RAGGED && wave == 0 && i < n_i && (threadIdx.x & 63) < 2)
      dma_b32(p.cand_off + imp_b(i) + (threadIdx.x & 63), sbase + Cv::kOffL0 + (i & 7) * kL0B);
  };
  auto issue_L1 = [&](int i) {
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const size_t base = (size_t)imp_b(i) * L + min(lane, L - 1);
    const unsigned l1 = sbase + Cv::kOffL1 + (i & 3) * Cv::kL1B;
    if (wave == 1) {
      dma_b32(p.his_ids + base, l1);
    } else if (wave == 2) {
      // the aligned word holding mask byte `base` (the reader picks the byte by address)
      const uintptr_t a = reinterpret_cast<uintptr_t>(p.mask + base) & ~(uintptr_t)3;
      dma_b32(reinterpret_cast<const void*>(a), l1 + 256);
    } else if (wave == 3) {
      if (bias) dma_b32(bias + base, l1 + 512);
    } else if (WITH_CAND && wave >= 4) {                 // candidate ids, 64 per DMA
      int off, cnt;
      cands(i, off, cnt);
      for (int j = wave - 4; j >= 0 && 64 * j < cnt; j += 4) {
        const int c = min(64 * j + lane, cnt - 1);
        dma_b32(p.cand_ids + off + c, l1 + Cv::kL1Cand + 256 * j);
      }
    }
  };
  // logit rows of impression i by UNIQUE history row (after its dedupe, below)
  auto issue_L2 = [&](int i) {
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const int U = __builtin_amdgcn_readfirstlane(dup_u(smem, i & 3)[0]);
    const int row = min(8 * wave + (lane >> 3), U - 1);
    const int piece = min(lane & 7, (KK >> 2) - 1);
    const int id = min(max(l1_his(smem, i & 3)[row], 0), p.n_news - 1);
    x2_dma_b128(p.logits + (size_t)id * KK + 4 * piece, sbase + Cv::kOffLog + (i & 1) * Cv::kLogB + wave * 1024);
  };
  // The masked history slots holding the same news id — the left padding: every pad slot is the pad
  // news, masked (reader.py:101-110, :369) — form one group: its row is gathered and contracted once,
  // and the softmax over the history (model.py:176-181) runs over the U groups with multiplicities,
  // A_u = m_u·exp(s_u − max) / Σ_v m_v·exp(s_v − max), exactly the slots' sum regrouped. Wave 7 (an
  // X wave: they wait at the barriers) replaces impression i's history ids in L1 by the groups' ids
  // (first-occurrence order) and writes each group's coefficients (±m, add): s_u = logit + bias with
  // weight m for a click (+m), s_u = 1e-30 with weight m for a pad slot (-m; model.py:176-180),
  // (0, -inf) past U — and U.
  // The groups' row units: loaded by one dedupe_prep call, merged into the codes by the next one (an
  // impression later: the loads have landed, nothing waits on them; the codes are read two
  // impressions after their dedupe). Wave 7 only; du_i = the impression whose units are pending.
  float du_E = 1.f, du_P = 1.f;
  int du_slot = -1, du_i = -1;
  // the merge of the pending units: the compiler waits for their loads here (vmcnt), so it is called
  // right after a barrier, when this wave's row DMAs have all landed, not behind the chunk DMAs it
  // has just issued
  auto dedupe_merge = [&]() {
    if (wave != kDedupeWave) return;
    if (du_i >= 0) {
      int* pcp = reinterpret_cast<int*>(prep_blk(smem, du_i));
      if (du_slot >= 0)
        pcp[du_slot] |= (((__float_as_int(du_E) >> 23) & 255) << 8) | (((__float_as_int(du_P) >> 23) & 255) << 16);
      du_i = -1;
    }
  };
  auto dedupe_prep = [&](int i) {
    if (wave != kDedupeWave) return;
    const int l = threadIdx.x & 63;
    dedupe_merge();
    if (i >= n_i) return;
    int* his = l1_his(smem, i & 3);
    const int ls = min(l, L - 1);
    const int id = his[ls];
    const int idc = min(max(id, 0), p.n_news - 1);
    du_E = p.unit_t[idc];
    du_P = WEIGHTED ? p.unit_p[idc] : 1.0f;
    const uint32_t mw = l1_mask(smem, i & 3)[ls];
    const int a = (int)(reinterpret_cast<uintptr_t>(p.mask + (size_t)imp_b(i) * L + ls) & 3);
    const bool keep = ((mw >> (8 * a)) & 0xffu) != 0u;
    const float bv = (keep && bias) ? l1_bias(smem, i & 3)[ls] : 0.f;
    // the group: the masked slots holding the first masked slot's news id (a masked slot's logit and
    // bias never enter its score, model.py:176-180); every other slot is a group of its own
    const unsigned long long pads = __ballot(l < L && !keep);
    const int f = pads ? (int)__builtin_ctzll(pads) : 0;
    const int idf = __builtin_amdgcn_readlane(id, f);
    const unsigned long long grp = pads & __ballot(id == idf);
    const int m = ((grp >> l) & 1ull) ? (int)__popcll(grp) : 1;   // read at the group's first slot only
    const bool uniq = l < L && (((grp >> l) & 1ull) == 0ull || l == f);
    const unsigned long long bal = __ballot(uniq);
    const int U = __popcll(bal);
    const int uidx = __popcll(bal & ((1ull << l) - 1ull));
    float* pr = prep_blk(smem, i);
    // (code, add) per group; code, an integer: bits 0-7 the multiplicity m, 8-15 / 16-23 the
    // exponent fields of the E / proj rows' units (powers of two; or'ed in by the next call), bit
    // 24 set for a click
    int* pc = reinterpret_cast<int*>(pr);
    if (uniq) {
      his[uidx] = id;
      pc[uidx] = m | (keep ? 1 << 24 : 0);
      pr[64 + uidx] = keep ? bv : 1e-30f;
    }
    if (l >= U) {                        // every coefficient past the groups (a unique lane may sit there):
      pc[l] = (113 << 8) | (113 << 16);  // m = 0, units 2^-14
      pr[64 + l] = -INFINITY;
    }
    if (l == 0) dup_u(smem, i & 3)[0] = U;
    du_slot = uniq ? uidx : -1;
    du_i = i;
  };
  // row DMAs of a chunk: wave w issues the 4-row blocks w and 8 + (w ^ 4) of every part (the rows
  // 32..47, live for L = 50 / C = 40, go to the X waves, the mostly-padding rows 48..63 to the mui
  // waves; all E rows on the mui waves and all proj / candidate rows on the X waves measured 10 %
  // slower). Lane l fills row 4b + (l >> 4), chunk slot l & 15 from source chunk slot ^ x2swz(row).
  // lv bit jj: history rows of block jj live; bit 4 + jj: its candidate rows live.
  auto dma_block = [&](int jj) { return jj ? 8 + (wave ^ 4) : wave; };
  constexpr bool dmaE = true, dmaP = WEIGHTED, dmaC = WITH_CAND;
  auto item_offsets = [&](int i, int pass, uint32_t* oH, uint32_t* oC, unsigned& lv) {
    const int lane = threadIdx.x & 63;
    const bool live = i < n_i;
    int off = 0, cnt = 1;
    if (live) cands(i, off, cnt);
    const int cntp = max(1, min(64, cnt - 64 * pass));
    const int U = live ? __builtin_amdgcn_readfirstlane(dup_u(smem, i & 3)[0]) : 1;
    lv = 0;
#pragma unroll
    for (int jj = 0; jj < kNB; ++jj) {
      const int row0 = 4 * dma_block(jj);
      if (live && (dmaE || dmaP) && row0 < U) lv |= 1u << jj;
      if (live && dmaC && row0 < cnt - 64 * pass) lv |= 16u << jj;
      const int row = row0 + (lane >> 4);
      const uint32_t poff = (uint32_t)(((lane & 15) ^ x2swz(row)) << 4);
      int h = 0, c = 0;
      if (live) {
        if (dmaE || dmaP) h = l1_his(smem, i & 3)[min(row, U - 1)];
        if (dmaC) c = l1_cand(smem, i & 3)[min(64 * pass + min(row, cntp - 1), kMaxCand - 1)];
      }
      h = min(max(h, 0), p.n_news - 1);
      c = min(max(c, 0), p.n_news - 1);
      const uint32_t rowBytes = (uint32_t)d * 4u;
      oH[jj] = (uint32_t)h * rowBytes + poff;
      oC[jj] = (uint32_t)c * rowBytes + poff;
    }
    lv = __builtin_amdgcn_readfirstlane(lv);
  };
  auto dma_chunk = [&](const uint32_t* oH, const uint32_t* oC, unsigned lv, int cc, int slot) {
    if (lv == 0 || (X2_ABL & 2)) return;
    const char* bE = tabB + cc * kRB;
    const char* bP = prjB + cc * kRB;
#pragma unroll
    for (int jj = 0; jj < kNB; ++jj) {
      const unsigned m = sbase + slot * Cv::kSlot + dma_block(jj) * 1024;
      if (lv & (1u << jj)) {
        if (dmaE) x2_dma_row(oH[jj], bE, m);
        if (dmaP) x2_dma_row(oH[jj], bP, m + Cv::kPart);
      }
      if (lv & (16u << jj)) x2_dma_row(oC[jj], bE, m + 2 * Cv::kPart + (dma_block(jj) >> 2) * 16);
    }
  };

  // ---- per-lane LDS read offsets (fixed for the launch) ----
  // transposed history reads: lane 4q + p of group g supplies (unique) row 16r + 4g + q (read r = 0, 1;
  // + 32 kb rows = 8192 B by immediate), columns 4p .. 4p + 3 of column tile 2ch + ctl; lane i of the
  // group receives column i of the 4 rows: contraction index 8g + e <-> row 32 kb + 16 (e >> 2) + 4g +
  // (e & 3), the order of the Ā tiles (softmax_inwave). Candidate reads: row i (+ 16 ct rows = 4096 B),
  // columns 32 ch + 16 ctl + 4g .. + 3 (8 B).
  // GS: the second block's rows 56..63 hold the Gram exchange (any bits, NaN included), so the
  // lanes that would read them (groups 2, 3 of read rr = 1) read rows 52..55 instead: zeros (no DMA
  // writes rows >= 52 at L <= 52), times the same zero attention weights (trH3 / trL3)
  uint32_t trH[2][2], trL[2][2], cfH[2], cfL[2], trH3[2], trL3[2];
  {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, i = lane & 15;
#pragma unroll
    for (int ctl = 0; ctl < 2; ++ctl) {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int row = 16 * rr + 4 * g + q;
        const int chunk = 4 * ch + 2 * ctl + (pp >> 1);
        trH[ctl][rr] = row * kRB + ((chunk ^ x2swz(row)) << 4) + 8 * (pp & 1);
        trL[ctl][rr] = row * kRB + (((chunk + 8) ^ x2swz(row)) << 4) + 8 * (pp & 1);
      }
      {
        const int row = g >= 2 ? 52 + q : 48 + 4 * g + q;
        const int chunk = 4 * ch + 2 * ctl + (pp >> 1);
        trH3[ctl] = row * kRB + ((chunk ^ x2swz(row)) << 4) + 8 * (pp & 1);
        trL3[ctl] = row * kRB + (((chunk + 8) ^ x2swz(row)) << 4) + 8 * (pp & 1);
      }
      const int chunk = 4 * ch + 2 * ctl + (g >> 1);
      cfH[ctl] = i * kRB + ((chunk ^ x2swz(i)) << 4) + 8 * (g & 1);
      cfL[ctl] = i * kRB + (((chunk + 8) ^ x2swz(i)) << 4) + 8 * (g & 1);
    }
  }

  // Aᵀ B operand of the history product, fp16 pairs: lane (g, i) holds A[16 kt + i][u] of the history
  // groups u = 32 kb + 16 (e >> 2) + 4g + (e & 3) (aH1 / aL1: interest tile 1, the Gram waves only)
  u32x4 aH[2], aL[2], aH1[2], aL1[2];

  // softmax over the history groups (model.py:176-181) of this wave's 16 interests, in registers:
  // lane (g, i) takes 16 groups, the 4 lane rows combined by permlanes
  // path pth (0: E rows, 1: proj rows) picks the units; kap = κ_k of this lane's interest
  auto softmax_inwave = [&](int i, int ktile, int pth, u32x4* dH, u32x4* dL, float& kap, auto nss_c) {
    constexpr int NSS = decltype(nss_c)::value;   // groups per lane: 16 (64 groups) or 8 (the first 32)
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const int k = 16 * ktile + j;
    const float* lgb = reinterpret_cast<const float*>(smem + Cv::kOffLog + (i & 1) * Cv::kLogB);
    const float* pr = prep_blk(smem, i);
    const int* pc = reinterpret_cast<const int*>(pr);
    const unsigned sh = pth ? 16u : 8u;
    float v[NSS], wm[NSS], un[NSS];
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < NSS; ++s) {
      const int u = 32 * (s >> 3) + 16 * ((s >> 2) & 1) + 4 * g + (s & 3);
      const unsigned code = (unsigned)pc[u];
      wm[s] = (float)(code & 255u);
      un[s] = __uint_as_float(__builtin_amdgcn_ubfe(code, sh, 8) << 23);     // the row's unit
      const float click = __uint_as_float((code >> 24) * 0x3f800000u);         // 1 for a click, else 0
      v[s] = __builtin_fmaf(lgb[u * 32 + k], click, pr[64 + u]);
      mx = fmaxf(mx, v[s]);
    }
    mx = x_rows4_max(mx);
    float sum = 0.f, tu = 0.f;
#pragma unroll
    for (int s = 0; s < NSS; ++s) {
      v[s] = x2_exp(v[s] - mx);              // 0 past U (v = -inf there; weight 0)
      const float we = wm[s] * v[s];
      sum += we;
      tu = __builtin_fmaf(we, un[s], tu);
    }
    sum = x_rows4_sum(sum);
    tu = x_rows4_sum(tu);
    // T_k = Σ_u A_ku·unit_u < 2^e: κ_k = 2^(14 - e) keeps every κ_k·A_ku·unit_u below 2^14
    int e;
    frexpf(tu / sum, &e);
    e = min(max(e, -100), 114);
    kap = __int_as_float((141 - e) << 23);              // 2^(14 - e)
    float inv = kap / sum;
    if (k >= KK) inv = 0.f;
#pragma unroll
    for (int m = 0; m < NSS / 2; ++m) {
      unsigned h, l;
      split2w(wm[2 * m], v[2 * m], inv * un[2 * m], wm[2 * m + 1], v[2 * m + 1], inv * un[2 * m + 1], h, l);
      dH[m >> 2][m & 3] = h;
      dL[m >> 2][m & 3] = l;
    }
  };

  // ring rows no DMA writes read as zeros; the prologue's first barrier orders these stores first
  for (int o = (int)threadIdx.x * 16; o < Cv::kRing; o += kThreads * 16)
    *reinterpret_cast<u32x4*>(smem + o) = u32x4{0u, 0u, 0u, 0u};
  for (int i = 0; i < 4; ++i) issue_L0(i);
  vm_wait_all();
  raw_barrier();
  issue_L1(0); issue_L1(1); issue_L1(2);
  vm_wait_all();
  raw_barrier();
  dedupe_prep(0);
  dedupe_prep(1);
  raw_barrier();
  issue_L2(0); issue_L2(1);
  vm_wait_all();
  raw_barrier();
  uint32_t cH[kNB], cC[kNB], nH[kNB], nC[kNB];
#pragma unroll
  for (int jj = 0; jj < kNB; ++jj) nH[jj] = nC[jj] = 0u;
  unsigned cLv = 0, nLv = 0;
  item_offsets(0, 0, cH, cC, cLv);
  dma_chunk(cH, cC, cLv, 0, 0);

  f32x4 acc[4];                                  // this wave's M / Lg partials, candidate tiles 0..3
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  int pend_off = -1, pend_cnt = 0;
  int t = 0;
  f32x4 gr[3];                                   // Gram tiles (0,0), (0,1), (1,1) of this wave's columns
#pragma unroll
  for (int q = 0; q < 3; ++q) gr[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  int pend_d = -1;                               // impression whose D is formed at the next chunk (wave 0)
  u32x4 gp = u32x4{0u, 0u, 0u, 0u};   // GS: this wave's operand of its off-diagonal columns, the last chunk
  int gs_step = 0, gs_b = 0;                     // GS (kernel-uniform): D of impression gs_b, step 1 / 2 pending
  int nkb = 2;                                   // 32-row blocks of unique history rows of the item
  bool d_pending = false;                        // wave-uniform: a Gram hand-off is waiting
  X2_STAMP_DECL

  // D of impression b from the Gram tiles (wave 0: its own + wave 2's from LDS): norms n_k = sqrt(G_kk),
  // S = Σ_{k != k'} G_kk' / (n_k n_k') over k, k' < K, D = S / K² (the diagonal zeroed as in the reference)
  auto form_d = [&](int b) {
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const float* pg = reinterpret_cast<const float*>(smem + Cv::kOffGram);
    float* nrm = reinterpret_cast<float*>(smem + Cv::kOffGram + 3 * 256 * 4);
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) gr[q][e] += pg[(q * 4 + e) * 64 + lane];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (4 * g + e == j) {
        nrm[j] = sqrtf(gr[0][e]);
        nrm[16 + j] = sqrtf(gr[2][e]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = 4 * g + e;
      const float nm0 = nrm[m], nm1 = nrm[16 + m], nn0 = nrm[j], nn1 = nrm[16 + j];
      if (m != j && m < KK && j < KK) sum += gr[0][e] / (nm0 * nn0);
      if (m < KK && 16 + j < KK) sum += 2.0f * (gr[1][e] / (nm0 * nn1));
      if (m != j && 16 + m < KK && 16 + j < KK) sum += gr[2][e] / (nm1 * nn1);
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if (lane == 0) dis_out[b] = sum / (float)(KK * KK);
#pragma unroll
    for (int q = 0; q < 3; ++q) gr[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // GS. The exchange block written by the wave of interest tile w in chunk tt, column half ch: 64
  // lanes x 16 B {hi, hi | lo, lo} of the columns the other wave takes, [16 (1 - w), +16)
  auto gs_xbuf = [&](int tt, int w) { return smem + (tt & 1) * Cv::kSlot + ch * Cv::kPart + 56 * kRB + w * 1024; };
  // the other wave's operand of this wave's off-diagonal columns in the chunk before, read right
  // after each chunk's barrier and used at the end of its products (with this wave's own operand
  // of those columns in that chunk, gp) or by the D step: its LDS latency hides behind the chunk
  u32x4 gx = u32x4{0u, 0u, 0u, 0u};
  auto gs_read = [&]() {
    if (X2_ABL & (128 | 256)) return;
    gx = *reinterpret_cast<const u32x4*>(gs_xbuf(t - 1, 1 - kt) + 16 * (threadIdx.x & 63));
  };
  // rows = this wave's own interests: the tile-1 wave's partial is the (0, 1) tile transposed, so
  // the D step weighs it with the norms the other way round
  auto gs_offdiag = [&]() {
    if (X2_ABL & (128 | 256)) return;
    gr[1] = mfma16_x2(gr[1], gp, gx);
  };
  // per chunk of a Gram pass, after the operand split (mui waves): the diagonal tile; the previous
  // chunk's off-diagonal partial; this wave's operand of its off-diagonal columns kept for the
  // next, the other columns' published as they are (a non-finite operand too: only this pass's
  // off-diagonal products read the block, and the wave's own diagonal tile carries it into the
  // norms anyway, so D is NaN / inf as the reference's). Round 6 A/B (tools/x2_ab.py):
  // the whole off-diagonal tile on the tile-0 waves +0.4 %; the published operand checked for
  // finiteness and zeroed, while the history products still read these rows, +3.2 %.
  auto gs_chunk = [&](int cc, const u32x4& bH, const u32x4& bL) {
    if (X2_ABL & 256) return;
    if (!(X2_ABL & 64)) gr[0] = mfma_x2(gr[0], bH, bL, bH, bL);
    if (X2_ABL & 128) return;
    if (cc > 0) gs_offdiag();
    const u32x4 c0 = u32x4{bH[0], bH[1], bL[0], bL[1]}, c1 = u32x4{bH[2], bH[3], bL[2], bL[3]};
    gp = kt ? c1 : c0;
    *reinterpret_cast<u32x4*>(gs_xbuf(t, kt) + 16 * (threadIdx.x & 63)) = kt ? c0 : c1;
  };
  // step 1 (the chunk after a Gram pass, after its barrier; mui waves): the last off-diagonal
  // partial, the norms n_k = sqrt(G_kk) from the four waves' diagonal partials (LDS [ch][kt][16],
  // written at the pass end), this wave's share Σ G_kk' / (n_k n_k') over its tiles (k != k' in the
  // diagonal tile, the off-diagonal partial twice) -> LDS; step 2 (a chunk later, wave 0): D = (Σ
  // of the four shares) / K²
  auto gs_step1 = [&]() {
    if (P != 0 || (X2_ABL & 512)) return;
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    gs_offdiag();
    // 1 / n_k = rsq(G_kk) (rsq(inf) = 0 and rsq(0) = inf keep a non-finite or zero mui NaN in D,
    // as the reference's cosines); lane (g, j) needs rows m = 4g..4g+3 of its tile, column j of its
    // tile (diagonal) and of the other (off-diagonal)
    const float* gdg = reinterpret_cast<const float*>(smem + Cv::kOffGram);
    const f32x4 dm0 = *reinterpret_cast<const f32x4*>(gdg + kt * 16 + 4 * g);
    const f32x4 dm1 = *reinterpret_cast<const f32x4*>(gdg + 32 + kt * 16 + 4 * g);
    const float rj = __builtin_amdgcn_rsqf(gdg[kt * 16 + j] + gdg[32 + kt * 16 + j]);
    const float rj1 = __builtin_amdgcn_rsqf(gdg[(1 - kt) * 16 + j] + gdg[32 + (1 - kt) * 16 + j]);
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float rm = __builtin_amdgcn_rsqf(dm0[e] + dm1[e]);
      if (4 * g + e != j) sum = __builtin_fmaf(gr[0][e] * rm, rj, sum);
      sum = __builtin_fmaf(2.0f * gr[1][e] * rm, rj1, sum);
    }
    // over the 16 lanes of a row (DPP row rotations), then the 4 rows (permlane swaps)
    sum += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sum), 0x128, 0xf, 0xf, false));
    sum += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sum), 0x124, 0xf, 0xf, false));
    sum += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sum), 0x122, 0xf, 0xf, false));
    sum += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sum), 0x121, 0xf, 0xf, false));
    sum = x_rows4_sum(sum);
    if (lane == 0) reinterpret_cast<float*>(smem + Cv::kOffGram + 256)[wave] = sum;
    gr[0] = gr[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto gs_step2 = [&]() {
    if (wave == 0 && (threadIdx.x & 63) == 0) {
      const float* sh = reinterpret_cast<const float*>(smem + Cv::kOffGram + 256);
      dis_out[gs_b] = ((sh[0] + sh[1]) + (sh[2] + sh[3])) / (float)(KK * KK);
    }
  };

  // S7 (model.py:128-136, :213-214) on the X waves 4-7: wave w candidates [16 (w - 4), +16) of the
  // finished pass, lane (kq, c) interests [8 kq, 8 kq + 8); the two column-half partials summed
  // here (ch 0 + ch 1), the 4 lane rows combined by permlanes
  auto s7 = [&]() {
    if (wave < 4) return;
    const int lane = threadIdx.x & 63;
    const int cl = lane & 15, kq = lane >> 4;
    const int c = 16 * (wave & 3) + cl;
    const float* F = reinterpret_cast<const float*>(smem + Cv::kOffF);
    const float uc_pend = uc_pend_r;
    const int sw = (c >> 1) & 31;
    float lg[8], m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = c * 32 + ((8 * kq + j) ^ sw);
      m[j] = (F[o] + F[Cv::kFBlk + o]) * uc_pend;                   // the candidate row's unit
      if constexpr (WEIGHTED) lg[j] = (F[2 * Cv::kFBlk + o] + F[3 * Cv::kFBlk + o]) * uc_pend;
    }
    float sc;
    if constexpr (WEIGHTED) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) mx = fmaxf(mx, lg[j]);
      mx = x_rows4_max(mx);
      float sm = 0.f, num = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (8 * kq + j < KK) {
          const float pe = x2_exp(lg[j] - mx);
          sm += pe;
          num = __builtin_fmaf(pe, m[j], num);
        }
      }
      sm = x_rows4_sum(sm);
      num = x_rows4_sum(num);
      sc = num * __builtin_amdgcn_rcpf(sm);   // sm >= 1 (the max term): one rounding more than num / sm
    } else {
      if (p.score_type == MINER_SCORE_MAX) {
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) mx = fmaxf(mx, m[j]);
        sc = x_rows4_max(mx);
      } else {
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) sm += m[j];
        sc = x_rows4_sum(sm) / (float)KK;
      }
    }
    if (kq == 0 && c < pend_cnt) p.scores[pend_off + c] = sc;
  };

  // the products of one chunk in slot t & 1 (after the next chunk's row DMAs, issued first so that
  // they land before the next barrier); mode: 1 history product, 2 candidate product, 4 mui out,
  // 8 Gram; NT candidate tiles compile-time (0: no candidate product)
  // the next chunk's row DMAs, issued by every wave right after the barrier. (Round 6 A/B,
  // tools/x2_ab.py, 1M impressions: the mui waves — which set the chunk length — issuing theirs
  // after their history product instead +3.1 %; the mui waves at priority 2 while they issue
  // +2.2 %; profiles/r06_x2_dma_ab.txt)
  int dn_cc = 0, dn_ni = 0, dn_np = 0;
  auto issue_dmas = [&]() {
    if (dn_cc + 1 < nchunk) {
      dma_chunk(cH, cC, cLv, dn_cc + 1, (t + 1) & 1);
    } else {
      item_offsets(dn_ni, dn_np, nH, nC, nLv);
      dma_chunk(nH, nC, nLv, 0, (t + 1) & 1);
    }
  };
  auto compute_t = [&](int ci, int cc, int mode, auto nt_c) {
    constexpr int NT = decltype(nt_c)::value;
    FRESH_LANE_IDS();
    const int g = lane >> 4, i = lane & 15;
    const char* slot = smem + (t & 1) * Cv::kSlot;
    const char* part = slot + P * Cv::kPart;
    f32x4 hx[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    [[maybe_unused]] f32x4 hy[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (kb == 1 && nkb < 2) break;    // <= 32 unique history rows: one 32-row block
      u32x4 eH[2], eL[2];
#pragma unroll
      for (int ctl = 0; ctl < 2; ++ctl) {
        const uint2 h0 = lds_tr(part + trH[ctl][0] + 8192 * kb);
        const uint2 h1 = lds_tr(part + ((GS && kb) ? trH3[ctl] : trH[ctl][1] + 8192 * kb));
        const uint2 l0 = lds_tr(part + trL[ctl][0] + 8192 * kb);
        const uint2 l1 = lds_tr(part + ((GS && kb) ? trL3[ctl] : trL[ctl][1] + 8192 * kb));
        eH[ctl] = u32x4{h0.x, h0.y, h1.x, h1.y};
        eL[ctl] = u32x4{l0.x, l0.y, l1.x, l1.y};
      }
#pragma unroll
      for (int ctl = 0; ctl < 2; ++ctl)
        hx[ctl] = (X2_ABL & 32) ? f32x4{__uint_as_float(eH[ctl][0] ^ aH[kb][0]), __uint_as_float(eL[ctl][1] ^ aL[kb][1]), 0.f, 0.f}
                                : mfma_x2(hx[ctl], eH[ctl], eL[ctl], aH[kb], aL[kb]);
      if (LOSS && !GS && (mode & 8)) {
#pragma unroll
        for (int ctl = 0; ctl < 2; ++ctl) hy[ctl] = mfma_x2(hy[ctl], eH[ctl], eL[ctl], aH1[kb], aL1[kb]);
      }
    }
    X2_STAMP(4);
    if (LOSS && !GS && (mode & 8)) {
      // Gram tiles over this wave's 32 columns: the operands of the candidate product's B side
      // (lane (g, i): columns 4g..4g+3 of both column tiles, interest i) serve as A (rows = k) and B
      float y0[8], y1[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y0[e] = hx[0][e] * (1.0f / kSA);       // the Gram waves are mui waves: |κ_k·mui_k| < 2^28
        y0[4 + e] = hx[1][e] * (1.0f / kSA);
        y1[e] = hy[0][e] * (1.0f / kSA);
        y1[4 + e] = hy[1][e] * (1.0f / kSA);
      }
      u32x4 g0H, g0L, g1H, g1L;
      split8h(y0, g0H, g0L);
      split8h(y1, g1H, g1L);
      gr[0] = mfma_x2(gr[0], g0H, g0L, g0H, g0L);
      gr[1] = mfma_x2(gr[1], g0H, g0L, g1H, g1L);
      gr[2] = mfma_x2(gr[2], g1H, g1L, g1H, g1L);
    }
    if ((mode & 4) && 16 * kt + i < KK) {
      const float mui_scale = __builtin_amdgcn_rcpf(kap);   // exact: κ is a power of two
      float* dst = mui_out + ((size_t)imp_b(ci) * KK + 16 * kt + i) * d + kCW * cc + 32 * ch + 4 * g;
#pragma unroll
      for (int ctl = 0; ctl < 2; ++ctl)
        *reinterpret_cast<float4*>(dst + 16 * ctl) =
            make_float4(hx[ctl][0] * mui_scale, hx[ctl][1] * mui_scale, hx[ctl][2] * mui_scale, hx[ctl][3] * mui_scale);
    }
    if constexpr (NT > 0) {
      // candidate operands: each tile's rows from its own base register (opaque to hipcc), so the
      // reads of tiles q and q + 1 are not paired into a ds_read2st64_b64, whose 16-lane groups bank
      // by dword mod 32 — a 2-way conflict on these 16-row reads (MI355X_MICROARCH.md §LDS) —
      // while ds_read_b64 banks mod 64 over 32 lanes: none
      const char* cpart = slot + 2 * Cv::kPart;
      uint2 cH_[NT][2], cL_[NT][2];
#pragma unroll
      for (int q = 0; q < NT; ++q) {
#pragma unroll
        for (int ctl = 0; ctl < 2; ++ctl) {
          cH_[q][ctl] = lds_u64(cpart + cfH[ctl] + kCTile * q);
          cL_[q][ctl] = lds_u64(cpart + cfL[ctl] + kCTile * q);
        }
      }
      float x[8];
      // mui path: κ·mui·2^-14 (< 2^14); X path: the GELU's input (A·proj)_k = acc / κ, then
      // gelu·κ·2^-14 (|gelu(y)| <= |y|)
      const float op_scale = P == 0 ? 1.0f / kSA : __builtin_amdgcn_rcpf(kap);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = hx[0][e] * op_scale;
        x[4 + e] = hx[1][e] * op_scale;
      }
      if (WEIGHTED && P == 1) {
        if (!(X2_ABL & 8)) gelu_as_pairs(x, 8);
        const float sPj = kap * (1.0f / kSA);
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] *= sPj;
      }
      u32x4 bH, bL;
      split8h(x, bH, bL);
      if (GS && (mode & 8)) gs_chunk(cc, bH, bL);
      X2_STAMP(5);
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const u32x4 ah = u32x4{cH_[q][0].x, cH_[q][0].y, cH_[q][1].x, cH_[q][1].y};
        const u32x4 al = u32x4{cL_[q][0].x, cL_[q][0].y, cL_[q][1].x, cL_[q][1].y};
        if (X2_ABL & 16) acc[q][0] += __uint_as_float(ah[0] ^ al[1] ^ bH[q] ^ bL[q]);
        else acc[q] = mfma_x2(acc[q], ah, al, bH, bL);
      }
      X2_STAMP(6);
    }
  };
  auto compute = [&](int ci, int cc, int mode, int ntile) {
    using std::integral_constant;
    if (!(mode & 1) || (X2_ABL & 4)) return;
    if (!(mode & 2)) compute_t(ci, cc, mode, integral_constant<int, 0>{});
    else if (ntile >= 4) compute_t(ci, cc, mode, integral_constant<int, 4>{});
    else if (ntile == 3) compute_t(ci, cc, mode, integral_constant<int, 3>{});
    else if (ntile == 2) compute_t(ci, cc, mode, integral_constant<int, 2>{});
    else compute_t(ci, cc, mode, integral_constant<int, 1>{});
  };

  // static priority for the X waves 4-7 (the GELU chain)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  for (int ci = 0; ci < n_i; ++ci) {
    int c_off, c_cnt;
    cands(ci, c_off, c_cnt);
    const int cn = max(1, (c_cnt + 63) >> 6);
    nkb = __builtin_amdgcn_readfirstlane(dup_u(smem, ci & 3)[0]) > 32 ? 2 : 1;
    for (int cp = 0; cp < cn; ++cp) {
      const int cntp = min(64, c_cnt - 64 * cp);
      const int ntile = (max(cntp, 1) + 15) >> 4;
      const bool need_mui = P == 0 && mui_out != nullptr && cp == 0;
      const bool need_c = WITH_CAND && path_live;
      const bool need_g = gram_w && dis_out != nullptr && cp == 0;
      const int mode = (k_live && path_live && (need_c || need_mui || need_g))
                           ? (1 | (need_c ? 2 : 0) | (need_mui ? 4 : 0) | (need_g ? 8 : 0)) : 0;
      const int ni = cp + 1 < cn ? ci : ci + 1, np = cp + 1 < cn ? cp + 1 : 0;
      bool did_s7 = false;
      for (int cc = 0; cc < nchunk; ++cc, ++t) {
        X2_STAMP(7);
        // this chunk's rows (and every older DMA) landed for this wave, then for every wave; the
        // slot of the last chunk is free
        vm_wait_all();
        X2_STAMP(0);
        raw_barrier();
        X2_STAMP(1);
        // the unit merge waits (compiler vmcnt) for the loads of the previous dedupe: here, before
        // this chunk's DMAs are issued, they have landed and the wait is free
        if ((!LOSS || SHP == 2) && cp == 0 && cc == 0) dedupe_merge();
        if (GS && gram_w && (need_g || gs_step == 1)) gs_read();
        // the next chunk's row DMAs right after the barrier, before a pass start's S7 / softmax / aux
        // work (round 4: -0.9 %)
        dn_cc = cc; dn_ni = ni; dn_np = np;
        issue_dmas();
        X2_STAMP(3);
        if (cc == 0) {
          did_s7 = (WITH_CAND && pend_off >= 0) || d_pending;
          if (WITH_CAND && pend_off >= 0) s7();
          pend_off = -1;
          if (LOSS && pend_d >= 0) form_d(pend_d);
          pend_d = -1;
          d_pending = false;
          if (cp == 0) {
            using std::integral_constant;
            // <= 32 history groups: the softmax over the first 32 only (the second block's A unused)
            if ((X2_ABL & 1024) && P == 0 && ci > 0) {                 // timing only: the mui waves keep the last A
            } else if ((X2_ABL & 2048) && P == 1 && ci > 0) {          // timing only: the X waves keep the last A
            } else if (nkb == 1) softmax_inwave(ci, kt, P, aH, aL, kap, integral_constant<int, 8>{});
            else softmax_inwave(ci, kt, P, aH, aL, kap, integral_constant<int, 16>{});
            if (LOSS && !GS && gram_w && dis_out) {
              float kap1;                // interest tile 1 of the Gram: the Gram's cosines are per-k scale free
              if (nkb == 1) softmax_inwave(ci, 1, 0, aH1, aL1, kap1, integral_constant<int, 8>{});
              else softmax_inwave(ci, 1, 0, aH1, aL1, kap1, integral_constant<int, 16>{});
            }
            dedupe_prep(ci + 2);       // L1 of ci + 2 landed; its logit rows are DMA'd by group next
            if (nchunk == 1) {
              raw_barrier();           // every wave has read impression ci's logit rows and coefficients
              issue_L2(ci + 2);
            }
            issue_L0(ci + 4);
            issue_L1(ci + 3);
          }
          if (GS && gs_step == 1) {
            gs_step1();
            gs_step = 2;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
        } else if (cc == 1 && cp == 0) {
          issue_L2(ci + 2);            // into the block impression ci's logits were read from
        }
        if (GS && cc == 1 && gs_step == 2) {
          gs_step2();
          gs_step = 0;
        }
        X2_STAMP(2);
        compute(ci, cc, mode, ntile);
      }
      if (WITH_CAND && wave >= 4) {
        // this pass's S7 (after the next barrier) needs its candidates' row units: one per lane
        const int c = 16 * (wave & 3) + (int)(threadIdx.x & 15);
        const int id = l1_cand(smem, ci & 3)[min(64 * cp + min(c, max(cntp, 1) - 1), kMaxCand - 1)];
        uc_pend_r = p.unit_t[min(max(id, 0), p.n_news - 1)];
      }
      if (nchunk == 1 && did_s7) raw_barrier();
      if (GS && dis_out && cp == 0) {
        // the four diagonal partials -> LDS [ch][kt][16] (read by step 1 after the next barrier)
        if (gram_w) {
          const int lane = threadIdx.x & 63;
          const int j = lane & 15, g = lane >> 4;
          float* gdg = reinterpret_cast<float*>(smem + Cv::kOffGram) + (2 * ch + kt) * 16;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * g + e == j) gdg[j] = gr[0][e];
        }
        gs_step = 1;
        gs_b = imp_b(ci);
      } else if (LOSS && dis_out && cp == 0) {
        // the Gram hand-off: wave 2 (columns 32..63 of each chunk) -> LDS -> wave 0 at the next chunk
        if (gram_w && ch == 1) {
          const int lane = threadIdx.x & 63;
          float* pg = reinterpret_cast<float*>(smem + Cv::kOffGram);
#pragma unroll
          for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) pg[(q * 4 + e) * 64 + lane] = gr[q][e];
#pragma unroll
          for (int q = 0; q < 3; ++q) gr[q] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if (gram_w && ch == 0) pend_d = imp_b(ci);
        d_pending = true;
      }
      if constexpr (WITH_CAND) {
        // pass done: every wave publishes its partial M / Lg [c][k ^ swizzle] into its own block
        // F[P][ch] without a barrier; S7, after the next chunk's barrier, reads them. The next
        // publish is at least one barrier after that S7 (one extra barrier when a pass is one chunk).
        const int lane = threadIdx.x & 63;
        const int j = lane & 15, g = lane >> 4;
        if (path_live && k_live) {
          // in true units over the candidate row's unit: M = M_s·unit_c·2^14/κ_k (Lg likewise)
          const float pub_scale = kSA * __builtin_amdgcn_rcpf(kap);
          float* F = reinterpret_cast<float*>(smem + Cv::kOffF) + (P * 2 + ch) * Cv::kFBlk;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (q < ntile) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int c = 16 * q + 4 * g + e;
                F[c * 32 + ((16 * kt + j) ^ ((c >> 1) & 31))] = acc[q][e] * pub_scale;
              }
            }
          }
        }
      }
      pend_off = c_off + 64 * cp;
      pend_cnt = cntp;
#pragma unroll
      for (int jj = 0; jj < kNB; ++jj) {
        cH[jj] = nH[jj];
        cC[jj] = nC[jj];
      }
      cLv = nLv;
    }
  }
  X2_STAMP_FLUSH(n_i);
  vm_wait_all();
  raw_barrier();
  if (WITH_CAND && pend_off >= 0) s7();
  if (LOSS && pend_d >= 0) form_d(pend_d);
  if (GS && gs_step == 1) {
    if (gram_w) gs_read();
    gs_step1();
    raw_barrier();
    gs_step2();
  }
}

// ================================================================================================
// wide shapes: K <= 64 interests, L <= 128 history slots (news_score_x2w)
// ================================================================================================
// The reference limits neither num_context_codes (model.py:18-21) nor the history length
// (model.py:159-185); news_score_x2's LDS carve stops at K <= 32, L <= 64. news_score_x2w is the
// same math on the same pair planes and per-news precompute, laid out for K <= 64 and up to 128
// history groups:
//   - 32-column steps: one 128-byte piece per row (32 hi | 32 lo fp16 of the 64-column chunk),
//     two LDS slots [E[his] 128 rows | proj[his] 128 rows | Cand 64 rows], LDS-DMA by id one step
//     ahead, one barrier per step; rows past the groups / the candidate count are not fetched;
//   - wave w = (path P = w >> 2, interest tile kq = w & 3): muiᵀ / Xᵀ [32 cols x 16 interests] =
//     part[his]ᵀ·Aᵀ over up to 4 history blocks of 32 (the history operand read transposed, Aᵀ pairs
//     in registers), then M / Lg [16 cands x 16 interests] += Cand·muiᵀ / Xᵀ per candidate tile;
//   - per impression, at its first step: the softmax over the history groups (each wave, its 16
//     interests), S7 of the previous pass (X waves, 16 candidates x 16 interests per lane row) and
//     the dedupe of the next impression (wave 7); the logit rows of the next impression land in
//     the single logit block at the second step.
// The masked slots holding the first masked slot's news id form one group (as news_score_x2).
constexpr int kWRB = 128;                              // bytes per staged row piece (32 hi | 32 lo)
constexpr int kWCTile = 16 * kWRB + 16;                // candidate tiles 16 B apart (see kCTile)
// The carve of the wide form (K <= 64, L <= 128, one workgroup of 8 waves per CU)
struct XW {
  static constexpr int kThr = 512;
  static constexpr int kMaxL = MINER_NEWS_X2W_MAX_L;
  static constexpr int kMaxK = MINER_NEWS_X2W_MAX_K;
  static constexpr int kMaxC = kMaxCand;
  static constexpr int kNKb = kMaxL / 32;                // history blocks of 32 groups
  static constexpr int kHalves = kMaxL / 64;             // 64-slot ballots of the dedupe
  static constexpr int kPart = kMaxL * kWRB;
  static constexpr int kSlot = 2 * kPart + 4 * kWCTile;
  static constexpr int kRing = 2 * kSlot;
  static constexpr int kOffF = kRing;                    // F[P] [c 64][k ^ (c & 15)] fp32
  static constexpr int kFP = 64 * kMaxK;                 // floats per path
  static constexpr int kOffLog = kOffF + 2 * kFP * 4;    // logit rows of one impression [group][kMaxK]
  static constexpr int kLogB = kMaxL * kMaxK * 4;
  static constexpr int kOffL1 = kOffLog + kLogB;         // 3 slots: his ids | mask words | bias | cand ids
  static constexpr int kL1B = 3 * 4 * kMaxL + 4 * kMaxC;
  static constexpr int kOffL0 = kOffL1 + 3 * kL1B;       // 8 slots: CSR offsets (ragged)
  static constexpr int kOffPrep = kOffL0 + 8 * kL0B;     // 2 blocks: code[kMaxL] | add[kMaxL]
  static constexpr int kPrepB = 2 * kMaxL * 4;
  static constexpr int kOffDup = kOffPrep + 2 * kPrepB;  // per L1 slot: U
  static constexpr int kLds = kOffDup + 3 * kDupB;
};
static_assert(XW::kMaxL == 128 && XW::kMaxK == 64, "the wide carve is laid out for L <= 128, K <= 64");
static_assert(XW::kLds <= 160 * 1024, "news_score_x2w LDS");

// 16-byte chunk swizzle of a staged 128-byte row (8 chunks: hi 0..3, lo 4..7): slot = chunk ^
// wswz(row). Over the 4 same-parity rows of a transposed read's 8-row group it takes the even
// values {0, 2, 4, 6} (rows 8..15 of a 16: the odd ones), so the chunk pairs of the two lanes'
// column halves land in 8 different slots; over the 8 same-parity rows of a 16-row candidate tile
// all 8 values: both reads are conflict-free (ds_read_b64 / _tr_b16 bank over 256 B per 32 lanes)
__host__ __device__ inline int wswz(int row) { return (((row >> 1) & 3) << 1) | ((row >> 3) & 1); }

template <int ST, bool RAGGED>
__global__ __launch_bounds__(512, 2) void news_score_x2w(X2Params p) {
  using Cw = XW;
  constexpr int NW = 8;                                   // waves
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool WEIGHTED = ST == MINER_SCORE_WEIGHTED;
  constexpr bool WITH_CAND = ST != MINER_SCORE_NONE;
  const int G = gridDim.x;
  const int n_i = (p.B - (int)blockIdx.x + G - 1) / G;
  const int L = p.L, KK = p.K, d = p.d;
  const int nst = d >> 5;                                 // 32-column steps
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P = wave / (NW / 2), kq = wave % (NW / 2);   // path, interest tile
  const bool k_live = 16 * kq < KK;
  const bool path_live = P == 0 || WEIGHTED;
  const char* tabB = static_cast<const char*>(p.table2);
  const char* prjB = WEIGHTED ? static_cast<const char*>(p.proj2) : tabB;
  const unsigned sbase = __builtin_amdgcn_readfirstlane(lds_offset(smem));
  float kap = kSA;                         // κ_k of this lane's interest (the wave's path), per impression
  float uc_pend[8 / NW] = {};              // S7 lane's candidate units (X waves), one per round

  auto imp_b = [&](int i) { return (int)blockIdx.x + i * G; };
  auto l1 = [&](int i) { return smem + Cw::kOffL1 + (i % 3) * Cw::kL1B; };
  auto w_his = [&](int i) { return reinterpret_cast<int*>(l1(i)); };
  auto w_mask = [&](int i) { return reinterpret_cast<uint32_t*>(l1(i) + 4 * Cw::kMaxL); };
  auto w_bias = [&](int i) { return reinterpret_cast<float*>(l1(i) + 8 * Cw::kMaxL); };
  auto w_cand = [&](int i) { return reinterpret_cast<int*>(l1(i) + 12 * Cw::kMaxL); };
  auto w_dup = [&](int i) { return reinterpret_cast<int*>(smem + Cw::kOffDup + (i % 3) * kDupB); };
  auto w_prep = [&](int i) { return reinterpret_cast<float*>(smem + Cw::kOffPrep + (i & 1) * Cw::kPrepB); };
  auto cands = [&](int i, int& off, int& cnt) {
    if constexpr (!WITH_CAND) { off = 0; cnt = 0; return; }
    if constexpr (RAGGED) {
      const int* o = reinterpret_cast<const int*>(smem + Cw::kOffL0 + (i & 7) * kL0B);
      off = __builtin_amdgcn_readfirstlane(o[0]);
      cnt = __builtin_amdgcn_readfirstlane(o[1]) - off;
    } else {
      off = imp_b(i) * p.C;
      cnt = p.C;
    }
    cnt = min(max(cnt, 0), Cw::kMaxC);
  };
  // ---- aux DMAs: L0 CSR offsets -> L1 ids / mask / bias / candidate ids -> L2 logit rows by group ----
  auto issue_L0 = [&](int i) {
    if (RAGGED && wave == 0 && i < n_i && (threadIdx.x & 63) < 2)
      dma_b32(p.cand_off + imp_b(i) + (threadIdx.x & 63), sbase + Cw::kOffL0 + (i & 7) * kL0B);
  };
  auto issue_L1 = [&](int i) {
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const unsigned dst = sbase + (unsigned)(l1(i) - smem);
    for (int hh = 0; hh < 2 && 64 * hh < L; ++hh) {
      const size_t base = (size_t)imp_b(i) * L + min(lane + 64 * hh, L - 1);
      if (wave == 1) {
        dma_b32(p.his_ids + base, dst + 256 * hh);
      } else if (wave == 2) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p.mask + base) & ~(uintptr_t)3;
        dma_b32(reinterpret_cast<const void*>(a), dst + 4 * Cw::kMaxL + 256 * hh);
      } else if (wave == 3) {
        if (p.bias) dma_b32(p.bias + base, dst + 8 * Cw::kMaxL + 256 * hh);
      }
    }
    if (WITH_CAND && wave >= 4) {                       // candidate ids, 64 per DMA
      int off, cnt;
      cands(i, off, cnt);
      for (int j = wave - 4; 64 * j < cnt; j += 4) {
        const int c = min(64 * j + lane, cnt - 1);
        dma_b32(p.cand_ids + off + c, dst + 12 * Cw::kMaxL + 256 * j);
      }
    }
  };
  auto issue_L2 = [&](int i) {             // 16-byte pieces of the groups' logit rows, 4 rows per DMA
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const int U = __builtin_amdgcn_readfirstlane(w_dup(i)[0]);
    const int* his = w_his(i);
    constexpr int PPR = Cw::kMaxK / 4;                  // 16-byte pieces per logit row
    constexpr int RPD = 64 / PPR;                         // rows per DMA
#pragma unroll
    for (int j = 0; j < Cw::kMaxL / RPD / NW; ++j) {
      const int n = wave + NW * j;                        // DMA n: rows RPD n .. RPD n + RPD - 1
      if (RPD * n >= U) break;
      const int row = min(RPD * n + lane / PPR, U - 1);
      const int pc = min(lane % PPR, (KK >> 2) - 1);
      const int id = min(max(his[row], 0), p.n_news - 1);
      x2_dma_b128(p.logits + (size_t)id * KK + 4 * pc, sbase + Cw::kOffLog + n * 1024);
    }
  };
  // the groups of impression i (wave 7; two 64-slot halves): its history ids are replaced by the
  // groups' ids, each group's code (multiplicity, click bit, row-unit exponents) and additive term
  // written; the units land a step later (dedupe_merge, right after a barrier)
  float du_E[2] = {1.f, 1.f}, du_P[2] = {1.f, 1.f};
  int du_slot[2] = {-1, -1}, du_i = -1;
  auto dedupe_merge = [&]() {
    if (wave != NW - 1 || du_i < 0) return;
    int* pcp = reinterpret_cast<int*>(w_prep(du_i));
#pragma unroll
    for (int hh = 0; hh < Cw::kHalves; ++hh)
      if (du_slot[hh] >= 0)
        pcp[du_slot[hh]] |= (((__float_as_int(du_E[hh]) >> 23) & 255) << 8) | (((__float_as_int(du_P[hh]) >> 23) & 255) << 16);
    du_i = -1;
  };
  auto dedupe_prep = [&](int i) {
    if (wave != NW - 1 || i >= n_i) return;
    const int l = threadIdx.x & 63;
    int* his = w_his(i);
    int id[2];
    bool keep[2], valid[2];
    float bv[2];
    unsigned long long pads[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int s = l + 64 * hh;
      const int ls = min(s, L - 1);
      valid[hh] = s < L;
      id[hh] = his[ls];
      const uint32_t mw = w_mask(i)[ls];
      const int a = (int)(reinterpret_cast<uintptr_t>(p.mask + (size_t)imp_b(i) * L + ls) & 3);
      keep[hh] = ((mw >> (8 * a)) & 0xffu) != 0u;
      bv[hh] = (keep[hh] && p.bias) ? w_bias(i)[ls] : 0.f;
      pads[hh] = __ballot(valid[hh] && !keep[hh]);
    }
    const int f = pads[0] ? (int)__builtin_ctzll(pads[0]) : pads[1] ? 64 + (int)__builtin_ctzll(pads[1]) : 0;
    const int idf = f >= 64 ? __builtin_amdgcn_readlane(id[1], f - 64) : __builtin_amdgcn_readlane(id[0], f);
    unsigned long long grp[2], bal[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) grp[hh] = pads[hh] & __ballot(id[hh] == idf);
    const int mg = __popcll(grp[0]) + __popcll(grp[1]);
    bool uniq[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const bool ing = ((grp[hh] >> l) & 1ull) != 0ull;
      uniq[hh] = valid[hh] && (!ing || l + 64 * hh == f);
      bal[hh] = __ballot(uniq[hh]);
    }
    const int U0 = __popcll(bal[0]);
    const int U = U0 + __popcll(bal[1]);
    float* pr = w_prep(i);
    int* pc = reinterpret_cast<int*>(pr);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int uidx = (hh ? U0 : 0) + __popcll(bal[hh] & ((1ull << l) - 1ull));
      const bool ing = ((grp[hh] >> l) & 1ull) != 0ull;
      const int idc = min(max(id[hh], 0), p.n_news - 1);
      du_E[hh] = p.unit_t[idc];
      du_P[hh] = WEIGHTED ? p.unit_p[idc] : 1.0f;
      if (uniq[hh]) {
        his[uidx] = id[hh];
        pc[uidx] = (ing ? mg : 1) | (keep[hh] ? 1 << 24 : 0);
        pr[Cw::kMaxL + uidx] = keep[hh] ? bv[hh] : 1e-30f;
      }
      du_slot[hh] = uniq[hh] ? uidx : -1;
      if (hh < Cw::kHalves && l + 64 * hh >= U) {   // past the groups: weight 0, units 2^-14
        pc[l + 64 * hh] = (113 << 8) | (113 << 16);
        pr[Cw::kMaxL + l + 64 * hh] = -INFINITY;
      }
    }
    if (l == 0) w_dup(i)[0] = U;
    du_i = i;
  };

  // ---- row DMAs of a step: wave w fills history rows 64 jj + 8w .. + 7 of E and proj (jj = 0, 1)
  // and candidate rows 8w .. 8w + 7; lane l: row 8 blk + (l >> 3), chunk slot l & 7 from source
  // chunk slot ^ wswz(row) (hi chunks 0..3 at +16 c, lo chunks at +128 + 16 (c - 4) of the
  // 64-column chunk, the step's half at +64)
  auto chunk_off = [](int row, int sl) {
    const int c = sl ^ wswz(row);
    return (uint32_t)((c & 4) * 32 + 16 * (c & 3));
  };
  constexpr int kCB = 8 / NW;                         // candidate DMA blocks (8 rows) per wave
  auto item_offsets = [&](int i, int pass, uint32_t* oH, uint32_t* oC, unsigned& lv) {
    const int lane = threadIdx.x & 63;
    const bool live = i < n_i;
    int off = 0, cnt = 1;
    if (live) cands(i, off, cnt);
    const int cntp = max(1, min(64, cnt - 64 * pass));
    const int U = live ? __builtin_amdgcn_readfirstlane(w_dup(i)[0]) : 1;
    const uint32_t rowBytes = (uint32_t)d * 4u;
    lv = 0;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row0 = 8 * NW * jj + 8 * wave;
      if (live && row0 < U) lv |= 1u << jj;
      const int row = row0 + (lane >> 3);
      int h = live ? w_his(i)[min(row, U - 1)] : 0;
      h = min(max(h, 0), p.n_news - 1);
      oH[jj] = (uint32_t)h * rowBytes + chunk_off(row, lane & 7);
    }
#pragma unroll
    for (int cj = 0; cj < kCB; ++cj) {
      const int row0 = 8 * NW * cj + 8 * wave;
      const int row = row0 + (lane >> 3);
      if (live && WITH_CAND && row0 < cnt - 64 * pass) lv |= 16u << cj;
      int c = (live && WITH_CAND) ? w_cand(i)[min(64 * pass + min(row, cntp - 1), Cw::kMaxC - 1)] : 0;
      c = min(max(c, 0), p.n_news - 1);
      oC[cj] = (uint32_t)c * rowBytes + chunk_off(row, lane & 7);
    }
    lv = __builtin_amdgcn_readfirstlane(lv);
  };
  auto dma_step = [&](const uint32_t* oH, const uint32_t* oC, unsigned lv, int sg, int slot) {
    if (lv == 0) return;
    const int so = (sg >> 1) * 256 + (sg & 1) * 64;
    const unsigned m = sbase + slot * Cw::kSlot;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      if (lv & (1u << jj)) {
        x2_dma_row(oH[jj], tabB + so, m + jj * 1024 * NW + wave * 1024);
        if (WEIGHTED) x2_dma_row(oH[jj], prjB + so, m + Cw::kPart + jj * 1024 * NW + wave * 1024);
      }
    }
#pragma unroll
    for (int cj = 0; cj < kCB; ++cj) {
      const int row0 = 8 * NW * cj + 8 * wave;
      if (lv & (16u << cj)) x2_dma_row(oC[cj], tabB + so, m + 2 * Cw::kPart + (row0 >> 4) * kWCTile + (row0 & 15) * kWRB);
    }
  };

  // ---- per-lane LDS read offsets (fixed for the launch): as news_score_x2, 128-byte rows ----
  uint32_t trH[2][2], trL[2][2], cfH[2], cfL[2];
  {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, i = lane & 15;
#pragma unroll
    for (int ctl = 0; ctl < 2; ++ctl) {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int row = 16 * rr + 4 * g + q;
        const int chunk = 2 * ctl + (pp >> 1);
        trH[ctl][rr] = row * kWRB + ((chunk ^ wswz(row)) << 4) + 8 * (pp & 1);
        trL[ctl][rr] = row * kWRB + (((chunk + 4) ^ wswz(row)) << 4) + 8 * (pp & 1);
      }
      const int chunk = 2 * ctl + (g >> 1);
      cfH[ctl] = i * kWRB + ((chunk ^ wswz(i)) << 4) + 8 * (g & 1);
      cfL[ctl] = i * kWRB + (((chunk + 4) ^ wswz(i)) << 4) + 8 * (g & 1);
    }
  }

  // Aᵀ B operand of the history product, fp16 pairs: lane (g, i) holds A[16 kq + i][u] of the groups
  // u = 32 kb + 16 (e >> 2) + 4g + (e & 3)
  u32x4 aH[Cw::kNKb], aL[Cw::kNKb];
  int nkb = Cw::kNKb;
  // softmax over the groups (model.py:176-181) of this wave's 16 interests, in registers (as
  // news_score_x2's softmax_inwave, up to 32 groups per lane)
  auto softmax_w = [&](int i, auto nss_c) {
    constexpr int NSS = decltype(nss_c)::value;   // groups per lane: 16 (<= 64 groups) or 32
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const int k = 16 * kq + j;
    const float* lgb = reinterpret_cast<const float*>(smem + Cw::kOffLog);
    const float* pr = w_prep(i);
    const int* pc = reinterpret_cast<const int*>(pr);
    const unsigned sh = P ? 16u : 8u;
    float v[NSS], wm[NSS], un[NSS];
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < NSS; ++s) {
      const int u = 32 * (s >> 3) + 16 * ((s >> 2) & 1) + 4 * g + (s & 3);
      const unsigned code = (unsigned)pc[u];
      wm[s] = (float)(code & 255u);
      un[s] = __uint_as_float(__builtin_amdgcn_ubfe(code, sh, 8) << 23);
      const float click = __uint_as_float((code >> 24) * 0x3f800000u);
      v[s] = __builtin_fmaf(lgb[u * Cw::kMaxK + min(k, KK - 1)], click, pr[Cw::kMaxL + u]);
      mx = fmaxf(mx, v[s]);
    }
    mx = x_rows4_max(mx);
    float sum = 0.f, tu = 0.f;
#pragma unroll
    for (int s = 0; s < NSS; ++s) {
      v[s] = x2_exp(v[s] - mx);
      const float we = wm[s] * v[s];
      sum += we;
      tu = __builtin_fmaf(we, un[s], tu);
    }
    sum = x_rows4_sum(sum);
    tu = x_rows4_sum(tu);
    int e;
    frexpf(tu / sum, &e);
    e = min(max(e, -100), 114);
    kap = __int_as_float((141 - e) << 23);
    float inv = kap / sum;
    if (k >= KK) inv = 0.f;
#pragma unroll
    for (int m = 0; m < NSS / 2; ++m) {
      unsigned hv, lv2;
      split2w(wm[2 * m], v[2 * m], inv * un[2 * m], wm[2 * m + 1], v[2 * m + 1], inv * un[2 * m + 1], hv, lv2);
      aH[m >> 2][m & 3] = hv;
      aL[m >> 2][m & 3] = lv2;
    }
#pragma unroll
    for (int kb = NSS / 8; kb < Cw::kNKb; ++kb) {
      aH[kb] = u32x4{0u, 0u, 0u, 0u};
      aL[kb] = u32x4{0u, 0u, 0u, 0u};
    }
  };

  // S7 (model.py:128-136, :213-214) on the X waves: wave w candidates [16 (w - 4), +16) of the
  // finished pass, lane (kq4, c) interests [16 kq4, 16 kq4 + 16), the 4 lane rows by permlanes
  int pend_off = -1, pend_cnt = 0;
  auto s7 = [&]() {
    if (wave < NW / 2) return;
    const int lane = threadIdx.x & 63;
    const int cl = lane & 15, kq4 = lane >> 4;
    const float* F = reinterpret_cast<const float*>(smem + Cw::kOffF);
#pragma unroll
    for (int rnd = 0; rnd < 8 / NW; ++rnd) {
      const int c = 16 * ((wave - NW / 2) + (NW / 2) * rnd) + cl;
      float lg[16], m[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int o = c * Cw::kMaxK + (((16 * kq4 + j) ^ cl) & (Cw::kMaxK - 1));
        m[j] = F[o] * uc_pend[rnd];
        if constexpr (WEIGHTED) lg[j] = F[Cw::kFP + o] * uc_pend[rnd];
      }
      float sc;
      if constexpr (WEIGHTED) {
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 16; ++j) if (16 * kq4 + j < KK) mx = fmaxf(mx, lg[j]);
        mx = x_rows4_max(mx);
        float sm = 0.f, num = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (16 * kq4 + j < KK) {
            const float pe = x2_exp(lg[j] - mx);
            sm += pe;
            num = __builtin_fmaf(pe, m[j], num);
          }
        }
        sm = x_rows4_sum(sm);
        num = x_rows4_sum(num);
        sc = num * __builtin_amdgcn_rcpf(sm);
      } else {
        if (p.score_type == MINER_SCORE_MAX) {
          float mx = -INFINITY;
#pragma unroll
          for (int j = 0; j < 16; ++j) if (16 * kq4 + j < KK) mx = fmaxf(mx, m[j]);
          sc = x_rows4_max(mx);
        } else {
          float sm = 0.f;
#pragma unroll
          for (int j = 0; j < 16; ++j) if (16 * kq4 + j < KK) sm += m[j];
          sc = x_rows4_sum(sm) / (float)KK;
        }
      }
      if (kq4 == 0 && c < pend_cnt) p.scores[pend_off + c] = sc;
    }
  };

  f32x4 acc[4];
  int t = 0;
  // the products of one step in slot t & 1; NT candidate tiles compile-time (0: none)
  auto compute_t = [&](int ci, int sg, bool mui_o, auto nt_c) {
    constexpr int NT = decltype(nt_c)::value;
    FRESH_LANE_IDS();
    const int g = lane >> 4, i = lane & 15;
    const char* slot = smem + (t & 1) * Cw::kSlot;
    const char* part = slot + P * Cw::kPart;
    f32x4 hx[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kb = 0; kb < Cw::kNKb; ++kb) {
      if (kb >= nkb) break;
      u32x4 eH[2], eL[2];
#pragma unroll
      for (int ctl = 0; ctl < 2; ++ctl) {
        const uint2 h0 = lds_tr(part + trH[ctl][0] + 4096 * kb), h1 = lds_tr(part + trH[ctl][1] + 4096 * kb);
        const uint2 l0 = lds_tr(part + trL[ctl][0] + 4096 * kb), l1v = lds_tr(part + trL[ctl][1] + 4096 * kb);
        eH[ctl] = u32x4{h0.x, h0.y, h1.x, h1.y};
        eL[ctl] = u32x4{l0.x, l0.y, l1v.x, l1v.y};
      }
#pragma unroll
      for (int ctl = 0; ctl < 2; ++ctl) hx[ctl] = mfma_x2(hx[ctl], eH[ctl], eL[ctl], aH[kb], aL[kb]);
    }
    if (mui_o && 16 * kq + i < KK) {
      const float mui_scale = __builtin_amdgcn_rcpf(kap);
      float* dst = p.mui_out + ((size_t)imp_b(ci) * KK + 16 * kq + i) * d + 32 * sg + 4 * g;
#pragma unroll
      for (int ctl = 0; ctl < 2; ++ctl)
        *reinterpret_cast<float4*>(dst + 16 * ctl) =
            make_float4(hx[ctl][0] * mui_scale, hx[ctl][1] * mui_scale, hx[ctl][2] * mui_scale, hx[ctl][3] * mui_scale);
    }
    if constexpr (NT > 0) {
      const char* cpart = slot + 2 * Cw::kPart;
      uint2 cH_[NT][2], cL_[NT][2];
#pragma unroll
      for (int q = 0; q < NT; ++q) {
#pragma unroll
        for (int ctl = 0; ctl < 2; ++ctl) {
          cH_[q][ctl] = lds_u64(cpart + cfH[ctl] + kWCTile * q);
          cL_[q][ctl] = lds_u64(cpart + cfL[ctl] + kWCTile * q);
        }
      }
      float x[8];
      const float op_scale = P == 0 ? 1.0f / kSA : __builtin_amdgcn_rcpf(kap);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = hx[0][e] * op_scale;
        x[4 + e] = hx[1][e] * op_scale;
      }
      if (WEIGHTED && P == 1) {
        gelu_as_pairs(x, 8);
        const float sPj = kap * (1.0f / kSA);
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] *= sPj;
      }
      u32x4 bH, bL;
      split8h(x, bH, bL);
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const u32x4 ah = u32x4{cH_[q][0].x, cH_[q][0].y, cH_[q][1].x, cH_[q][1].y};
        const u32x4 al = u32x4{cL_[q][0].x, cL_[q][0].y, cL_[q][1].x, cL_[q][1].y};
        acc[q] = mfma_x2(acc[q], ah, al, bH, bL);
      }
    }
  };
  auto compute = [&](int ci, int sg, bool need_c, bool mui_o, int ntile) {
    using std::integral_constant;
    if (!need_c && !mui_o) return;
    if (!need_c) compute_t(ci, sg, mui_o, integral_constant<int, 0>{});
    else if (ntile >= 4) compute_t(ci, sg, mui_o, integral_constant<int, 4>{});
    else if (ntile == 3) compute_t(ci, sg, mui_o, integral_constant<int, 3>{});
    else if (ntile == 2) compute_t(ci, sg, mui_o, integral_constant<int, 2>{});
    else compute_t(ci, sg, mui_o, integral_constant<int, 1>{});
  };

  // ---- prologue ----
  for (int o = (int)threadIdx.x * 16; o < Cw::kRing; o += Cw::kThr * 16)      // rows no DMA writes read as 0
    *reinterpret_cast<u32x4*>(smem + o) = u32x4{0u, 0u, 0u, 0u};
  for (int o = (int)threadIdx.x * 16; o < Cw::kLogB; o += Cw::kThr * 16)      // stale logit rows stay finite
    *reinterpret_cast<u32x4*>(smem + Cw::kOffLog + o) = u32x4{0u, 0u, 0u, 0u};
  for (int i = 0; i < 3; ++i) issue_L0(i);
  vm_wait_all();
  raw_barrier();
  issue_L1(0); issue_L1(1);
  vm_wait_all();
  raw_barrier();
  dedupe_prep(0);
  raw_barrier();
  dedupe_merge();
  issue_L2(0);
  vm_wait_all();
  raw_barrier();
  uint32_t cH[2], cC[kCB], nH[2] = {0u, 0u}, nC[kCB] = {};
  unsigned cLv = 0, nLv = 0;
  item_offsets(0, 0, cH, cC, cLv);
  dma_step(cH, cC, cLv, 0, 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  for (int ci = 0; ci < n_i; ++ci) {
    int c_off, c_cnt;
    cands(ci, c_off, c_cnt);
    const int cn = max(1, (c_cnt + 63) >> 6);
    const int U = __builtin_amdgcn_readfirstlane(w_dup(ci)[0]);
    nkb = (U + 31) >> 5;
    for (int cp = 0; cp < cn; ++cp) {
      const int cntp = min(64, c_cnt - 64 * cp);
      const int ntile = (max(cntp, 1) + 15) >> 4;
      const bool mui_o = P == 0 && p.mui_out != nullptr && cp == 0 && k_live;
      const bool need_c = WITH_CAND && path_live && k_live;
      const int ni = cp + 1 < cn ? ci : ci + 1, np = cp + 1 < cn ? cp + 1 : 0;
      for (int sg = 0; sg < nst; ++sg, ++t) {
        vm_wait_all();
        raw_barrier();
        if (cp == 0 && sg == 1) dedupe_merge();      // before this step's DMAs: the unit loads have landed
        if (sg == 0) {                // the candidate units' load waited for here, not behind the DMAs
#pragma unroll
          for (int rnd = 0; rnd < 8 / NW; ++rnd) asm volatile("" : "+v"(uc_pend[rnd]));
        }
        if (sg + 1 < nst) {
          dma_step(cH, cC, cLv, sg + 1, (t + 1) & 1);
        } else {
          item_offsets(ni, np, nH, nC, nLv);
          dma_step(nH, nC, nLv, 0, (t + 1) & 1);
        }
        if (sg == 0) {
          if (WITH_CAND && pend_off >= 0) s7();
          pend_off = -1;
          if (cp == 0) {
            using std::integral_constant;
            if (nkb <= 2) softmax_w(ci, integral_constant<int, 16>{});
            else softmax_w(ci, integral_constant<int, 32>{});
            dedupe_prep(ci + 1);
            issue_L0(ci + 3);
            issue_L1(ci + 2);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
        } else if (sg == 1 && cp == 0) {
          issue_L2(ci + 1);                          // every wave has read impression ci's logit rows
        }
        compute(ci, sg, need_c, mui_o, ntile);
      }
      if (WITH_CAND && wave >= NW / 2) {
#pragma unroll
        for (int rnd = 0; rnd < 8 / NW; ++rnd) {
          const int c = 16 * ((wave - NW / 2) + (NW / 2) * rnd) + (int)(threadIdx.x & 15);
          const int id = w_cand(ci)[min(64 * cp + min(c, max(cntp, 1) - 1), Cw::kMaxC - 1)];
          uc_pend[rnd] = p.unit_t[min(max(id, 0), p.n_news - 1)];
        }
      }
      if constexpr (WITH_CAND) {
        // pass done: the partial M / Lg of every wave -> F[P][c][k ^ (c & 15)] (S7 after the next barrier)
        const int lane = threadIdx.x & 63;
        const int j = lane & 15, g = lane >> 4;
        if (path_live && k_live) {
          const float pub_scale = kSA * __builtin_amdgcn_rcpf(kap);
          float* F = reinterpret_cast<float*>(smem + Cw::kOffF) + P * Cw::kFP;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (q < ntile) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int c = 16 * q + 4 * g + e;
                F[c * Cw::kMaxK + (((16 * kq + j) ^ (c & 15)) & (Cw::kMaxK - 1))] = acc[q][e] * pub_scale;
              }
            }
          }
        }
      }
      pend_off = c_off + 64 * cp;
      pend_cnt = cntp;
      cH[0] = nH[0];
      cH[1] = nH[1];
#pragma unroll
      for (int cj = 0; cj < kCB; ++cj) cC[cj] = nC[cj];
      cLv = nLv;
    }
  }
  vm_wait_all();
  raw_barrier();
  if (WITH_CAND && pend_off >= 0) s7();
}

// ================================================================================================
// host side
// ================================================================================================
int x2_num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}

inline bool al16(const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15u) == 0; }

int x2w_launch(void* stream, const X2Params& prm) {
  void (*kern)(X2Params) = nullptr;
  const bool rg = prm.cand_off != nullptr;
  switch (prm.score_type) {
    case MINER_SCORE_WEIGHTED: kern = rg ? news_score_x2w<MINER_SCORE_WEIGHTED, true> : news_score_x2w<MINER_SCORE_WEIGHTED, false>; break;
    case MINER_SCORE_NONE: kern = news_score_x2w<MINER_SCORE_NONE, false>; break;
    default: kern = rg ? news_score_x2w<MINER_SCORE_MAX, true> : news_score_x2w<MINER_SCORE_MAX, false>; break;
  }
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, XW::kLds);
  if (e != hipSuccess) return (int)e;
  int grid = x2_num_cus();
  if (grid > prm.B) grid = prm.B;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(XW::kThr), XW::kLds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

// The kernel for a launch: the MIND shape (history 50, K = 32, 'weighted', no category bias, no mui
// output; the bench and the reference's eval) with its chunk count and shape compile-time, every
// other shape the run-time form
int x2_launch(void* stream, const X2Params& prm) {
  if (prm.L > kMaxL || prm.K > kMaxK) return x2w_launch(stream, prm);
  void (*kern)(X2Params) = nullptr;
  const bool rg = prm.cand_off != nullptr;
  const bool mind = prm.L == 50 && prm.K == 32 && !prm.bias && !prm.mui_out && prm.score_type == MINER_SCORE_WEIGHTED;
#define X2_PICK(NCHV, LOSSV)                                                                                 \
  switch (prm.score_type) {                                                                                  \
    case MINER_SCORE_WEIGHTED: kern = rg ? news_score_x2<MINER_SCORE_WEIGHTED, true, NCHV, 0, LOSSV> : news_score_x2<MINER_SCORE_WEIGHTED, false, NCHV, 0, LOSSV>; break; \
    case MINER_SCORE_NONE: kern = news_score_x2<MINER_SCORE_NONE, false, NCHV, 0, LOSSV>; break;              \
    default: kern = rg ? news_score_x2<MINER_SCORE_MAX, true, NCHV, 0, LOSSV> : news_score_x2<MINER_SCORE_MAX, false, NCHV, 0, LOSSV>; break; \
  }
#define X2_MIND(NCHV, LOSSV) kern = rg ? news_score_x2<MINER_SCORE_WEIGHTED, true, NCHV, 2, LOSSV> : news_score_x2<MINER_SCORE_WEIGHTED, false, NCHV, 2, LOSSV>
  if (prm.dis_out) {                   // eval with the eval loss (config/eval_miner.txt: metrics + loss)
    if (prm.d == 768) {
      if (mind) { X2_MIND(12, true); } else { X2_PICK(12, true) }
    } else if (prm.d == 256 && mind) {   // config 2 (MIND-small)
      X2_MIND(4, true);
    } else {
      X2_PICK(0, true)
    }
  } else {
    if (prm.d == 768) {                // config 3 (MIND-large)
      if (mind) { X2_MIND(12, false); } else { X2_PICK(12, false) }
    } else if (prm.d == 256) {         // config 2 (MIND-small)
      if (mind) { X2_MIND(4, false); } else { X2_PICK(4, false) }
    } else {
      X2_PICK(0, false)
    }
  }
#undef X2_PICK
#undef X2_MIND
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kX2Lds);
  if (e != hipSuccess) return (int)e;
  int grid = x2_num_cus();
  if (grid > prm.B) grid = prm.B;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), kX2Lds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

}  // namespace

extern "C" {

#ifdef MINER_STAMPS
// diagnostic build only: read (and reset) the per-wave stage cycles of news_score_x2;
// out[8 w + i] = cycles of stage i of wave w summed over workgroups, out[64] = impressions
int miner_news_x2_debug_stage_cycles(unsigned long long* out) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x2_stage), 64 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(g_x2_items), sizeof(unsigned long long));
  unsigned long long z[64] = {0};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_x2_stage), z, 64 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_x2_items), z, sizeof(unsigned long long));
  return (int)e;
}
#endif

int miner_news_split_x2(void* stream, const float* src, int n, int d, void* dst, float* row_unit) {
  if (!src || !dst || !row_unit || n <= 0 || d <= 0) return MINER_EINVAL;
  if (d % 64 || d > 64 * 8 * kSplitMaxG) return MINER_ESHAPE;
  if (!al16(src) || !al16(dst)) return MINER_EALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int grid = (n + 3) / 4 < 8192 ? (n + 3) / 4 : 8192;
  hipLaunchKernelGGL(x2_split_rows, dim3(grid), dim3(256), 0, s, src, n, d, static_cast<unsigned short*>(dst), row_unit);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

int miner_score_news_x2(void* stream, int score_type, const void* table2, const float* table_unit,
                        const float* news_logits, const void* proj2, const float* proj_unit, int n_news,
                        const int32_t* his_ids, const uint8_t* his_mask, const float* his_bias,
                        const int32_t* cand_ids, const int32_t* cand_offsets, int B, int L, int C, int d, int K,
                        float* scores, float* user_out, float* disagree_out) {
  if (score_type < MINER_SCORE_WEIGHTED || score_type > MINER_SCORE_NONE) return MINER_EINVAL;
  if (!table2 || !table_unit || !news_logits || !his_ids || !his_mask || n_news <= 0 || B < 0) return MINER_EINVAL;
  if (L <= 0 || d <= 0 || K <= 0) return MINER_EINVAL;
  if (L > XW::kMaxL || K > XW::kMaxK || (K & 3) || d % 64 || d > 1024) return MINER_ESHAPE;
  if ((L > kMaxL || K > kMaxK) && disagree_out) return MINER_ESHAPE;   // the wide kernel writes mui instead
  if ((uint64_t)n_news * (uint64_t)d * 4u > 0xffffffffull) return MINER_ESHAPE;   // 32-bit row offsets
  if (score_type == MINER_SCORE_WEIGHTED && (!proj2 || !proj_unit)) return MINER_EINVAL;
  if (score_type != MINER_SCORE_NONE) {
    if (!scores || !cand_ids) return MINER_EINVAL;
    if (!cand_offsets && (C < 0 || C > kMaxCand)) return MINER_ESHAPE;
  } else if (!user_out && !disagree_out) {
    return MINER_EINVAL;
  }
  if (!al16(table2) || !al16(news_logits) || !al16(proj2)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  X2Params prm{table2, news_logits, proj2, table_unit, proj_unit ? proj_unit : table_unit, his_ids, his_mask, his_bias,
               score_type == MINER_SCORE_NONE ? nullptr : cand_ids,
               score_type == MINER_SCORE_NONE ? nullptr : cand_offsets,
               scores, user_out, disagree_out, n_news, B, L, score_type == MINER_SCORE_NONE ? 0 : C, d, K, score_type};
  return x2_launch(stream, prm);
}

}  // extern "C"
