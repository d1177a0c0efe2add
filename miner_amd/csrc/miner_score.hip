// miner_score.hip — fused MINER scoring kernel for MI355X (gfx950 / CDNA4).
//
// One workgroup (8 waves, 512 threads, one per CU) scores one impression at a time and walks
// impressions b = blockIdx.x, blockIdx.x + gridDim.x, ...  Everything between the HBM reads of an
// impression's history/candidate rows and its fp32 score writes stays on chip:
//
//   S0  history rows E[L,d] + mask/bias -> LDS by LDS-DMA, issued during the previous impression
//       (bf16; the fp32 parity mode reads them from L2)
//   S1  Pᵀ = tanh(W1 · Eᵀ)        [Dc,L]  MFMA, wave w owns Dc-tile w                 (model.py:171)
//   S2  S_w = P_w · Q_wᵀ          [L,K]   bf16: fused into S1's epilogue, the tanh'd accumulator
//       is the A operand; per-wave partials -> LDS (fp32: separate stage)          (model.py:174)
//   S3  A  = softmax_L(fill(S))   [K,L]   bf16: 16 lanes per interest, DPP row reductions;
//       masked -> 1e-30                                                           (model.py:178-181)
//   S4  muiᵀ = Eᵀ · Aᵀ            [d,K]   MFMA, Eᵀ read with ds_read_b64_tr_b16; the candidate
//       rows are then DMA'd into the (dead) history image, landing during S5        (model.py:182)
//   S5  X  = gelu(W2 · muiᵀ)      [d,K]   MFMA, wave w owns d-tiles w, w+8, w+16   (model.py:212)
//   S6  Lgᵀ = Xᵀ·Candᵀ, Mᵀ = mui·Candᵀ  [K,C]  MFMA split over the waves' d-tiles, reduced
//       through LDS with plain stores in two rounds; the next history DMA is issued here (model.py:127,213)
//   S7  score_c = Σ_k softmax_K(Lg)_k · M_k  (or max_k / mean_k of M)      (model.py:128-134,213-214)
//
// Operand layout (both dtypes) — a "slab" is 32 consecutive contraction indices: lane
// l = 32h + r (h = l>>5, r = l&31) holds 16 contiguous elements [16h, 16h+16) of row r of the
// slab. bf16: two v_mfma_f32_32x32x16_bf16 steps (8 elements each); fp32: sixteen
// v_mfma_f32_32x32x2_f32 steps (one element each, an exact fp32 fma chain). A 32x32 MFMA
// accumulator keeps row (e&3)+8(e>>2)+4h of column r in register e; when the A-operand rows of a
// GEMM are taken in the order pi(r) = 16((r>>2)&1) + (r&3) + 4(r>>3), register e of lane half h
// holds row 16h+e: the accumulator IS a slab fragment of a following contraction over its rows
// (S5 -> S6), and its 16 registers are 16 contiguous elements of an LDS row (S1 -> P).
//
// Weights are pre-packed once (miner_pack_weights) into 32-row x 32-column tiles, rows in pi
// order, so each wave-instruction of a weight slab reads 2 KiB (bf16) contiguous bytes: reading
// the row-major [Dc,d] / [d,d] matrices directly put every wave's 32 row segments on 4 of an XCD
// L2's 16 channels (row stride 1536 B) and ran S5 3x slower.
//
// Hot-loop rules learned on this kernel (ROCm 7.2 hipcc):
//   * no LDS float atomics on the bf16 path: ds_add_f32 cost ~180 cycles each and serialise;
//   * every global load in a slab loop is unconditional (addresses clamped): a predicated load
//     makes hipcc wait vmcnt(0) and drains the prefetch ring; a loop back-edge does the same, so
//     the slab loops are fully unrolled on a compile-time d (NS = d/32 template);
//   * lane ids are re-derived from an opaque threadIdx.x in every stage so no per-lane address
//     is hoisted across stages (the hoisted values were spilled; scratch reloads wait vmcnt(0)).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include "../../include/miner_score.h"
#include "cdna4_common.h"

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kMaxL = 64;        // history positions per impression (two 32-row tiles)
constexpr int kMaxK = 32;        // interest vectors (one 32-row tile)
constexpr int kMaxDc = 256;      // context-code dim (one 32-row tile per wave)
constexpr int kMaxD = 768;       // embedding dim (<= 3 d-tiles per wave)
constexpr int kMaxJ = kMaxD / 32 / kWaves;
constexpr int kCChunk = 64;      // candidates per S6/S7 pass (two 32-column tiles)
constexpr int kLdsMax = 160 * 1024;
constexpr int kLgS = kCChunk + 1;      // fp32-path Lg/Mt row stride (floats)
constexpr int kPartS = 36;             // bf16-path partial slab row stride (floats): [c][k] rows
constexpr int kPartTile = 32 * kPartS; // one 32x32 tile, floats
constexpr int kPartWave = 4 * kPartTile;  // Lg ct0, Lg ct1, Mt ct0, Mt ct1
constexpr int kSPS = kMaxL + 4;        // bf16-path S-partial row stride (floats): [k][l] rows
constexpr int kSPTile = kMaxK * kSPS;  // one wave's S partial (floats)

enum Mode { kFull = 0, kTaa = 1 };

#ifndef MINER_PF_S1
#define MINER_PF_S1 3      // register prefetch depth of the W1 ring (S1; 6 and 8 measured slower)
#endif

struct Params {
  const void* hist;      // kFull: history [B,L,d]; kTaa: query (mui) [B,K,d]
  const uint8_t* mask;
  const float* bias;
  const void* cand;
  const int32_t* cand_off;
  const void* wp;        // packed weights (miner_pack_weights)
  const float* value;    // kTaa: [sum C_b, K]
  float* scores;
  float* mui_out;
  int B, L, C, d, Dc, K, score_type;
  // LDS carve (bytes)
  int MS;       // mui row stride
  int PS;       // P row stride (elements)
  int offE, offZ, offP, offS, offMui, offAw, offPart, offLg, offMt, offAux;
  // news-table gather mode (miner_score_gather): hist and cand point to the table [n_news, d]
  const int32_t* his_ids;    // [B, L] rows of the table, or null (dense history)
  const int32_t* cand_ids;   // [sum C_b] rows of the table, or null (dense candidates)
  int n_news;
  int eimg;     // bytes of the history image (bf16): the candidate rows may be staged there
  int dbg;      // ablation bits, honoured only by the -DMINER_STAMPS diagnostic build
  int part_ok;  // fp32: the mui region holds the S6 partial slabs (plain-store reduce); else LDS atomics
  int offS1;    // fp32 full (bf16x6): the S1 history-operand planes (kS1Bytes)
};

// ---------------------------------------------------------------------------------------------
// packed weight layout (elements of T):  [W1p | Qp | W2p]
//   W1p: ceil(Dc/32) x (d/32) blocks of 32x32 (block (ct, j) = rows 32ct + pi(r) of W1, columns
//        32j .. 32j+31), zero padded past Dc;
//   Qp : 32 x 32*ceil(Dc/32), row-major, zero padded;
//   W2p: (d/32) x (d/32) blocks, block (jt, j) = rows 32jt + pi(r) of W2, columns 32j .. 32j+31.
// Each block is stored FRAGMENT-MAJOR: 16-byte piece q of lane l = 32h + r sits at byte
// (64q + l)*16 and holds columns 16h + q*(16/sizeof(T)) ... of row r — exactly what
// frag_load_tile reads, so each wave-instruction reads 1 KiB contiguous (8 whole cache lines).
// ---------------------------------------------------------------------------------------------
__host__ __device__ inline int n_ctiles(int Dc) { return (Dc + 31) >> 5; }
__host__ __device__ inline size_t w1p_elems(int d, int Dc) { return (size_t)n_ctiles(Dc) * (d >> 5) * 1024; }
__host__ __device__ inline size_t qp_elems(int Dc) { return (size_t)n_ctiles(Dc) * 1024; }
__host__ __device__ inline size_t w2p_elems(int d) { return (size_t)(d >> 5) * (d >> 5) * 1024; }

template <class T> __device__ __forceinline__ float act_tanh(float x) {
  if constexpr (sizeof(T) == 2) return tanh_fast(x); else return tanhf(x);
}
template <class T> __device__ __forceinline__ float act_gelu(float x) {
  if constexpr (sizeof(T) == 2) return gelu_fast(x); else return gelu_erf(x);
}
template <class T> __device__ __forceinline__ float act_exp(float x) {
  if constexpr (sizeof(T) == 2) return __expf(x); else return expf(x);
}

// ---------------------------------------------------------------------------------------------
// history image in LDS (bf16 mode)
// ---------------------------------------------------------------------------------------------

// nrows rows of d elements -> the swizzled image (whole 1 KiB blocks, one per wave-instruction)
// Gather mode: row r is table row ids[r] (ids in LDS), clamped to [0, n_news) so a bad id can
// never address outside the table (the host wrapper validates ids and raises).
template <class T>
__device__ __forceinline__ void dma_rows(const T* src, int nrows, int d, char* img, int wave, int lane,
                                         const int32_t* idsL = nullptr, int n_news = 0) {
  const int cpr = d >> 3;                 // 16-byte chunks per row
  const int g16 = (cpr & 15) == 0;
  const int total = nrows * cpr;
  const int nblk = (total + 63) >> 6;
  for (int blk = wave; blk < nblk; blk += kWaves) {
    const int pos = blk * 64 + lane;
    const int row = pos / cpr;
    const int c = pos - row * cpr;
    const size_t r = idsL ? (size_t)min(max(idsL[min(row, nrows - 1)], 0), n_news - 1) : (size_t)row;
    const T* g = (pos < total) ? src + r * d + (size_t)((c ^ eswz(row, g16)) << 3) : src;
    dma_b128(g, __builtin_amdgcn_readfirstlane(lds_offset(img + blk * 1024)));
  }
}

// Per-impression aux block (1 KiB): [0,256) the mask bytes (as the aligned words covering them),
// [256,512) fp32 bias, [512,768) history ids, [768,1024) the first 64 candidate ids (gather mode)
constexpr int kAuxBytes = 1024;
template <class P>
__device__ __forceinline__ void dma_aux(const P& p, int b, char* aux, int wave, int lane) {
  const int L = p.L;
  if (wave == 0) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p.mask + (size_t)b * L) & ~(uintptr_t)3;
    const uintptr_t last = reinterpret_cast<uintptr_t>(p.mask + (size_t)p.B * L - 1) & ~(uintptr_t)3;
    const uintptr_t w = a + 4 * (uintptr_t)lane;
    dma_b32(reinterpret_cast<const void*>(w < last ? w : last), __builtin_amdgcn_readfirstlane(lds_offset(aux)));
  } else if (wave == 1 && p.bias) {
    dma_b32(p.bias + (size_t)b * L + min(lane, L - 1), __builtin_amdgcn_readfirstlane(lds_offset(aux + 256)));
  } else if (wave == 2 && p.his_ids) {
    dma_b32(p.his_ids + (size_t)b * L + min(lane, L - 1), __builtin_amdgcn_readfirstlane(lds_offset(aux + 512)));
  } else if (wave == 3 && p.cand_ids) {
    const int cb = p.cand_off ? p.cand_off[b] : b * p.C;
    const int n = p.cand_off ? p.cand_off[b + 1] - cb : p.C;
    if (n > 0)
      dma_b32(p.cand_ids + cb + min(lane, n - 1), __builtin_amdgcn_readfirstlane(lds_offset(aux + 768)));
  }
}

// B-operand slab fragment of history row `row` (contraction over d), from the swizzled image
__device__ __forceinline__ void frag_load_E(Frag<__bf16>& f, const char* ldsE, int row, int kb, int h, int rowB, int g16) {
  const int c0 = (kb + 16 * h) >> 3;
  const int sw = eswz(row, g16);
  const char* base = ldsE + row * rowB;
  f.q[0] = *reinterpret_cast<const u32x4*>(base + ((c0 ^ sw) << 4));
  f.q[1] = *reinterpret_cast<const u32x4*>(base + (((c0 + 1) ^ sw) << 4));
}

// ---------------------------------------------------------------------------------------------
// diagnostic stamps (-DMINER_STAMPS only)
// ---------------------------------------------------------------------------------------------
#ifdef MINER_STAMPS
// thread 0 of every workgroup sums the s_memtime cycles each stage takes (between the barriers
// that delimit it) into g_stage_cycles; p.dbg enables ablations.  Never in the product library.
__device__ unsigned long long g_stage_cycles[16];
__device__ unsigned long long g_stage_imps;
#define STAMP_DECL unsigned long long st_acc[12] = {0}; unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { if (threadIdx.x == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } } while (0)
#define STAMP_FLUSH(n) do { if (threadIdx.x == 0) { for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&g_stage_cycles[i_], st_acc[i_]); atomicAdd(&g_stage_imps, (unsigned long long)(n)); } } while (0)
#define DBG(bit) (p.dbg & (1 << (bit)))
#define STAMP_SYNC() __syncthreads()
#else
#define STAMP_SYNC() do {} while (0)
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH(n) do {} while (0)
#define DBG(bit) 0
#endif

// slab product: fp32 MFMA, or (X6, the fp32 kernel's default) the six bf16 partial products of
// split16 operands — see cdna4_common.h (bf16x6)
#ifndef MINER_X6_STAGES
#define MINER_X6_STAGES 5   // bf16x6 stages of the fp32 kernel: 1 S1, 2 S4, 4 S5, 8 S6 (S4 spills 12-21 VGPRs, S6 61-74: off)
#endif
#ifndef MINER_S1_P2
#define MINER_S1_P2 1   // fp32 (bf16x6 form, cooperative S1 cut): S1 on fp16 pairs (0: bf16x6, A/B builds)
#endif
#ifndef MINER_S5_P2
#define MINER_S5_P2 1   // fp32 (bf16x6 form): S5 on fp16 pairs (0: bf16x6, A/B builds)
#endif
template <class T, bool X6>
__device__ __forceinline__ void mma_f(f32x16& acc, const Frag<T>& a, const Frag<T>& b) {
  if constexpr (X6 && sizeof(T) == 4) mma_slab_x6(acc, a, b);
  else mma_slab<T>(acc, a, b);
}

// ---------------------------------------------------------------------------------------------
// fp16 pairs (the fp32 kernel's S5, news_x2.hip's operand form): an fp32 value x of a row with unit
// u (a power of two, max|row| < 2^14·u) is carried as hi = f16(x/u), lo = f16(x/u - hi), and a
// product as lo·hi + hi·lo + hi·hi on the f16 MFMA: three v_mfma_f32_32x32x16_f16 per 16-element
// step instead of bf16x6's six, the weights pre-cut at pack time (same bytes as fp32: no split VALU
// for them). The accumulator is rescaled by the two rows' units (powers of two: exact).
// ---------------------------------------------------------------------------------------------
// row unit exponent: max|row| < 2^e (a non-finite max is clamped to FLT_MAX: e = 128)
__host__ __device__ inline int p2_exp(float mx) {
  int e;
  frexpf(mx, &e);
  return e < -100 ? -100 : (e > 128 ? 128 : e);
}
// 2^(e - 14) and 2^(14 - e), the unit and the splitting scale of a row with max|row| < 2^e
__host__ __device__ inline float p2_unit(int e) { return ldexpf(1.0f, e - 14); }
__host__ __device__ inline float p2_scale(int e) { return ldexpf(1.0f, 14 - e); }
// the unit of a row with max|row| = mx: +inf when the row holds an infinity (its finite elements
// scale to 0 and the infinity is clamped, p2_split2), so its products come out ±inf — or NaN for a
// zero weight — as the reference's w·inf
__host__ __device__ inline float p2_unit_of(float mx, int e) { return mx > 3.40282347e38f ? INFINITY : p2_unit(e); }
// an infinity clamped to ±65504 by v_med3, a NaN kept by a select: v_med3 does not return a NaN
// operand (a NaN table row came out finite in news.hip's pair precompute before the select)
__device__ __forceinline__ float p2_clamp(float x) {
  return x != x ? x : __builtin_amdgcn_fmed3f(x, -65504.0f, 65504.0f);
}
// (x0, x1), scaled so that a finite row's |x| < 2^14, -> packed (hi, lo) fp16 pairs; the residual
// against hi as packed (one conversion of hi). An infinite x is clamped to ±65504 (p2_clamp),
// hi = ±65504 and lo = 0, so no inf - inf; its row's unit is +inf (p2_unit_of). A NaN stays NaN.
template <bool CLAMP = true>   // false: the caller has clamped
__device__ __forceinline__ void p2_split2(float x0, float x1, unsigned& hi, unsigned& lo) {
  if constexpr (CLAMP) {
    x0 = p2_clamp(x0);
    x1 = p2_clamp(x1);
  }
  const f16x2v h = __builtin_convertvector((f32x2v){x0, x1}, f16x2v);
  unsigned hb = __builtin_bit_cast(unsigned, h);
  asm volatile("" : "+v"(hb));
  const f16x2v hh = __builtin_bit_cast(f16x2v, hb);
  hi = hb;
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){x0 - (float)hh[0], x1 - (float)hh[1]}, f16x2v));
}
__device__ __forceinline__ f32x16 mfma32_f16(const u32x4& a, const u32x4& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// acc += A·B over one 32-wide slab: A a pair-packed weight fragment (pieces {hi, lo} of elements
// 0..7, then of 8..15), B an fp32 fragment already scaled and clamped, cut here (smallest products
// first)
__device__ __forceinline__ void mma_slab_p2(f32x16& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    u32x4 bh, bl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = 8 * st + 2 * i;
      unsigned h, l;
      p2_split2<false>(__uint_as_float(b.q[e >> 2][e & 3]), __uint_as_float(b.q[(e + 1) >> 2][(e + 1) & 3]), h, l);
      bh[i] = h;
      bl[i] = l;
    }
    acc = mfma32_f16(a.q[2 * st + 1], bh, acc);
    acc = mfma32_f16(a.q[2 * st], bl, acc);
    acc = mfma32_f16(a.q[2 * st], bh, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// S5 body, specialised on NM = number of d-tiles the wave owns (tiles wave + 8m)
// ---------------------------------------------------------------------------------------------
// X_m = gelu(W2[tile m] · muiᵀ) over the whole contraction d; packed W2 slabs stream from L2
// through a PF-deep register ring (unconditional loads, clamped at the end), muiᵀ fragments come
// from LDS.  The result stays in registers as slab fragments of the S6 contraction.
// P2 (fp32): W2p is the pair-packed copy, u2 its row units, s2 + 32 the units of the 32 mui rows
// (muiL scaled in place by their inverses, infinities clamped)
template <class T, int PF, int NM, bool X6, bool P2 = false>
__device__ __forceinline__ void s5_gelu(Frag<T> (&xf)[kMaxJ], const T* __restrict__ W2p, const T* muiL,
                                        int msE, int d, int wave, int lane, const float* __restrict__ u2 = nullptr,
                                        const float* s2 = nullptr) {
  const int ns = d >> 5;
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[NM];
  const T* w2t[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    acc[m] = zero16();
    w2t[m] = W2p + (size_t)(wave + kWaves * m) * ns * 1024;   // block (tile, slab 0)
  }
  Frag<T> ring[PF][NM];
#pragma unroll
  for (int s = 0; s < PF; ++s)
#pragma unroll
    for (int m = 0; m < NM; ++m) frag_load_tile(ring[s][m], w2t[m] + min(s, ns - 1) * 1024, lane);
  int j = 0;
#pragma unroll
  for (; j + PF <= ns; j += PF) {
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      Frag<T> bm;
      frag_load(bm, muiL + r * msE + (j + s) * 32 + 16 * h);
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        if constexpr (P2) mma_slab_p2(acc[m], ring[s][m], bm);
        else mma_f<T, X6 && (MINER_X6_STAGES & 4)>(acc[m], ring[s][m], bm);
      }
#pragma unroll
      for (int m = 0; m < NM; ++m) frag_load_tile(ring[s][m], w2t[m] + min(j + s + PF, ns - 1) * 1024, lane);
      __builtin_amdgcn_sched_barrier(0);   // keep the refill right behind the MFMAs it waits on
    }
  }
#pragma unroll
  for (int s = 0; s < PF; ++s) {
    if (j + s < ns) {
      Frag<T> bm;
      frag_load(bm, muiL + r * msE + (j + s) * 32 + 16 * h);
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        if constexpr (P2) mma_slab_p2(acc[m], ring[s][m], bm);
        else mma_f<T, X6 && (MINER_X6_STAGES & 4)>(acc[m], ring[s][m], bm);
      }
    }
  }
  if constexpr (P2) {
    // the units back: register e of lane half h is W2 row 32 tile + 16h + e, column r is mui row r
    const float ub = s2[32 + r];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const float* ur = u2 + (wave + kWaves * m) * 32 + 16 * h;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][e] = acc[m][e] * ur[e] * ub;
    }
  }
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    gelu_tile<T>(acc[m]);
    acc_to_frag(xf[m], acc[m]);
  }
}

// S6 partial products over the wave's d-tiles for candidates [cc, cc+64): lg = Xᵀ·Candᵀ and
// mt = mui·Candᵀ restricted to those tiles.  Candidate rows past the end are clamped to a real
// row (finite data, never read back by S7).
template <class T, int NM, bool WEIGHTED, bool FULL, bool X6>
__device__ __forceinline__ void s6_products(f32x16 (&lg)[2], f32x16 (&mt)[2], const Frag<T> (&xf)[kMaxJ],
                                            const Frag<T> (&amr)[kMaxJ], const T* __restrict__ cand,
                                            const char* cimg, int Cb, int cc, int d, int wave, int r, int h,
                                            const T* muiL, int msE, const int32_t* cids, int n_news) {
  // mui fragments of the wave's d-tiles: bf16 preloads them (amr) before the chunk loop, because
  // the partial slabs overwrite mui; fp32 reads them here
  Frag<T> am[NM];
  if constexpr (FULL) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      if constexpr (sizeof(T) == 2) am[m] = amr[m];
      else frag_load(am[m], muiL + r * msE + (wave + kWaves * m) * 32 + 16 * h);
    }
  }
  // one 32-candidate tile at a time (NM fragments live, not 2·NM)
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int c = min(cc + ct * 32 + r, Cb - 1);
    Frag<T> bc[NM];
    if constexpr (sizeof(T) == 2) {
      if (cimg) {   // candidate rows DMA'd into the swizzled image
        const int g16 = ((d >> 3) & 15) == 0;
#pragma unroll
        for (int m = 0; m < NM; ++m)
          frag_load_E(reinterpret_cast<Frag<__bf16>&>(bc[m]), cimg, c, (wave + kWaves * m) * 32, h, d * 2, g16);
      }
    }
    if (!cimg || sizeof(T) != 2) {   // gather mode: table row cids[c] (ids from global)
      const size_t cr = cids ? (size_t)min(max(cids[c], 0), n_news - 1) : (size_t)c;
      const T* crow = cand + cr * d + 16 * h;
#pragma unroll
      for (int m = 0; m < NM; ++m) frag_load_stream(bc[m], crow + (wave + kWaves * m) * 32);
    }
    lg[ct] = zero16();
    mt[ct] = zero16();
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      if constexpr (WEIGHTED) mma_f<T, X6 && (MINER_X6_STAGES & 8)>(lg[ct], xf[m], bc[m]);
      if constexpr (FULL) mma_f<T, X6 && (MINER_X6_STAGES & 8)>(mt[ct], am[m], bc[m]);
    }
  }
}

template <class T, bool WEIGHTED, bool FULL, bool X6>
__device__ __forceinline__ void s6_dispatch(int nm, f32x16 (&lg)[2], f32x16 (&mt)[2], const Frag<T> (&xf)[kMaxJ],
                                            const Frag<T> (&am)[kMaxJ], const T* cand, const char* cimg, int Cb,
                                            int cc, int d, int wave, int r, int h, const T* muiL, int msE,
                                            const int32_t* cids, int n_news) {
  if (nm == 3) s6_products<T, 3, WEIGHTED, FULL, X6>(lg, mt, xf, am, cand, cimg, Cb, cc, d, wave, r, h, muiL, msE, cids, n_news);
  else if (nm == 2) s6_products<T, 2, WEIGHTED, FULL, X6>(lg, mt, xf, am, cand, cimg, Cb, cc, d, wave, r, h, muiL, msE, cids, n_news);
  else if (nm == 1) s6_products<T, 1, WEIGHTED, FULL, X6>(lg, mt, xf, am, cand, cimg, Cb, cc, d, wave, r, h, muiL, msE, cids, n_news);
}

// one 32x32 accumulator tile -> rows [c][k] of a partial slab (4 x 16-byte stores per lane):
// register e of lane (r=c, h) is k = (e&3) + 8(e>>2) + 4h, so registers 4g..4g+3 are 4 contiguous k
__device__ __forceinline__ void part_store(float* tile, const f32x16& a, int r, int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(tile + r * kPartS + 8 * g + 4 * h) = float4{a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]};
}
__device__ __forceinline__ void part_add(float* tile, const f32x16& a, int r, int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float4* q = reinterpret_cast<float4*>(tile + r * kPartS + 8 * g + 4 * h);
    const float4 v = *q;
    *q = float4{v.x + a[4 * g], v.y + a[4 * g + 1], v.z + a[4 * g + 2], v.w + a[4 * g + 3]};
  }
}

// S6 reduction, bf16: two rounds through LDS with plain stores — waves 0-3 store their partial
// tiles, waves 4-7 add theirs onto the same slots (contains the barrier between the rounds)
__device__ __forceinline__ void s6_reduce_bf16(float* part, const f32x16 (&lg)[2], const f32x16 (&mt)[2], int wave,
                                               int r, int h, bool skip) {
  float* slot = part + (wave & 3) * kPartWave;
  if (wave < 4 && !skip) {
    part_store(slot, lg[0], r, h);
    part_store(slot + kPartTile, lg[1], r, h);
    part_store(slot + 2 * kPartTile, mt[0], r, h);
    part_store(slot + 3 * kPartTile, mt[1], r, h);
  }
  __syncthreads();
  if (wave >= 4 && !skip) {
    part_add(slot, lg[0], r, h);
    part_add(slot + kPartTile, lg[1], r, h);
    part_add(slot + 2 * kPartTile, mt[0], r, h);
    part_add(slot + 3 * kPartTile, mt[1], r, h);
  }
}

// S7 load, bf16: candidate cl's Lg and M for interests 4sub .. 4sub+3, summed over the 4 slots
__device__ __forceinline__ void s7_load_bf16(const float* part, int cl, int sub, float (&lgv)[4], float (&mtv)[4]) {
  const int ct = cl >> 5, cr = cl & 31;
  float4 a = float4{0.f, 0.f, 0.f, 0.f}, mm = a;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float* slot = part + w * kPartWave + cr * kPartS + 4 * sub;
    const float4 x = *reinterpret_cast<const float4*>(slot + ct * kPartTile);
    const float4 y = *reinterpret_cast<const float4*>(slot + (2 + ct) * kPartTile);
    a = float4{a.x + x.x, a.y + x.y, a.z + x.z, a.w + x.w};
    mm = float4{mm.x + y.x, mm.y + y.y, mm.z + y.z, mm.w + y.w};
  }
  lgv[0] = a.x; lgv[1] = a.y; lgv[2] = a.z; lgv[3] = a.w;
  mtv[0] = mm.x; mtv[1] = mm.y; mtv[2] = mm.z; mtv[3] = mm.w;
}

// S7 arithmetic for one candidate held by 8 lanes (interests 4sub .. 4sub+3 each):
// weighted: Σ_k softmax_K(Lg)_k · M_k (model.py:213-214); max_k M (:128-129); mean_k M (:130-132)
template <class T>
__device__ __forceinline__ float s7_score(const float (&lgv)[4], const float (&mtv)[4], const bool (&kv)[4],
                                          int score_type, int K) {
  if (score_type == MINER_SCORE_WEIGHTED) {
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) if (kv[j]) mx = fmaxf(mx, lgv[j]);
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
    float ex[4], den = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ex[j] = kv[j] ? act_exp<T>(lgv[j] - mx) : 0.f;
      den += ex[j];
    }
    den += __shfl_xor(den, 1, 64);
    den += __shfl_xor(den, 2, 64);
    den += __shfl_xor(den, 4, 64);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += (ex[j] / den) * mtv[j];   // softmax weights · value
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    return acc;
  }
  if (score_type == MINER_SCORE_MAX) {
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) if (kv[j]) mx = fmaxf(mx, mtv[j]);
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
    return mx;
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += kv[j] ? mtv[j] : 0.f;
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  return s / (float)K;
}

// ---------------------------------------------------------------------------------------------
// the fused kernel
// ---------------------------------------------------------------------------------------------
// SHP 1: the MIND model shape compile-time (L = 50, Dc = 200, K = 32); X6 (fp32 only): S1 and
// S5 on the bf16 matrix cores as bf16x6 (S4 stays on the fp32 MFMA) (the fp32-MFMA form stays selectable: MINER_DENSE_FP32=mfma32)
#ifndef MINER_S1_COOP
#define MINER_S1_COOP 1   // fp32 bf16x6: the history operand of S1 split once per slab into LDS by all threads
#endif
constexpr int kS1Row = 80;                       // bytes per row of a split plane (32 bf16 + 16 pad: conflict-free b128)
constexpr int kS1Plane = 64 * kS1Row;            // one plane of one slab (64 history rows)
constexpr int kS1Slab = 3 * kS1Plane;            // hi | mid | lo
constexpr int kS1Bytes = 4 * kS1Slab;            // two buffers of two slabs

template <class T, int MODE, int NS, bool GATHER, int SHP = 0, bool X6 = false, bool S1C = false>
__global__ __launch_bounds__(kThreads) void miner_fused(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool kBf16 = sizeof(T) == 2;
  // S1C: the fp32 bf16x6 form with S1's history operand cut once per slab into LDS (the host picks
  // it where the carve holds one workgroup per CU anyway)
  constexpr bool kS1Coop = S1C && !kBf16 && X6 && (MINER_X6_STAGES & 1) && MODE == kFull;
  // news-table gather mode (compile-time, so the dense instantiations carry no gather code)
  const int32_t* const his_ids = GATHER ? p.his_ids : nullptr;
  const int32_t* const cand_ids = GATHER ? p.cand_ids : nullptr;
  constexpr bool kDma = kBf16 && MODE == kFull;  // history staged in LDS by DMA
#ifndef MINER_PF
#define MINER_PF 3
#endif
  constexpr int PF = kBf16 ? MINER_PF : 1;        // register prefetch depth of streamed weight slabs
  // S1 has 4 MFMAs per W1 slab and wave (S5: 6): it needs a deeper ring to cover L2 latency
  constexpr int PF1 = kBf16 ? MINER_PF_S1 : 1;
  // NS > 0: the embedding dim is a compile-time 32*NS and every slab loop fully unrolls
  const int L = SHP ? 50 : p.L, d = NS ? 32 * NS : p.d, Dc = SHP ? 200 : p.Dc, K = SHP ? 32 : p.K;
  const int ns = d >> 5;
  const int nct = n_ctiles(Dc);
  const T* __restrict__ W1p = static_cast<const T*>(p.wp);
  const T* __restrict__ Qp = W1p + w1p_elems(d, Dc);
  const T* __restrict__ W2p = Qp + qp_elems(Dc);
  // fp32 (bf16x6 form): S5 on fp16 pairs — the pair-packed W2 copy and its row units follow W2p
  constexpr bool kP2 = !kBf16 && X6 && MODE == kFull && MINER_S5_P2;
  const T* __restrict__ W2x = W2p + w2p_elems(d);
  const float* __restrict__ u2 = reinterpret_cast<const float*>(W2x + w2p_elems(d));
  // ... and S1 (the cooperative cut form) likewise: the pair-packed W1 copy and its row units
  constexpr bool kP1 = kS1Coop && MINER_S1_P2;
  const T* __restrict__ W1x = reinterpret_cast<const T*>(u2 + d);
  const float* __restrict__ u1 = reinterpret_cast<const float*>(W1x + w1p_elems(d, Dc));
  const bool weighted = (p.score_type == MINER_SCORE_WEIGHTED);
  const bool need_scores = (p.score_type != MINER_SCORE_NONE);
  const int rowB = d * 2;
  const int g16 = ((d >> 3) & 15) == 0;
  char* ldsE = smem + p.offE;
  T* muiL = reinterpret_cast<T*>(smem + p.offMui);        // [32][MS bytes]
  const int msE = p.MS / (int)sizeof(T);
  float* Lg = reinterpret_cast<float*>(smem + p.offLg);   // fp32 path: [32][kLgS], atomically summed
  float* Mt = reinterpret_cast<float*>(smem + p.offMt);
  float* part = reinterpret_cast<float*>(smem + p.offPart);  // bf16 path: 4 waves x kPartWave
  constexpr int AwS = kBf16 ? 72 : 68;

  {
    FRESH_LANE_IDS();
    if constexpr (kDma) {
      if (tid < 4) reinterpret_cast<u32x4*>(smem + p.offZ)[tid] = u32x4{0u, 0u, 0u, 0u};
      if (blockIdx.x < p.B) {   // aux (ids) first: the gathered history DMA reads them
        dma_aux(p, blockIdx.x, smem + p.offAux, wave, lane);
        vm_wait_all();
        __syncthreads();
        dma_rows(static_cast<const T*>(p.hist) + (his_ids ? 0 : (size_t)blockIdx.x * L * d), L, d, ldsE, wave, lane,
                 his_ids ? reinterpret_cast<const int32_t*>(smem + p.offAux + 512) : nullptr, p.n_news);
      }
    }
    if constexpr (!kBf16)
      for (int i = tid; i < 2 * kMaxK * kLgS; i += kThreads) Lg[i] = 0.f;   // Lg and Mt are adjacent
  }
  STAMP_DECL
  int n_done = 0;

  for (int b = blockIdx.x; b < p.B; b += gridDim.x) {
    ++n_done;
    const int cbase = p.cand_off ? p.cand_off[b] : b * p.C;
    const int Cb = p.cand_off ? (p.cand_off[b + 1] - cbase) : p.C;
    // gather mode: cand = the table, cids = this impression's candidate ids (global)
    const int32_t* cids = cand_ids ? cand_ids + cbase : nullptr;
    const T* __restrict__ cand = static_cast<const T*>(p.cand) + ((DBG(2) || cids) ? (size_t)0 : (size_t)cbase * d);
    const int bnext = b + gridDim.x;
    bool prefetched = false;   // next impression's history DMA already issued
    const char* cimg = nullptr;   // candidate rows staged in the history image (bf16)
    // aux blocks alternate by iteration: the next impression's aux lands while this one's is read
    char* aux = smem + p.offAux + ((n_done - 1) & 1) * kAuxBytes;
    char* auxn = smem + p.offAux + (n_done & 1) * kAuxBytes;

    if constexpr (MODE == kFull) {
      const T* __restrict__ E = static_cast<const T*>(p.hist) + (his_ids ? 0 : (size_t)b * L * d);
      // fp32 path: history row l (gather mode: table row his_ids[b][l], staged in LDS below)
      const int32_t* hidL = reinterpret_cast<const int32_t*>(smem + p.offAux);
      auto erow = [&](int l) -> const T* {
        return his_ids ? E + (size_t)min(max(hidL[l], 0), p.n_news - 1) * d : E + (size_t)l * d;
      };
      if constexpr (!kBf16 && GATHER) {
        FRESH_LANE_IDS();
        __syncthreads();   // the previous impression's readers of the id block are done
        if (tid < L) reinterpret_cast<int32_t*>(smem + p.offAux)[tid] = his_ids[(size_t)b * L + tid];
      }
      T* Ps = reinterpret_cast<T*>(smem + p.offP);         // P[l][c], row stride PS (aliases mui)
      float* S = reinterpret_cast<float*>(smem + p.offS);  // Sᵀ[k][l], [32][kMaxL] (aliases mui)
      T* Aw = reinterpret_cast<T*>(smem + p.offAw);        // A[k][l], [32][AwS]

      if constexpr (kDma) vm_wait_all();   // this impression's history / mask / bias DMA landed
      __syncthreads();                      // ... for every wave; last impression's LDS reads done
      STAMP(0);

      // ---- S1: Pᵀ = tanh(W1[ct] · Eᵀ) -> P[l][c] in LDS -------------------------------------
      {
        FRESH_LANE_IDS();
        // fp32 bf16x6 (kS1Coop): the history operand is the same for every wave, so its three bf16
        // terms are cut once per slab by all 512 threads into LDS (two slabs per round, planes of
        // 80-byte rows) instead of by each of the 7 MFMA waves in registers; products and their
        // order per accumulator unchanged (bit-identical)
        f32x16 cacc0 = zero16(), cacc1 = zero16();
        [[maybe_unused]] int ep0 = 0, ep1 = 0;   // kP1: the accumulators' unit exponents (history rows r, 32 + r)
        constexpr bool coop = kS1Coop;
        if constexpr (coop) {
          // kP1: each history row's unit exponent per round of two slabs (max|row piece| < 2^e, from
          // the 8 lanes that cut it), [2 buffers][64] ints in the S region (free until S2); the MFMA
          // waves carry their accumulators from round to round by the exponent difference (exact)
          [[maybe_unused]] int* reL = reinterpret_cast<int*>(smem + p.offS);
          // rounds of two slabs through two LDS buffers: round g + 1 is cut (its global loads in
          // flight) while round g's products run, one barrier per round
          const T* w1t = (kP1 ? W1x : W1p) + (size_t)min(wave, nct - 1) * ns * 1024;
          Frag<T> ring1;
          frag_load_tile(ring1, w1t, lane);
          auto cut = [&](int g) {          // slabs g, g + 1 -> buffer (g / 2) & 1
            char* sb = smem + p.offS1 + ((g >> 1) & 1) * (2 * kS1Slab);
            const int row = tid >> 3, cb = tid & 7, sl = cb >> 2, c8 = (cb & 3) * 8;
            float4 x0 = float4{0.f, 0.f, 0.f, 0.f}, x1 = x0;
            if (g + sl < ns) {
              const float4* src = reinterpret_cast<const float4*>(erow(min(row, L - 1)) + (g + sl) * 32 + c8);
              x0 = src[0];
              x1 = src[1];
            }
            [[maybe_unused]] float sc = 1.f;
            if constexpr (kP1) {         // the round's unit of the row: max over its 8 lanes
              float mx = fmaxf(fmaxf(fmaxf(fabsf(x0.x), fabsf(x0.y)), fmaxf(fabsf(x0.z), fabsf(x0.w))),
                               fmaxf(fmaxf(fabsf(x1.x), fabsf(x1.y)), fmaxf(fabsf(x1.z), fabsf(x1.w))));
              mx = fmaxf(mx, __shfl_xor(mx, 1));
              mx = fmaxf(mx, __shfl_xor(mx, 2));
              mx = fmaxf(mx, __shfl_xor(mx, 4));
              const int e = p2_exp(fminf(mx, 3.40282347e38f));
              if (cb == 0) reL[((g >> 1) & 1) * 64 + row] = e;
              sc = p2_scale(e);
            }
            if (g + sl < ns) {
              const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
              char* dst = sb + sl * kS1Slab + row * kS1Row + c8 * 2;
              if constexpr (kP1) {       // fp16 pairs: planes hi | lo
                u32x4 hi, lo;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                  unsigned a, b;
                  p2_split2(xv[2 * m] * sc, xv[2 * m + 1] * sc, a, b);
                  hi[m] = a;
                  lo[m] = b;
                }
                *reinterpret_cast<u32x4*>(dst) = hi;
                *reinterpret_cast<u32x4*>(dst + kS1Plane) = lo;
              } else {
                u32x4 hi, md, lo;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                  unsigned a, b, c;
                  split3_pair<true>(xv[2 * m], xv[2 * m + 1], a, b, c);
                  hi[m] = a;
                  md[m] = b;
                  lo[m] = c;
                }
                *reinterpret_cast<u32x4*>(dst) = hi;
                *reinterpret_cast<u32x4*>(dst + kS1Plane) = md;
                *reinterpret_cast<u32x4*>(dst + 2 * kS1Plane) = lo;
              }
            }
          };
          cut(0);
          __syncthreads();
          for (int g = 0; g < ns; g += 2) {
            if (g + 2 < ns) cut(g + 2);
            if (wave < nct) {
              const char* sb = smem + p.offS1 + ((g >> 1) & 1) * (2 * kS1Slab);
              if constexpr (kP1) {
                // this round's exponents; the accumulators (in units 2^(ep - 14)) brought to them
                const int e0 = reL[((g >> 1) & 1) * 64 + r], e1 = reL[((g >> 1) & 1) * 64 + 32 + r];
                if (g > 0) {
#pragma unroll
                  for (int e = 0; e < 16; ++e) {
                    cacc0[e] = ldexpf(cacc0[e], ep0 - e0);
                    cacc1[e] = ldexpf(cacc1[e], ep1 - e1);
                  }
                }
                ep0 = e0;
                ep1 = e1;
              }
#pragma unroll
              for (int s2 = 0; s2 < 2; ++s2) {
                if (g + s2 < ns) {
                  const Frag<T> a = ring1;
                  frag_load_tile(ring1, w1t + min(g + s2 + 1, ns - 1) * 1024, lane);
                  const char* base = sb + s2 * kS1Slab;
#pragma unroll
                  for (int st = 0; st < 2; ++st) {
                    if constexpr (kP1) {   // a: pair pieces {hi, lo} of step st; lo·hi + hi·lo + hi·hi
#pragma unroll
                      for (int rt = 0; rt < 2; ++rt) {
                        const char* q = base + (32 * rt + r) * kS1Row + (16 * h + 8 * st) * 2;
                        const u32x4 bh = *reinterpret_cast<const u32x4*>(q);
                        const u32x4 bl = *reinterpret_cast<const u32x4*>(q + kS1Plane);
                        f32x16& c = rt ? cacc1 : cacc0;
                        c = mfma32_f16(a.q[2 * st + 1], bh, c);
                        c = mfma32_f16(a.q[2 * st], bl, c);
                        c = mfma32_f16(a.q[2 * st], bh, c);
                      }
                    } else {
                      u32x4 ah, am, al;
                      split8_step<false>(a, st, ah, am, al);
#pragma unroll
                      for (int rt = 0; rt < 2; ++rt) {
                        const char* q = base + (32 * rt + r) * kS1Row + (16 * h + 8 * st) * 2;
                        const u32x4 bh = *reinterpret_cast<const u32x4*>(q);
                        const u32x4 bm = *reinterpret_cast<const u32x4*>(q + kS1Plane);
                        const u32x4 bl = *reinterpret_cast<const u32x4*>(q + 2 * kS1Plane);
                        mma6_step(rt ? cacc1 : cacc0, ah, am, al, bh, bm, bl);
                      }
                    }
                  }
                }
              }
            }
            __syncthreads();                 // round g + 2 cut; round g's buffer read by every wave
          }
        }
        if (wave < nct) {
          f32x16 acc0 = cacc0, acc1 = cacc1;
          const T* w1t = W1p + (size_t)wave * ns * 1024;   // block (tile, slab 0)
          // rows >= L: finite, dropped in S3.  bf16: lane r takes history row pi(r), so the tanh'd
          // accumulator is directly the A operand of the fused S2 product (rows l in pi order)
          const int lr = kBf16 ? pi_row(r) : r;
          const int l0 = min(lr, L - 1), l1 = min(32 + lr, L - 1);
          Frag<T> qa;   // bf16 fused S2: Q[k = r][32 wave + 16h ...]
          if constexpr (kBf16) frag_load(qa, Qp + r * (nct * 32) + wave * 32 + 16 * h);
          Frag<T> ring[PF1];
#pragma unroll
          for (int s = 0; s < PF1; ++s)
            if (!coop) frag_load_tile(ring[s], w1t + min(s, ns - 1) * 1024, lane);
          if constexpr (kBf16) {
            // the history fragments of slab s+1 are read from LDS before slab s's MFMAs: read right
            // before use, every MFMA waited one LDS latency (lgkmcnt) — S1 was LDS-latency bound
            Frag<T> c0, c1, n0, n1;
            frag_load_E(c0, ldsE, l0, 0, h, rowB, g16);
            frag_load_E(c1, ldsE, l1, 0, h, rowB, g16);
            int j = 0;
#pragma unroll
            for (; j + PF1 <= ns; j += PF1) {
#pragma unroll
              for (int s = 0; s < PF1; ++s) {
                if (j + s + 1 < ns) {
                  frag_load_E(n0, ldsE, l0, (j + s + 1) * 32, h, rowB, g16);
                  frag_load_E(n1, ldsE, l1, (j + s + 1) * 32, h, rowB, g16);
                }
                mma_slab<T>(acc0, ring[s], c0);
                mma_slab<T>(acc1, ring[s], c1);
                frag_load_tile(ring[s], w1t + min(j + s + PF1, ns - 1) * 1024, lane);
                c0 = n0;
                c1 = n1;
                __builtin_amdgcn_sched_barrier(0);   // keep the refill right behind the MFMAs it waits on
              }
            }
#pragma unroll
            for (int s = 0; s < PF1; ++s) {
              if (j + s < ns) {
                if (j + s + 1 < ns) {
                  frag_load_E(n0, ldsE, l0, (j + s + 1) * 32, h, rowB, g16);
                  frag_load_E(n1, ldsE, l1, (j + s + 1) * 32, h, rowB, g16);
                }
                mma_slab<T>(acc0, ring[s], c0);
                mma_slab<T>(acc1, ring[s], c1);
                c0 = n0;
                c1 = n1;
              }
            }
          } else if (!coop) {
            int j = 0;
#pragma unroll
            for (; j + PF1 <= ns; j += PF1) {
#pragma unroll
              for (int s = 0; s < PF1; ++s) {
                const int kk = (j + s) * 32;
                Frag<T> b0, b1;
                frag_load(b0, erow(l0) + kk + 16 * h);
                frag_load(b1, erow(l1) + kk + 16 * h);
                mma_f<T, X6 && (MINER_X6_STAGES & 1)>(acc0, ring[s], b0);
                mma_f<T, X6 && (MINER_X6_STAGES & 1)>(acc1, ring[s], b1);
                frag_load_tile(ring[s], w1t + min(j + s + PF1, ns - 1) * 1024, lane);
                __builtin_amdgcn_sched_barrier(0);
              }
            }
#pragma unroll
            for (int s = 0; s < PF1; ++s) {
              if (j + s < ns) {
                const int kk = (j + s) * 32;
                Frag<T> b0, b1;
                frag_load(b0, erow(l0) + kk + 16 * h);
                frag_load(b1, erow(l1) + kk + 16 * h);
                mma_f<T, X6 && (MINER_X6_STAGES & 1)>(acc0, ring[s], b0);
                mma_f<T, X6 && (MINER_X6_STAGES & 1)>(acc1, ring[s], b1);
              }
            }
          }
          STAMP(10);
          if constexpr (kP1) {
            // the units back: register e of lane half h is W1 row 32 wave + 16h + e, column r (+ 32)
            // history row r (32 + r), the last round's unit 2^(ep - 14)
            const float v0 = p2_unit(ep0), v1 = p2_unit(ep1);
            const float* ur = u1 + wave * 32 + 16 * h;
            // (the padded rows c >= Dc stay 0, also beside a history row of unit +inf: Q is zero
            // there, and 0·NaN would poison S)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const bool cv = 32 * wave + 16 * h + e < Dc;
              acc0[e] = cv ? acc0[e] * ur[e] * v0 : 0.f;
              acc1[e] = cv ? acc1[e] * ur[e] * v1 : 0.f;
            }
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) { acc0[e] = act_tanh<T>(acc0[e]); acc1[e] = act_tanh<T>(acc1[e]); }
          STAMP(11);
          // register e of lane (r, h) is c = 32*wave + 16h + e: 16 contiguous c of history row lr
          Frag<T> pf;
          if constexpr (kBf16) {
            // fused S2 partial over this wave's 32 context dims: S_w[l][k] = Σ_c P[l][c] Q[k][c];
            // register e of lane (h, k) is l = 16h + e (A rows in pi order) -> 4 b128 stores of row k
            float* sp = reinterpret_cast<float*>(smem + p.offS) + wave * kSPTile + r * kSPS + 16 * h;
            f32x16 sacc = zero16();
            acc_to_frag(pf, acc0);
            mma_slab<T>(sacc, pf, qa);
#pragma unroll
            for (int g = 0; g < 4; ++g)
              reinterpret_cast<float4*>(sp)[g] = float4{sacc[4 * g], sacc[4 * g + 1], sacc[4 * g + 2], sacc[4 * g + 3]};
            if (L > 32) {
              sacc = zero16();
              acc_to_frag(pf, acc1);
              mma_slab<T>(sacc, pf, qa);
#pragma unroll
              for (int g = 0; g < 4; ++g)
                reinterpret_cast<float4*>(sp + 32)[g] = float4{sacc[4 * g], sacc[4 * g + 1], sacc[4 * g + 2], sacc[4 * g + 3]};
            }
          } else {
            acc_to_frag(pf, acc0);
            frag_store(Ps + r * p.PS + wave * 32 + 16 * h, pf);
            if (L > 32) {
              acc_to_frag(pf, acc1);
              frag_store(Ps + (32 + r) * p.PS + wave * 32 + 16 * h, pf);
            }
          }
        }
      }
      __syncthreads();
      STAMP(1);

      // ---- S2 (fp32; fused into S1 for bf16): Sᵀ[k][l] = Σ_c Q[k][c] P[l][c] ------------------
      if constexpr (!kBf16 && kS1Coop) {
        // the contraction over the context tiles split over all 8 waves (history tile wave & 1, tile
        // group wave >> 1: tiles cg, cg + 4): four partials [4][K][kMaxL] from offS on (the S region
        // and the S1 planes behind it, both free here; P ends where they start), summed in S3 —
        // two waves over all nct tiles left six idle: 12.6k cycles per impression
        FRESH_LANE_IDS();
        const int lt = wave & 1, cg = wave >> 1;
        if (lt * 32 < L) {
          f32x16 acc = zero16();
          const T* qrow = Qp + r * (nct * 32) + 16 * h;
          const T* prow = Ps + (lt * 32 + r) * p.PS + 16 * h;
          for (int j = cg; j < nct; j += 4) {
            Frag<T> qa, pb;
            frag_load(qa, qrow + j * 32);
            frag_load(pb, prow + j * 32);
            mma_slab<T>(acc, qa, pb);
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) S[(cg * kMaxK + acc_row(e, h)) * kMaxL + lt * 32 + r] = acc[e];
        }
      } else if constexpr (!kBf16) {
        FRESH_LANE_IDS();
        if (wave * 32 < L) {
          f32x16 acc = zero16();
          const T* qrow = Qp + r * (nct * 32) + 16 * h;
          const T* prow = Ps + (wave * 32 + r) * p.PS + 16 * h;
          for (int j = 0; j < nct; ++j) {
            Frag<T> qa, pb;
            frag_load(qa, qrow + j * 32);
            frag_load(pb, prow + j * 32);
            mma_slab<T>(acc, qa, pb);
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) S[acc_row(e, h) * kMaxL + wave * 32 + r] = acc[e];
        }
      }
      if constexpr (!kBf16) __syncthreads();
      STAMP(2);

      // ---- S3: masked softmax over the history ----------------------------------------------
      if constexpr (kBf16) {
        // 16 lanes (a DPP row) per interest k = 4 wave + row, 4 positions l = 4j..4j+3 per lane;
        // S = Σ of the nct per-wave partials of S1
        FRESH_LANE_IDS();
        const int k = 4 * wave + (lane >> 4), j = lane & 15;
        const float* sp = reinterpret_cast<const float*>(smem + p.offS) + k * kSPS + 4 * j;
        float4 sv = *reinterpret_cast<const float4*>(sp);
        for (int w = 1; w < nct; ++w) {
          const float4 t = *reinterpret_cast<const float4*>(sp + w * kSPTile);
          sv = float4{sv.x + t.x, sv.y + t.y, sv.z + t.z, sv.w + t.w};
        }
        float v[4] = {sv.x, sv.y, sv.z, sv.w};
        float mx = -INFINITY;
        const int shift = (int)(reinterpret_cast<uintptr_t>(p.mask + (size_t)b * L) & 3);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int l = 4 * j + t;
          const bool in = l < L;
          const bool real = in && aux[shift + l] != 0;
          const float bl = (p.bias && in) ? reinterpret_cast<const float*>(aux + 256)[l] : 0.f;
          v[t] = in ? (real ? v[t] + bl : 1e-30f) : -INFINITY;   // model.py:180
          mx = fmaxf(mx, v[t]);
        }
        mx = row16_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          v[t] = (4 * j + t < L) ? act_exp<T>(v[t] - mx) : 0.f;
          sum += v[t];
        }
        sum = row16_sum(sum);
        const float inv = (k < K) ? 1.0f / sum : 0.f;
        *reinterpret_cast<uint2*>(Aw + k * AwS + 4 * j) = uint2{pack_bf16x2(v[0] * inv, v[1] * inv), pack_bf16x2(v[2] * inv, v[3] * inv)};
      } else {
        FRESH_LANE_IDS();
        const int l = lane;
        const bool in = l < L;
        const bool real = in && p.mask[(size_t)b * L + l] != 0;
        const float bl = (p.bias && in) ? p.bias[(size_t)b * L + l] : 0.f;
        constexpr int RK = kMaxK / kWaves;
        float v[RK], m[RK], ex[RK], sum[RK];
#pragma unroll
        for (int q = 0; q < RK; ++q) {
          const int k = wave + kWaves * q;
          float sv = S[k * kMaxL + l];
          if constexpr (kS1Coop)      // the four partials of the split S2
            sv = ((sv + S[(kMaxK + k) * kMaxL + l]) + S[(2 * kMaxK + k) * kMaxL + l]) + S[(3 * kMaxK + k) * kMaxL + l];
          v[q] = in ? (real ? sv + bl : 1e-30f) : -INFINITY;   // model.py:180
          m[q] = v[q];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
          for (int q = 0; q < RK; ++q) m[q] = fmaxf(m[q], __shfl_xor(m[q], o, 64));
#pragma unroll
        for (int q = 0; q < RK; ++q) { ex[q] = in ? act_exp<T>(v[q] - m[q]) : 0.f; sum[q] = ex[q]; }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
          for (int q = 0; q < RK; ++q) sum[q] += __shfl_xor(sum[q], o, 64);
#pragma unroll
        for (int q = 0; q < RK; ++q) {
          const int k = wave + kWaves * q;
          Aw[k * AwS + l] = from_f32<T>((k < K) ? ex[q] / sum[q] : 0.f);
        }
      }
      __syncthreads();
      STAMP(3);

      // ---- S4: mui = A · E  (rows k, columns i) ---------------------------------------------
      {
        FRESH_LANE_IDS();
        const int nLs = (L + 31) >> 5;
        Frag<T> af0, af1;
        frag_load(af0, Aw + r * AwS + 16 * h);
        if (nLs > 1) frag_load(af1, Aw + r * AwS + 32 + 16 * h); else frag_zero(af1);
#ifndef MINER_S4_PF
#define MINER_S4_PF 1   // fp32: the next d-tile's Eᵀ fragments (global loads) in flight during this tile's MFMAs
#endif
        if constexpr (!kBf16 && MINER_S4_PF) {
          // Eᵀ fragment of d-tile `it`: lane (h, r) holds column 32·it + r of history rows 32·ls + 16h + e
          // (rows >= L clamped: finite data times a zero weight). Every load unconditional (the tile index
          // clamped), so hipcc's vmcnt waits stay counted instead of draining to 0.
          auto load_e = [&](Frag<T>& bf, int it, int ls) {
            const int i0 = min(it, ns - 1) * 32;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int l = min(32 * ls + 16 * h + e, L - 1);
              bf.q[e >> 2][e & 3] = __float_as_uint(erow(l)[i0 + r]);
            }
          };
          // two stages: rows 32..63 of tile it load during the MFMAs on rows 0..31, and rows 0..31 of
          // tile it + 8 during those on rows 32..63 (one fragment in flight, no extra registers)
          Frag<T> b0, b1;
          load_e(b0, wave, 0);
          for (int it = wave; it < ns; it += kWaves) {
            const int i0 = it * 32;
            load_e(b1, it, 1);
            f32x16 acc = zero16();
            mma_f<T, X6 && (MINER_X6_STAGES & 2)>(acc, af0, b0);
            load_e(b0, it + kWaves, 0);
            if (nLs > 1) mma_f<T, X6 && (MINER_X6_STAGES & 2)>(acc, af1, b1);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int k = acc_row(e, h);
              muiL[k * msE + i0 + r] = from_f32<T>(acc[e]);
              if (p.mui_out && k < K) p.mui_out[((size_t)b * K + k) * d + i0 + r] = acc[e];
            }
          }
        } else
        for (int it = wave; it < ns; it += kWaves) {
          const int i0 = it * 32;
          f32x16 acc = zero16();
#pragma unroll
          for (int ls = 0; ls < 2; ++ls) {
            if (ls < nLs) {
              Frag<T> bf;
              const int lb = ls * 32;
              if constexpr (kBf16) {
                // Eᵀ fragment via ds_read_b64_tr_b16: lane group g = lane>>4 reads 4 rows x 16 cols
                const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
                // output lane j of group g receives column i0 + pi(16(g&1) + j) (A rows in pi order)
                const int col = i0 + 16 * (pp & 1) + 8 * (g & 1) + 4 * (pp >> 1);
                const int ch = col >> 3, sub8 = (col & 7) * 2;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
#pragma unroll
                  for (int u = 0; u < 2; ++u) {
                    const int row = lb + 16 * (g >> 1) + 8 * s + 4 * u + q;
                    const int off = (row < L) ? (p.offE + row * rowB + ((ch ^ eswz(row, g16)) << 4) + sub8) : p.offZ;
                    const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)((lds_char*)smem + off));
                    bf.q[s][2 * u] = (unsigned)(unsigned short)v[0] | ((unsigned)(unsigned short)v[1] << 16);
                    bf.q[s][2 * u + 1] = (unsigned)(unsigned short)v[2] | ((unsigned)(unsigned short)v[3] << 16);
                  }
                }
              } else {
#pragma unroll
                for (int e = 0; e < 16; ++e) {   // rows >= L: finite data times a zero weight
                  const int l = min(lb + 16 * h + e, L - 1);
                  bf.q[e >> 2][e & 3] = __float_as_uint(erow(l)[i0 + r]);
                }
              }
              if constexpr (kBf16) mma_slab<T>(acc, bf, ls == 0 ? af0 : af1);   // muiᵀ = Eᵀ·Aᵀ
              else mma_f<T, X6 && (MINER_X6_STAGES & 2)>(acc, ls == 0 ? af0 : af1, bf);
            }
          }
          if constexpr (kBf16) {
            // register e of lane (h, k) is muiᵀ[i0 + 16h + e][k]: 16 contiguous elements of row k
            Frag<T> mf;
            acc_to_frag(mf, acc);
            frag_store(muiL + r * msE + i0 + 16 * h, mf);
            if (p.mui_out && r < K) {
              float4* o = reinterpret_cast<float4*>(p.mui_out + ((size_t)b * K + r) * d + i0 + 16 * h);
#pragma unroll
              for (int g = 0; g < 4; ++g) o[g] = float4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
            }
          } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int k = acc_row(e, h);
              muiL[k * msE + i0 + r] = from_f32<T>(acc[e]);
              if (p.mui_out && k < K) p.mui_out[((size_t)b * K + k) * d + i0 + r] = acc[e];
            }
          }
        }
      }
      __syncthreads();  // history region free from here on
      if constexpr (kDma) {
        // This impression's candidate rows -> the (dead) history image, landing during S5.  Issued
        // before S5's ring: an untracked DMA issued inside the ring, older than later ring loads,
        // would make each of their waits cover its HBM latency too (measured: S5 +6K cycles).
        FRESH_LANE_IDS();
        if (need_scores && Cb > 0 && Cb <= kCChunk && ((Cb * rowB + 1023) & ~1023) <= p.eimg) {
          dma_rows(cand, Cb, d, ldsE, wave, lane, cids ? reinterpret_cast<const int32_t*>(aux + 768) : nullptr,
                   p.n_news);
          cimg = ldsE;
        }
        // the next impression's mask / bias / ids -> the other aux block (read by its DMAs and S3)
        if (bnext < p.B) dma_aux(p, bnext, auxn, wave, lane);
      }
      STAMP(4);
    } else {  // MODE == kTaa: multi_user_interest comes from global (query)
      FRESH_LANE_IDS();
      const T* __restrict__ qy = static_cast<const T*>(p.hist) + (size_t)b * K * d;
      const int per_row = d * (int)sizeof(T) / 16;
      __syncthreads();  // last impression's LDS reads done
      for (int i = tid; i < kMaxK * per_row; i += kThreads) {
        const int k = i / per_row, c = i - k * per_row;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (k < K) v = reinterpret_cast<const u32x4*>(qy + (size_t)k * d)[c];
        *reinterpret_cast<u32x4*>(smem + p.offMui + k * p.MS + c * 16) = v;
      }
      __syncthreads();
    }

    if (need_scores) {
      // ---- S5: X = gelu(W2 · muiᵀ), wave-owned d-tiles kept in registers ---------------------
      Frag<T> xf[kMaxJ];
      // kP2: each mui row's unit (s2L[32 + k], in the dead Aw region); mui scaled in place by its inverse
      float* s2L = reinterpret_cast<float*>(smem + p.offAw);
      if constexpr (kP2) {
        if (weighted) {
          FRESH_LANE_IDS();
          const int k = tid >> 4, c = tid & 15;     // 16 lanes (a DPP row) per mui row
          float mx = 0.f;
          for (int i = 4 * c; i < d; i += 64) {
            const float4 v = *reinterpret_cast<const float4*>(muiL + k * msE + i);
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          }
          mx = row16_max(mx);
          const int e = p2_exp(fminf(mx, 3.40282347e38f));
          if (c == 0) s2L[32 + k] = p2_unit_of(mx, e);
          // the row scaled in place (a power of two: exact) and an infinity clamped (p2_split2), once
          // here instead of in each wave's S5 split; S6 takes the units back from its products
          const float sc = p2_scale(e);
          for (int i = 4 * c; i < d; i += 64) {
            float4* q = reinterpret_cast<float4*>(muiL + k * msE + i);
            const float4 v = *q;
            *q = float4{p2_clamp(v.x * sc), p2_clamp(v.y * sc), p2_clamp(v.z * sc), p2_clamp(v.w * sc)};
          }
          __syncthreads();
        }
      }
      {
        FRESH_LANE_IDS();
        const int nm = (ns - wave + kWaves - 1) / kWaves;
        const T* w2s = kP2 ? W2x : W2p;
        if (weighted) {
          if (nm == 3) s5_gelu<T, PF, 3, X6, kP2>(xf, w2s, muiL, msE, d, wave, lane, u2, s2L);
          else if (nm == 2) s5_gelu<T, PF, 2, X6, kP2>(xf, w2s, muiL, msE, d, wave, lane, u2, s2L);
          else if (nm == 1) s5_gelu<T, PF, 1, X6, kP2>(xf, w2s, muiL, msE, d, wave, lane, u2, s2L);
        }
      }
      Frag<T> am[kMaxJ];   // bf16 full: the wave's mui fragments, held across the candidate chunks
      if constexpr (kDma) {
        FRESH_LANE_IDS();
        const int nm = (ns - wave + kWaves - 1) / kWaves;
#pragma unroll
        for (int m = 0; m < kMaxJ; ++m)
          if (m < nm) frag_load(am[m], muiL + r * msE + (wave + kWaves * m) * 32 + 16 * h);
      }
      if (cimg) { vm_wait_all(); __syncthreads(); }   // candidate rows landed for every wave
      STAMP_SYNC();
      STAMP(5);

      // ---- S6/S7 over candidate chunks ---------------------------------------------------------
      for (int cc = 0; cc < Cb; cc += kCChunk) {
        {
          FRESH_LANE_IDS();
          const int nm = (ns - wave + kWaves - 1) / kWaves;
          f32x16 lg[2], mt[2];
          lg[0] = lg[1] = mt[0] = mt[1] = zero16();
          if (weighted) s6_dispatch<T, true, MODE == kFull, X6>(nm, lg, mt, xf, am, cand, cimg, Cb, cc, d, wave, r, h, muiL, msE, cids, p.n_news);
          else s6_dispatch<T, false, MODE == kFull, X6>(nm, lg, mt, xf, am, cand, cimg, Cb, cc, d, wave, r, h, muiL, msE, cids, p.n_news);
          if constexpr (kP2) {
            // mui was scaled in place for S5 (weighted): its rows' units back on M (row k of the tile
            // in register e of lane half h: acc_row)
            if (weighted) {
              const float* un = reinterpret_cast<const float*>(smem + p.offAw) + 32;
#pragma unroll
              for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int e = 0; e < 16; ++e) mt[ct][e] *= un[acc_row(e, h)];
            }
          }
          STAMP_SYNC();
          STAMP(6);
          if constexpr (kDma) {
            // the partial slabs overwrite mui; every wave is done with mui and the candidate image;
            // the next impression's aux (its history ids) has landed for every wave
            vm_wait_all();
            __syncthreads();
            if (cimg && bnext < p.B && !DBG(4)) {   // single chunk: next impression's history now
              dma_rows(static_cast<const T*>(p.hist) + (his_ids ? 0 : (size_t)bnext * L * d), L, d, ldsE, wave, lane,
                       his_ids ? reinterpret_cast<const int32_t*>(auxn + 512) : nullptr, p.n_news);
              prefetched = true;
            }
          }
          // fp32: the last chunk (TAA: every chunk) reduces through the dead mui region with plain
          // stores like bf16; the earlier chunks of a C > 64 impression still read mui, so they sum
          // into Lg / Mt with LDS atomics (~190 cycles each: 18 % of the kernel when every chunk did)
          const bool plain = kBf16 || (p.part_ok && (MODE == kTaa || cc + kCChunk >= Cb));
          if (!kBf16 && plain) __syncthreads();   // every wave's mui reads (S6 products) done
          if (plain) {
            s6_reduce_bf16(part, lg, mt, wave, r, h, DBG(3));
          } else {
            if (nm > 0) {
#pragma unroll
              for (int ct = 0; ct < 2; ++ct) {
                if (cc + ct * 32 < Cb) {
#pragma unroll
                  for (int e = 0; e < 16; ++e) {
                    const int k = acc_row(e, h);
                    if (weighted) atomicAdd(&Lg[k * kLgS + ct * 32 + r], lg[ct][e]);
                    if (MODE == kFull) atomicAdd(&Mt[k * kLgS + ct * 32 + r], mt[ct][e]);
                  }
                }
              }
            }
          }
        }
        __syncthreads();
        STAMP(7);
        // S7: 8 lanes per candidate, 4 interests per lane
        {
          FRESH_LANE_IDS();
          const int cl = tid >> 3, sub = tid & 7;
          const int c = cc + cl;
          const bool cval = c < Cb;
          float lgv[4], mtv[4];
          if (kBf16 || (p.part_ok && (MODE == kTaa || cc + kCChunk >= Cb))) {
            s7_load_bf16(part, cl, sub, lgv, mtv);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int k = 4 * sub + j;
              lgv[j] = Lg[k * kLgS + cl];
              mtv[j] = Mt[k * kLgS + cl];
              Lg[k * kLgS + cl] = 0.f;
              Mt[k * kLgS + cl] = 0.f;
            }
          }
          bool kv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int k = 4 * sub + j;
            kv[j] = k < K;
            if (MODE == kTaa) mtv[j] = (cval && kv[j]) ? p.value[(size_t)(cbase + c) * K + k] : 0.f;
          }
          const float sc = s7_score<T>(lgv, mtv, kv, p.score_type, K);
          if (sub == 0 && cval) p.scores[cbase + c] = sc;
        }
        __syncthreads();
        STAMP(8);
      }
    }

    if constexpr (kDma) {
      FRESH_LANE_IDS();
      if (!prefetched && bnext < p.B && !DBG(4)) {   // the history region is free now
        vm_wait_all();
        __syncthreads();   // the next impression's aux (history ids) landed for every wave
        dma_rows(static_cast<const T*>(p.hist) + (his_ids ? 0 : (size_t)bnext * L * d), L, d, ldsE, wave, lane,
                 his_ids ? reinterpret_cast<const int32_t*>(auxn + 512) : nullptr, p.n_news);
      }
    }
    STAMP(9);
  }
  STAMP_FLUSH(n_done);
}

// ---------------------------------------------------------------------------------------------
// weight packing
// ---------------------------------------------------------------------------------------------

template <class T>
__global__ void pack_weights_kernel(const T* __restrict__ W1, const T* __restrict__ Q, const T* __restrict__ W2,
                                    int d, int Dc, int K, T* __restrict__ out) {
  const size_t n1 = w1p_elems(d, Dc), nq = qp_elems(Dc), n2 = W2 ? w2p_elems(d) : 0;
  const int ns = d >> 5, nct = n_ctiles(Dc);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + nq + n2; i += (size_t)gridDim.x * blockDim.x) {
    T v = (T)0.f;
    if (i < n1) {
      const size_t tile = i >> 10;
      int rr, cc;
      block_pos<T>((int)(i & 1023), rr, cc);
      const int ct = (int)(tile / ns), j = (int)(tile % ns);
      const int row = ct * 32 + pi_row(rr);
      if (row < Dc) v = W1[(size_t)row * d + j * 32 + cc];
    } else if (i < n1 + nq) {
      const size_t q = i - n1;
      const int k = (int)(q / (nct * 32)), c = (int)(q % (nct * 32));
      if (k < K && c < Dc) v = Q[(size_t)k * Dc + c];
    } else {
      const size_t q = i - n1 - nq;
      const size_t tile = q >> 10;
      int rr, cc;
      block_pos<T>((int)(q & 1023), rr, cc);
      const int jt = (int)(tile / ns), j = (int)(tile % ns);
      v = W2[(size_t)(jt * 32 + pi_row(rr)) * d + j * 32 + cc];
    }
    out[i] = v;
  }
}

// fp32 W2 as fp16 pairs: row units (one thread per row), then the pair tiles — the fp32 tiles'
// fragment-major geometry (a 16-byte piece per lane and q), piece 2st + plane of lane l holding
// plane (hi, lo) of that lane's elements 8st..8st+7: [16 (l >> 5) + 8st, +8) of tile row pi(l & 31)
// W [rows, d] row-major; units for the padded rows (up to 32 per tile) are 1, their pieces 0
__global__ void pair_units_kernel(const float* __restrict__ W, int rows, int rows_pad, int cols,
                                  float* __restrict__ units) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_pad) return;
  float mx = 0.f;
  if (i < rows)
    for (int j = 0; j < cols; ++j) mx = fmaxf(mx, fabsf(W[(size_t)i * cols + j]));
  units[i] = i < rows ? p2_unit_of(mx, p2_exp(fminf(mx, 3.40282347e38f))) : 1.0f;
}
__global__ void pack_pairs_kernel(const float* __restrict__ W, const float* __restrict__ units, int rows, int ntr,
                                  int d, u32x4* __restrict__ out) {
  const int ns = d >> 5;
  const size_t n = (size_t)ntr * ns * 256;          // 16-byte pieces
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t tile = i >> 8;
    const int q = (int)((i >> 6) & 3), l = (int)(i & 63);
    const int st = q >> 1, plane = q & 1;
    const int jt = (int)(tile / ns), j = (int)(tile % ns);
    const int row = jt * 32 + pi_row(l & 31);
    const int c0 = j * 32 + 16 * (l >> 5) + 8 * st;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (row < rows) {
      const float s = 1.0f / units[row];             // a power of two: exact
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        unsigned hi, lo;
        p2_split2(W[(size_t)row * d + c0 + 2 * m] * s, W[(size_t)row * d + c0 + 2 * m + 1] * s, hi, lo);
        v[m] = plane ? lo : hi;
      }
    }
    out[i] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
inline int round16(int x) { return (x + 15) & ~15; }

struct Carve {
  int MS, PS, offE, offZ, offP, offS, offMui, offAw, offPart, offLg, offMt, offAux, eimg, total;
  int part_ok;
  int offS1;
};

// LDS carve (bytes).
//   bf16 full:  [history image (partial slabs alias it after S4) | zero block | mui (P, S alias it
//               before S4) | Aw]
//   fp32 full:  [Lg Mt | mui (P, S alias) | Aw]
//   bf16 TAA:   [partial slabs | mui];   fp32 TAA: [Lg Mt | mui]
Carve carve(int dtype, int mode, int L, int d, int Dc) {
  Carve c{};
  const bool bf = dtype == MINER_DTYPE_BF16;
  const int es = bf ? 2 : 4;
  const int lgmt = 2 * kMaxK * kLgS * 4;
  const int parts = 4 * kPartWave * 4;
  c.MS = d * es + 16;
  c.PS = n_ctiles(Dc) * 32 + (bf ? 8 : 4);
  const int pbytes = round16(64 * c.PS * es);
  const int r2a = 32 * c.MS;
  int r2b = bf ? n_ctiles(Dc) * kSPTile * 4 : pbytes + kMaxK * kMaxL * 4;
  if (parts > r2b) r2b = parts;            // the S6 partial slabs live here too (after the mui reads)
  // TAA keeps its mui region at r2a (bf16 TAA has its partial slabs in front of mui, r1). fp32 TAA
  // reduces through it with plain stores only where it holds the slabs (d >= ~570); below, the
  // chunks sum with LDS atomics, so the carve (and the two workgroups per CU it allows at small d)
  // does not grow
  const int r2 = round16(mode == kFull ? (r2a > r2b ? r2a : r2b) : r2a);
  c.part_ok = bf || mode == kFull || r2a >= parts;
  const int aw = mode == kFull ? (bf ? 32 * 72 * 2 : 32 * 68 * 4) : 0;
  int off = 0;
  if (bf) {
    const int eimg = mode == kFull ? (L * d * 2 + 1023) & ~1023 : 0;   // whole 1 KiB DMA blocks
    c.offE = 0;
    c.eimg = eimg;
    c.offPart = 0;                                  // TAA: [partial slabs | mui]
    const int r1 = mode == kFull ? eimg : parts;
    c.offZ = round16(r1);
    c.offAux = c.offZ + 64;                         // 2 aux blocks (mask | bias | ids), by parity
    off = mode == kFull ? c.offAux + 2 * kAuxBytes : c.offZ;
    c.offLg = c.offMt = 0;
  } else {
    c.offE = c.offZ = c.offPart = 0;
    c.offLg = 0;
    c.offMt = kMaxK * kLgS * 4;
    off = lgmt;
  }
  c.offMui = round16(off);
  c.offP = c.offMui;                       // P lives in the mui region until S4 overwrites it
  c.offS = bf ? c.offMui : c.offMui + pbytes;   // S too (bf16: the per-wave S partials of S1)
  if (bf && mode == kFull) c.offPart = c.offMui;   // full: after S6 products mui is dead
  if (!bf) c.offPart = c.offMui;                   // fp32: the last chunk's partials (after its products)
  c.offAw = round16(c.offMui + r2);
  c.total = c.offAw + aw;
  if (!bf && mode == kFull && MINER_S1_COOP && (MINER_X6_STAGES & 1) && c.total > kLdsMax / 2) {
    // the S1 history-operand planes: in the mui region behind P and S (free until S4; P is written
    // after the S1 loop, S in S2), running on into Aw (written in S3) and past it where needed; only
    // where the carve already holds one workgroup per CU (the planes would cost a second one)
    c.offS1 = round16(c.offS + kMaxK * kMaxL * 4);
    if (c.offS1 + kS1Bytes > c.total) c.total = c.offS1 + kS1Bytes;
  }
  if (!bf && mode == kFull) {   // fp32 gather mode: the impression's history ids (read during S1: after its planes)
    c.offAux = round16(c.total);
    c.total = c.offAux + kMaxL * 4;
  }
  return c;
}

int check_shape(int dtype_in, int mode, int L, int d, int Dc, int K) {
  const int dtype = dtype_in == MINER_DTYPE_F32_MFMA ? MINER_DTYPE_F32 : dtype_in;
  if (dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) return MINER_EINVAL;
  if (d <= 0 || K <= 0) return MINER_EINVAL;
  if (mode == kFull && (L <= 0 || Dc <= 0)) return MINER_EINVAL;
  if (K > kMaxK || d % 32 != 0 || d > kMaxD) return MINER_ESHAPE;
  if (dtype == MINER_DTYPE_BF16 && mode == kFull && d % 64 != 0) return MINER_ESHAPE;
  if (mode == kFull && (L > kMaxL || Dc > kMaxDc)) return MINER_ESHAPE;
  if (carve(dtype, mode, L, d, mode == kFull ? Dc : 1).total > kLdsMax) return MINER_ELDS;
  return MINER_OK;
}

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

inline bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <class T, int MODE, int NS, bool GATHER = false, int SHP = 0, bool X6 = false, bool S1C = false>
int launch(void* stream, const Params& prm, int lds) {
  auto kern = miner_fused<T, MODE, NS, GATHER, SHP, X6, S1C>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return (int)e;
  const int per_cu = kLdsMax / lds > 0 ? (kLdsMax / lds > 2 ? 2 : kLdsMax / lds) : 1;
  int grid = num_cus() * per_cu;
  if (grid > prm.B) grid = prm.B;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

// MINER_DTYPE_F32_MFMA is MINER_DTYPE_F32 with every product on the fp32 MFMA (exact fp32 fma
// chains) instead of the bf16x6 default: the same operands, layouts and carve
int base_dtype(int dtype) { return dtype == MINER_DTYPE_F32_MFMA ? MINER_DTYPE_F32 : dtype; }

int run(void* stream, int dtype_in, int mode, Params prm) {
  const bool exact32 = dtype_in == MINER_DTYPE_F32_MFMA;
  const int dtype = base_dtype(dtype_in);
#ifdef MINER_STAMPS
  if (const char* e = getenv("MINER_DBG")) prm.dbg = atoi(e);
#endif
  const Carve c = carve(dtype, mode, prm.L, prm.d, prm.Dc);
  prm.MS = c.MS; prm.PS = c.PS; prm.offE = c.offE; prm.offZ = c.offZ; prm.offP = c.offP; prm.offS = c.offS;
  prm.offMui = c.offMui; prm.offAw = c.offAw; prm.offPart = c.offPart; prm.offLg = c.offLg; prm.offMt = c.offMt;
  prm.offAux = c.offAux; prm.eimg = c.eimg; prm.part_ok = c.part_ok; prm.offS1 = c.offS1;
  const bool gather = prm.his_ids != nullptr;
  if (dtype == MINER_DTYPE_BF16) {
    // config 3's model (d = 768, history 50, Dc = 200, K = 32), dense rows: the shape compile-time
    if (prm.d == 768 && mode == kFull && !gather && prm.L == 50 && prm.Dc == 200 && prm.K == 32)
      return launch<__bf16, kFull, 24, false, 1>(stream, prm, c.total);
    // bf16 kernels specialised on the embedding dim (d = 32*NS) so the slab loops fully unroll
    switch (prm.d) {
#define MINER_NS_CASE(ns)                                                                        \
  case 32 * ns:                                                                                  \
    if (mode == kTaa) return launch<__bf16, kTaa, ns>(stream, prm, c.total);                     \
    return gather ? launch<__bf16, kFull, ns, true>(stream, prm, c.total) : launch<__bf16, kFull, ns>(stream, prm, c.total);
      MINER_NS_CASE(2) MINER_NS_CASE(4) MINER_NS_CASE(6) MINER_NS_CASE(8) MINER_NS_CASE(12)
      MINER_NS_CASE(16) MINER_NS_CASE(24)
#undef MINER_NS_CASE
      default:
        if (mode == kTaa) return launch<__bf16, kTaa, 0>(stream, prm, c.total);
        return gather ? launch<__bf16, kFull, 0, true>(stream, prm, c.total) : launch<__bf16, kFull, 0>(stream, prm, c.total);
    }
  }
  // fp32: bf16x6 products by default, the exact fp32-MFMA form for MINER_DTYPE_F32_MFMA
  if (exact32) {
    if (mode == kTaa) return launch<float, kTaa, 0>(stream, prm, c.total);
    return gather ? launch<float, kFull, 0, true>(stream, prm, c.total) : launch<float, kFull, 0>(stream, prm, c.total);
  }
  if (mode == kTaa) return launch<float, kTaa, 0, false, 0, true>(stream, prm, c.total);
  if (c.offS1 > 0)
    return gather ? launch<float, kFull, 0, true, 0, true, true>(stream, prm, c.total)
                  : launch<float, kFull, 0, false, 0, true, true>(stream, prm, c.total);
  return gather ? launch<float, kFull, 0, true, 0, true>(stream, prm, c.total) : launch<float, kFull, 0, false, 0, true>(stream, prm, c.total);
}

// fp32: [W1p | Qp | W2p | W2 pair-packed | W2 row units | W1 pair-packed | W1 row units (n_ctiles·32)];
// bf16: [W1p | Qp | W2p]
size_t packed_bytes(int dtype, int d, int Dc) {
  const size_t es = dtype == MINER_DTYPE_BF16 ? 2 : 4;
  const size_t pairs = dtype == MINER_DTYPE_BF16 ? 0 : w2p_elems(d) + (size_t)d + w1p_elems(d, Dc) + qp_elems(Dc) / 32;
  return (w1p_elems(d, Dc) + qp_elems(Dc) + w2p_elems(d) + pairs) * es;
}

}  // namespace

extern "C" {

size_t miner_packed_weights_bytes(int dtype, int d, int Dc, int K) {
  if ((dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) || d <= 0 || d % 32 || Dc <= 0 || K <= 0 || K > kMaxK)
    return 0;
  return packed_bytes(dtype, d, Dc);
}

int miner_pack_weights(void* stream, int dtype, const void* w_poly, const void* context_codes, const void* w_target,
                       int d, int Dc, int K, void* packed) {
  if (dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) return MINER_EINVAL;
  if (d <= 0 || Dc <= 0 || K <= 0) return MINER_EINVAL;
  if (d % 32 || K > kMaxK || Dc > kMaxDc || d > kMaxD) return MINER_ESHAPE;
  if (!w_poly || !context_codes || !packed) return MINER_EINVAL;
  if (!aligned16(packed)) return MINER_EALIGN;
  const size_t n = w1p_elems(d, Dc) + qp_elems(Dc) + (w_target ? w2p_elems(d) : 0);
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  if (dtype == MINER_DTYPE_BF16)
    hipLaunchKernelGGL(pack_weights_kernel<__bf16>, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const __bf16*>(w_poly), static_cast<const __bf16*>(context_codes),
                       static_cast<const __bf16*>(w_target), d, Dc, K, static_cast<__bf16*>(packed));
  else {
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(pack_weights_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<const float*>(w_poly),
                       static_cast<const float*>(context_codes), static_cast<const float*>(w_target), d, Dc, K,
                       static_cast<float*>(packed));
    // the fp16-pair copies of W2 (S5) and W1 (S1) with their row units
    float* w2x = static_cast<float*>(packed) + w1p_elems(d, Dc) + qp_elems(Dc) + w2p_elems(d);
    float* u2 = w2x + w2p_elems(d);
    float* w1x = u2 + d;
    float* u1 = w1x + w1p_elems(d, Dc);
    auto pairs = [&](const float* W, int rows, int ntr, float* x, float* units) {
      hipLaunchKernelGGL(pair_units_kernel, dim3((ntr * 32 + 255) / 256), dim3(256), 0, s, W, rows, ntr * 32, d, units);
      const size_t pieces = (size_t)ntr * (d >> 5) * 256;
      const int g2 = (int)((pieces + 255) / 256 < 4096 ? (pieces + 255) / 256 : 4096);
      hipLaunchKernelGGL(pack_pairs_kernel, dim3(g2), dim3(256), 0, s, W, units, rows, ntr, d, reinterpret_cast<u32x4*>(x));
    };
    if (w_target) pairs(static_cast<const float*>(w_target), d, d >> 5, w2x, u2);
    pairs(static_cast<const float*>(w_poly), Dc, n_ctiles(Dc), w1x, u1);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

size_t miner_target_weights_bytes(int dtype, int d) {
  if ((dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) || d <= 0 || d % 32 || d > kMaxD) return 0;
  return w2p_elems(d) * (dtype == MINER_DTYPE_BF16 ? 2 : 4);
}

// W2 alone (TargetAwareAttention.linear.weight, model.py:198) in the tiled layout: the packed
// buffer of miner_pack_weights with an empty PolyAttention part (Dc = 0), for miner_target_aware
int miner_pack_target_weights(void* stream, int dtype, const void* w_target, int d, void* packed) {
  if (dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) return MINER_EINVAL;
  if (d <= 0 || !w_target || !packed) return MINER_EINVAL;
  if (d % 32 || d > kMaxD) return MINER_ESHAPE;
  if (!aligned16(packed)) return MINER_EALIGN;
  const size_t n = w2p_elems(d);
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  if (dtype == MINER_DTYPE_BF16)
    hipLaunchKernelGGL(pack_weights_kernel<__bf16>, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       nullptr, nullptr, static_cast<const __bf16*>(w_target), d, 0, 0, static_cast<__bf16*>(packed));
  else
    hipLaunchKernelGGL(pack_weights_kernel<float>, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       nullptr, nullptr, static_cast<const float*>(w_target), d, 0, 0, static_cast<float*>(packed));
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

int miner_score(void* stream, int dtype, int score_type, const void* history, const uint8_t* his_mask,
                const float* his_bias, const void* candidates, const int32_t* cand_offsets,
                const void* packed_weights, int B, int L, int C, int d, int Dc, int K, float* scores,
                float* user_out) {
  if (score_type < MINER_SCORE_WEIGHTED || score_type > MINER_SCORE_NONE) return MINER_EINVAL;
  if (B < 0 || C < 0) return MINER_EINVAL;
  const int sh = check_shape(dtype, kFull, L, d, Dc, K);
  if (sh != MINER_OK) return sh;
  if (!history || !his_mask || !packed_weights) return MINER_EINVAL;
  if (score_type != MINER_SCORE_NONE && (!candidates || !scores)) return MINER_EINVAL;
  if (score_type == MINER_SCORE_NONE && !user_out) return MINER_EINVAL;
  if (!aligned16(history) || !aligned16(candidates) || !aligned16(packed_weights)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  Params prm{};
  prm.hist = history; prm.mask = his_mask; prm.bias = his_bias; prm.cand = candidates;
  prm.cand_off = cand_offsets; prm.wp = packed_weights; prm.value = nullptr; prm.scores = scores;
  prm.mui_out = user_out;
  prm.B = B; prm.L = L; prm.C = C; prm.d = d; prm.Dc = Dc; prm.K = K; prm.score_type = score_type;
  return run(stream, dtype, kFull, prm);
}

int miner_score_gather(void* stream, int dtype, int score_type, const void* news_table, int n_news,
                       const int32_t* his_ids, const uint8_t* his_mask, const float* his_bias,
                       const int32_t* cand_ids, const int32_t* cand_offsets, const void* packed_weights,
                       int B, int L, int C, int d, int Dc, int K, float* scores, float* user_out) {
  if (score_type < MINER_SCORE_WEIGHTED || score_type > MINER_SCORE_NONE) return MINER_EINVAL;
  if (B < 0 || C < 0 || n_news <= 0) return MINER_EINVAL;
  const int sh = check_shape(dtype, kFull, L, d, Dc, K);
  if (sh != MINER_OK) return sh;
  if (!news_table || !his_ids || !his_mask || !packed_weights) return MINER_EINVAL;
  if (score_type != MINER_SCORE_NONE && (!cand_ids || !scores)) return MINER_EINVAL;
  if (score_type == MINER_SCORE_NONE && !user_out) return MINER_EINVAL;
  if (!aligned16(news_table) || !aligned16(packed_weights)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  Params prm{};
  prm.hist = news_table; prm.mask = his_mask; prm.bias = his_bias; prm.cand = news_table;
  prm.cand_off = cand_offsets; prm.wp = packed_weights; prm.value = nullptr; prm.scores = scores;
  prm.mui_out = user_out; prm.his_ids = his_ids; prm.cand_ids = score_type != MINER_SCORE_NONE ? cand_ids : nullptr;
  prm.n_news = n_news;
  prm.B = B; prm.L = L; prm.C = C; prm.d = d; prm.Dc = Dc; prm.K = K; prm.score_type = score_type;
  return run(stream, dtype, kFull, prm);
}

int miner_target_aware(void* stream, int dtype, const void* query, const void* key, const float* value,
                       const int32_t* cand_offsets, const void* packed_weights, int Dc, int B, int C, int d, int K,
                       float* out) {
  if (B < 0 || C < 0 || Dc < 0) return MINER_EINVAL;     // Dc = 0: a miner_pack_target_weights buffer
  const int sh = check_shape(dtype, kTaa, 1, d, 1, K);
  if (sh != MINER_OK) return sh;
  if (!query || !key || !value || !packed_weights || !out) return MINER_EINVAL;
  if (!aligned16(query) || !aligned16(key) || !aligned16(packed_weights)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  Params prm{};
  prm.hist = query; prm.mask = nullptr; prm.bias = nullptr; prm.cand = key; prm.cand_off = cand_offsets;
  prm.wp = packed_weights; prm.value = value; prm.scores = out; prm.mui_out = nullptr;
  prm.B = B; prm.L = 1; prm.C = C; prm.d = d; prm.Dc = Dc; prm.K = K; prm.score_type = MINER_SCORE_WEIGHTED;
  return run(stream, dtype, kTaa, prm);
}

int miner_supported(int dtype, int L, int d, int Dc, int K) { return check_shape(dtype, kFull, L, d, Dc, K); }

int miner_lds_bytes(int dtype, int score_type, int L, int d, int Dc) {
  (void)score_type;
  return carve(base_dtype(dtype), kFull, L, d, Dc).total;
}

const char* miner_strerror(int code) {
  switch (code) {
    case MINER_OK: return "ok";
    case MINER_EINVAL: return "invalid argument (null pointer, bad enum or non-positive size)";
    case MINER_ESHAPE: return "shape not supported by this build (K<=32, L<=64, Dc<=256, d%32==0 (bf16: d%64==0), d<=768)";
    case MINER_EALIGN: return "device pointer not 16-byte aligned";
    case MINER_ELDS: return "shape needs more LDS than one CU has (160 KiB)";
    default: return code > 0 ? hipGetErrorString(static_cast<hipError_t>(code)) : "unknown error";
  }
}

int miner_abi_version(void) { return MINER_ABI_VERSION; }

#ifdef MINER_STAMPS
// diagnostic build only: read (and reset) the per-stage cycle sums; out[0..11] cycles, out[12] impressions
int miner_debug_stage_cycles(unsigned long long* out) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stage_cycles), 12 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 12, HIP_SYMBOL(g_stage_imps), sizeof(unsigned long long));
  unsigned long long z[16] = {0};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_stage_cycles), z, 16 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_stage_imps), z, sizeof(unsigned long long));
  return (int)e;
}
#endif

}  // extern "C"
