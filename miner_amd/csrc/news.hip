// news.hip — MINER scoring from news ids with a news-side precompute, MI355X
// (gfx950 / CDNA4). Two kernels:
//
//   news_pre   per news row n of the table (one workgroup per 64 rows, 32 in fp32):
//                logits[n] = tanh(W1·e_n)·Qᵀ       (model.py:171-174)           fp32 [n_news, K]
//                proj[n]   = W2·e_n                 (model.py:212, pre-GELU)     T    [n_news, d]
//              the rows of the tile are staged in LDS (LDS-DMA, XOR-swizzled), the packed weight
//              tiles (miner_pack_weights) stream from L2 through a register ring: wave w owns the
//              output column tiles w, w+8, ... of [W1 (Dc) | W2 (d)]; the W1 tiles go on through
//              tanh and their Q contraction in registers, the per-tile logit partials are summed
//              through LDS in a fixed order.
//
//   news_score per impression (one persistent workgroup of 8 waves per CU), from the history /
//              candidate ids:
//                A   = softmax_L(logits[his] + bias, masked slots = 1e-30)   (model.py:176-181)
//                mui = A·E[his]                                              (model.py:182)
//                X   = gelu(A·proj[his])  = gelu(mui·W2ᵀ)                    (model.py:212)
//                M   = Cand·muiᵀ,  Lg = Cand·Xᵀ                              (model.py:127, :213)
//                score = Σ_k softmax_k(Lg)·M  | max_k M | mean_k M           (model.py:128-136, :214)
//              No weight is touched per impression: the kernel is a gather stream. The history rows
//              of E and proj and the candidate rows are streamed in 64-column chunks through a ring
//              of LDS slots (LDS-DMA by id, one 128-byte line per row per chunk in bf16), PD chunks
//              in flight, one barrier per chunk. Per chunk wave w = (path P, slab sl, cand tile ct):
//                P = 0:  muiᵀ[slab] = E[his]ᵀ·Aᵀ  (4 MFMA, E read transposed with
//                        ds_read_b64_tr_b16), then M[ct] += Cand[ct]·muiᵀ[slab]
//                P = 1:  Xᵀ[slab] = gelu(proj[his]ᵀ·Aᵀ), then Lg[ct] += Cand[ct]·Xᵀ[slab]
//              The accumulator of a product is the operand of the next (rows taken in pi order, see
//              cdna4_common.h): nothing but the rows themselves goes through LDS. The per-impression
//              ids, mask, bias and logit rows ride in small LDS "aux" blocks, DMA'd one to three
//              impressions ahead, so no load the compiler can see is ever waited on in the loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>

#include "../../include/miner_news.h"
#include "cdna4_common.h"

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kMaxL = 64;
constexpr int kMaxK = 32;
constexpr int kMaxCand = MINER_NEWS_MAX_CAND;
constexpr int kMaxD = 1024;
constexpr int kMaxDc = 256;
constexpr int kLdsMax = 160 * 1024;

__device__ __forceinline__ void raw_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <class T> __device__ __forceinline__ float nx_exp(float x) {
  if constexpr (sizeof(T) == 2) return __expf(x); else return expf(x);
}
template <class T> __device__ __forceinline__ float nx_tanh(float x) {
  if constexpr (sizeof(T) == 2) return tanh_fast(x); else return tanhf(x);
}

// 32-lane (one half of the wave) all-reduce: DPP inside the 16-lane rows, then rows 0<->1, 2<->3
__device__ __forceinline__ float half_max(float x) {
  x = row16_max(x);
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  x = row16_sum(x);
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
// combine the two lane halves (permlane32_swap of x with itself: one result holds the low half's
// value in every lane, the other the high half's)
__device__ __forceinline__ float both_max(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float both_sum(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// all-reduce over the 4 16-lane rows (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float rows4_max(float x) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return both_max(fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1])));
}
__device__ __forceinline__ float rows4_sum(float x) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return both_sum(__uint_as_float(s[0]) + __uint_as_float(s[1]));
}

__device__ __forceinline__ uint32_t lds_u32(const char* p) { return *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ u32x4 lds_u32x4(const char* p) { return *reinterpret_cast<const u32x4*>(p); }

#ifndef NS_ABL
#define NS_ABL 0         // timing ablations of news_score (wrong scores): 2 no row DMAs, 4 no products
#endif
#ifndef NS_EARLY
#define NS_EARLY 0       // 1: operand reads issued before the chunk's row DMAs (measured 25 % slower at d = 768)
#endif
// wait until at most N LDS operations are in flight, the 4 transposed pieces of a slab tied to it
template <int N>
__device__ __forceinline__ void ns_wait_tr(uint2 (&r)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]) : "i"(N));
}
template <int NT>
__device__ __forceinline__ void ns_wait_c(u32x4 (&c)[NT][2]) {
  if constexpr (NT == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c[0][0]), "+v"(c[0][1]));
  else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c[0][0]), "+v"(c[0][1]), "+v"(c[1][0]), "+v"(c[1][1]));
}

// LDS-DMA of 16 bytes per lane with the default cache policy (table rows may be re-read by other
// impressions: keep them in L2 / the Infinity Cache)
__device__ __forceinline__ void dma_b128_c(const void* g, unsigned lds) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(g), "s"(lds) : "memory");
}

// ================================================================================================
// per-news precompute
// ================================================================================================
// packed weight layout of miner_pack_weights (miner_score.hip): [W1p | Qp | W2p]
__host__ __device__ inline int n_ct(int Dc) { return (Dc + 31) >> 5; }
__host__ __device__ inline size_t w1p_el(int d, int Dc) { return (size_t)n_ct(Dc) * (d >> 5) * 1024; }
__host__ __device__ inline size_t qp_el(int Dc) { return (size_t)n_ct(Dc) * 1024; }

struct PreParams {
  const void* table;
  const void* wp;
  float* logits;   // [N, K]
  void* proj;      // [N, d] or null
  int N, d, Dc, K;
};

// fp16 pairs for the fp32 precompute (miner_score.hip's operand form, §4 "Round 6"): a row with
// max|row| < 2^e is carried as x·2^(14-e) = hi + lo, hi = f16, lo = f16(residual), and a product as
// lo·hi + hi·lo + hi·hi on v_mfma_f32_32x32x16_f16; the accumulator is rescaled by the two rows'
// units 2^(e-14) (powers of two: exact). The weights' pair copies and units are the ones
// miner_pack_weights writes for fp32 after W2p: [W2x | u2 (d) | W1x | u1 (32 nct)].
__device__ __forceinline__ int pre_p2_exp(float mx) {
  int e;
  frexpf(mx, &e);
  return e < -100 ? -100 : (e > 128 ? 128 : e);
}
__device__ __forceinline__ f32x16 pre_mfma_f16(const u32x4& a, const u32x4& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// acc += A·B over one 32-wide slab: A a pair-packed weight tile fragment (pieces {hi, lo} of elements
// 0..7, then of 8..15), B an fp32 fragment already scaled into |x| ≤ 65504, cut here
__device__ __forceinline__ void pre_slab_p2(f32x16& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    u32x4 bh, bl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = 8 * st + 2 * i;
      const float x0 = __uint_as_float(b.q[e >> 2][e & 3]), x1 = __uint_as_float(b.q[(e + 1) >> 2][(e + 1) & 3]);
      const f16x2v hv = __builtin_convertvector((f32x2v){x0, x1}, f16x2v);
      unsigned hb = __builtin_bit_cast(unsigned, hv);
      asm volatile("" : "+v"(hb));
      const f16x2v hh = __builtin_bit_cast(f16x2v, hb);
      bh[i] = hb;
      bl[i] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){x0 - (float)hh[0], x1 - (float)hh[1]}, f16x2v));
    }
    acc = pre_mfma_f16(a.q[2 * st + 1], bh, acc);
    acc = pre_mfma_f16(a.q[2 * st], bl, acc);
    acc = pre_mfma_f16(a.q[2 * st], bh, acc);
  }
}

template <class T> constexpr int kPreRows = sizeof(T) == 2 ? 64 : 32;   // news rows per tile

// XOR swizzle of the 16-byte chunks of a tile row (cpr chunks per row, a multiple of 8): the 16
// rows of a ds_read_b128 lane group land in 16 different bank slots
__device__ __forceinline__ int pre_swz(int row, int cpr) { return (cpr & 15) ? (row & 7) : (row & 15); }

// P2 (fp32 only, MINER_DTYPE_F32): the W1 / W2 products on fp16 pairs (pre_slab_p2) with the
// pair copies of the packed weights and one unit per table row (the staged rows scaled in place);
// !P2: every product on the fp32 MFMA (MINER_DTYPE_F32_MFMA)
template <class T, int NS, bool P2 = false>
__global__ __launch_bounds__(kThreads) void news_pre(PreParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(!P2 || sizeof(T) == 4, "pairs: fp32 tables");
  constexpr int R = kPreRows<T>;
  constexpr int NRT = R / 32;
  const int d = p.d;
  const int ns = NS > 0 ? NS : (d >> 5);
  const int nct = n_ct(p.Dc);
  const int J = nct + (p.proj ? ns : 0);
  const int rowB = d * (int)sizeof(T);
  const int cpr = rowB >> 4;
  const int imgB = R * rowB;
  char* img = smem;
  float* xch = reinterpret_cast<float*>(smem + imgB);     // [nct][NRT][16 regs][64 lanes]
  float* uE = xch + (size_t)nct * NRT * 16 * 64;          // P2: the staged rows' units
  const T* __restrict__ W1p = static_cast<const T*>(p.wp);
  const T* __restrict__ Qp = W1p + w1p_el(d, p.Dc);
  const T* __restrict__ W2p = Qp + qp_el(p.Dc);
  const T* __restrict__ W2x = W2p + (size_t)(d >> 5) * (d >> 5) * 1024;
  const float* __restrict__ u2 = reinterpret_cast<const float*>(W2x + (size_t)(d >> 5) * (d >> 5) * 1024);
  const T* __restrict__ W1x = reinterpret_cast<const T*>(u2 + d);
  const float* __restrict__ u1 = reinterpret_cast<const float*>(W1x + w1p_el(d, p.Dc));
  const T* __restrict__ tab = static_cast<const T*>(p.table);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (p.N + R - 1) / R;
  const unsigned sbase = __builtin_amdgcn_readfirstlane(lds_offset(smem));

  auto issue_rows = [&](int tile) {
    const int lane = threadIdx.x & 63;
    const int n0 = tile * R;
    for (int k = wave; k < (imgB >> 10); k += kWaves) {
      const int o = (k << 10) + (lane << 4);
      const int row = o / rowB;
      const int piece = (o - row * rowB) >> 4;
      const int n = min(n0 + row, p.N - 1);
      const char* src = reinterpret_cast<const char*>(tab + (size_t)n * d) + ((piece ^ pre_swz(row, cpr)) << 4);
      dma_b128(src, sbase + (k << 10));
    }
  };

  int tile = blockIdx.x;
  if (tile < ntiles) issue_rows(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const int n0 = tile * R;
    vm_wait_all();
    raw_barrier();     // the tile's rows landed for every wave; last tile's partial readers done
    if constexpr (P2) {
      // each wave scales R / 8 rows in place by 2^(14-e) (an element order inside a row is the
      // chunk swizzle's: irrelevant to a max and a scale), an infinity clamped to ±65504 by v_med3 and
      // a NaN kept by a select (v_med3 does not return a NaN operand: a NaN row came out finite,
      // test_precompute_pairs_heavy_tailed); the row's unit 2^(e-14), +inf for a row holding an infinity
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int i = 0; i < R / kWaves; ++i) {
        const int row = (R / kWaves) * wave + i;
        float* rp = reinterpret_cast<float*>(img + row * rowB);
        float mx = 0.f;
        for (int c = lane; c < d; c += 64) mx = fmaxf(mx, fabsf(rp[c]));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        const int e = pre_p2_exp(fminf(mx, 3.40282347e38f));
        const float sc = ldexpf(1.0f, 14 - e);
        for (int c = lane; c < d; c += 64) {
          const float x = rp[c] * sc;
          rp[c] = x != x ? x : __builtin_amdgcn_fmed3f(x, -65504.0f, 65504.0f);
        }
        if (lane == 0) uE[row] = mx > 3.40282347e38f ? INFINITY : ldexpf(1.0f, e - 14);
      }
      raw_barrier();
    }

    for (int u = wave; u < J; u += kWaves) {
      FRESH_LANE_IDS();
      const bool w1 = u < nct;
      const T* blk0 = P2 ? (w1 ? W1x + (size_t)u * ns * 1024 : W2x + (size_t)(u - nct) * ns * 1024)
                         : (w1 ? W1p + (size_t)u * ns * 1024 : W2p + (size_t)(u - nct) * ns * 1024);
      f32x16 acc[NRT];
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt) acc[rt] = zero16();
      auto step = [&](const Frag<T>& wf, int s) {
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
          const int row = 32 * rt + r;
          const int ch = (32 * s + 16 * h) * (int)sizeof(T) / 16;   // first 16-byte chunk of columns [32s+16h, +16)
          Frag<T> ef;
#pragma unroll
          for (int q = 0; q < kNQ<T>; ++q)
            ef.q[q] = lds_u32x4(img + row * rowB + (((ch + q) ^ pre_swz(row, cpr)) << 4));
          if constexpr (P2) pre_slab_p2(acc[rt], wf, ef);
          else mma_slab(acc[rt], wf, ef);
        }
      };
      if constexpr (NS > 0) {
        constexpr int PF = NS < 4 ? NS : 4;
        Frag<T> ring[PF];
#pragma unroll
        for (int s = 0; s < PF; ++s) frag_load_tile(ring[s], blk0 + (size_t)s * 1024, lane);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const Frag<T> wf = ring[s % PF];
          if (s + PF < NS) frag_load_tile(ring[s % PF], blk0 + (size_t)(s + PF) * 1024, lane);
          step(wf, s);
        }
      } else {
        for (int s = 0; s < ns; ++s) {
          Frag<T> wf;
          frag_load_tile(wf, blk0 + (size_t)s * 1024, lane);
          step(wf, s);
        }
      }
      if constexpr (P2) {
        // register e of lane half h: weight row 32 tile + 16 h + e; column: staged row 32 rt + r
        const float* uw = (w1 ? u1 + 32 * u : u2 + 32 * (u - nct)) + 16 * h;
        float wu[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 v = reinterpret_cast<const float4*>(uw)[i];
          wu[4 * i] = v.x;
          wu[4 * i + 1] = v.y;
          wu[4 * i + 2] = v.z;
          wu[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
          const float ue = uE[32 * rt + r];
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[rt][e] = acc[rt][e] * wu[e] * ue;
        }
      }
      if (w1) {
        // Sᵀ partial [k, news] = Q[:, tile u] · tanh(Pᵀ)[tile u, news]; Q rows in pi order
        Frag<T> qf;
        frag_load(qf, Qp + (size_t)pi_row(r) * (nct * 32) + 32 * u + 16 * h);
        // W1's padded rows (c >= Dc) are 0 whatever the table row holds: their zero weights times an
        // infinite element (or an infinite pair unit) are NaN, and Q's zero columns would carry it
        // into every logit of the row (the reference has no such rows: tanh(±inf) = ±1)
        const int cpad = p.Dc - (32 * u + 16 * h);
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[rt][e] = e < cpad ? nx_tanh<T>(acc[rt][e]) : 0.f;
          Frag<T> pf;
          acc_to_frag<T>(pf, acc[rt]);
          f32x16 sacc = zero16();
          mma_slab(sacc, qf, pf);
          float* dst = xch + ((size_t)(u * NRT + rt) * 16) * 64 + lane;
#pragma unroll
          for (int e = 0; e < 16; ++e) dst[e * 64] = sacc[e];
        }
      } else {
        const int jt = u - nct;
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
          const int n = n0 + 32 * rt + r;
          if (n < p.N) {
            Frag<T> of;
            acc_to_frag<T>(of, acc[rt]);
            frag_store(static_cast<T*>(p.proj) + (size_t)n * d + 32 * jt + 16 * h, of);
          }
        }
      }
    }
    raw_barrier();     // partials written; the row image is free
    if (tile + (int)gridDim.x < ntiles) issue_rows(tile + gridDim.x);
    if (wave < NRT) {
      FRESH_LANE_IDS();
      const int n = n0 + 32 * wave + r;
      float s[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) s[e] = 0.f;
      for (int u = 0; u < nct; ++u) {
        const float* src = xch + ((size_t)(u * NRT + wave) * 16) * 64 + lane;
#pragma unroll
        for (int e = 0; e < 16; ++e) s[e] += src[e * 64];
      }
      if (n < p.N) {
#pragma unroll
        for (int e = 0; e < 16; ++e)
          if (16 * h + e < p.K) p.logits[(size_t)n * p.K + 16 * h + e] = s[e];
      }
    }
  }
  vm_wait_all();
}

// GEMM-shaped precompute (bf16): one persistent workgroup per CU walks 256-row x 256-column output
// tiles of [n_news, W1 (Dc, padded to 8 tiles) | W2 (d)], tile t -> (row tile, column tile) so that
// the 4 column tiles of a row tile land on one XCD (blocks b, b+8, b+16, b+24) and re-read the rows
// from its L2. Per 32-column slab of d (one "step") the 8 packed weight tiles of the column tile
// (2 KiB each, fragment-major) and the 256 row pieces (64 B each, XOR-swizzled) are LDS-DMA'd into a
// 4-slot ring, 3 steps ahead, across tile boundaries; every weight byte staged serves 256 rows (the
// register-streamed news_pre re-reads all weights per 64 rows). Wave w owns rows [32w, 32w+32) and
// all 8 column tiles, so for the W1 tile the logits tanh(P)·Qᵀ are summed over the Dc tiles in
// registers (Q staged in LDS once); W2 tiles store proj straight from the accumulators.
constexpr int kP2Rows = 256;
constexpr int kP2RowB = 64;                                 // bytes of one staged row piece (32 bf16)
constexpr int kP2Slot = kP2Rows * kP2RowB + 8 * 2048;       // rows | 8 weight tiles
constexpr int kP2NS = 4;
constexpr int kP2QOff = kP2NS * kP2Slot;                    // packed Q (32 x nct*32 bf16) after the ring
__device__ __forceinline__ int p2_swz(int row) { return (row >> 2) & 3; }

template <int NSL>
__global__ __launch_bounds__(kThreads) void news_pre2(PreParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using T = __bf16;
  const int d = p.d;
  const int ns = NSL > 0 ? NSL : (d >> 5);
  const int nct = n_ct(p.Dc);
  const int ncol = 1 + (p.proj ? (d + 255) / 256 : 0);
  const int nrt = (p.N + kP2Rows - 1) / kP2Rows;
  const int ntile = ((nrt + 7) & ~7) * ncol;
  const T* __restrict__ W1p = static_cast<const T*>(p.wp);
  const T* __restrict__ Qp = W1p + w1p_el(d, p.Dc);
  const T* __restrict__ W2p = Qp + qp_el(p.Dc);
  const T* __restrict__ tab = static_cast<const T*>(p.table);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned sbase = __builtin_amdgcn_readfirstlane(lds_offset(smem));
  const int G = gridDim.x;
  const int my_tiles = ((int)blockIdx.x < ntile) ? (ntile - (int)blockIdx.x + G - 1) / G : 0;
  const int nq = my_tiles * ns;
  auto tile_pos = [&](int t, int& rt, int& ct) {
    const int grp = t / (8 * ncol), i = t - grp * 8 * ncol;
    rt = grp * 8 + (i & 7);
    ct = i >> 3;
  };
  // step q of this workgroup -> its 4 DMAs per wave (2 weight-tile halves, 2 row instructions);
  // out-of-range tiles and rows are clamped to valid memory, never consumed
  auto issue = [&](int q) {
    const int lane = threadIdx.x & 63;
    int rt, ct;
    tile_pos((int)blockIdx.x + (q / ns) * G, rt, ct);
    const int sl = q % ns;
    const unsigned slot = sbase + (q & (kP2NS - 1)) * kP2Slot;
    const T* blk = W1p;
    if (ct == 0) {
      if (wave < nct) blk = W1p + ((size_t)wave * ns + sl) * 1024;
    } else {
      const int j2 = 8 * (ct - 1) + wave;
      if (j2 < ns) blk = W2p + ((size_t)j2 * ns + sl) * 1024;
    }
    dma_b128_c(blk + lane * 8, slot + kP2Rows * kP2RowB + wave * 2048);
    dma_b128_c(blk + 512 + lane * 8, slot + kP2Rows * kP2RowB + wave * 2048 + 1024);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * wave + h;
      const int row = 16 * j + (lane >> 2), pc = lane & 3;
      const int n = min(rt * kP2Rows + row, p.N - 1);
      dma_b128_c(tab + (size_t)n * d + 32 * sl + 8 * (pc ^ p2_swz(row)), slot + j * 1024);
    }
  };

  // packed Q -> LDS (plain loads; the first barrier below publishes it)
  {
    const int nqe = 32 * nct * 32;                         // bf16 elements
    const u32x4* src = reinterpret_cast<const u32x4*>(Qp);
    u32x4* dst = reinterpret_cast<u32x4*>(smem + kP2QOff);
    for (int i = threadIdx.x; i < nqe / 8; i += kThreads) dst[i] = src[i];
  }
  for (int q = 0; q < min(kP2NS - 1, nq); ++q) issue(q);

  f32x16 acc[8];
  for (int q = 0; q < nq; ++q) {
    const int sl = q % ns;
    if (sl == 0) {
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) acc[jt] = zero16();
    }
    const int younger = min(nq - 1 - q, kP2NS - 2);       // steps issued after q (4 DMAs each)
    if (younger >= 2) vm_wait<8>();
    else if (younger == 1) vm_wait<4>();
    else vm_wait<0>();
    raw_barrier();                                         // step q landed for all; slot of q-1 free
    if (q + kP2NS - 1 < nq) issue(q + kP2NS - 1);
    int rt, ct;
    tile_pos((int)blockIdx.x + (q / ns) * G, rt, ct);
    const int nvalid = ct == 0 ? nct : min(8, ns - 8 * (ct - 1));   // column tiles of this tile
    {
      FRESH_LANE_IDS();
      const char* slot = smem + (q & (kP2NS - 1)) * kP2Slot;
      const int row = 32 * wave + r;
      Frag<T> ef;
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) ef.q[qq] = lds_u32x4(slot + row * kP2RowB + (((2 * h + qq) ^ p2_swz(row)) << 4));
      const char* wst = slot + kP2Rows * kP2RowB;
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) {
        if (jt < nvalid) {
          Frag<T> wf;
          wf.q[0] = lds_u32x4(wst + jt * 2048 + lane * 16);
          wf.q[1] = lds_u32x4(wst + jt * 2048 + 1024 + lane * 16);
          mma_slab(acc[jt], wf, ef);
        }
      }
    }
    if (sl == ns - 1) {                                    // tile done: epilogue
      FRESH_LANE_IDS();
      const int n = rt * kP2Rows + 32 * wave + r;
      if (ct == 0) {
        // Sᵀ [k, news] = Σ_tiles Q[:, tile] · tanh(Pᵀ)[tile, news]; Q rows in pi order (model.py:171-174)
        f32x16 sacc = zero16();
        const char* ql = smem + kP2QOff;
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {
          if (jt < nct) {
            // padded W1 rows: 0 (news_pre); a NaN kept (tanh_fast's clamp of the exponent drops it)
            const int cpad = p.Dc - (32 * jt + 16 * h);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const float x = acc[jt][e];
              acc[jt][e] = e < cpad ? (x != x ? x : tanh_fast(x)) : 0.f;
            }
            Frag<T> pf, qf;
            acc_to_frag<T>(pf, acc[jt]);
            const char* qa = ql + ((size_t)pi_row(r) * (nct * 32) + 32 * jt + 16 * h) * 2;
            qf.q[0] = lds_u32x4(qa);
            qf.q[1] = lds_u32x4(qa + 16);
            mma_slab(sacc, qf, pf);
          }
        }
        if (n < p.N) {
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (16 * h + e < p.K) p.logits[(size_t)n * p.K + 16 * h + e] = sacc[e];
        }
      } else if (n < p.N) {
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {
          if (jt < nvalid) {
            Frag<T> of;
            acc_to_frag<T>(of, acc[jt]);
            frag_store(static_cast<T*>(p.proj) + (size_t)n * d + 32 * (8 * (ct - 1) + jt) + 16 * h, of);
          }
        }
      }
    }
  }
  vm_wait_all();
}

// ================================================================================================
// per-impression scoring
// ================================================================================================
struct NsParams {
  const void* table;
  const float* logits;
  const void* proj;
  const int32_t* his_ids;
  const uint8_t* mask;
  const float* bias;
  const int32_t* cand_ids;
  const int32_t* cand_off;
  float* scores;
  float* mui_out;
  int n_news, B, L, C, d, K, score_type;
  int abl;      // experiment bits (MINER_NEWS_ABL, A/B in one process): 1 = no priority for waves 4-7

};

#ifdef MINER_NEWS_DEBUG
// diagnostic build only: every DMA / store address is range-checked, a violation is recorded in
// g_news_dbg (kind bit, first offending value) and the access skipped
__device__ unsigned long long g_news_dbg[4];
__device__ __forceinline__ bool dbg_ok(int kind, const void* a, size_t n, const void* lo, size_t range, unsigned lds,
                                       unsigned lds_n) {
  const char* c = static_cast<const char*>(a);
  const char* l = static_cast<const char*>(lo);
  const bool ok = c >= l - 3 && c + n <= l + range && lds + lds_n <= (unsigned)(160 * 1024);
  if (!ok) {
    atomicOr(&g_news_dbg[0], 1ull << kind);
    atomicCAS(&g_news_dbg[1 + (kind & 1)], 0ull, (unsigned long long)(c - l) + 1);
    atomicCAS(&g_news_dbg[3], 0ull, (unsigned long long)lds + 1);
  }
  return ok;
}
#define NEWS_CHK(kind, a, n, lo, range, lds, lds_n) if (dbg_ok(kind, a, n, lo, range, lds, lds_n))
#else
#define NEWS_CHK(kind, a, n, lo, range, lds, lds_n)
#endif

// diagnostic build only (-DMINER_STAMPS): per-wave stage cycles of news_score32 (lane 0 of each wave
// sums s_memtime deltas; read with miner_news_debug_stage_cycles)
#ifdef MINER_STAMPS
__device__ unsigned long long g_ns_stage[kWaves][8];
__device__ unsigned long long g_ns_items;
#define NS_STAMP_DECL unsigned long long st_acc[8] = {0}; unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define NS_STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } while (0)
#define NS_STAMP_FLUSH(n) do { if ((threadIdx.x & 63) == 0) { for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_ns_stage[threadIdx.x >> 6][i_], st_acc[i_]); if (threadIdx.x == 0) atomicAdd(&g_ns_items, (unsigned long long)(n)); } } while (0)
#else
#define NS_STAMP_DECL
#define NS_STAMP(i) do {} while (0)
#define NS_STAMP_FLUSH(n) do {} while (0)
#endif

template <class T, int CW = 64> struct NCfg {   // CW: columns per chunk (64, or 128 for 16-bit)
  static constexpr int RB = CW * (int)sizeof(T);     // bytes of one row of a chunk
  static constexpr int PART = 64 * RB;               // 64 rows: E[his] | proj[his] | Cand
  static constexpr int SLOT = 3 * PART;
  static constexpr int NSLOT = RB == 128 ? 4 : 2;      // 128-byte chunk rows: 4 slots of 24 KiB
  static constexpr int NI = RB / 128;                // DMA instructions per part per wave
  static constexpr int RPI = 1024 / RB;              // rows per DMA instruction
  static constexpr int PPR = RB / 16;                // 16-byte pieces per row
  static constexpr int NSLAB = CW / 32;              // 32-column slabs per chunk
};

// LDS carve (bytes): [ring | xchg | logit blocks x2 | aux L1 x4 | aux L0 x4]
constexpr int kRingB = 98304;                        // NSLOT * SLOT for both dtypes
constexpr int kXchB = kWaves * 32 * 32 * 4;          // candidate partials [wave][c][k], 32x32 fp32 each
constexpr int kLogB = 64 * 128;                      // 64 history rows x K (<= 32) fp32; then A in place
constexpr int kL1B = 4 * 64 * 3 + 4 * kMaxCand;      // his ids | mask words | bias | cand ids
constexpr int kL0B = 16;                             // CSR offsets (2 ints) of one impression
constexpr int kPrepB = 2 * 64 * 4;                   // softmax coefficients (mul | add) per history slot
constexpr int kOffX = kRingB;
constexpr int kOffLog = kOffX + kXchB;
constexpr int kOffL1 = kOffLog + 2 * kLogB;
constexpr int kOffL0 = kOffL1 + 4 * kL1B;
constexpr int kOffPrep = kOffL0 + 8 * kL0B;
constexpr int kOffSoft = kOffPrep + 2 * kPrepB;      // cooperative softmax partials [wave][k][max, sum]
constexpr int kOffDup = kOffSoft + kWaves * 32 * 2 * 4;   // news_score: U (history groups) per L1 slot
constexpr int kNewsLds = kOffDup + 4 * 16;
static_assert(kNewsLds <= kLdsMax, "news_score LDS");
static_assert(NCfg<__bf16>::NSLOT * NCfg<__bf16>::SLOT == kRingB && NCfg<float>::NSLOT * NCfg<float>::SLOT == kRingB &&
              NCfg<__bf16, 128>::NSLOT * NCfg<__bf16, 128>::SLOT == kRingB &&
              NCfg<float, 32>::NSLOT * NCfg<float, 32>::SLOT == kRingB, "ring");

// chunk swizzle of a slot row: bf16 (8 chunks per row, 2 rows per 256-byte bank row): rows 4q..4q+3
// of a transposed read hit disjoint banks and 16 rows of a ds_read_b128 group distinct slots;
// bf16 with 256-byte rows (CW = 128): chunk ^ ((row & 3) << 2 | (row >> 2) & 3) — the row & 15 of
// the fp32 layout leaves the 32x32x16 transposed reads 4-way (cdna_hip_programming.md T10), this
// XOR makes them and the candidate ds_read_b128 conflict-free (PMC: 2.9k conflict cycles per
// impression before); fp32 (16 chunks per row): row & 15
template <class T, int CW = 64> __device__ __forceinline__ int nswz(int row) {
  if constexpr (NCfg<T, CW>::PPR == 8) return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
  else if constexpr (sizeof(T) == 2) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return row & 15;
}
// A-operand fragment of a part's transpose: rows = columns 32 sl + pi(r) of the chunk, contraction
// over the 32 part rows 32 ls .. 32 ls + 31 (bf16: ds_read_b64_tr_b16)
template <class T>
__device__ __forceinline__ void load_partT(Frag<T>& f, const char* part, int ls, int sl, int lane) {
  if constexpr (sizeof(T) == 2) {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int col = 32 * sl + 16 * (pp & 1) + 8 * (g & 1) + 4 * (pp >> 1);
    const int ch = col >> 3, sub = (col & 7) * 2;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int row = 32 * ls + 16 * (g >> 1) + 8 * s + 4 * u + q;
        const char* a = part + row * 128 + ((ch ^ nswz<T>(row)) << 4) + sub;
        const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds_char*)a);
        f.q[s][2 * u] = (unsigned)(unsigned short)v[0] | ((unsigned)(unsigned short)v[1] << 16);
        f.q[s][2 * u + 1] = (unsigned)(unsigned short)v[2] | ((unsigned)(unsigned short)v[3] << 16);
      }
    }
  } else {
    const int r = lane & 31, h = lane >> 5;
    const int col = 32 * sl + pi_row(r);
    const int ch = col >> 2, sub = (col & 3) * 4;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = 32 * ls + 16 * h + i;
      f.q[i >> 2][i & 3] = lds_u32(part + row * 256 + ((ch ^ nswz<T>(row)) << 4) + sub);
    }
  }
}

// A-operand fragment of candidate rows 32 ct + pi(r), columns [32 sl + 16 h, +16) of the chunk
template <class T>
__device__ __forceinline__ void load_cand(Frag<T>& f, const char* part, int ct, int sl, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int row = 32 * ct + pi_row(r);
  const int ch0 = sizeof(T) == 2 ? 4 * sl + 2 * h : 8 * sl + 4 * h;
#pragma unroll
  for (int q = 0; q < kNQ<T>; ++q)
    f.q[q] = lds_u32x4(part + row * NCfg<T>::RB + (((ch0 + q) ^ nswz<T>(row)) << 4));
}

__device__ __forceinline__ int* l1_his(char* smem, int slot) { return reinterpret_cast<int*>(smem + kOffL1 + slot * kL1B); }
__device__ __forceinline__ uint32_t* l1_mask(char* smem, int slot) { return reinterpret_cast<uint32_t*>(smem + kOffL1 + slot * kL1B + 256); }
__device__ __forceinline__ float* l1_bias(char* smem, int slot) { return reinterpret_cast<float*>(smem + kOffL1 + slot * kL1B + 512); }
__device__ __forceinline__ int* l1_cand(char* smem, int slot) { return reinterpret_cast<int*>(smem + kOffL1 + slot * kL1B + 768); }
__device__ __forceinline__ int* l0_off(char* smem, int slot) { return reinterpret_cast<int*>(smem + kOffL0 + slot * kL0B); }
__device__ __forceinline__ int* grp_u(char* smem, int slot) { return reinterpret_cast<int*>(smem + kOffDup + slot * 16); }

// row DMAs of one chunk for this wave (saddr form: the chunk's scalar base + a 32-bit per-lane row
// offset), parts E[his] / proj[his] / Cand at M0 = mE, mE + PART, mE + 2 PART; one statement, M0
// saved and restored around it
// The MINER_NEWS_ABL experiment bits news_score32 honours. Production builds compile them out (0):
// the uniform branches cost 6 % (15.11 -> 14.17 ms per 131k impressions, bit-identical scores,
// tools/bisect_news.py); diagnostic builds (tools/stage_profile.py, A/B scripts) pass 0x7fffffff.
#ifndef MINER_NEWS_ABL_MASK
#define MINER_NEWS_ABL_MASK 0
#endif
#ifndef MINER_NEWS_NT
#define MINER_NEWS_NT 0
#endif
#if MINER_NEWS_NT
#define NEWS_CP_STR " nt"
#else
#define NEWS_CP_STR ""
#endif
// one row DMA (saddr form) into M0 = m, M0 saved and restored around it
__device__ __forceinline__ void dma_row(uint32_t off, const char* base, unsigned m) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" NEWS_CP_STR "\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(t) : "v"(off), "s"(base), "s"(m) : "memory");
}

// SKIP (PD == 1 only, where the slot wait is vmcnt(0) and no count depends on how many DMAs a chunk
// issued): a DMA instruction whose rows all lie past L (history) or past the pass's candidate count is
// not issued (bit jj of `live`: history rows of E and proj; bit NI + jj: candidate rows). Those ring
// rows keep the zeros written at kernel start (or a finite row of an earlier chunk): they meet only
// A = 0 history slots and candidate rows whose scores are never stored. proj rows only for 'weighted'.
// SKIP: instruction jj lands at mE + jj * jstep (the block map is the caller's).
template <class T, int CW, bool SKIP, bool WITH_PROJ>
__device__ __forceinline__ void dma_chunk(const uint32_t* oH, const uint32_t* oC, const char* bE, const char* bY,
                                          unsigned mE, unsigned live, unsigned jstep = kWaves * 1024) {
  using Cf = NCfg<T, CW>;
  [[maybe_unused]] unsigned t;
  if constexpr (SKIP) {
#pragma unroll
    for (int jj = 0; jj < Cf::NI; ++jj) {
      if (live & (1u << jj)) {
        dma_row(oH[jj], bE, mE + jj * jstep);
        if constexpr (WITH_PROJ) dma_row(oH[jj], bY, mE + Cf::PART + jj * jstep);
      }
      if (live & (1u << (Cf::NI + jj))) dma_row(oC[jj], bE, mE + 2 * Cf::PART + jj * jstep);
    }
  } else if constexpr (Cf::NI == 1) {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %4" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(t)
        : "v"(oH[0]), "v"(oC[0]), "s"(bE), "s"(bY), "s"(mE), "s"(mE + Cf::PART), "s"(mE + 2 * Cf::PART)
        : "memory");
  } else {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %8\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %9\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %6" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %10\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %6" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %11\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %12\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5" NEWS_CP_STR "\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(t)
        : "v"(oH[0]), "v"(oH[1]), "v"(oC[0]), "v"(oC[1]), "s"(bE), "s"(bY),
          "s"(mE), "s"(mE + 8192), "s"(mE + Cf::PART), "s"(mE + Cf::PART + 8192),
          "s"(mE + 2 * Cf::PART), "s"(mE + 2 * Cf::PART + 8192)
        : "memory");
  }
}

template <class T, int ST, bool RAGGED, int PD, int CW, int NCH = 0, int SHP = 0>   // NCH: chunks per row (0: d / CW at
// run time); SHP 1: the MIND shape L = 50, K = 32 compile-time (0: at run time)
__global__ __launch_bounds__(kThreads) void news_score(NsParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using Cf = NCfg<T, CW>;
  constexpr int NSLAB = Cf::NSLAB;
  constexpr int NT = NSLAB == 4 ? 2 : 1;      // candidate tiles per wave
  constexpr int NI = Cf::NI;
  constexpr int NS = Cf::NSLOT;
  static_assert(PD >= 1 && PD <= NS - 1, "prefetch depth");
  constexpr bool WEIGHTED = ST == MINER_SCORE_WEIGHTED;
  constexpr bool WITH_CAND = ST != MINER_SCORE_NONE;
  constexpr bool SKIP = PD == 1;              // padding-row DMAs not issued (dma_chunk)
  // 128-column chunks (config 3): the second DMA block of wave w is block 8 + (w ^ 4), so the rows
  // 32..47 (live for L = 50, C = 40) go to the X-path waves 4-7 and the rows 48..63 (mostly padding,
  // not fetched) to the mui-path waves 0-3; S7 runs on waves 4-7. With the X waves prioritised the
  // mui waves are the critical path: this moves 8 of the 36 live DMAs per chunk and S7 off it.
  constexpr bool SWAP = SKIP && NSLAB == 4;
  const int G = gridDim.x;
  const int n_i = (p.B - (int)blockIdx.x + G - 1) / G;      // impressions of this workgroup
  const int L = SHP == 1 ? 50 : p.L, d = NCH > 0 ? NCH * CW : p.d;
  const int KK = SHP == 1 ? 32 : p.K;
  const int nchunk = NCH > 0 ? NCH : d / CW;
  // cooperative softmax one impression ahead (always for 128-column chunks: the host picks them for d >= 512)
  // (its two phases ride on chunks 1 and 2: 128-column chunks with fewer than 3 chunks per row, d = 256,
  // compute A in-wave)
  const bool coop = (CW == 128 && nchunk >= 3) || (nchunk >= PD + 1 && nchunk >= 4);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int w4 = SWAP ? (wave ^ 4) : wave;
  const char* tabB = static_cast<const char*>(p.table);
  const char* prjB = WEIGHTED ? static_cast<const char*>(p.proj) : tabB;
  const unsigned sbase = __builtin_amdgcn_readfirstlane(lds_offset(smem));

  auto imp_b = [&](int i) { return (int)blockIdx.x + i * G; };
  // candidates of impression i (scores offset, count <= kMaxCand); L0 must have landed (ragged)
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

  // ---- aux DMA jobs (issued after a barrier, before that iteration's row DMAs) ----
  auto issue_L0 = [&](int i) {           // CSR offsets of impression i
    if (RAGGED && wave == 0 && i < n_i && (threadIdx.x & 63) < 2)
      dma_b32(p.cand_off + imp_b(i) + (threadIdx.x & 63), sbase + kOffL0 + (i & 7) * kL0B);
  };
  auto issue_L1 = [&](int i) {           // ids / mask / bias of impression i (needs its L0)
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const size_t base = (size_t)imp_b(i) * L + min(lane, L - 1);
    const unsigned l1 = sbase + kOffL1 + (i & 3) * kL1B;
    if (wave == 1) {
      NEWS_CHK(1, p.his_ids + base, 4, p.his_ids, (size_t)p.B * L * 4, l1, 256)
      dma_b32(p.his_ids + base, l1);
    } else if (wave == 2) {
      // the aligned word holding mask byte `base` (the reader picks the byte by address)
      const uintptr_t a = reinterpret_cast<uintptr_t>(p.mask + base) & ~(uintptr_t)3;
      NEWS_CHK(2, reinterpret_cast<const void*>(a), 4, p.mask, (size_t)p.B * L + 3, l1 + 256, 256)
      dma_b32(reinterpret_cast<const void*>(a), l1 + 256);
    } else if (wave == 3) {
      if (p.bias) dma_b32(p.bias + base, l1 + 512);
    } else if (WITH_CAND && wave >= 4) { // waves 4..7: candidate ids, 64 per DMA (j >= 0)
      int off, cnt;
      cands(i, off, cnt);
      for (int j = wave - 4; j >= 0 && 64 * j < cnt; j += 4) {
        const int c = min(64 * j + lane, cnt - 1);
        NEWS_CHK(3, p.cand_ids + off + c, 4, p.cand_ids, (size_t)(RAGGED ? 1 << 30 : p.B * p.C) * 4, l1 + 768 + 256 * j, 256)
        dma_b32(p.cand_ids + off + c, l1 + 768 + 256 * j);
      }
    }
  };
  auto issue_L2 = [&](int i) {           // logit rows of impression i's history groups (needs its dedupe)
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const int U = __builtin_amdgcn_readfirstlane(grp_u(smem, i & 3)[0]);
    const int row = min(8 * wave + (lane >> 3), U - 1);
    const int piece = min(lane & 7, (KK >> 2) - 1);
    const int id = min(max(l1_his(smem, i & 3)[row], 0), p.n_news - 1);
    NEWS_CHK(4, p.logits + (size_t)id * KK + 4 * piece, 16, p.logits, (size_t)p.n_news * KK * 4, sbase + kOffLog + (i & 1) * kLogB + wave * 1024, 1024)
    dma_b128_c(p.logits + (size_t)id * KK + 4 * piece, sbase + kOffLog + (i & 1) * kLogB + wave * 1024);
  };
  // The masked history slots holding the same news id — the left padding: every pad slot is the pad
  // news, masked (reader.py:101-110, :369) — form one group, gathered and contracted once; the softmax
  // over the history (model.py:176-181) runs over the U groups with multiplicities m_u, the slots' sum
  // regrouped. Wave 7 (after its L1 landed) replaces impression i's history ids in L1 by the groups'
  // ids and writes each group's coefficients (±m, add): s_u = logit + bias with weight m for a click
  // (+m), s_u = 1e-30 with weight m for a pad slot (-m; model.py:176-180), (0, -inf) past U — and U
  auto dedupe_prep = [&](int i) {
    if (wave != 7 || i >= n_i) return;
    const int l = threadIdx.x & 63;
    int* his = l1_his(smem, i & 3);
    const int ls = min(l, L - 1);
    const int id = his[ls];
    const uint32_t mw = l1_mask(smem, i & 3)[ls];
    const int a = (int)(reinterpret_cast<uintptr_t>(p.mask + (size_t)imp_b(i) * L + ls) & 3);
    const bool keep = ((mw >> (8 * a)) & 0xffu) != 0u;
    const float bv = (keep && p.bias) ? l1_bias(smem, i & 3)[ls] : 0.f;
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
    float* pr = reinterpret_cast<float*>(smem + kOffPrep + (i & 1) * kPrepB);
    if (uniq) {                          // (±m, add): the sign says click / pad, |.| the multiplicity
      his[uidx] = id;
      pr[uidx] = keep ? (float)m : -(float)m;
      pr[64 + uidx] = keep ? bv : 1e-30f;
    }
    if (l >= U) {
      pr[l] = 0.f;
      pr[64 + l] = -INFINITY;
    }
    if (l == 0) grp_u(smem, i & 3)[0] = U;
  };
  // cooperative softmax over the history (model.py:176-181), one impression ahead: phase 1 — wave w
  // takes history slots [8w, 8w+8), lane (h, k) four of them: partial (max, Σexp) per interest k;
  // phase 2 (after a barrier) — merge the 8 partials, write A[l][k] over the logit rows the wave
  // read (its own rows only: no wave reads another's), bf16 / fp32 as the MFMA operand
  auto soft_phase = [&](int i, int phase) {
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const int k = lane & 31, h = lane >> 5;
    char* lg = smem + kOffLog + (i & 1) * kLogB;
    const float* pr = reinterpret_cast<const float*>(smem + kOffPrep + (i & 1) * kPrepB);
    float* part = reinterpret_cast<float*>(smem + kOffSoft);
    const int l0 = 8 * wave + 4 * h;
    const float4 mu = *reinterpret_cast<const float4*>(pr + l0);
    const float4 ad = *reinterpret_cast<const float4*>(pr + 64 + l0);
    const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, a4[4] = {ad.x, ad.y, ad.z, ad.w};
    float x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      x[j] = __builtin_fmaf(reinterpret_cast<const float*>(lg + (l0 + j) * 128)[k], m4[j] > 0.f ? 1.f : 0.f, a4[j]);
    if (phase == 1) {
      float m = fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3]));
      float s = 0.f;
      if (m != -INFINITY) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s = __builtin_fmaf(fabsf(m4[j]), nx_exp<T>(x[j] - m), s);
      }
      const float mo = both_max(m);      // combine the two lane halves
      const float so = (m == -INFINITY ? 0.f : s * nx_exp<T>(m - mo));
      const float st = mo == -INFINITY ? 0.f : both_sum(so);
      if (h == 0) {
        part[(wave * 32 + k) * 2] = mo;
        part[(wave * 32 + k) * 2 + 1] = st;
      }
    } else {
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) M = fmaxf(M, part[(w * 32 + k) * 2]);
      float S = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const float mw = part[(w * 32 + k) * 2];
        if (mw != -INFINITY) S += part[(w * 32 + k) * 2 + 1] * nx_exp<T>(mw - M);
      }
      float inv;
      if constexpr (sizeof(T) == 2) inv = __builtin_amdgcn_rcpf(S); else inv = 1.0f / S;
      if (k >= KK) inv = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = fabsf(m4[j]) * nx_exp<T>(x[j] - M) * inv;
        if constexpr (sizeof(T) == 2) reinterpret_cast<T*>(lg + (l0 + j) * 128)[k] = (T)a;
        else reinterpret_cast<float*>(lg + (l0 + j) * 128)[k] = a;
      }
    }
  };
  // this lane's row offsets (bytes, + its swizzled 16-byte piece) for item (i, pass): the history
  // row (E and proj parts) and the candidate row of each of its NI DMA blocks
  auto item_offsets = [&](int i, int pass, uint32_t* oH, uint32_t* oC, unsigned& lv) {
    const int lane = threadIdx.x & 63;
    const bool live = i < n_i;
    int off = 0, cnt = 1;
    if (live) cands(i, off, cnt);
    const int cntp = max(1, min(64, cnt - 64 * pass));
    const int U = live ? __builtin_amdgcn_readfirstlane(grp_u(smem, i & 3)[0]) : 1;
    lv = 0;                            // live DMA instructions of this wave (dma_chunk, SKIP)
#pragma unroll
    for (int jj = 0; jj < NI; ++jj) {
      const int row0 = (jj ? w4 + 8 * jj : wave) * Cf::RPI;   // first row of instruction jj
      if (live && row0 < U) lv |= 1u << jj;
      if (live && WITH_CAND && row0 < cnt - 64 * pass) lv |= 1u << (NI + jj);
    }
    lv = __builtin_amdgcn_readfirstlane(lv);
    const int* hid = l1_his(smem, i & 3);
    const int* cid = l1_cand(smem, i & 3);
    const uint32_t rowBytes = (uint32_t)d * sizeof(T);
#pragma unroll
    for (int jj = 0; jj < NI; ++jj) {
      const int rowp = (jj ? w4 + 8 * jj : wave) * Cf::RPI + lane / Cf::PPR;
      const uint32_t poff = (uint32_t)(((lane % Cf::PPR) ^ nswz<T, CW>(rowp)) << 4);
      int h = 0, c = 0;
      if (live) {
        h = hid[min(rowp, U - 1)];
        if (WITH_CAND) c = cid[min(64 * pass + min(rowp, cntp - 1), kMaxCand - 1)];
      }
      h = min(max(h, 0), p.n_news - 1);
      c = min(max(c, 0), p.n_news - 1);
      oH[jj] = (uint32_t)h * rowBytes + poff;
      oC[jj] = (uint32_t)c * rowBytes + poff;
    }
  };

  // ---- per-lane LDS read offsets of this wave's operands (fixed for the whole launch) ----
  // wave roles: P = path (0: E -> mui -> M, 1: proj -> X -> Lg), sl = slab of the chunk, ct = candidate
  // tile (64-column chunks: 2 slabs x 2 tiles, the X slab computed by both tile waves; 128-column
  // chunks: 4 slabs, each wave both tiles). Waves w and w+4 share a SIMD: one of each path.
  const int P = wave >> 2;
  const int sl = NSLAB == 4 ? (wave & 3) : ((wave >> 1) & 1);
  const int ct = NSLAB == 4 ? 0 : (wave & 1);
  uint32_t trOff[8];                   // bf16: transposed reads [ls][s][u] of part rows
  uint32_t cOff[NT][kNQ<T>];           // candidate rows 32 tile + pi(r), columns [32 sl + 16 h, +16)
  uint32_t aOff[4];                    // bf16 coop: A[l][k] rows 16 h + .., transposed reads [s][u]
  {
    const int lane = threadIdx.x & 63;
    const int r = lane & 31, h = lane >> 5;
    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
      const int col = 32 * sl + 16 * (pp & 1) + 8 * (g & 1) + 4 * (pp >> 1);
      const int ch = col >> 3, sub = (col & 7) * 2;
#pragma unroll
      for (int ls = 0; ls < 2; ++ls)
#pragma unroll
        for (int su = 0; su < 4; ++su) {
          const int row = 32 * ls + 16 * (g >> 1) + 8 * (su >> 1) + 4 * (su & 1) + q;
          trOff[4 * ls + su] = row * Cf::RB + ((ch ^ nswz<T, CW>(row)) << 4) + sub;
        }
      // A stored [l][k] (bf16, row stride 128 B): block rows l, columns k = 16 (g & 1) + 4 pp ..
#pragma unroll
      for (int su = 0; su < 4; ++su) {
        const int row = 16 * (g >> 1) + 8 * (su >> 1) + 4 * (su & 1) + q;
        aOff[su] = row * 128 + (16 * (g & 1) + 4 * pp) * 2;
      }
    }
#pragma unroll
    for (int tl = 0; tl < NT; ++tl) {
      const int row = 32 * (NT == 2 ? tl : ct) + pi_row(r);
      const int ch0 = sizeof(T) == 2 ? 4 * sl + 2 * h : 8 * sl + 4 * h;
#pragma unroll
      for (int q = 0; q < kNQ<T>; ++q) cOff[tl][q] = row * Cf::RB + (((ch0 + q) ^ nswz<T, CW>(row)) << 4);
    }
  }

  Frag<T> af[2];                       // attention weights A [K, 64] as two B-operand slabs
  // A of impression i -> af: from the A rows written by soft_phase (coop), else computed in-wave
  auto load_af = [&](int i) {
    const int lane = threadIdx.x & 63;
    const int r = lane & 31, h = lane >> 5;
    const char* lg = smem + kOffLog + (i & 1) * kLogB;
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int su = 0; su < 4; ++su) {
          const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds_char*)(lg + 32 * ls * 128 + aOff[su]));
          const auto w2 = __builtin_bit_cast(uint2, v);
          af[ls].q[su >> 1][2 * (su & 1)] = w2.x;
          af[ls].q[su >> 1][2 * (su & 1) + 1] = w2.y;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e)
          af[ls].q[e >> 2][e & 3] = __float_as_uint(reinterpret_cast<const float*>(lg + (32 * ls + 16 * h + e) * 128)[r]);
      }
    }
  };
  auto softmax_inwave = [&](int i) {   // small d: every wave computes A of impression i itself
    const int lane = threadIdx.x & 63;
    const int r = lane & 31, h = lane >> 5;
    const float* lgb = reinterpret_cast<const float*>(smem + kOffLog + (i & 1) * kLogB);
    const float* pr = reinterpret_cast<const float*>(smem + kOffPrep + (i & 1) * kPrepB);
    float v[32], wm[32];
    float mx = -INFINITY;
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int l0 = 32 * ls + 16 * h + 4 * j4;
        const float4 mu = *reinterpret_cast<const float4*>(pr + l0);
        const float4 ad = *reinterpret_cast<const float4*>(pr + 64 + l0);
        const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, a4[4] = {ad.x, ad.y, ad.z, ad.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float s = __builtin_fmaf(lgb[(l0 + u) * 32 + r], m4[u] > 0.f ? 1.f : 0.f, a4[u]);
          v[16 * ls + 4 * j4 + u] = s;
          wm[16 * ls + 4 * j4 + u] = fabsf(m4[u]);
          mx = fmaxf(mx, s);
        }
      }
    }
    mx = both_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      v[j] = wm[j] * nx_exp<T>(v[j] - mx);     // exp(-inf) = 0 past U (weight 0)
      sum += v[j];
    }
    sum = both_sum(sum);
    float inv;
    if constexpr (sizeof(T) == 2) inv = __builtin_amdgcn_rcpf(sum); else inv = 1.0f / sum;
    if (r >= KK) inv = 0.f;
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int m = 0; m < 8; ++m) af[ls].q[m >> 2][m & 3] = pack_bf16x2(v[16 * ls + 2 * m] * inv, v[16 * ls + 2 * m + 1] * inv);
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) af[ls].q[e >> 2][e & 3] = __float_as_uint(v[16 * ls + e] * inv);
      }
    }
  };

  // ring rows no DMA writes (history slots >= L, candidates past the count) read as zeros; the
  // prologue's first barrier (lgkmcnt(0)) orders these stores before every ring DMA
  if constexpr (SKIP) {
    for (int o = (int)threadIdx.x * 16; o < kRingB; o += kThreads * 16)
      *reinterpret_cast<u32x4*>(smem + o) = u32x4{0u, 0u, 0u, 0u};
  }
  // ---- prologue: aux for the first impressions, A of impression 0, then the first PD chunks ----
  for (int i = 0; i < 4; ++i) issue_L0(i);
  vm_wait_all();
  raw_barrier();
  issue_L1(0); issue_L1(1); issue_L1(2);
  vm_wait_all();
  raw_barrier();
  dedupe_prep(0); dedupe_prep(1);
  raw_barrier();
  issue_L2(0); issue_L2(1);
  vm_wait_all();
  raw_barrier();
  if (coop) {
    soft_phase(0, 1);
    raw_barrier();
    soft_phase(0, 2);
    raw_barrier();
  }
  uint32_t cH[NI], cC[NI], nH[NI], nC[NI];   // row offsets of the current / next item
  unsigned cLv = 0, nLv = 0;                 // and their live DMA instructions
  item_offsets(0, 0, cH, cC, cLv);
#pragma unroll
  for (int k = 0; k < PD; ++k)
    dma_chunk<T, CW, SKIP, WEIGHTED>(cH, cC, tabB + k * CW * sizeof(T), prjB + k * CW * sizeof(T),
                                     sbase + k * Cf::SLOT + wave * 1024, cLv, (w4 + 8 - wave) * 1024);

  f32x16 acc[NT];                      // this wave's M / Lg partials, 32x32 candidate tiles
#pragma unroll
  for (int tl = 0; tl < NT; ++tl) acc[tl] = zero16();
  int pend_off = -1, pend_cnt = 0;     // a finished pass waiting for S7 (pend_off >= 0)
  int t = 0;

  // S7 (model.py:128-136, :213-214) on waves 0..3: wave w takes candidates [16 w, 16 w + 16) of the
  // pass, lane (kq, c) = (lane >> 4, lane & 15) interests [8 kq, 8 kq + 8); partials of the 8 waves
  // are summed here (M: waves ct, 2+ct; Lg: 4+ct, 6+ct), the 4 lane rows combined by permlanes
  auto s7 = [&]() {
    if (SWAP ? wave < 4 : wave >= 4) return;
    const int lane = threadIdx.x & 63;
    const int cl = lane & 15, kq = lane >> 4;
    const int c = 16 * (wave & 3) + cl;        // candidate of the pass
    const int tct = c >> 5, cr = c & 31;       // c-tile, row in the tile
    const float* X = reinterpret_cast<const float*>(smem + kOffX);
    const int sw = (cr >> 1) & 31;
    float lg[8], m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * kq + j;
      const int o = cr * 32 + (k ^ sw);
      m[j] = X[(tct) * 1024 + o] + X[(2 + tct) * 1024 + o];
      if constexpr (WEIGHTED) lg[j] = X[(4 + tct) * 1024 + o] + X[(6 + tct) * 1024 + o];
    }
    float sc;
    if constexpr (WEIGHTED) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) mx = fmaxf(mx, lg[j]);
      mx = rows4_max(mx);
      float s = 0.f, num = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (8 * kq + j < KK) {
          const float pe = nx_exp<T>(lg[j] - mx);
          s += pe;
          num = __builtin_fmaf(pe, m[j], num);
        }
      }
      s = rows4_sum(s);
      num = rows4_sum(num);
      if constexpr (sizeof(T) == 2) sc = num * __builtin_amdgcn_rcpf(s); else sc = num / s;
    } else {
      if (p.score_type == MINER_SCORE_MAX) {
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) mx = fmaxf(mx, m[j]);
        sc = rows4_max(mx);
      } else {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) s += m[j];
        sc = rows4_sum(s) / (float)KK;
      }
    }
    if (kq == 0 && c < pend_cnt) {
      NEWS_CHK(8, p.scores + pend_off + c, 4, p.scores, (size_t)(RAGGED ? 1 << 30 : p.B * p.C) * 4, 0, 0)
      p.scores[pend_off + c] = sc;
    }
  };

  // static priority for the X-path waves 4-7 (the GELU chain, the longer one of each SIMD's pair):
  // MI355X_MICROARCH.md §Two waves per SIMD, item 4. Config 3: 4.37 -> 4.20 ms, bit-identical.
  if (!(p.abl & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);

  // one 64-column chunk: the row DMAs of chunk `ich` of the item whose offsets are (iH, iC), PD
  // chunks ahead, then the X / mui slab and the candidate product of this chunk.
  // `mode`: 1 X, 2 candidate product, 4 mui out
  NS_STAMP_DECL
  // the item's history groups fit one 32-slot slab (<= 32 groups: the left padding is one group):
  // the second slab's attention weights are all 0, its transposed reads and MFMAs are skipped
  bool one_slab = false;
  auto chunk = [&](int ci, int cc, int mode, int ncand, const uint32_t* iH, const uint32_t* iC, unsigned iLv,
                   int ich) {
    NS_STAMP(2);
    if constexpr (sizeof(T) == 2 && NS_EARLY) {
      // every LDS operand read of the chunk first (asm: issued together, not split around the
      // MFMAs), then the row DMAs PD chunks ahead, whose issue covers the reads' latency, then the
      // products behind counted lgkmcnt waits (the history reads are the oldest in flight)
      const unsigned sb = sbase + (unsigned)((t & (NS - 1)) * Cf::SLOT);
      const unsigned hb = sb + (unsigned)(P * Cf::PART);
      const bool do_x = mode & 1, do_c = (mode & 3) == 3;
      const bool two_sl = !one_slab, two_t = NT == 2 && ncand > 32;
      uint2 tr[2][4];
      u32x4 cf_[NT][2];
      if (do_x) {
#pragma unroll
        for (int su = 0; su < 4; ++su)
          asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(tr[0][su]) : "v"(hb + trOff[su]));
        if (two_sl) {
#pragma unroll
          for (int su = 0; su < 4; ++su)
            asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(tr[1][su]) : "v"(hb + trOff[4 + su]));
        }
        if (do_c) {
#pragma unroll
          for (int tl = 0; tl < NT; ++tl) {
            if (tl == 0 || two_t) {
#pragma unroll
              for (int q = 0; q < 2; ++q)
                asm volatile("ds_read_b128 %0, %1" : "=v"(cf_[tl][q]) : "v"(sb + 2 * Cf::PART + cOff[tl][q]));
            }
          }
        }
      }
      dma_chunk<T, CW, SKIP, WEIGHTED>(iH, iC, tabB + ich * CW * sizeof(T), prjB + ich * CW * sizeof(T),
                                       sbase + ((t + PD) & (NS - 1)) * Cf::SLOT + wave * 1024, iLv, (w4 + 8 - wave) * 1024);
      NS_STAMP(3);
      if (!do_x) return;
      FRESH_LANE_IDS();
      if (!do_c) ns_wait_tr<0>(tr[0]);
      else if (two_t) ns_wait_tr<4>(tr[0]);
      else ns_wait_tr<2>(tr[0]);
      if (two_sl) {                    // younger than slab 0's reads: covered by the same count
        if (!do_c) ns_wait_tr<0>(tr[1]);
        else if (two_t) ns_wait_tr<4>(tr[1]);
        else ns_wait_tr<2>(tr[1]);
      }
      f32x16 ax = zero16();
#pragma unroll
      for (int ls = 0; ls < 2; ++ls) {
        if (ls == 1 && !two_sl) break;
        Frag<T> ef;
#pragma unroll
        for (int su = 0; su < 4; ++su) {
          ef.q[su >> 1][2 * (su & 1)] = tr[ls][su].x;
          ef.q[su >> 1][2 * (su & 1) + 1] = tr[ls][su].y;
        }
        mma_slab(ax, ef, af[ls]);
      }
      NS_STAMP(4);
      if ((mode & 4) && r < KK) {
        float* dst = p.mui_out + ((size_t)imp_b(ci) * KK + r) * d + CW * cc + 32 * sl + 16 * h;
#pragma unroll
        for (int e = 0; e < 16; e += 4) *reinterpret_cast<float4*>(dst + e) = make_float4(ax[e], ax[e + 1], ax[e + 2], ax[e + 3]);
      }
      if (do_c) {
        if (WEIGHTED && P == 1) gelu_tile<T>(ax);
        Frag<T> xf;
        acc_to_frag<T>(xf, ax);
        NS_STAMP(5);
        ns_wait_c<NT>(cf_);
#pragma unroll
        for (int tl = 0; tl < NT; ++tl) {
          if (tl == 0 || two_t) {
            Frag<T> cf;
            cf.q[0] = cf_[tl][0];
            cf.q[1] = cf_[tl][1];
            mma_slab(acc[tl], cf, xf);
          }
        }
      }
      return;
    }
    if (!(NS_ABL & 2))
      dma_chunk<T, CW, SKIP, WEIGHTED>(iH, iC, tabB + ich * CW * sizeof(T), prjB + ich * CW * sizeof(T),
                                       sbase + ((t + PD) & (NS - 1)) * Cf::SLOT + wave * 1024, iLv, (w4 + 8 - wave) * 1024);
    NS_STAMP(3);
    if ((mode & 1) && !(NS_ABL & 4)) {
      FRESH_LANE_IDS();
      const char* slot = smem + (t & (NS - 1)) * Cf::SLOT;
      const char* part = slot + P * Cf::PART;
      f32x16 ax = zero16();
#pragma unroll
      for (int ls = 0; ls < 2; ++ls) {
        if (ls == 1 && one_slab) break;
        Frag<T> ef;
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int su = 0; su < 4; ++su) {
            const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds_char*)(part + trOff[4 * ls + su]));
            const auto w2 = __builtin_bit_cast(uint2, v);
            ef.q[su >> 1][2 * (su & 1)] = w2.x;
            ef.q[su >> 1][2 * (su & 1) + 1] = w2.y;
          }
        } else {
          load_partT<T>(ef, part, ls, sl, lane);
        }
        mma_slab(ax, ef, af[ls]);
      }
      NS_STAMP(4);
      if ((mode & 4) && r < KK) {
        float* dst = p.mui_out + ((size_t)imp_b(ci) * KK + r) * d + CW * cc + 32 * sl + 16 * h;
#pragma unroll
        for (int e = 0; e < 16; e += 4) *reinterpret_cast<float4*>(dst + e) = make_float4(ax[e], ax[e + 1], ax[e + 2], ax[e + 3]);
      }
      if (mode & 2) {
        const char* cpart = slot + 2 * Cf::PART;
        if (WEIGHTED && P == 1) gelu_tile<T>(ax);
        Frag<T> xf;
        acc_to_frag<T>(xf, ax);
        NS_STAMP(5);
#pragma unroll
        for (int tl = 0; tl < NT; ++tl) {
          if (tl == 0 || ncand > 32) {
            Frag<T> cf;
#pragma unroll
            for (int q = 0; q < kNQ<T>; ++q) cf.q[q] = lds_u32x4(cpart + cOff[tl][q]);
            mma_slab(acc[tl], cf, xf);
          }
        }
      }
    }
  };
  auto wait_slot = [&]() {
    // slot t landed (this wave's DMAs: all but the PD-1 younger chunks), then for every wave
    NS_STAMP(6);
    vm_wait<3 * NI * (PD - 1)>();
    raw_barrier();
    NS_STAMP(0);
  };

  for (int ci = 0; ci < n_i; ++ci) {
    int c_off, c_cnt;
    cands(ci, c_off, c_cnt);
    const int cn = max(1, (c_cnt + 63) >> 6);
    one_slab = __builtin_amdgcn_readfirstlane(grp_u(smem, ci & 3)[0]) <= 32;
    for (int cp = 0; cp < cn; ++cp) {
      const int cntp = min(64, c_cnt - 64 * cp);
      const bool need_c = WITH_CAND && (ct == 0 || cntp > 32) && (P == 0 || WEIGHTED);
      const bool need_mui = P == 0 && p.mui_out != nullptr && cp == 0 && ct == 0;   // NSLAB 4: ct == 0
      const bool need_x = (P == 0) ? (WITH_CAND || need_mui) : WEIGHTED;
      const int mode = ((need_x && (need_c || need_mui)) ? 1 : 0) | (need_c ? 2 : 0) | (need_mui ? 4 : 0);
      // the item after this one, for the DMAs that run ahead into it
      const int ni = cp + 1 < cn ? ci : ci + 1, np = cp + 1 < cn ? cp + 1 : 0;
      bool did_s7 = false;
      // per-item work riding on the first chunks of the item
      auto extras = [&](int cc) {
        if (cc == 0) {
          did_s7 = WITH_CAND && pend_off >= 0;
          NS_STAMP(1);
          if (did_s7) s7();
          NS_STAMP(7);
          pend_off = -1;
          if (cp == 0) {
            if (coop) {
              load_af(ci);
            } else {
              softmax_inwave(ci);
              dedupe_prep(ci + 2);
              raw_barrier();           // every wave has read impression ci's logit rows; ci + 2 grouped
              issue_L2(ci + 2);
            }
            issue_L0(ci + 4);
            issue_L1(ci + 3);
            if (coop) dedupe_prep(ci + 2);   // its logit rows go out at the next chunk
          }
#pragma unroll
          for (int tl = 0; tl < NT; ++tl) acc[tl] = zero16();
        } else if (coop && cp == 0) {
          if (cc == 1) {
            issue_L2(ci + 2);          // into the rows A of ci was read from (free since the barrier)
            NS_STAMP(1);
            soft_phase(ci + 1, 1);
            NS_STAMP(2);
          } else if (cc == 2) {
            NS_STAMP(1);
            soft_phase(ci + 1, 2);
            NS_STAMP(2);
          }
        }
      };
      int cc = 0;
      for (; cc < nchunk - PD; ++cc, ++t) {
        wait_slot();
        extras(cc);
        NS_STAMP(1);
        chunk(ci, cc, mode, cntp, cH, cC, cLv, cc + PD);
      }
      item_offsets(ni, np, nH, nC, nLv);
      for (; cc < nchunk; ++cc, ++t) {
        wait_slot();
        extras(cc);
        NS_STAMP(1);
        chunk(ci, cc, mode, cntp, nH, nC, nLv, cc + PD - nchunk);
      }
      // pass done: partials -> LDS blocks [c][k ^ swizzle] (block = 4P + 2 sl + tile for the two
      // slab halves that survive), S7 at the next item's first chunk
      if (nchunk == 1 && did_s7) raw_barrier();
      {
        const int lane = threadIdx.x & 63;
        const int r = lane & 31, h = lane >> 5;
        float* X = reinterpret_cast<float*>(smem + kOffX);
        auto put = [&](int blk, const f32x16& a) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int cr = 16 * h + e;
            X[blk * 1024 + cr * 32 + (r ^ ((cr >> 1) & 31))] = a[e];
          }
        };
        if constexpr (NSLAB == 4) {
          // slabs 2, 3 hand their partials to slabs 0, 1 (same path), which add and publish
          if (sl >= 2) {
#pragma unroll
            for (int tl = 0; tl < 2; ++tl) put(4 * P + 2 * (sl - 2) + tl, acc[tl]);
          }
          raw_barrier();
          if (sl < 2) {
#pragma unroll
            for (int tl = 0; tl < 2; ++tl) {
              const int blk = 4 * P + 2 * sl + tl;
#pragma unroll
              for (int e = 0; e < 16; ++e) {
                const int cr = 16 * h + e;
                acc[tl][e] += X[blk * 1024 + cr * 32 + (r ^ ((cr >> 1) & 31))];
              }
              put(blk, acc[tl]);
            }
          }
        } else {
          put(wave, acc[0]);
        }
      }
      pend_off = c_off + 64 * cp;
      pend_cnt = cntp;
#pragma unroll
      for (int jj = 0; jj < NI; ++jj) { cH[jj] = nH[jj]; cC[jj] = nC[jj]; }
      cLv = nLv;
    }
  }
  vm_wait_all();
  raw_barrier();
  if (WITH_CAND && pend_off >= 0) s7();
  NS_STAMP_FLUSH(n_i);
}

// ================================================================================================
// fp32 scoring (the parity mode and the bench headline): news_score32<ST, RAGGED>
// ================================================================================================
// The per-impression math of news_score (model.py:113-138, :176-182, :200-216 on the gathered
// rows) laid out for the fp32 matrix cores: v_mfma_f32_16x16x4_f32 is an exact fp32 fma chain at
// the fp32 peak (64 FLOP/clk/SIMD, the rate of 32x32x2 but in 16-row tiles), so the history pads
// only to a multiple of 4 (50 -> 52, not 64) and the candidates to 16 (40 -> 48, not 64).
//   * the rows stream in 32-column chunks (128-byte row pieces, 8 rows per LDS-DMA instruction)
//     through a 4-slot ring, two chunks per barrier: one pair is computed while the next lands;
//     rows past L / past the candidate count are never fetched (the ring starts zeroed; such rows
//     meet A = 0 or unstored scores);
//   * wave w = (path P = w >> 2, column tile ct = (w >> 1) & 1, interest tile kt = w & 1), so each
//     SIMD pairs a mui wave (P = 0) with an X wave (P = 1, carries the GELU). Per chunk:
//       muiᵀ / Xᵀ [16 cols x 16 interests] = part[his]ᵀ · Aᵀ     ceil(L/4) MFMAs (model.py:182, :212)
//       M / Lg [16 cands x 16 interests] += Cand · muiᵀ / Xᵀ      4 MFMAs per candidate tile (:127, :213)
//     the accumulator of the first product is the B operand of the second (D rows = its k steps);
//   * per pass (<= 64 candidates) the two column-tile waves of each (P, kt) combine their partials
//     through LDS (one barrier), the final M / Lg go to LDS, and S7 (:128-136, :214) runs on waves
//     0-3 at the next item's first chunk.
// X6 = true (MINER_NEWS_F32X6=1): the same stream and the same products on the bf16 matrix cores
// at fp32 accuracy (bf16x6, cdna4_common.h: every fp32 operand cut exactly into three bf16 terms,
// six v_mfma_f32_16x16x32_bf16 per 32-index contraction). Wave w = (P, chunk cc = (w >> 1) & 1 of the
// pair, kt); per pair each wave takes ONE whole 32-column chunk:
//       muiᵀ / Xᵀ [32 cols x 16 interests] = part[his]ᵀ · Aᵀ   2 column tiles (even / odd columns,
//           one ds_read_b64 per row) x ceil(L/32) x 6 MFMAs; history padded to 32 / 64
//       M / Lg [16 cands x 16 interests] += Cand · muiᵀ / Xᵀ    6 MFMAs per candidate tile
//     the two accumulators of the first product are the B operand of the second as they stand:
//     lane (j, g) holds columns 2(4g + e) and 2(4g + e) + 1 = the contraction indices 8g .. 8g + 7.
//     The fp32 MFMA cannot co-issue with VALU; the bf16 MFMA does, so one SIMD's GELU / split VALU
//     work runs beside the other wave's MFMAs. Measured (tools/news_stages.py): equal to the fp32
//     MFMA form at config 3 (15.5 vs 15.6 ms per 131k): the MFMA time saved (1344 vs 3200 cycles
//     per pair per SIMD) goes to the split VALU (2x redundant for the history rows, 4x for the
//     candidate rows across the waves), and both share ~2.3k cycles per pair of DMA issue, softmax,
//     S7 and pass-end work.
constexpr int kF32CW = 32;
// chunk-row swizzle over the 8 16-byte pieces of a 128-byte row: conflict-free ds_read_b128 of the
// candidate operand (rows 16t + l, pieces 4ct + g) and ds_read_b32 of the history operand (rows
// 4s + g of a half wave); found by exhaustive search over GF(2)-linear maps of the row bits
__host__ __device__ inline int f32swz(int row) { return (((row >> 1) & 1) << 1) | (((row ^ (row >> 2)) & 1) << 2); }
// bf16x6 layout of a part: physical row 8b + i holds logical row 8b + (i ^ (b & 1)) (x6row, an
// involution), and its 16-byte piece slot s holds logical piece s ^ x6swz(physical row). Then the
// ds_read_b64 of the history operand (lanes g = 0, 1 of a half read logical rows 8g + i, whole
// 128-byte rows) puts the half's two rows in different 128-byte bank halves, and the ds_read_b128 of
// the candidate operand (rows 16q + j, pieces 2g + u) is conflict-free in all four lane groups
// (exhaustive search over GF(2)-linear maps of the physical row bits)
__host__ __device__ inline int x6row(int row) { return row ^ ((row >> 3) & 1); }
__host__ __device__ inline int x6swz(int prow) { return ((prow >> 1) & 1) | (prow & 4); }

__device__ __forceinline__ void vm_wait_n(int n) {      // s_waitcnt vmcnt(n), n wave-uniform in [0, 6]
  switch (n) {
    case 6: vm_wait<6>(); break;
    case 5: vm_wait<5>(); break;
    case 4: vm_wait<4>(); break;
    case 3: vm_wait<3>(); break;
    case 2: vm_wait<2>(); break;
    case 1: vm_wait<1>(); break;
    default: vm_wait<0>(); break;
  }
}

typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int ST, bool RAGGED, bool X6, int NCH, int SHP = 0>   // NCH: 32-column chunks per row (0: d / 32 at run time);
// SHP 1: the MIND shape L = 50, K = 32 compile-time (0: at run time); SHP 2: that shape, no category
// bias and no mui output (plain scoring: the bench, the eval without eval loss)
__global__ __launch_bounds__(kThreads) void news_score32(NsParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using T = float;
  using Cf = NCfg<float, kF32CW>;
  constexpr int NS = Cf::NSLOT;
  static_assert(NS == 4, "ring: a pair of chunks computed while the next pair lands");
  constexpr bool WEIGHTED = ST == MINER_SCORE_WEIGHTED;
  constexpr bool WITH_CAND = ST != MINER_SCORE_NONE;
  const int G = gridDim.x;
  const int n_i = (p.B - (int)blockIdx.x + G - 1) / G;      // impressions of this workgroup
  const int abl = p.abl & MINER_NEWS_ABL_MASK;              // experiment bits (MINER_NEWS_ABL)
  const int L = SHP >= 1 ? 50 : p.L, d = p.d;
  const int KK = SHP >= 1 ? 32 : p.K;
  const float* const bias = SHP == 2 ? nullptr : p.bias;
  float* const mui_out = SHP == 2 ? nullptr : p.mui_out;
  const int nchunk = NCH > 0 ? NCH : d / kF32CW;
  // softmax over the history (model.py:176-181): smode 2 (d >= 128): every wave computes its own A slice
  // (16 interests) at the item's first pair, the next logit rows and softmax coefficients are staged
  // at the second pair (the block it read is free after that barrier). An fp32 wave needs 16 exps per
  // lane either way, and the cooperative form (smode 1, MINER_NEWS_ABL bit 256) adds two LDS round
  // trips and a partial exchange; smode 0 (one pair per item): in-wave + a barrier before the L2 DMA
  const int npair0 = nchunk >> 1;
  const int smode = (abl & 256) && nchunk >= 6 ? 1 : (npair0 >= 2 ? 2 : 0);
  const bool coop = smode == 1;
  const bool split_f = npair0 >= 2 && !(abl & 512);    // pass end without a barrier (see the pass end)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* tabB = static_cast<const char*>(p.table);
  const char* prjB = WEIGHTED ? static_cast<const char*>(p.proj) : tabB;
  const unsigned sbase = __builtin_amdgcn_readfirstlane(lds_offset(smem));
  const int P = wave >> 2, ct = (wave >> 1) & 1, kt = wave & 1;   // X6: ct = the chunk of the pair
  const int nsteps = (L + 3) >> 2;
  const bool k_live = 16 * kt < KK;
  const bool path_live = P == 0 || WEIGHTED;

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
  // ---- aux DMA jobs, as news_score ----
  auto issue_L0 = [&](int i) {
    if (RAGGED && wave == 0 && i < n_i && (threadIdx.x & 63) < 2)
      dma_b32(p.cand_off + imp_b(i) + (threadIdx.x & 63), sbase + kOffL0 + (i & 7) * kL0B);
  };
  auto issue_L1 = [&](int i) {
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const size_t base = (size_t)imp_b(i) * L + min(lane, L - 1);
    const unsigned l1 = sbase + kOffL1 + (i & 3) * kL1B;
    if (wave == 1) {
      dma_b32(p.his_ids + base, l1);
    } else if (wave == 2) {
      const uintptr_t a = reinterpret_cast<uintptr_t>(p.mask + base) & ~(uintptr_t)3;
      dma_b32(reinterpret_cast<const void*>(a), l1 + 256);
    } else if (wave == 3) {
      if (bias) dma_b32(bias + base, l1 + 512);
    } else if (WITH_CAND && wave >= 4) {
      int off, cnt;
      cands(i, off, cnt);
      for (int j = wave - 4; j >= 0 && 64 * j < cnt; j += 4) {
        const int c = min(64 * j + lane, cnt - 1);
        dma_b32(p.cand_ids + off + c, l1 + 768 + 256 * j);
      }
    }
  };
  auto issue_L2 = [&](int i) {
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const int row = min(8 * wave + (lane >> 3), L - 1);
    const int piece = min(lane & 7, (KK >> 2) - 1);
    const int id = min(max(l1_his(smem, i & 3)[row], 0), p.n_news - 1);
    dma_b128_c(p.logits + (size_t)id * KK + 4 * piece, sbase + kOffLog + (i & 1) * kLogB + wave * 1024);
  };
  auto prep_softmax = [&](int i) {
    if (wave != 3 || i >= n_i) return;
    const int l = threadIdx.x & 63;
    const uint32_t mw = l1_mask(smem, i & 3)[l];
    const int a = (int)(reinterpret_cast<uintptr_t>(p.mask + (size_t)imp_b(i) * L + l) & 3);
    const bool keep = ((mw >> (8 * a)) & 0xffu) != 0u;
    float mul = 0.f, add = -INFINITY;
    if (l < L) {
      mul = keep ? 1.f : 0.f;
      add = keep ? (bias ? l1_bias(smem, i & 3)[l] : 0.f) : 1e-30f;
    }
    float* pr = reinterpret_cast<float*>(smem + kOffPrep + (i & 1) * kPrepB);
    pr[l] = mul;
    pr[64 + l] = add;
  };
  auto soft_phase = [&](int i, int phase) {
    if (i >= n_i) return;
    const int lane = threadIdx.x & 63;
    const int k = lane & 31, h = lane >> 5;
    char* lg = smem + kOffLog + (i & 1) * kLogB;
    const float* pr = reinterpret_cast<const float*>(smem + kOffPrep + (i & 1) * kPrepB);
    float* part = reinterpret_cast<float*>(smem + kOffSoft);
    const int l0 = 8 * wave + 4 * h;
    const float4 mu = *reinterpret_cast<const float4*>(pr + l0);
    const float4 ad = *reinterpret_cast<const float4*>(pr + 64 + l0);
    const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, a4[4] = {ad.x, ad.y, ad.z, ad.w};
    float x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = __builtin_fmaf(reinterpret_cast<const float*>(lg + (l0 + j) * 128)[k], m4[j], a4[j]);
    if (phase == 1) {
      float m = fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3]));
      float s = 0.f;
      if (m != -INFINITY) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s += expf(x[j] - m);
      }
      const float mo = both_max(m);
      const float so = (m == -INFINITY ? 0.f : s * expf(m - mo));
      const float st = mo == -INFINITY ? 0.f : both_sum(so);
      if (h == 0) {
        part[(wave * 32 + k) * 2] = mo;
        part[(wave * 32 + k) * 2 + 1] = st;
      }
    } else {
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) M = fmaxf(M, part[(w * 32 + k) * 2]);
      float S = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const float mw = part[(w * 32 + k) * 2];
        if (mw != -INFINITY) S += part[(w * 32 + k) * 2 + 1] * expf(mw - M);
      }
      float inv = 1.0f / S;
      if (k >= KK) inv = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) reinterpret_cast<float*>(lg + (l0 + j) * 128)[k] = expf(x[j] - M) * inv;
    }
  };
  // this lane's row offsets for item (i, pass). The row DMAs are issued by the mui-path waves 0-3
  // only (no GELU: the shorter compute), each two 8-row blocks b = 2 (w & 3) + jj of every part, so
  // the X waves 4-7 start their products right after the barrier, alone on their SIMDs while the
  // partner waits on the address path. lv bit jj: history rows of block jj live (E, and proj when
  // weighted), bit 2 + jj: its candidate rows live
  const bool dma8 = (abl & 64) != 0;   // experiment: every wave issues one block of each part
  auto dma_block = [&](int jj) { return dma8 ? wave : 2 * (wave & 3) + jj; };
  auto item_offsets = [&](int i, int pass, uint32_t* oH, uint32_t* oC, unsigned& lv) {
    const int lane = threadIdx.x & 63;
    const bool live = i < n_i && (dma8 || wave < 4);
    int off = 0, cnt = 1;
    if (live) cands(i, off, cnt);
    const int cntp = max(1, min(64, cnt - 64 * pass));
    lv = 0;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      if (dma8 && jj == 1) break;
      const int row0 = 8 * dma_block(jj);
      if (live && row0 < L) lv |= 1u << jj;
      if (live && WITH_CAND && row0 < cnt - 64 * pass) lv |= 4u << jj;
      const int prow = row0 + (lane >> 3);                    // the ring row this lane fills
      const int rowp = X6 ? x6row(prow) : prow;                // the logical row it fetches
      const uint32_t poff = (uint32_t)(((lane & 7) ^ (X6 ? x6swz(prow) : f32swz(rowp))) << 4);
      int h = 0, c = 0;
      if (live) {
        h = l1_his(smem, i & 3)[min(rowp, L - 1)];
        if (WITH_CAND) c = l1_cand(smem, i & 3)[min(64 * pass + min(rowp, cntp - 1), kMaxCand - 1)];
      }
      h = min(max(h, 0), p.n_news - 1);
      c = min(max(c, 0), p.n_news - 1);
      const uint32_t rowBytes = (uint32_t)d * 4u;
      oH[jj] = (uint32_t)h * rowBytes + poff;
      oC[jj] = (uint32_t)c * rowBytes + poff;
    }
    lv = __builtin_amdgcn_readfirstlane(lv);
  };
  const bool abl_nodma = (abl & 2) != 0, abl_nocomp = (abl & 4) != 0;   // timing ablations (outputs wrong)
  NS_STAMP_DECL
  auto dma32 = [&](const uint32_t* oH, const uint32_t* oC, unsigned lv, int ich, int slot) {
    if (abl_nodma || lv == 0) return;
    const char* bE = tabB + ich * kF32CW * 4;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const unsigned m = sbase + slot * Cf::SLOT + dma_block(jj) * 1024;
      if (lv & (1u << jj)) {
        dma_row(oH[jj], bE, m);
        if constexpr (WEIGHTED) dma_row(oH[jj], prjB + ich * kF32CW * 4, m + Cf::PART);
      }
      if (lv & (4u << jj)) dma_row(oC[jj], bE, m + 2 * Cf::PART);
    }
  };

  // ---- per-lane LDS offsets (fixed for the launch) ----
  uint32_t hOff[2], cOff;
  {
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {       // history operand rows 4s + g, s of parity sp
      const int row = 4 * sp + g;
      hOff[sp] = row * 128 + (((4 * ct + (j >> 2)) ^ f32swz(row)) << 4) + (j & 3) * 4;
    }
    cOff = j * 128 + (((4 * ct + g) ^ f32swz(j)) << 4);
  }
  // X6: history operand rows 8g + i of a 32-row block, columns 2j, 2j + 1 (one ds_read_b64; the
  // block offset 4096 kb is added at the read); candidate operand rows 16q + j, pieces 2g + u
  uint32_t xeOff[8], xcOff[2];
  if constexpr (X6) {
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pr = x6row(8 * g + i);
      xeOff[i] = pr * 128 + (((j >> 1) ^ x6swz(pr)) << 4) + (j & 1) * 8;
    }
    const int prc = x6row(j);
#pragma unroll
    for (int u = 0; u < 2; ++u) xcOff[u] = prc * 128 + (((2 * g + u) ^ x6swz(prc)) << 4);
  }
  // Aᵀ B operand: aw[s] = A[16 kt + j][aw_row(s)]; fp32 MFMA: history slot 4s + g; X6: slot
  // 32 (s >> 3) + 8g + (s & 7), split per 32-slot block into awx[kb]
  float aw[16];
  Split8 awx[2];
  auto aw_row = [&](int s, int g) { return X6 ? 32 * (s >> 3) + 8 * g + (s & 7) : 4 * s + g; };
  auto split_aw = [&]() {
    if constexpr (X6) {
      awx[0] = split8(aw);
      awx[1] = split8(aw + 8);
    }
  };
  auto load_aw = [&](int i) {
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const float* lg = reinterpret_cast<const float*>(smem + kOffLog + (i & 1) * kLogB);
#pragma unroll
    for (int s = 0; s < 16; ++s) aw[s] = lg[aw_row(s, g) * 32 + 16 * kt + j];
    split_aw();
  };
  auto softmax_inwave = [&](int i) {       // small d: every wave computes its A slice itself
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const int k = 16 * kt + j;
    const float* lgb = reinterpret_cast<const float*>(smem + kOffLog + (i & 1) * kLogB);
    const float* pr = reinterpret_cast<const float*>(smem + kOffPrep + (i & 1) * kPrepB);
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int l = aw_row(s, g);
      aw[s] = __builtin_fmaf(lgb[l * 32 + k], pr[l], pr[64 + l]);
      mx = fmaxf(mx, aw[s]);
    }
    mx = rows4_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      aw[s] = expf(aw[s] - mx);            // exp(-inf) = 0 past L
      sum += aw[s];
    }
    sum = rows4_sum(sum);
    float inv = 1.0f / sum;
    if (k >= KK) inv = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) aw[s] *= inv;
    split_aw();
  };

  if constexpr (true) {                    // ring rows no DMA writes read as zeros
    for (int o = (int)threadIdx.x * 16; o < kRingB; o += kThreads * 16)
      *reinterpret_cast<u32x4*>(smem + o) = u32x4{0u, 0u, 0u, 0u};
  }
  // ---- prologue: aux for the first impressions, A of impression 0, then the first pair ----
  for (int i = 0; i < 4; ++i) issue_L0(i);
  vm_wait_all();
  raw_barrier();
  issue_L1(0); issue_L1(1); issue_L1(2);
  vm_wait_all();
  raw_barrier();
  issue_L2(0); issue_L2(1);
  prep_softmax(0); prep_softmax(1);
  vm_wait_all();
  raw_barrier();
  if (coop) {
    soft_phase(0, 1);
    raw_barrier();
    soft_phase(0, 2);
    raw_barrier();
  }
  uint32_t cH[2], cC[2], nH[2] = {0u, 0u}, nC[2] = {0u, 0u};
  unsigned cLv = 0, nLv = 0;
  item_offsets(0, 0, cH, cC, cLv);
  dma32(cH, cC, cLv, 0, 0);
  dma32(cH, cC, cLv, 1, 1);

  f32x4v acc[4];                               // M / Lg partials of this wave, candidate tiles 0..3
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f32x4v{0.f, 0.f, 0.f, 0.f};
  int pend_off = -1, pend_cnt = 0;
  int t = 0;

  // S7 on waves 4-7 (the X waves, which wait at the barrier otherwise): wave w candidates [16(w-4), +16) of the finished pass, lane (kq, c) interests
  // [8kq, 8kq+8); the 4 lane rows combined by permlanes (model.py:128-136, :213-214)
  const bool s7lo = (abl & 128) != 0;  // experiment: S7 on waves 0-3
  auto s7 = [&]() {
    if (s7lo ? wave >= 4 : wave < 4) return;
    const int lane = threadIdx.x & 63;
    const int cl = lane & 15, kq = lane >> 4;
    const int c = 16 * (wave & 3) + cl;
    const float* F0 = reinterpret_cast<const float*>(smem + kOffX + 16384);
    const float* F1 = F0 + 2048;
    const float* G = reinterpret_cast<const float*>(smem + kOffX);    // split_f: [P][ct] blocks of 2048
    const int sw = (c >> 1) & 31;
    float lg[8], m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = c * 32 + ((8 * kq + j) ^ sw);
      if (split_f) {
        m[j] = G[o] + G[2048 + o];
        if constexpr (WEIGHTED) lg[j] = G[4096 + o] + G[6144 + o];
      } else {
        m[j] = F0[o];
        if constexpr (WEIGHTED) lg[j] = F1[o];
      }
    }
    float sc;
    if constexpr (WEIGHTED) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) mx = fmaxf(mx, lg[j]);
      mx = rows4_max(mx);
      float sm = 0.f, num = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (8 * kq + j < KK) {
          const float pe = expf(lg[j] - mx);
          sm += pe;
          num = __builtin_fmaf(pe, m[j], num);
        }
      }
      sm = rows4_sum(sm);
      num = rows4_sum(num);
      sc = num / sm;
    } else {
      if (p.score_type == MINER_SCORE_MAX) {
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) mx = fmaxf(mx, m[j]);
        sc = rows4_max(mx);
      } else {
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) if (8 * kq + j < KK) sm += m[j];
        sc = rows4_sum(sm) / (float)KK;
      }
    }
    if (kq == 0 && c < pend_cnt) p.scores[pend_off + c] = sc;
  };


  // the history and candidate products of the chunk PAIR (cc0, cc0 + 1) in slots t, t + 1; mode: 1
  // history product, 2 candidate product, 4 mui out. NST history steps (rows 4s + g, s < NST: A = 0
  // past L) and NT candidate tiles are compile-time, so all LDS reads issue before the MFMAs, and the
  // two chunks' chains interleave (one chunk's GELU beside the other's MFMAs).
  auto compute_t = [&](int ci, int cc0, int mode, auto nst_c, auto nt_c) {
    constexpr int NST = decltype(nst_c)::value;
    constexpr int NT = decltype(nt_c)::value;
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const char* s0 = smem + (t & (NS - 1)) * Cf::SLOT;
    const char* s1 = smem + ((t + 1) & (NS - 1)) * Cf::SLOT;
    float a0[NST], a1[NST];
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      a0[s] = *reinterpret_cast<const float*>(s0 + P * Cf::PART + hOff[s & 1] + (s >> 1) * 1024);
      a1[s] = *reinterpret_cast<const float*>(s1 + P * Cf::PART + hOff[s & 1] + (s >> 1) * 1024);
    }
    f32x4v h00 = f32x4v{0.f, 0.f, 0.f, 0.f}, h01 = h00, h10 = h00, h11 = h00;
    // (the ablation branch below also shapes the schedule: without it, and with the chains
    // started on an inline-zero accumulator instead, the kernel measured 7 % slower in a clean
    // per-commit A/B, tools/bisect_news.py; one chain per chunk +5 %)
    if (abl & 32) { h00[0] = a0[0]; h10[0] = a1[0]; } else
#pragma unroll
    for (int s = 0; s < NST; s += 2) {
      h00 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], aw[s], h00, 0, 0, 0);
      h10 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], aw[s], h10, 0, 0, 0);
      if (s + 1 < NST) {
        h01 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s + 1], aw[s + 1], h01, 0, 0, 0);
        h11 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s + 1], aw[s + 1], h11, 0, 0, 0);
      }
    }
    f32x4v x0 = h00 + h01, x1 = h10 + h11;
    if ((mode & 4) && 16 * kt + j < KK) {
      float* dst = mui_out + ((size_t)imp_b(ci) * KK + 16 * kt + j) * d + kF32CW * cc0 + 16 * ct + 4 * g;
      *reinterpret_cast<float4*>(dst) = make_float4(x0[0], x0[1], x0[2], x0[3]);
      *reinterpret_cast<float4*>(dst + kF32CW) = make_float4(x1[0], x1[1], x1[2], x1[3]);
    }
    if (mode & 2) {
      f32x4v cf0[NT], cf1[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        cf0[q] = *reinterpret_cast<const f32x4v*>(s0 + 2 * Cf::PART + cOff + q * 2048);
        cf1[q] = *reinterpret_cast<const f32x4v*>(s1 + 2 * Cf::PART + cOff + q * 2048);
      }
      if (WEIGHTED && P == 1 && !(abl & 8)) {
        if (abl & 2048) {            // A/B: the Numerical Recipes erfc form
#pragma unroll
          for (int e = 0; e < 4; ++e) x0[e] = gelu_erfc_nr(x0[e]);
        } else {
          gelu_as_pairs(x0, 4);
        }
      }
      if (abl & 16) {
#pragma unroll
        for (int q = 0; q < NT; ++q) acc[q] += cf0[q] * x0 + cf1[q] * x1;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int q = 0; q < NT; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(cf0[q][e], x0[e], acc[q], 0, 0, 0);
        }
        if (WEIGHTED && P == 1 && !(abl & 8)) {
          if (abl & 2048) {
#pragma unroll
            for (int e = 0; e < 4; ++e) x1[e] = gelu_erfc_nr(x1[e]);
          } else {
            gelu_as_pairs(x1, 4);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int q = 0; q < NT; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(cf1[q][e], x1[e], acc[q], 0, 0, 0);
        }
      }
    }
  };
  // X6: this wave's chunk cc0 + ct of the pair (slot t + ct); NKB 32-slot history blocks, NT
  // candidate tiles, compile-time
  auto compute_x6 = [&](int ci, int cc0, int mode, auto nkb_c, auto nt_c) {
    constexpr int NKB = decltype(nkb_c)::value;
    constexpr int NT = decltype(nt_c)::value;
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const char* sl = smem + ((t + ct) & (NS - 1)) * Cf::SLOT;
    const char* hp = sl + P * Cf::PART;
    f32x4v h0 = f32x4v{0.f, 0.f, 0.f, 0.f}, h1 = h0;    // columns 2(4g + e) and 2(4g + e) + 1
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      float e0[8], e1[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float2 v = *reinterpret_cast<const float2*>(hp + kb * 4096 + xeOff[i]);
        e0[i] = v.x;
        e1[i] = v.y;
      }
      if (abl & 32) {                        // timing ablation: no history product
        h0[0] += e0[0];
        h1[0] += e1[0];
      } else {
        h0 = mma_x6(h0, split8(e0), awx[kb]);
        h1 = mma_x6(h1, split8(e1), awx[kb]);
      }
      __builtin_amdgcn_sched_barrier(0);       // one block's operands live at a time (VGPR budget)
    }
    NS_STAMP(4);
    const int col0 = kF32CW * (cc0 + ct) + 8 * g;          // this lane's columns col0 .. col0 + 7
    if ((mode & 4) && 16 * kt + j < KK) {
      float* dst = mui_out + ((size_t)imp_b(ci) * KK + 16 * kt + j) * d + col0;
      *reinterpret_cast<float4*>(dst) = make_float4(h0[0], h1[0], h0[1], h1[1]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(h0[2], h1[2], h0[3], h1[3]);
    }
    if (mode & 2) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[2 * e] = h0[e];
        x[2 * e + 1] = h1[e];
      }
      if (WEIGHTED && P == 1 && !(abl & 8)) {
        gelu_as_pairs(x, 8);
      }
      const Split8 sb = split8(x);
      NS_STAMP(5);
      const char* cpart = sl + 2 * Cf::PART;
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        float c[8];
        *reinterpret_cast<float4*>(c) = *reinterpret_cast<const float4*>(cpart + q * 2048 + xcOff[0]);
        *reinterpret_cast<float4*>(c + 4) = *reinterpret_cast<const float4*>(cpart + q * 2048 + xcOff[1]);
        if (abl & 16) acc[q][0] += c[0] + sb.hi[0];   // timing ablation: no candidate product
        else acc[q] = mma_x6(acc[q], split8(c), sb);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  using I4 = std::integral_constant<int, 4>;
  auto compute = [&](int ci, int cc0, int mode, int ntile) {
    if (!(mode & 1) || abl_nocomp) return;
    if constexpr (X6) {
      auto by_nt = [&](auto nkb_c) {
        if (!(mode & 2) || ntile >= 4) compute_x6(ci, cc0, mode, nkb_c, I4{});
        else if (ntile == 3) compute_x6(ci, cc0, mode, nkb_c, std::integral_constant<int, 3>{});
        else if (ntile == 2) compute_x6(ci, cc0, mode, nkb_c, std::integral_constant<int, 2>{});
        else compute_x6(ci, cc0, mode, nkb_c, std::integral_constant<int, 1>{});
      };
      if (L <= 32) by_nt(std::integral_constant<int, 1>{});
      else by_nt(std::integral_constant<int, 2>{});
      return;
    }
    auto by_nt = [&](auto nst_c) {
      if (!(mode & 2) || ntile >= 4) compute_t(ci, cc0, mode, nst_c, I4{});
      else if (ntile == 3) compute_t(ci, cc0, mode, nst_c, std::integral_constant<int, 3>{});
      else if (ntile == 2) compute_t(ci, cc0, mode, nst_c, std::integral_constant<int, 2>{});
      else compute_t(ci, cc0, mode, nst_c, std::integral_constant<int, 1>{});
    };
    if (nsteps <= 8) by_nt(std::integral_constant<int, 8>{});
    else if (nsteps <= 13) by_nt(std::integral_constant<int, 13>{});
    else by_nt(std::integral_constant<int, 16>{});
  };

  // static priority for the X-path waves 4-7 (the GELU chain, the longer one of each SIMD's pair)
  if (!(abl & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int npair = nchunk >> 1;
  for (int ci = 0; ci < n_i; ++ci) {
    int c_off, c_cnt;
    cands(ci, c_off, c_cnt);
    const int cn = max(1, (c_cnt + 63) >> 6);
    for (int cp = 0; cp < cn; ++cp) {
      const int cntp = min(64, c_cnt - 64 * cp);
      const int ntile = (max(cntp, 1) + 15) >> 4;
      const bool need_mui = P == 0 && mui_out != nullptr && cp == 0;
      const bool need_c = WITH_CAND && path_live;
      const int mode = (k_live && path_live && (need_c || need_mui)) ? (1 | (need_c ? 2 : 0) | (need_mui ? 4 : 0)) : 0;
      const int ni = cp + 1 < cn ? ci : ci + 1, np = cp + 1 < cn ? cp + 1 : 0;
      for (int u = 0; u < npair; ++u, t += 2) {
        NS_STAMP(7);
        vm_wait_all();                 // this pair's rows (and every older DMA) landed for this wave,
        NS_STAMP(0);
        raw_barrier();                 // then for every wave; the previous pair's slots are free
        NS_STAMP(1);
        if (u == 0) {
          if (!X6) NS_STAMP(2);
          if (WITH_CAND && pend_off >= 0) s7();
          if (!X6) NS_STAMP(4);          // fp32-MFMA form: stage 4 = S7, stage 5 = in-wave softmax
          pend_off = -1;
          if (cp == 0) {
            if (smode == 1) {
              load_aw(ci);
            } else if (smode == 2) {
              softmax_inwave(ci);
              if (!X6) NS_STAMP(5);
            } else {
              softmax_inwave(ci);
              raw_barrier();           // every wave has read impression ci's logit rows
              issue_L2(ci + 2);
            }
            issue_L0(ci + 4);
            issue_L1(ci + 3);
            if (smode != 2) prep_softmax(ci + 2);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] = f32x4v{0.f, 0.f, 0.f, 0.f};
        } else if (smode == 2 && cp == 0 && u == 1) {
          issue_L2(ci + 2);            // into the block impression ci's logits were read from
          prep_softmax(ci + 2);
        } else if (coop && cp == 0) {
          if (u == 1) {
            issue_L2(ci + 2);          // into the rows A of ci was read from (free since the barrier)
            soft_phase(ci + 1, 1);
          } else if (u == 2) {
            soft_phase(ci + 1, 2);
          }
        }
        NS_STAMP(2);
        if (u + 1 < npair) {           // the next pair of this item, else the first pair of the next one
          dma32(cH, cC, cLv, 2 * u + 2, (t + 2) & (NS - 1));
          dma32(cH, cC, cLv, 2 * u + 3, (t + 3) & (NS - 1));
        } else {
          item_offsets(ni, np, nH, nC, nLv);
          dma32(nH, nC, nLv, 0, (t + 2) & (NS - 1));
          dma32(nH, nC, nLv, 1, (t + 3) & (NS - 1));
        }
        NS_STAMP(3);
        compute(ci, 2 * u, mode, ntile);
        NS_STAMP(6);
      }
      if (WITH_CAND && split_f) {
        // pass done (npair >= 2): every wave publishes its partial M / Lg [c][k ^ swizzle] into its
        // own block F[P][ct], no barrier; S7, after the next pair's barrier, sums the two column-tile
        // partials in the order of the hand-off below (ct 0 + ct 1). The next pass end is at least
        // one barrier after that S7.
        const int lane = threadIdx.x & 63;
        const int j = lane & 15, g = lane >> 4;
        if (path_live && k_live) {
          float* F = reinterpret_cast<float*>(smem + kOffX) + (P * 2 + ct) * 2048;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (q < ntile) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int c = 16 * q + 4 * g + e;
                F[c * 32 + ((16 * kt + j) ^ ((c >> 1) & 31))] = acc[q][e];
              }
            }
          }
        }
      } else if constexpr (WITH_CAND) {
        // pass done: the ct = 1 waves hand their partials to the ct = 0 waves of the same (P, kt),
        // which publish the final M / Lg [c][k ^ swizzle] for S7
        const int lane = threadIdx.x & 63;
        const int j = lane & 15, g = lane >> 4;
        float* R = reinterpret_cast<float*>(smem + kOffX) + (P * 2 + kt) * 1024;
        if (path_live && k_live && ct == 1) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (q < ntile) {
#pragma unroll
              for (int e = 0; e < 4; ++e) R[(16 * q + 4 * g + e) * 16 + j] = acc[q][e];
            }
          }
        }
        raw_barrier();
        if (path_live && k_live && ct == 0) {
          float* F = reinterpret_cast<float*>(smem + kOffX + 16384) + P * 2048;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (q < ntile) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int c = 16 * q + 4 * g + e;
                F[c * 32 + ((16 * kt + j) ^ ((c >> 1) & 31))] = acc[q][e] + R[c * 16 + j];
              }
            }
          }
        }
      }
      pend_off = c_off + 64 * cp;
      pend_cnt = cntp;
      cH[0] = nH[0]; cH[1] = nH[1]; cC[0] = nC[0]; cC[1] = nC[1]; cLv = nLv;
      NS_STAMP(7);
    }
  }
  NS_STAMP_FLUSH(n_i);
  vm_wait_all();
  raw_barrier();
  if (WITH_CAND && pend_off >= 0) s7();
}

// ================================================================================================
// host side
// ================================================================================================
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

inline bool aligned16(const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15u) == 0; }

int check_news(int dtype, int L, int d, int Dc, int K) {
  if (dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16 && dtype != MINER_DTYPE_F32_X6) return MINER_EINVAL;
  if (L <= 0 || d <= 0 || K <= 0 || Dc <= 0) return MINER_EINVAL;
  if (L > kMaxL || K > kMaxK || (K & 3) || d % 64 || d > kMaxD || Dc > kMaxDc) return MINER_ESHAPE;
  return MINER_OK;
}

int pre_lds(int dtype, int d, int Dc) {
  const int es = dtype == MINER_DTYPE_BF16 ? 2 : 4;
  const int R = dtype == MINER_DTYPE_BF16 ? 64 : 32;
  return R * d * es + n_ct(Dc) * (R / 32) * 16 * 64 * 4;
}
constexpr int kPreUnitB = 32 * 4;   // fp32 pairs: the 32 staged rows' units after the partials

template <class T, int NS, bool P2 = false>
int launch_pre(void* stream, const PreParams& prm, int lds) {
  auto kern = news_pre<T, NS, P2>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return (int)e;
  const int R = kPreRows<T>;
  int grid = (prm.N + R - 1) / R;
  if (grid > num_cus()) grid = num_cus();
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

template <int NSL>
int launch_pre2(void* stream, const PreParams& prm) {
  auto kern = news_pre2<NSL>;
  const int lds = kP2QOff + 32 * n_ct(prm.Dc) * 32 * 2;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(kern, dim3(num_cus()), dim3(kThreads), lds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

// P2: fp32 on fp16 pairs (MINER_DTYPE_F32); fp32 with P2 false: the fp32 MFMA (MINER_DTYPE_F32_MFMA)
template <class T, bool P2 = false>
int run_pre(void* stream, const PreParams& prm, int lds) {
  if constexpr (sizeof(T) == 2) {     // bf16: the GEMM-shaped news_pre2 (round 1 v7: 0.34 -> 0.23 ms)
    return prm.d == 768 ? launch_pre2<24>(stream, prm) : launch_pre2<0>(stream, prm);
  } else {
    switch (prm.d >> 5) {
      case 2: return launch_pre<T, 2, P2>(stream, prm, lds);
      case 4: return launch_pre<T, 4, P2>(stream, prm, lds);
      case 8: return launch_pre<T, 8, P2>(stream, prm, lds);
      case 16: return launch_pre<T, 16, P2>(stream, prm, lds);
      case 24: return launch_pre<T, 24, P2>(stream, prm, lds);
      default: return launch_pre<T, 0, P2>(stream, prm, lds);
    }
  }
}

// x6: news_score32's bf16x6 form (dtype MINER_DTYPE_F32_X6) instead of the fp32-MFMA one
template <class T>
int launch_score(void* stream, const NsParams& prm, bool x6 = false) {
  void (*kern)(NsParams) = nullptr;
  const bool rg = prm.cand_off != nullptr;
#define NEWS_PICK_NS(PDV, CWV, NCHV, SHPV)                                                               \
  switch (prm.score_type) {                                                                            \
    case MINER_SCORE_WEIGHTED: kern = rg ? news_score<T, MINER_SCORE_WEIGHTED, true, PDV, CWV, NCHV, SHPV> : news_score<T, MINER_SCORE_WEIGHTED, false, PDV, CWV, NCHV, SHPV>; break; \
    case MINER_SCORE_NONE: kern = news_score<T, MINER_SCORE_NONE, false, PDV, CWV, NCHV, SHPV>; break;                   \
    default: kern = rg ? news_score<T, MINER_SCORE_MAX, true, PDV, CWV, NCHV, SHPV> : news_score<T, MINER_SCORE_MAX, false, PDV, CWV, NCHV, SHPV>; break; \
  }
#define NEWS_PICK_N(PDV, CWV, NCHV) NEWS_PICK_NS(PDV, CWV, NCHV, 0)
#define NEWS_PICK(PDV, CWV) NEWS_PICK_N(PDV, CWV, 0)
  if constexpr (sizeof(T) == 2) {
    const int nchunk = prm.d >> 6;
    const bool mind = prm.L == 50 && prm.K == 32;   // MIND: history 50, 32 interests
    if (prm.d % 128 == 0 && prm.d >= 512) {
      // config 3: compile-time chunk count (the compile-time shape measured 1.1 % slower here)
      if (prm.d == 768) { NEWS_PICK_N(1, 128, 6) }
      else { NEWS_PICK(1, 128) }       // 128-column chunks, double-buffered
    } else if (prm.d == 256) {         // config 2
      if (mind) { NEWS_PICK_NS(3, 64, 4, 1) } else { NEWS_PICK_N(3, 64, 4) }
    } else if (nchunk >= 3) {
      NEWS_PICK(3, 64)
    } else if (nchunk == 2) {
      NEWS_PICK(2, 64)
    } else {
      NEWS_PICK(1, 64)
    }
  } else {
    // fp32: news_score32 on the fp32 matrix cores (exact fp32 fma chains, 16x16x4 tiles, 32-column
    // chunks computed in pairs); dtype MINER_DTYPE_F32_X6 selects the bf16x6 form (same accuracy
    // class, bf16 matrix cores; measured equal speed at config 3)
#define NEWS_PICK32S(X6V, NCH, SHPV)                                                                     \
    switch (prm.score_type) {                                                                            \
      case MINER_SCORE_WEIGHTED: kern = rg ? news_score32<MINER_SCORE_WEIGHTED, true, X6V, NCH, SHPV> : news_score32<MINER_SCORE_WEIGHTED, false, X6V, NCH, SHPV>; break; \
      case MINER_SCORE_NONE: kern = news_score32<MINER_SCORE_NONE, false, X6V, NCH, SHPV>; break;               \
      default: kern = rg ? news_score32<MINER_SCORE_MAX, true, X6V, NCH, SHPV> : news_score32<MINER_SCORE_MAX, false, X6V, NCH, SHPV>; break; \
    }
#define NEWS_PICK32(X6V, NCH) NEWS_PICK32S(X6V, NCH, 0)
    const bool mind = prm.L == 50 && prm.K == 32;          // MIND: history 50, 32 interests
    const bool plain = !prm.bias && !prm.mui_out;          // no bias, no mui output
    if (prm.d == 768) {                // config 3 (MIND-large): the chunk count compile-time
      if (x6) { NEWS_PICK32(true, 24) }
      else if (mind && plain) { NEWS_PICK32S(false, 24, 2) }
      else if (mind) { NEWS_PICK32S(false, 24, 1) }
      else { NEWS_PICK32(false, 24) }
    } else if (prm.d == 256) {         // config 2 (MIND-small)
      if (x6) { NEWS_PICK32(true, 8) }
      else if (mind && plain) { NEWS_PICK32S(false, 8, 2) }
      else if (mind) { NEWS_PICK32S(false, 8, 1) }
      else { NEWS_PICK32(false, 8) }
    } else {
      if (x6) { NEWS_PICK32(true, 0) } else { NEWS_PICK32(false, 0) }
    }
#undef NEWS_PICK32
#undef NEWS_PICK32S
  }
#undef NEWS_PICK
#undef NEWS_PICK_N
#undef NEWS_PICK_NS
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kNewsLds);
  if (e != hipSuccess) return (int)e;
  int grid = num_cus();
  if (grid > prm.B) grid = prm.B;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), kNewsLds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
#ifdef MINER_NEWS_DEBUG
  unsigned long long h[4] = {0, 0, 0, 0};
  hipStreamSynchronize(static_cast<hipStream_t>(stream));
  hipMemcpyFromSymbol(h, HIP_SYMBOL(g_news_dbg), sizeof(h));
  fprintf(stderr, "[news_score debug] kinds=0x%llx off_odd=%lld off_even=%lld lds=%lld\n", h[0], (long long)h[1] - 1,
          (long long)h[2] - 1, (long long)h[3] - 1);
  unsigned long long z[4] = {0, 0, 0, 0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_news_dbg), z, sizeof(z));
#endif
  return e == hipSuccess ? MINER_OK : (int)e;
}

}  // namespace

extern "C" {

#ifdef MINER_STAMPS
// diagnostic build only: read (and reset) the per-wave stage cycles of news_score32;
// out[8 w + i] = cycles of stage i of wave w summed over workgroups, out[64] = impressions
int miner_news_debug_stage_cycles(unsigned long long* out) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ns_stage), 64 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(g_ns_items), sizeof(unsigned long long));
  unsigned long long z[64] = {0};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_ns_stage), z, 64 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_ns_items), z, sizeof(unsigned long long));
  return (int)e;
}
#endif

int miner_news_supported(int dtype, int L, int d, int Dc, int K) {
  const int rc = check_news(dtype, L, d, Dc, K);
  if (rc != MINER_OK) return rc;
  return pre_lds(dtype, d, Dc) > kLdsMax ? MINER_ELDS : MINER_OK;
}

int miner_news_precompute(void* stream, int dtype, const void* news_table, int n_news, const void* packed_weights,
                          int d, int Dc, int K, float* news_logits, void* news_proj) {
  if (!news_table || !packed_weights || !news_logits || n_news <= 0 || dtype == MINER_DTYPE_F32_X6) return MINER_EINVAL;
  const bool mfma32 = dtype == MINER_DTYPE_F32_MFMA;   // fp32 tables, every product on the fp32 MFMA
  if (mfma32) dtype = MINER_DTYPE_F32;
  const int rc = miner_news_supported(dtype, 1, d, Dc, K);
  if (rc != MINER_OK) return rc;
  if (!aligned16(news_table) || !aligned16(packed_weights) || !aligned16(news_logits) || !aligned16(news_proj))
    return MINER_EALIGN;
  PreParams prm{news_table, packed_weights, news_logits, news_proj, n_news, d, Dc, K};
  const int lds = pre_lds(dtype, d, Dc);
  if (dtype == MINER_DTYPE_BF16) return run_pre<__bf16>(stream, prm, lds);
  // the pair form needs 128 more bytes: at the one shape where the fp32 carve is the whole 160 KiB
  // (d = 1024, Dc = 256) the fp32-MFMA form runs instead
  if (mfma32 || lds + kPreUnitB > kLdsMax) return run_pre<float, false>(stream, prm, lds);
  return run_pre<float, true>(stream, prm, lds + kPreUnitB);
}

int miner_score_news(void* stream, int dtype, int score_type, const void* news_table, const float* news_logits,
                     const void* news_proj, int n_news, const int32_t* his_ids, const uint8_t* his_mask,
                     const float* his_bias, const int32_t* cand_ids, const int32_t* cand_offsets, int B, int L,
                     int C, int d, int K, float* scores, float* user_out) {
  if (score_type < MINER_SCORE_WEIGHTED || score_type > MINER_SCORE_NONE) return MINER_EINVAL;
  if (!news_table || !news_logits || !his_ids || !his_mask || n_news <= 0 || B < 0) return MINER_EINVAL;
  const int rc = check_news(dtype, L, d, 1, K);
  if (rc != MINER_OK) return rc;
  if (score_type == MINER_SCORE_WEIGHTED && !news_proj) return MINER_EINVAL;
  if (score_type != MINER_SCORE_NONE) {
    if (!scores || !cand_ids) return MINER_EINVAL;
    if (!cand_offsets && (C < 0 || C > kMaxCand)) return MINER_ESHAPE;
  } else if (!user_out) {
    return MINER_EINVAL;
  }
  if (!aligned16(news_table) || !aligned16(news_logits) || !aligned16(news_proj)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  // timing-ablation bits of the diagnostic tools (tools/news_ablate.py): read once per process;
  // news_score32 compiles them out of the product build (MINER_NEWS_ABL_MASK = 0)
  static const int abl = [] { const char* e = getenv("MINER_NEWS_ABL"); return e ? atoi(e) : 0; }();
  NsParams prm{news_table, news_logits, news_proj, his_ids, his_mask, his_bias,
               score_type == MINER_SCORE_NONE ? nullptr : cand_ids,
               score_type == MINER_SCORE_NONE ? nullptr : cand_offsets,
               scores, user_out, n_news, B, L, score_type == MINER_SCORE_NONE ? 0 : C, d, K, score_type,
               abl};
  return dtype == MINER_DTYPE_BF16 ? launch_score<__bf16>(stream, prm)
                                   : launch_score<float>(stream, prm, dtype == MINER_DTYPE_F32_X6);
}

}  // extern "C"
