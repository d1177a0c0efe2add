// miner_score.hip — fused MINER scoring kernel for MI355X (gfx950 / CDNA4).
//
// One workgroup (8 waves, 512 threads) scores one impression at a time and walks impressions
// b = blockIdx.x, blockIdx.x + gridDim.x, ...  Everything between the HBM reads of the
// impression's history/candidate rows and the fp32 score writes stays on chip:
//
//   S0  history rows E[L,d] -> LDS (bf16 mode; fp32 mode streams them from L2 instead)
//   S1  Pᵀ = tanh(W1 · Eᵀ)          [Dc,L]   MFMA, wave w owns Dc-tile w          (model.py:171)
//   S2  Sᵀ = Q · Pᵀ                 [K,L]    MFMA on the S1 accumulators, ds_add  (model.py:174)
//   S3  A  = softmax_L(fill(Sᵀ))   [K,L]    wave shuffles; masked -> 1e-30       (model.py:178-181)
//   S4  mui = A · E                 [K,d]    MFMA (E read transposed from LDS)    (model.py:182)
//   S5  X  = gelu(W2 · muiᵀ)       [d,K]    MFMA, wave w owns d-tiles w, w+8, .. (model.py:212)
//   S6  Lgᵀ = Xᵀ·Candᵀ, Mᵀ = mui·Candᵀ [K,C] MFMA on the S5 accumulators, ds_add (model.py:127,213)
//   S7  score_c = Σ_k softmax_K(Lg)_k · M_k  (or max_k / mean_k of M)            (model.py:128-134,213-214)
//
// Operand layout (both dtypes) — "slab" = 32 consecutive contraction indices:
//   lane l = 32h + r (h = l>>5, r = l&31) holds 16 contiguous elements [16h, 16h+16) of row r of
//   the slab.  bf16: two v_mfma_f32_32x32x16_bf16 steps (8 elements each); fp32: sixteen
//   v_mfma_f32_32x32x2_f32 steps (1 element each, exact fp32 fma chain).  The accumulator of a
//   32x32 MFMA tile keeps row (e&3)+8(e>>2)+4h of column r in register e; loading the A-operand
//   rows of a GEMM in the order pi(r) = 16((r>>2)&1) + (r&3) + 4(r>>3) makes register e of lane
//   half h hold row 16h+e — i.e. the accumulator IS a slab fragment of the next contraction, with
//   no LDS round trip (S1->S2, S5->S6).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/miner_score.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kMaxL = 64;        // history positions per impression (two 32-row tiles)
constexpr int kMaxK = 32;        // interest vectors (one 32-row tile)
constexpr int kMaxDc = 256;      // context-code dim (one 32-row tile per wave)
constexpr int kMaxD = 768;       // embedding dim (<= 3 d-tiles per wave in S5)
constexpr int kMaxJ = kMaxD / 32 / kWaves;
constexpr int kCChunk = 64;      // candidates per S6/S7 pass
constexpr int kLdsMax = 160 * 1024;

enum Mode { kFull = 0, kTaa = 1 };

struct Params {
  const void* hist;
  const uint8_t* mask;
  const float* bias;
  const void* cand;
  const int32_t* cand_off;
  const void* W1;
  const void* Q;
  const void* W2;
  const float* value;  // TAA mode: [sum C_b, K]
  float* scores;
  float* mui_out;
  int B, L, C, d, Dc, K, score_type;
  // LDS carve (bytes)
  int ES;      // history row stride (bf16 mode)
  int MS;      // mui row stride
  int offE, offZ, offLg, offMt, offMui, offS, offAw;
};

// ---------------------------------------------------------------------------------------------
// element helpers
// ---------------------------------------------------------------------------------------------
template <class T> struct Frag;            // one lane's 16-element slab fragment
template <> struct Frag<__bf16> { u32x4 q[2]; };
template <> struct Frag<float> { u32x4 q[4]; };

template <class T>
__device__ __forceinline__ void frag_zero(Frag<T>& f) {
#pragma unroll
  for (int i = 0; i < (int)(sizeof(f.q) / sizeof(u32x4)); ++i) f.q[i] = u32x4{0u, 0u, 0u, 0u};
}

// 16 contiguous elements from a 16-byte-aligned address (global or LDS).
template <class T>
__device__ __forceinline__ void frag_load(Frag<T>& f, const T* p) {
  const u32x4* s = reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(f.q) / sizeof(u32x4)); ++i) f.q[i] = s[i];
}

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__bf16 x) { return (float)x; }
template <class T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  __bf16 a = (__bf16)lo, b = (__bf16)hi;
  unsigned short ua = __builtin_bit_cast(unsigned short, a);
  unsigned short ub = __builtin_bit_cast(unsigned short, b);
  return (unsigned)ua | ((unsigned)ub << 16);
}

// 16 elements with a per-element bound (unaligned / ragged rows, e.g. context codes).
template <class T>
__device__ __forceinline__ void frag_load_pred(Frag<T>& f, const T* row, int start, int limit) {
  float v[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = (start + e < limit) ? to_f32(row[start + e]) : 0.f;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int m = 0; m < 8; ++m) f.q[m >> 2][m & 3] = pack_bf16x2(v[2 * m], v[2 * m + 1]);
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) f.q[e >> 2][e & 3] = __float_as_uint(v[e]);
  }
}

// accumulator tile (rows permuted by pi at load time) -> slab fragment of the next contraction
template <class T>
__device__ __forceinline__ void acc_to_frag(Frag<T>& f, const f32x16& x) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int m = 0; m < 8; ++m) f.q[m >> 2][m & 3] = pack_bf16x2(x[2 * m], x[2 * m + 1]);
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) f.q[e >> 2][e & 3] = __float_as_uint(x[e]);
  }
}

// acc += A(slab) · B(slab) over 32 contraction indices
template <class T>
__device__ __forceinline__ void mma_slab(f32x16& acc, const Frag<T>& a, const Frag<T>& b) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a.q[s]),
                                                    __builtin_bit_cast(bf16x8, b.q[s]), acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.q[t >> 2][t & 3]),
                                                 __uint_as_float(b.q[t >> 2][t & 3]), acc, 0, 0, 0);
  }
}

__device__ __forceinline__ int pi_row(int r) { return 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3); }
__device__ __forceinline__ int acc_row(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// torch.nn.functional.gelu(approximate='none')
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

// bf16-mode transcendentals: branch-free, a handful of VALU ops each.  Their error (tanh: a few
// fp32 ulp of 1; erf: <= 1.5e-7 absolute, Abramowitz & Stegun 7.1.26) is far below the bf16
// operand rounding of that mode.  The fp32 parity mode uses the libm tanhf / erff / expf.
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(fminf(2.8853900817779268f * fabsf(x), 126.f));  // e^{2|x|}
  const float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
  return copysignf(t, x);
}
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float erfz = 1.0f - poly * __builtin_amdgcn_exp2f(-1.4426950408889634f * z * z);
  return 0.5f * x * (1.0f + copysignf(erfz, x));
}
template <class T> __device__ __forceinline__ float act_tanh(float x) {
  if constexpr (sizeof(T) == 2) return tanh_fast(x); else return tanhf(x);
}
template <class T> __device__ __forceinline__ float act_gelu(float x) {
  if constexpr (sizeof(T) == 2) return gelu_fast(x); else return gelu_erf(x);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  return z;
}

// ---------------------------------------------------------------------------------------------
// the fused kernel
// ---------------------------------------------------------------------------------------------
template <class T, int MODE>
__global__ __launch_bounds__(kThreads) void miner_fused(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool kBf16 = sizeof(T) == 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int L = p.L, d = p.d, Dc = p.Dc, K = p.K;
  const T* __restrict__ W1 = static_cast<const T*>(p.W1);
  const T* __restrict__ Qc = static_cast<const T*>(p.Q);
  const T* __restrict__ W2 = static_cast<const T*>(p.W2);
  const bool weighted = (p.score_type == MINER_SCORE_WEIGHTED);
  const bool need_scores = (p.score_type != MINER_SCORE_NONE);

  T* muiL = reinterpret_cast<T*>(smem + p.offMui);   // [K_pad=32][MS bytes]
  float* Lg = reinterpret_cast<float*>(smem + p.offLg);  // [32][kCChunk]
  float* Mt = reinterpret_cast<float*>(smem + p.offMt);  // [32][kCChunk]
  const int msE = p.MS / (int)sizeof(T);                 // mui row stride in elements

  if constexpr (kBf16 && MODE == kFull) {
    if (tid < 4) reinterpret_cast<u32x4*>(smem + p.offZ)[tid] = u32x4{0u, 0u, 0u, 0u};
  }

  for (int b = blockIdx.x; b < p.B; b += gridDim.x) {
    const int cbase = p.cand_off ? p.cand_off[b] : b * p.C;
    const int Cb = p.cand_off ? (p.cand_off[b + 1] - cbase) : p.C;
    const T* __restrict__ cand = static_cast<const T*>(p.cand) + (size_t)cbase * d;

    if constexpr (MODE == kFull) {
      const T* __restrict__ E = static_cast<const T*>(p.hist) + (size_t)b * L * d;
      float* S = reinterpret_cast<float*>(smem + p.offS);  // [32][kMaxL]
      T* Aw = reinterpret_cast<T*>(smem + p.offAw);        // [32][AwS]
      constexpr int AwS = kBf16 ? 72 : 68;

      // ---- S0: history -> LDS (bf16), zero S ------------------------------------------------
      if constexpr (kBf16) {
        const int per_row = d / 8;
        const int n = L * per_row;
        for (int i = tid; i < n; i += kThreads) {
          const int row = i / per_row, c8 = i - row * per_row;
          const u32x4 v = reinterpret_cast<const u32x4*>(E + (size_t)row * d)[c8];
          *reinterpret_cast<u32x4*>(smem + p.offE + row * p.ES + c8 * 16) = v;
        }
      }
      for (int i = tid; i < kMaxK * kMaxL; i += kThreads) S[i] = 0.f;
      __syncthreads();

      // ---- S1 + S2: Sᵀ += Q[:,ct] · tanh(W1[ct,:] · Eᵀ) -------------------------------------
      {
        const int c0 = wave * 32;
        if (c0 < Dc) {
          const int nLt = (L + 31) >> 5;
          f32x16 acc0 = zero16(), acc1 = zero16();
          const int crow = c0 + pi_row(r);
          const bool cvalid = crow < Dc;
          const T* w1row = W1 + (size_t)(cvalid ? crow : 0) * d + 16 * h;
          const int l0 = r, l1 = 32 + r;
          Frag<T> an;
          if (cvalid) frag_load(an, w1row); else frag_zero(an);
          for (int kb = 0; kb < d; kb += 32) {
            Frag<T> a = an, b0, b1;
            if (cvalid && kb + 32 < d) frag_load(an, w1row + kb + 32);
            if constexpr (kBf16) {
              if (l0 < L) frag_load(b0, reinterpret_cast<const T*>(smem + p.offE + l0 * p.ES) + kb + 16 * h);
              else frag_zero(b0);
              if (l1 < L) frag_load(b1, reinterpret_cast<const T*>(smem + p.offE + l1 * p.ES) + kb + 16 * h);
              else frag_zero(b1);
            } else {
              if (l0 < L) frag_load(b0, E + (size_t)l0 * d + kb + 16 * h); else frag_zero(b0);
              if (l1 < L) frag_load(b1, E + (size_t)l1 * d + kb + 16 * h); else frag_zero(b1);
            }
            mma_slab<T>(acc0, a, b0);
            if (nLt > 1) mma_slab<T>(acc1, a, b1);
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) { acc0[e] = act_tanh<T>(acc0[e]); acc1[e] = act_tanh<T>(acc1[e]); }
          // context codes: A operand rows k, contraction over this wave's 32 Dc columns
          Frag<T> qa;
          if (r < K) frag_load_pred(qa, Qc + (size_t)r * Dc, c0 + 16 * h, Dc); else frag_zero(qa);
          Frag<T> pf;
          acc_to_frag(pf, acc0);
          f32x16 s0 = zero16();
          mma_slab<T>(s0, qa, pf);
#pragma unroll
          for (int e = 0; e < 16; ++e) atomicAdd(&S[acc_row(e, h) * kMaxL + r], s0[e]);
          if (nLt > 1) {
            acc_to_frag(pf, acc1);
            f32x16 s1 = zero16();
            mma_slab<T>(s1, qa, pf);
#pragma unroll
            for (int e = 0; e < 16; ++e) atomicAdd(&S[acc_row(e, h) * kMaxL + 32 + r], s1[e]);
          }
        }
      }
      __syncthreads();

      // ---- S3: masked softmax over the history ----------------------------------------------
      {
        const int l = lane;
        const bool in = l < L;
        const bool real = in && p.mask[(size_t)b * L + l] != 0;
        const float bl = (p.bias && in) ? p.bias[(size_t)b * L + l] : 0.f;
#pragma unroll
        for (int kk = 0; kk < kMaxK / kWaves; ++kk) {
          const int k = wave + kWaves * kk;
          float v = in ? (real ? S[k * kMaxL + l] + bl : 1e-30f) : -INFINITY;
          const float m = wave_max(v);
          const float ex = in ? (kBf16 ? __expf(v - m) : expf(v - m)) : 0.f;
          const float sum = wave_sum(ex);
          const float a = (k < K) ? ex / sum : 0.f;
          Aw[k * AwS + l] = from_f32<T>(a);
        }
      }
      __syncthreads();

      // ---- S4: mui = A · E  (rows k, columns i) ---------------------------------------------
      {
        const int nLs = (L + 31) >> 5;
        Frag<T> af0, af1;
        frag_load(af0, Aw + r * AwS + 16 * h);
        if (nLs > 1) frag_load(af1, Aw + r * AwS + 32 + 16 * h); else frag_zero(af1);
        const int nIt = d >> 5;
        for (int it = wave; it < nIt; it += kWaves) {
          const int i0 = it * 32;
          f32x16 acc = zero16();
#pragma unroll
          for (int ls = 0; ls < 2; ++ls) {
            if (ls < nLs) {
              Frag<T> bf;
              const int lb = ls * 32;
              if constexpr (kBf16) {
                // E^T fragment via ds_read_b64_tr_b16: group g = lane>>4 reads 4 rows x 16 cols
                const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
                const int col = i0 + 16 * (g & 1) + 4 * pp;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
#pragma unroll
                  for (int u = 0; u < 2; ++u) {
                    const int row = lb + 16 * (g >> 1) + 8 * s + 4 * u + q;
                    const int off = (row < L) ? (p.offE + row * p.ES + col * 2) : p.offZ;
                    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
                    typedef __attribute__((address_space(3))) char lds_char;
                    const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_i16x4*)((lds_char*)smem + off));
                    const unsigned lo = (unsigned)(unsigned short)v[0] | ((unsigned)(unsigned short)v[1] << 16);
                    const unsigned hi = (unsigned)(unsigned short)v[2] | ((unsigned)(unsigned short)v[3] << 16);
                    bf.q[s][2 * u] = lo;
                    bf.q[s][2 * u + 1] = hi;
                  }
                }
              } else {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                  const int l = lb + 16 * h + e;
                  const float v = (l < L) ? E[(size_t)l * d + i0 + r] : 0.f;
                  bf.q[e >> 2][e & 3] = __float_as_uint(v);
                }
              }
              mma_slab<T>(acc, ls == 0 ? af0 : af1, bf);
            }
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int k = acc_row(e, h);
            muiL[k * msE + i0 + r] = from_f32<T>(acc[e]);
            if (p.mui_out && k < K) p.mui_out[((size_t)b * K + k) * d + i0 + r] = acc[e];
          }
        }
      }
      __syncthreads();
    } else {  // MODE == kTaa: multi_user_interest comes from global (query)
      const T* __restrict__ qy = static_cast<const T*>(p.hist) + (size_t)b * K * d;
      const int per_row = d * (int)sizeof(T) / 16;
      for (int i = tid; i < kMaxK * per_row; i += kThreads) {
        const int k = i / per_row, c = i - k * per_row;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (k < K) v = reinterpret_cast<const u32x4*>(qy + (size_t)k * d)[c];
        *reinterpret_cast<u32x4*>(smem + p.offMui + k * p.MS + c * 16) = v;
      }
      __syncthreads();
    }

    if (!need_scores) continue;  // PolyAttention only (uniform branch; S4's barrier is behind us)

    // ---- S5: X = gelu(W2 · muiᵀ), wave-owned d-tiles kept in registers -----------------------
    const int nJt = d >> 5;
    Frag<T> xf[kMaxJ];
    if (weighted) {
      f32x16 acc[kMaxJ];
#pragma unroll
      for (int m = 0; m < kMaxJ; ++m) acc[m] = zero16();
      const T* w2row[kMaxJ];
#pragma unroll
      for (int m = 0; m < kMaxJ; ++m) {
        const int jt = wave + kWaves * m;
        w2row[m] = W2 + (size_t)((jt < nJt ? jt : 0) * 32 + pi_row(r)) * d + 16 * h;
      }
      const int nm = (nJt - wave + kWaves - 1) / kWaves;  // d-tiles owned by this wave
      Frag<T> an[kMaxJ];
#pragma unroll
      for (int m = 0; m < kMaxJ; ++m) {
        if (m < nm) frag_load(an[m], w2row[m]); else frag_zero(an[m]);
      }
      for (int kb = 0; kb < d; kb += 32) {
        Frag<T> a[kMaxJ];
#pragma unroll
        for (int m = 0; m < kMaxJ; ++m) a[m] = an[m];
        if (kb + 32 < d) {
#pragma unroll
          for (int m = 0; m < kMaxJ; ++m)
            if (m < nm) frag_load(an[m], w2row[m] + kb + 32);
        }
        Frag<T> bm;
        frag_load(bm, muiL + r * msE + kb + 16 * h);
#pragma unroll
        for (int m = 0; m < kMaxJ; ++m)
          if (m < nm) mma_slab<T>(acc[m], a[m], bm);
      }
#pragma unroll
      for (int m = 0; m < kMaxJ; ++m) {
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[m][e] = act_gelu<T>(acc[m][e]);
        acc_to_frag(xf[m], acc[m]);
      }
    }
    for (int i = tid; i < 2 * kMaxK * kCChunk; i += kThreads) Lg[i] = 0.f;  // Lg and Mt are adjacent
    __syncthreads();

    // ---- S6/S7 over candidate chunks ---------------------------------------------------------
    for (int cc = 0; cc < Cb; cc += kCChunk) {
#pragma unroll
      for (int ct = 0; ct < kCChunk / 32; ++ct) {
        const int c = cc + ct * 32 + r;
        if (cc + ct * 32 < Cb) {
          f32x16 lg = zero16(), mt = zero16();
          const bool cvalid = c < Cb;
          const T* crow = cand + (size_t)(cvalid ? c : 0) * d + 16 * h;
#pragma unroll
          for (int m = 0; m < kMaxJ; ++m) {
            const int jt = wave + kWaves * m;
            if (jt < nJt) {
              Frag<T> bc;
              if (cvalid) frag_load(bc, crow + jt * 32); else frag_zero(bc);
              if (weighted) mma_slab<T>(lg, xf[m], bc);
              if (MODE == kFull) {
                Frag<T> am;
                frag_load(am, muiL + r * msE + jt * 32 + 16 * h);
                mma_slab<T>(mt, am, bc);
              }
            }
          }
          if (wave < nJt) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int k = acc_row(e, h);
              if (weighted) atomicAdd(&Lg[k * kCChunk + ct * 32 + r], lg[e]);
              if (MODE == kFull) atomicAdd(&Mt[k * kCChunk + ct * 32 + r], mt[e]);
            }
          }
        }
      }
      __syncthreads();
      if (tid < kCChunk) {
        const int c = cc + tid;
        if (c < Cb) {
          float sc;
          if (MODE == kTaa) {
            const float* val = p.value + (size_t)(cbase + c) * K;
            float mx = -INFINITY;
            for (int k = 0; k < K; ++k) mx = fmaxf(mx, Lg[k * kCChunk + tid]);
            float den = 0.f, num = 0.f;
            for (int k = 0; k < K; ++k) {
              const float ex = expf(Lg[k * kCChunk + tid] - mx);
              den += ex;
              num += ex * val[k];
            }
            sc = num / den;
          } else if (p.score_type == MINER_SCORE_WEIGHTED) {
            float mx = -INFINITY;
            for (int k = 0; k < K; ++k) mx = fmaxf(mx, Lg[k * kCChunk + tid]);
            float den = 0.f;
            for (int k = 0; k < K; ++k) den += expf(Lg[k * kCChunk + tid] - mx);
            float acc = 0.f;
            for (int k = 0; k < K; ++k) acc += (expf(Lg[k * kCChunk + tid] - mx) / den) * Mt[k * kCChunk + tid];
            sc = acc;
          } else if (p.score_type == MINER_SCORE_MAX) {
            float mx = -INFINITY;
            for (int k = 0; k < K; ++k) mx = fmaxf(mx, Mt[k * kCChunk + tid]);
            sc = mx;
          } else {
            float s = 0.f;
            for (int k = 0; k < K; ++k) s += Mt[k * kCChunk + tid];
            sc = s / (float)K;
          }
          p.scores[cbase + c] = sc;
        }
        for (int k = 0; k < kMaxK; ++k) { Lg[k * kCChunk + tid] = 0.f; Mt[k * kCChunk + tid] = 0.f; }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
inline int round16(int x) { return (x + 15) & ~15; }

struct Carve {
  int ES, MS, offE, offZ, offLg, offMt, offMui, offS, offAw, total;
};

Carve carve(int dtype, int mode, int L, int d) {
  Carve c{};
  const bool bf = dtype == MINER_DTYPE_BF16;
  const int es = bf ? 2 : 4;
  const int lgmt = 2 * kMaxK * kCChunk * 4;
  c.MS = d * es + 16;
  if (mode == kFull && bf) {
    c.ES = d * es + 16;
    c.offE = 0;
    c.offZ = round16(L * c.ES);
    const int r1 = c.offZ + 64 > lgmt ? c.offZ + 64 : lgmt;  // Lg/Mt alias the history region
    c.offLg = 0;
    c.offMt = kMaxK * kCChunk * 4;
    c.offMui = round16(r1);
  } else {
    c.ES = 0;
    c.offE = 0;
    c.offZ = 0;
    c.offLg = 0;
    c.offMt = kMaxK * kCChunk * 4;
    c.offMui = lgmt;
  }
  const int r2 = 32 * c.MS > kMaxK * kMaxL * 4 ? 32 * c.MS : kMaxK * kMaxL * 4;
  c.offS = c.offMui;  // S lives in the mui region until S4 overwrites it
  c.offAw = round16(c.offMui + r2);
  const int aw = mode == kFull ? (bf ? 32 * 72 * 2 : 32 * 68 * 4) : 0;
  c.total = c.offAw + aw;
  return c;
}

int check_shape(int dtype, int mode, int L, int d, int Dc, int K) {
  if (dtype != MINER_DTYPE_F32 && dtype != MINER_DTYPE_BF16) return MINER_EINVAL;
  if (d <= 0 || K <= 0) return MINER_EINVAL;
  if (mode == kFull && (L <= 0 || Dc <= 0)) return MINER_EINVAL;
  if (K > kMaxK || d % 32 != 0 || d > kMaxD) return MINER_ESHAPE;
  if (mode == kFull && (L > kMaxL || Dc > kMaxDc)) return MINER_ESHAPE;
  if (carve(dtype, mode, L, d).total > kLdsMax) return MINER_ELDS;
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

template <class T, int MODE>
int launch(void* stream, const Params& prm, int lds) {
  auto kern = miner_fused<T, MODE>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return (int)e;
  const int per_cu = kLdsMax / lds > 0 ? (kLdsMax / lds > 2 ? 2 : kLdsMax / lds) : 1;
  int grid = num_cus() * per_cu;
  if (grid > prm.B) grid = prm.B;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

int run(void* stream, int dtype, int mode, Params prm) {
  const Carve c = carve(dtype, mode, prm.L, prm.d);
  prm.ES = c.ES; prm.MS = c.MS; prm.offE = c.offE; prm.offZ = c.offZ; prm.offLg = c.offLg;
  prm.offMt = c.offMt; prm.offMui = c.offMui; prm.offS = c.offS; prm.offAw = c.offAw;
  if (dtype == MINER_DTYPE_BF16)
    return mode == kFull ? launch<__bf16, kFull>(stream, prm, c.total) : launch<__bf16, kTaa>(stream, prm, c.total);
  return mode == kFull ? launch<float, kFull>(stream, prm, c.total) : launch<float, kTaa>(stream, prm, c.total);
}

}  // namespace

extern "C" {

int miner_score(void* stream, int dtype, int score_type, const void* history, const uint8_t* his_mask,
                const float* his_bias, const void* candidates, const int32_t* cand_offsets,
                const void* w_poly, const void* context_codes, const void* w_target, int B, int L, int C,
                int d, int Dc, int K, float* scores, float* user_out) {
  if (score_type < MINER_SCORE_WEIGHTED || score_type > MINER_SCORE_NONE) return MINER_EINVAL;
  if (B < 0 || C < 0) return MINER_EINVAL;
  const int sh = check_shape(dtype, kFull, L, d, Dc, K);
  if (sh != MINER_OK) return sh;
  if (!history || !his_mask || !w_poly || !context_codes) return MINER_EINVAL;
  if (score_type != MINER_SCORE_NONE && (!candidates || !scores)) return MINER_EINVAL;
  if (score_type == MINER_SCORE_WEIGHTED && !w_target) return MINER_EINVAL;
  if (score_type == MINER_SCORE_NONE && !user_out) return MINER_EINVAL;
  if (!aligned16(history) || !aligned16(candidates) || !aligned16(w_poly) || !aligned16(w_target))
    return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  Params prm{};
  prm.hist = history; prm.mask = his_mask; prm.bias = his_bias; prm.cand = candidates;
  prm.cand_off = cand_offsets; prm.W1 = w_poly; prm.Q = context_codes; prm.W2 = w_target;
  prm.value = nullptr; prm.scores = scores; prm.mui_out = user_out;
  prm.B = B; prm.L = L; prm.C = C; prm.d = d; prm.Dc = Dc; prm.K = K; prm.score_type = score_type;
  return run(stream, dtype, kFull, prm);
}

int miner_target_aware(void* stream, int dtype, const void* query, const void* key, const float* value,
                       const int32_t* cand_offsets, const void* w_target, int B, int C, int d, int K,
                       float* out) {
  if (B < 0 || C < 0) return MINER_EINVAL;
  const int sh = check_shape(dtype, kTaa, 1, d, 1, K);
  if (sh != MINER_OK) return sh;
  if (!query || !key || !value || !w_target || !out) return MINER_EINVAL;
  if (!aligned16(query) || !aligned16(key) || !aligned16(w_target)) return MINER_EALIGN;
  if (B == 0) return MINER_OK;
  Params prm{};
  prm.hist = query; prm.mask = nullptr; prm.bias = nullptr; prm.cand = key; prm.cand_off = cand_offsets;
  prm.W1 = nullptr; prm.Q = nullptr; prm.W2 = w_target; prm.value = value; prm.scores = out;
  prm.mui_out = nullptr; prm.B = B; prm.L = 1; prm.C = C; prm.d = d; prm.Dc = 1; prm.K = K;
  prm.score_type = MINER_SCORE_WEIGHTED;
  return run(stream, dtype, kTaa, prm);
}

int miner_supported(int dtype, int L, int d, int Dc, int K) { return check_shape(dtype, kFull, L, d, Dc, K); }

int miner_lds_bytes(int dtype, int score_type, int L, int d) {
  (void)score_type;
  return carve(dtype, kFull, L, d).total;
}

const char* miner_strerror(int code) {
  switch (code) {
    case MINER_OK: return "ok";
    case MINER_EINVAL: return "invalid argument (null pointer, bad enum or non-positive size)";
    case MINER_ESHAPE: return "shape not supported by this build (K<=32, L<=64, Dc<=256, d%32==0, d<=768)";
    case MINER_EALIGN: return "device pointer not 16-byte aligned";
    case MINER_ELDS: return "shape needs more LDS than one CU has (160 KiB)";
    default: return code > 0 ? hipGetErrorString(static_cast<hipError_t>(code)) : "unknown error";
  }
}

int miner_abi_version(void) { return MINER_ABI_VERSION; }

}  // extern "C"
