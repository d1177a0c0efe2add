// corpus.hip — full-corpus ranking for MI355X (gfx950 / CDNA4): BASELINE config 5, SURVEY.md §7
// step 6 ("a users x news GEMM with fused softmax-over-K and a top-k epilogue; output never
// materialised"). Two kernels:
//
//   ue_fused  user encoder, one workgroup (8 waves) per user, any L <= 256 and K <= 64:
//             PolyAttention (model.py:159-185) -> mui [K,d] and proj = gelu(mui·W2ᵀ) (model.py:212)
//     S1+S2  wave w owns history rows [32w, 32w+32): Pᵀ = tanh(W1·Eᵀ) for all 8 Dc-tiles (Dc padded
//            to 256 with zero weights) and then Sᵀ = Q·Pᵀ straight from the accumulators — no
//            cross-wave exchange; Sᵀ (+ bias) -> LDS
//     S3     masked softmax over L per interest (masked logits = 1e-30, model.py:180)
//     S4     muiᵀ = Eᵀ·Aᵀ over 32-row slabs of E LDS-DMA'd twice-buffered (16-bit: ds_read_b64_tr_b16
//            Eᵀ fragments), wave w owning d-tiles w, w+8, ...
//     S5     per interest tile: the mui image in LDS, projᵀ = gelu(W2·muiᵀ), W2 streamed (packed)
//
//   rk_fused  ranker: workgroup tile = 2 users x 256 news per step, contraction over d in 128-byte
//             chunks staged through LDS by LDS-DMA (double buffered, XOR-swizzled rows); wave w owns
//             user w>>2 and news [64(w&3), +64) and holds all of that user's K-row tiles (proj and
//             mui) for its 64 news, so the click score (softmax over K of proj·e weighting mui·e,
//             model.py:127-134, 213-214) is an in-register epilogue plus one lane-half exchange. Each
//             workgroup owns whole users: a running top-k per user in LDS, threshold-filtered, so
//             the U x N scores never leave the CU.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>
#include <math.h>

#include "../../include/miner_corpus.h"
#include "cdna4_common.h"

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kMaxL = MINER_CORPUS_MAX_L;
constexpr int kMaxK = MINER_CORPUS_MAX_K;
constexpr int kMaxTopk = MINER_CORPUS_MAX_TOPK;
constexpr int kDcT = 8;          // Dc padded to 8 tiles of 32
constexpr int kMaxD = 768;

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

__device__ __forceinline__ int fresh_lane() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t & 63;
}

template <class T> __device__ __forceinline__ float cx_exp(float x) {
  if constexpr (sizeof(T) == 2) return __expf(x); else return expf(x);
}
template <class T> __device__ __forceinline__ float cx_tanh(float x) {
  if constexpr (sizeof(T) == 2) return tanh_fast(x); else return tanhf(x);
}
__device__ __forceinline__ float xor32_max(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float wave_max(float x) {
  x = row16_max(x);
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return xor32_max(fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1])));
}
__device__ __forceinline__ float wave_sum(float x) {
  x = row16_sum(x);
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return xor32_sum(__uint_as_float(s[0]) + __uint_as_float(s[1]));
}

// ================================================================================================
// user encoder
// ================================================================================================
// packed weights (T elements): W1p [8 ct][ns] blocks (rows 32ct + pi(rr) of W1, zero past Dc),
// Qp [nkt][8 c] blocks (rows 32kt + pi(rr) of Q, columns 32c.., zero past K / Dc),
// W2p [ns][ns] blocks (rows 32jt + pi(rr) of W2); each block fragment-major (cdna4_common.h)
__host__ __device__ inline size_t ue_w1_elems(int d) { return (size_t)kDcT * (d >> 5) * 1024; }
__host__ __device__ inline size_t ue_q_elems(int K) { return (size_t)((K + 31) >> 5) * kDcT * 1024; }
__host__ __device__ inline size_t ue_w2_elems(int d) { return (size_t)(d >> 5) * (d >> 5) * 1024; }

template <class T>
__global__ void ue_pack_kernel(const T* __restrict__ W1, const T* __restrict__ Q, const T* __restrict__ W2, int d,
                               int Dc, int K, T* __restrict__ out) {
  const size_t n1 = ue_w1_elems(d), nq = ue_q_elems(K), n2 = W2 ? ue_w2_elems(d) : 0;
  const int ns = d >> 5;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + nq + n2; i += (size_t)gridDim.x * blockDim.x) {
    T v = (T)0.f;
    int rr, cc;
    block_pos<T>((int)(i & 1023), rr, cc);
    if (i < n1) {
      const int tile = (int)(i >> 10), ct = tile / ns, j = tile % ns;
      const int row = 32 * ct + pi_row(rr);
      if (row < Dc) v = W1[(size_t)row * d + 32 * j + cc];
    } else if (i < n1 + nq) {
      const int tile = (int)((i - n1) >> 10), kt = tile / kDcT, c = tile % kDcT;
      const int row = 32 * kt + pi_row(rr), col = 32 * c + cc;
      if (row < K && col < Dc) v = Q[(size_t)row * Dc + col];
    } else {
      const int tile = (int)((i - n1 - nq) >> 10), jt = tile / ns, j = tile % ns;
      v = W2[(size_t)(32 * jt + pi_row(rr)) * d + 32 * j + cc];
    }
    out[i] = v;
  }
}

struct UeParams {
  const void* hist;        // dense [U, L, d], or the news table (gather)
  const int32_t* his_ids;  // [U, L] or null
  int n_news;
  const uint8_t* mask;
  const float* bias;
  const void* wp;
  float* mui_f32;          // [U, K, d] or null
  void* user_mui;          // [U, K, d] T
  void* user_proj;         // [U, K, d] T or null
  int U, L, d, Dc, K;
};

// LDS carve (bytes)
constexpr int kSS = kMaxL + 4;                          // S / fp32-A row stride (floats)
constexpr int kSBytes = kMaxK * kSS * 4;                // logits; fp32 mode: A in place
// mui image row stride (elements): an odd number of 16-byte units, so the 16 rows of a ds_read_b128
// lane group land in 16 different bank slots
template <class T> constexpr int kMS = kMaxD + 16 / (int)sizeof(T);
template <class T> constexpr int kMuiImg = 32 * kMS<T> * (int)sizeof(T);  // one interest tile
template <class T> constexpr int kEBuf = sizeof(T) == 2 ? 32 * kMaxD * 2 : 0;  // one E slab image (16-bit)
template <class T> constexpr int kR1 = ((kSBytes > kMuiImg<T> ? kSBytes : kMuiImg<T>) > 2 * kEBuf<T>
                                            ? (kSBytes > kMuiImg<T> ? kSBytes : kMuiImg<T>) : 2 * kEBuf<T>);
constexpr int kAS = kMaxL + 8;                          // 16-bit A row stride (elements)
template <class T> constexpr int kABytes = sizeof(T) == 2 ? kMaxK * kAS * 2 : 0;
template <class T> constexpr int kOffA = kR1<T>;
template <class T> constexpr int kOffIds = kOffA<T> + kABytes<T>;
template <class T> constexpr int kOffZero = kOffIds<T> + kMaxL * 4;
template <class T> constexpr int kUeLds = kOffZero<T> + 64;
static_assert(kUeLds<__bf16> <= 160 * 1024 && kUeLds<float> <= 160 * 1024, "encoder LDS");

// A-operand fragment of Eᵀ (rows = columns i0 + pi(..) of E, contraction over the 32 rows of an
// E slab image) via ds_read_b64_tr_b16; rows >= nvalid read the zero block
template <class T>
__device__ __forceinline__ void frag_load_Et(Frag<T>& bf, unsigned img_off, unsigned zero_off, int i0, int rowB,
                                             int g16, int nvalid, int lane) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int col = i0 + 16 * (pp & 1) + 8 * (g & 1) + 4 * (pp >> 1);
  const int ch = col >> 3, sub8 = (col & 7) * 2;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = 16 * (g >> 1) + 8 * s + 4 * u + q;
      const unsigned off = row < nvalid ? img_off + row * rowB + ((ch ^ eswz(row, g16)) << 4) + sub8 : zero_off;
      const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)((lds_char*)smem + off));
      bf.q[s][2 * u] = (unsigned)(unsigned short)v[0] | ((unsigned)(unsigned short)v[1] << 16);
      bf.q[s][2 * u + 1] = (unsigned)(unsigned short)v[2] | ((unsigned)(unsigned short)v[3] << 16);
    }
  }
}

// nrows rows of d elements (dense from src, or table rows ids[r]) -> an E slab image (whole 1 KiB
// DMA blocks; chunk c of row `row` at c ^ eswz(row))
template <class T>
__device__ __forceinline__ void ue_dma_slab(const T* src, const int32_t* idsL, int n_news, int nrows, int d,
                                            char* img, int wave, int lane) {
  const int cpr = d >> 3;
  const int g16 = (cpr & 15) == 0;
  const int total = nrows * cpr;
  const int nblk = (total + 63) >> 6;
  for (int blk = wave; blk < nblk; blk += kWaves) {
    const int pos = blk * 64 + lane;
    const int row = pos / cpr;
    const int c = pos - row * cpr;
    const int rr = min(row, nrows - 1);
    const size_t r = idsL ? (size_t)min(max(idsL[rr], 0), n_news - 1) : (size_t)rr;
    const T* g = (pos < total) ? src + r * d + (size_t)((c ^ eswz(row, g16)) << 3) : src;
    dma_b128(g, __builtin_amdgcn_readfirstlane(lds_offset(img + blk * 1024)));
  }
}

template <class T, int NKT, bool GATHER>
__global__ __launch_bounds__(kThreads) void ue_fused(UeParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool k16 = sizeof(T) == 2;
  const int L = p.L, d = p.d, K = p.K, ns = d >> 5;
  const int nLt = (L + 31) >> 5;
  const T* __restrict__ W1p = static_cast<const T*>(p.wp);
  const T* __restrict__ Qp = W1p + ue_w1_elems(d);
  const T* __restrict__ W2p = Qp + ue_q_elems(K);
  float* S = reinterpret_cast<float*>(smem);
  int32_t* idsL = reinterpret_cast<int32_t*>(smem + kOffIds<T>);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x < 16) reinterpret_cast<float*>(smem + kOffZero<T>)[threadIdx.x] = 0.f;

  for (int u = blockIdx.x; u < p.U; u += gridDim.x) {
    const T* __restrict__ base = static_cast<const T*>(p.hist) + (GATHER ? (size_t)0 : (size_t)u * L * d);
    if constexpr (GATHER) {
      __syncthreads();      // the previous user's readers of the id block are done
      for (int i = threadIdx.x; i < L; i += kThreads) idsL[i] = p.his_ids[(size_t)u * L + i];
    }
    __syncthreads();

    // ---- S1 + S2: wave w = history rows [32w, 32w + 32) ----
    if (wave < nLt) {
      const int lane = fresh_lane();
      const int r = lane & 31, h = lane >> 5;
      const int m = min(32 * wave + r, L - 1);
      const T* erow = GATHER ? base + (size_t)min(max(idsL[m], 0), p.n_news - 1) * d : base + (size_t)m * d;
      f32x16 acc[kDcT];
#pragma unroll
      for (int c = 0; c < kDcT; ++c) acc[c] = zero16();
      for (int j = 0; j < ns; ++j) {
        Frag<T> eb;
        frag_load<T>(eb, erow + 32 * j + 16 * h);
#pragma unroll
        for (int c = 0; c < kDcT; ++c) {
          Frag<T> wa;
          frag_load_tile<T>(wa, W1p + (size_t)(c * ns + j) * 1024, lane);
          mma_slab<T>(acc[c], wa, eb);          // Pᵀ[dc][l] over this d slab
        }
      }
      f32x16 sacc[NKT];
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) sacc[kt] = zero16();
#pragma unroll
      for (int c = 0; c < kDcT; ++c) {
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[c][e] = cx_tanh<T>(acc[c][e]);     // model.py:171
        Frag<T> pf;
        acc_to_frag<T>(pf, acc[c]);            // lane (h, l): 16 consecutive Dc of row l
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
          Frag<T> qa;
          frag_load_tile<T>(qa, Qp + (size_t)(kt * kDcT + c) * 1024, lane);
          mma_slab<T>(sacc[kt], qa, pf);        // Sᵀ[k][l] (model.py:174)
        }
      }
      const int l = 32 * wave + r;
      const float bl = (p.bias && l < L) ? p.bias[(size_t)u * L + l] : 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
        for (int e = 0; e < 16; ++e) S[(32 * kt + 16 * h + e) * kSS + l] = sacc[kt][e] + bl;   // + bias (model.py:176)
      }
    }
    __syncthreads();

    // ---- S3: masked softmax over the history (model.py:178-181), 8 interests per wave ----
    {
      const int lane = fresh_lane();
      const uint8_t* mrow = p.mask + (size_t)u * L;
      bool real[kMaxL / 64];
#pragma unroll
      for (int i = 0; i < kMaxL / 64; ++i) {
        const int l = lane + 64 * i;
        real[i] = l < L && mrow[min(l, L - 1)] != 0;
      }
#pragma unroll
      for (int q = 0; q < 32 * NKT / kWaves; ++q) {
        const int k = wave * (32 * NKT / kWaves) + q;
        float v[kMaxL / 64];
        float mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < kMaxL / 64; ++i) {
          const int l = lane + 64 * i;
          v[i] = l < L ? (real[i] ? S[k * kSS + l] : 1e-30f) : -INFINITY;
          mx = fmaxf(mx, v[i]);
        }
        mx = wave_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < kMaxL / 64; ++i) {
          v[i] = (lane + 64 * i < L) ? cx_exp<T>(v[i] - mx) : 0.f;
          sum += v[i];
        }
        sum = wave_sum(sum);
        const float inv = k < K ? 1.0f / sum : 0.f;
#pragma unroll
        for (int i = 0; i < kMaxL / 64; ++i) {
          const int l = lane + 64 * i;
          if constexpr (k16) reinterpret_cast<T*>(smem + kOffA<T>)[k * kAS + l] = (T)(v[i] * inv);
          else S[k * kSS + l] = v[i] * inv;    // in place: this lane read exactly these entries
        }
      }
    }
    __syncthreads();

    // ---- S4: muiᵀ = Eᵀ · Aᵀ, wave w owning d-tiles w, w + 8, ... ----
    constexpr int kDt = kMaxD / 32 / kWaves;    // d-tiles per wave (<= 3)
    f32x16 macc[kDt][NKT];
#pragma unroll
    for (int i = 0; i < kDt; ++i)
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) macc[i][kt] = zero16();
    if constexpr (k16) {
      const int rowB = 2 * d, g16 = (((d >> 3) & 15) == 0);
      const int nls = nLt;
      {
        const int lane = fresh_lane();
        ue_dma_slab<T>(base, GATHER ? idsL : nullptr, p.n_news, min(32, L), d, smem, wave, lane);
      }
      for (int s = 0; s < nls; ++s) {
        vm_wait_all();
        __syncthreads();      // slab s landed; slab s - 1's buffer is free
        const int lane = fresh_lane();
        const int r = lane & 31, h = lane >> 5;
        if (s + 1 < nls) {
          const int r0 = 32 * (s + 1);
          ue_dma_slab<T>(GATHER ? base : base + (size_t)r0 * d, GATHER ? idsL + r0 : nullptr, p.n_news,
                         min(32, L - r0), d, smem + ((s + 1) & 1) * kEBuf<T>, wave, lane);
        }
        const unsigned img = lds_offset(smem + (s & 1) * kEBuf<T>);
        const unsigned zoff = lds_offset(smem + kOffZero<T>);
        const int nvalid = min(32, L - 32 * s);
        Frag<T> af[NKT];
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
          frag_load<T>(af[kt], reinterpret_cast<const T*>(smem + kOffA<T>) + (32 * kt + r) * kAS + 32 * s + 16 * h);
#pragma unroll
        for (int i = 0; i < kDt; ++i) {
          const int dt = wave + kWaves * i;
          if (dt < ns) {
            Frag<T> ef;
            frag_load_Et<T>(ef, img, zoff, 32 * dt, rowB, g16, nvalid, lane);
#pragma unroll
            for (int kt = 0; kt < NKT; ++kt) mma_slab<T>(macc[i][kt], ef, af[kt]);   // lane (h,k): d 16h..
          }
        }
      }
    } else {
      // fp32 parity mode: E columns straight from L2 (one element per register), A rows natural
      const int lane = fresh_lane();
      const int r = lane & 31, h = lane >> 5;
      for (int s = 0; s < nLt; ++s) {
        Frag<T> af[NKT];
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) frag_load<T>(af[kt], S + (32 * kt + r) * kSS + 32 * s + 16 * h);
#pragma unroll
        for (int i = 0; i < kDt; ++i) {
          const int dt = wave + kWaves * i;
          if (dt < ns) {
            Frag<T> ef;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int l = min(32 * s + 16 * h + e, L - 1);      // rows >= L: finite x zero weight
              const size_t row = GATHER ? (size_t)min(max(idsL[l], 0), p.n_news - 1) : (size_t)l;
              ef.q[e >> 2][e & 3] = __float_as_uint(base[row * d + 32 * dt + r]);
            }
#pragma unroll
            for (int kt = 0; kt < NKT; ++kt) mma_slab<T>(macc[i][kt], af[kt], ef);   // lane (h,d): k rows
          }
        }
      }
    }
    __syncthreads();          // E slab buffers / A free: the mui images go there

    // ---- outputs: mui, then S5 per interest tile ----
    {
      const int lane = fresh_lane();
      const int r = lane & 31, h = lane >> 5;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        T* img = reinterpret_cast<T*>(smem);         // [32 k][kMS]
#pragma unroll
        for (int i = 0; i < kDt; ++i) {
          const int dt = wave + kWaves * i;
          if (dt >= ns) continue;
          if constexpr (k16) {
            const int k = 32 * kt + r;
            Frag<T> mf;
            acc_to_frag<T>(mf, macc[i][kt]);
            frag_store<T>(img + r * kMS<T> + 32 * dt + 16 * h, mf);
            if (k < K) {
              frag_store<T>(static_cast<T*>(p.user_mui) + ((size_t)u * K + k) * d + 32 * dt + 16 * h, mf);
              if (p.mui_f32) {
                float4* o = reinterpret_cast<float4*>(p.mui_f32 + ((size_t)u * K + k) * d + 32 * dt + 16 * h);
#pragma unroll
                for (int g = 0; g < 4; ++g)
                  o[g] = float4{macc[i][kt][4 * g], macc[i][kt][4 * g + 1], macc[i][kt][4 * g + 2], macc[i][kt][4 * g + 3]};
              }
            }
          } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int kl = acc_row(e, h), k = 32 * kt + kl;
              img[kl * kMS<T> + 32 * dt + r] = macc[i][kt][e];
              if (k < K) {
                static_cast<T*>(p.user_mui)[((size_t)u * K + k) * d + 32 * dt + r] = macc[i][kt][e];
                if (p.mui_f32) p.mui_f32[((size_t)u * K + k) * d + 32 * dt + r] = macc[i][kt][e];
              }
            }
          }
        }
        if (p.user_proj) {
          __syncthreads();    // the mui image of this interest tile is complete
          // projᵀ = gelu(W2 · muiᵀ): wave w owns W2 row tiles w, w + 8, ...
#pragma unroll
          for (int i = 0; i < kDt; ++i) {
            const int jt = wave + kWaves * i;
            if (jt >= ns) continue;
            f32x16 pacc = zero16();
            for (int j = 0; j < ns; ++j) {
              Frag<T> wa, mb;
              frag_load_tile<T>(wa, W2p + (size_t)(jt * ns + j) * 1024, lane);
              frag_load<T>(mb, img + r * kMS<T> + 32 * j + 16 * h);
              mma_slab<T>(pacc, wa, mb);
            }
            gelu_tile<T>(pacc);                         // model.py:212 (exact erf in fp32 mode)
            const int k = 32 * kt + r;
            if (k < K) {
              Frag<T> pf;
              acc_to_frag<T>(pf, pacc);
              frag_store<T>(static_cast<T*>(p.user_proj) + ((size_t)u * K + k) * d + 32 * jt + 16 * h, pf);
            }
          }
        }
        __syncthreads();      // before the next interest tile's image (or the next user) reuses LDS
      }
    }
  }
}

// ================================================================================================
// ranker
// ================================================================================================
constexpr int kUT = 2;            // users per workgroup tile
constexpr int kNT = 256;          // news per step

struct RkParams {
  const void* mui;
  const void* proj;
  const void* news;
  float* top_s;
  int32_t* top_i;
  float* ws_s;             // S > 1: per (user, news slice) top-k lists [U][S][topk], merged by rk_merge
  int32_t* ws_i;
  size_t ws_bytes;         // the caller's workspace size (the split form needs U·S·topk·8)
  int U, N, d, K, topk, score_type;
};

// S > 1 (S = 8, grid = 256): the news steps are dealt to S slices (step st of slice s is news step
// s + S·st) and 8 consecutive user tiles x 8 slices go to the 32 workgroups b that share b % 8 — one
// XCD under the round-robin placement (speed only, never correctness): workgroup b takes slice
// (b >> 3) & 7 of the tiles 32 r + 4 (b & 7) + ((b >> 6) & 3), r = 0, 1, ... So an XCD's L2 holds the
// user rows of 8 users (1.5 MB at K = 64, d = 768, both mui and proj) that its 32 CUs all read,
// and every news row it fetches serves 8 users; with S = 1 every CU streams its own 2 users' rows
// (12 MB per XCD, beyond its 4 MB L2) and the table once per 2 users.
constexpr int kSplit = 8;

// diagnostic builds only (tools/rk_ablate.py): bit 1 no DMAs, 2 no MFMAs, 4 no epilogue, 8 no
// per-chunk barrier (the results are wrong, only the time is read)
#ifndef MINER_RK_ABL
#define MINER_RK_ABL 0
#endif
#ifndef MINER_RK_DMAW
#define MINER_RK_DMAW 4   // 91.5 -> 86.9 ms per config-5 step against 8 (tools/rk_ablate.py)
#endif

// one LDS-DMA (saddr form: scalar base + 32-bit per-lane offset) into M0 = m, M0 saved / restored;
// default cache policy (nt on the ranker's rows cost 18 %, tools/rk_ablate.py)
__device__ __forceinline__ void rk_dma(uint32_t off, const char* base, unsigned m) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(off), "s"(base), "s"(m) : "memory");
}

// image geometry: rows of RB bytes per chunk; 16-byte unit c of row `row` at c ^ rk_swz(row) —
// RB = 128: (row >> 1) & 7, RB = 64: (row >> 2) & 3. Either way the 16 rows of a ds_read_b128 lane
// group (natural or pi order: lanes {0-3, 12-15, 20-27} read rows {0-3, 12-15, 20-27}) land in 16
// different 16-byte bank slots.
template <int RB>
__device__ __forceinline__ int rk_swz(int row) { return RB == 128 ? (row >> 1) & 7 : (row >> 2) & 3; }

template <class T, int RB>
__device__ __forceinline__ void rk_frag(Frag<T>& f, const char* img, int row, int c0) {
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i)
    f.q[i] = *reinterpret_cast<const u32x4*>(img + row * RB + (((c0 + i) ^ rk_swz<RB>(row)) << 4));
}

// a wave's vector-memory operations down to N outstanding
template <int N>
__device__ __forceinline__ void vm_wait_n() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

// stream geometry: GEO 0 rows of 128 B, a ring of 2 stages (the next chunk in flight); GEO 1 (16-bit,
// at least two row tiles per user) rows of 64 B, a ring of 4 stages of the same total size (three
// chunks in flight)
template <int GEO> constexpr int kRB = GEO ? 64 : 128;
template <int GEO> constexpr int kRing = GEO ? 4 : 2;

// total order of ranked entries: higher score first, then lower news id
__device__ __forceinline__ bool better(float s, int i, float s2, int i2) { return s > s2 || (s == s2 && i < i2); }

template <int NR, int GEO = 0>
struct RkLds {
  static constexpr int kARows = kUT * NR * 32;
  static constexpr int kStage = (kARows + kNT) * kRB<GEO>;
  static constexpr int kOffList = kRing<GEO> * kStage;              // [kUT][kMaxTopk] float + int
  static constexpr int kOffStage = kOffList + kUT * kMaxTopk * 8;  // staged candidates [2 bufs][kUT][kNT]
  static constexpr int kOffCnt = kOffStage + 2 * kUT * kNT * 8;     // list counts [kUT], staged [2][kUT]
  static constexpr int kTotal = kOffCnt + 64;
};

// NCH: RB-byte d-chunks per row (0: at run time); GEO: the stream geometry (kRB / kRing)
template <class T, int NKT, int SCORE, int NCH = 0, int S = 1, int GEO = 0, int KC = 0>   // KC: K compile-time (0: run time)
__global__ __launch_bounds__(kThreads) void rk_fused(RkParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool kW = SCORE == MINER_SCORE_WEIGHTED;
  constexpr int NR = kW ? 2 * NKT : NKT;            // row tiles per user: mui (and proj)
  constexpr int RB = kRB<GEO>, RING = kRing<GEO>, PD = RING - 1;   // PD: chunks in flight
  using LD = RkLds<NR, GEO>;
  constexpr int kChunkSlabs = RB / (32 * (int)sizeof(T));          // 32-index slabs per chunk
  static_assert(kChunkSlabs >= 1, "a chunk holds whole slabs");
  const int d = NCH > 0 ? NCH * RB / (int)sizeof(T) : p.d, K = KC > 0 ? KC : p.K, N = p.N;
  const int nchunk = NCH > 0 ? NCH : d * (int)sizeof(T) / RB;
  const int nsteps = ((N + kNT - 1) / kNT + S - 1) / S;            // news steps per slice
  const int ntiles = (p.U + kUT - 1) / kUT;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int uu = wave >> 2, nsub = wave & 3;
  float* list_s = reinterpret_cast<float*>(smem + LD::kOffList);
  int* list_i = reinterpret_cast<int*>(smem + LD::kOffList + kUT * kMaxTopk * 4);
  float* stg_s = reinterpret_cast<float*>(smem + LD::kOffStage);                    // [buf][uu][kNT]
  int* stg_i = reinterpret_cast<int*>(smem + LD::kOffStage + 2 * kUT * kNT * 4);
  int* cnt = reinterpret_cast<int*>(smem + LD::kOffCnt);   // [0, kUT) list sizes, kUT + buf * kUT + uu staged
  // the user's merging wave: 0 and 5 (two SIMDs under the wave -> SIMD w % 4 placement)
  const bool merger = wave == 5 * uu;
  const T* __restrict__ mui = static_cast<const T*>(p.mui);
  const T* __restrict__ proj = static_cast<const T*>(p.proj);
  const T* __restrict__ news = static_cast<const T*>(p.news);
  const int b = blockIdx.x;
  const int first = S == 1 ? b : 4 * (b & 7) + ((b >> 6) & 3);    // this workgroup's first tile
  const int tstride = S == 1 ? (int)gridDim.x : 32;
  const int slice = S == 1 ? 0 : (b >> 3) & 7;
  if (first >= ntiles) return;
  const int ntile_mine = (ntiles - first + tstride - 1) / tstride;
  const int total_chunks = ntile_mine * nsteps * nchunk;
  auto news_step = [&](int st) { return S == 1 ? st : slice + S * st; };

  // Row DMAs. Wave w issues the 1 KiB blocks w + 8 j of every stage: j < NR are user k-rows (A),
  // the rest news rows (B). The per-lane byte offsets are fixed for the launch (A: within the user's
  // [K, d] array; B: from the step's first news row); the user, step and chunk go into the scalar
  // base of the saddr form. A chunk's blocks are issued spread over the previous chunk's MFMAs.
  constexpr int kBlk = (LD::kARows + kNT) * RB / 1024;              // 1 KiB DMA blocks per stage
  static_assert(kBlk % kWaves == 0, "whole DMA blocks per wave");
  constexpr int kJ = kBlk / kWaves;
  constexpr int kUnits = RB / 16;                                    // 16-byte units per row
  constexpr int kRpb = 1024 / RB;                                    // rows per DMA block
  constexpr int kAJ = LD::kARows / (kWaves * kRpb);                  // A blocks per wave (jj < kAJ)
  static_assert(LD::kARows % (kWaves * kRpb) == 0, "A blocks split evenly over the waves");
  uint32_t voff[kJ];
#pragma unroll
  for (int jj = 0; jj < kJ; ++jj) {
    const int lane = fresh_lane();
    const int P = (wave + kWaves * jj) * 64 + lane;
    const int row = P / kUnits, cl = (P % kUnits) ^ rk_swz<RB>(row);
    if (jj < kAJ) {
      const int k = min(32 * (((row >> 5) % NR) % NKT) + (row & 31), K - 1);
      voff[jj] = (uint32_t)(k * d) * (uint32_t)sizeof(T) + cl * 16;
    } else {
      voff[jj] = (uint32_t)((row - LD::kARows) * d) * (uint32_t)sizeof(T) + cl * 16;
    }
  }
  // the next chunk to issue: (tile nti, slice step nsl, chunk nc), advanced after each issue
  int nti = first, nsl = 0, nc = 0;
  auto dma_block = [&](int jj, int stage) {
    const unsigned la = __builtin_amdgcn_readfirstlane(lds_offset(smem + stage * LD::kStage + (wave + kWaves * jj) * 1024));
    if (jj < kAJ) {
      const int row0 = (wave + kWaves * jj) * kRpb;
      const int t = (row0 >> 5) % NR, ou = row0 / (NR * 32);
      const int user = min(nti * kUT + ou, p.U - 1);
      const T* src = (kW && t >= NKT) ? proj : mui;
      rk_dma(voff[jj], reinterpret_cast<const char*>(src + (size_t)user * K * d) + nc * RB, la);
    } else {
      const int st = news_step(nsl);
      if (st * kNT + kNT <= N) {
        rk_dma(voff[jj], reinterpret_cast<const char*>(news + (size_t)st * kNT * d) + nc * RB, la);
      } else {                           // the table's last (partial) step: rows clamped to N - 1
        const int lane = fresh_lane();
        const int P = (wave + kWaves * jj) * 64 + lane;
        const int row = P / kUnits, cl = (P % kUnits) ^ rk_swz<RB>(row);
        const int n = min(st * kNT + (row - LD::kARows), N - 1);
        dma_b128_rt(news + (size_t)n * d + nc * (RB / (int)sizeof(T)) + cl * (16 / (int)sizeof(T)), la);
      }
    }
  };
  auto advance = [&]() {
    if (++nc == nchunk) {
      nc = 0;
      if (++nsl == nsteps) { nsl = 0; nti += tstride; }
    }
  };

  if (wave >= 4) __builtin_amdgcn_s_setprio(1);   // static priority for the second half (-0.8 %)
  if (threadIdx.x < 3 * kUT) cnt[threadIdx.x] = 0;

  // merge the candidates staged in buffer `buf` into user uu's running top-k (one wave). The list
  // (best first) and the staged entries are ranked in parallel: an entry's new position is the
  // number of entries of both sets better than it (a total order on distinct news ids); entries
  // ranked past topk drop out. Every LDS read comes before the first write (one wave, in order).
  auto merge = [&](int buf) {
    const int ns = cnt[kUT + buf * kUT + uu];
    if (ns == 0) return;
    const int lane = fresh_lane();
    const int c = cnt[uu];
    float* ls = list_s + uu * kMaxTopk;
    int* li = list_i + uu * kMaxTopk;
    const float* ss = stg_s + (buf * kUT + uu) * kNT;
    const int* si = stg_i + (buf * kUT + uu) * kNT;
    constexpr int kLT = kMaxTopk / 64, kST = kNT / 64;
    float lv[kLT], sv[kST];
    int lid[kLT], sid[kST], lr[kLT], sr[kST];
#pragma unroll
    for (int t = 0; t < kLT; ++t) {
      const int i = min(lane + 64 * t, kMaxTopk - 1);
      lv[t] = ls[i];
      lid[t] = li[i];
      lr[t] = lane + 64 * t;
    }
#pragma unroll
    for (int v = 0; v < kST; ++v) {
      const int j = min(lane + 64 * v, kNT - 1);
      sv[v] = ss[j];
      sid[v] = si[j];
      sr[v] = 0;
    }
    for (int j2 = 0; j2 < ns; ++j2) {
      const float s2 = ss[j2];
      const int i2 = si[j2];
      int nl = 0;                              // list entries better than staged entry j2
#pragma unroll
      for (int t = 0; t < kLT; ++t) {
        lr[t] += better(s2, i2, lv[t], lid[t]) ? 1 : 0;   // staged entries better than each entry
        nl += __popcll(__ballot(lane + 64 * t < c && better(lv[t], lid[t], s2, i2)));
      }
#pragma unroll
      for (int v = 0; v < kST; ++v) {
        sr[v] += better(s2, i2, sv[v], sid[v]) ? 1 : 0;
        if (j2 == lane + 64 * v) sr[v] += nl;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < kLT; ++t) {
      if (lane + 64 * t < c && lr[t] < p.topk) {
        ls[lr[t]] = lv[t];
        li[lr[t]] = lid[t];
      }
    }
#pragma unroll
    for (int v = 0; v < kST; ++v) {
      if (lane + 64 * v < ns && sr[v] < p.topk) {
        ls[sr[v]] = sv[v];
        li[sr[v]] = sid[v];
      }
    }
    if (lane == 0) {
      cnt[uu] = min(c + ns, p.topk);
      cnt[kUT + buf * kUT + uu] = 0;
    }
  };

  for (int q0 = 0; q0 < PD && q0 < total_chunks; ++q0) {   // prologue: the first PD chunks
    if (!(MINER_RK_ABL & 1)) {
#pragma unroll
      for (int jj = 0; jj < kJ; ++jj) dma_block(jj, q0);
    }
    advance();
  }
  int q = 0;
  for (int ti = first; ti < ntiles; ti += tstride) {
    for (int sl = 0; sl < nsteps; ++sl) {
      const int st = news_step(sl);
      f32x16 acc[NR][2];
#pragma unroll
      for (int t = 0; t < NR; ++t) { acc[t][0] = zero16(); acc[t][1] = zero16(); }
      for (int c = 0; c < nchunk; ++c, ++q) {
        // chunk q landed (this wave's DMAs of chunks q + 1 .. q + PD - 1 may stay in flight), then
        // for every wave; chunk q - 1's stage is free
        if (!(MINER_RK_ABL & 1)) {
          if (PD > 1 && q + PD - 1 < total_chunks) vm_wait_n<(PD - 1) * kJ>();
          else vm_wait_all();
        }
        if (!(MINER_RK_ABL & 8)) __syncthreads();
        // the previous step's staged candidates (its epilogue is behind this barrier); the next
        // epilogue reads the list only after this chunk's barriers
        if (c == 0 && sl > 0 && merger && !(MINER_RK_ABL & 4)) merge((sl - 1) & 1);
        const bool pre = !(MINER_RK_ABL & 1) && q + PD < total_chunks;
        const int lane = fresh_lane();
        const int r = lane & 31, h = lane >> 5;
        const char* img = smem + (q % RING) * LD::kStage;
        const char* bimg = img + LD::kARows * RB;
        constexpr int kPairs = kChunkSlabs * NR;
#pragma unroll
        for (int s = 0; s < kChunkSlabs; ++s) {
          const int c0 = (2 * s + h) * kNQ<T>;
          Frag<T> bf[2];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) rk_frag<T, RB>(bf[nt], bimg, 64 * nsub + 32 * nt + r, c0);
#pragma unroll
          for (int t = 0; t < NR; ++t) {
            Frag<T> af;
            rk_frag<T, RB>(af, img, (uu * NR + t) * 32 + pi_row(r), c0);
            if (!(MINER_RK_ABL & 2)) {
              mma_slab<T>(acc[t][0], af, bf[0]);
              mma_slab<T>(acc[t][1], af, bf[1]);
            } else {
              acc[t][0][0] += __builtin_bit_cast(float, af.q[0][0]);   // keep the reads
              acc[t][1][0] += __builtin_bit_cast(float, bf[1].q[0][0]);
            }
            // the next chunk's DMA blocks, spread over this chunk's first kWin MFMA pairs
            constexpr int kWin = MINER_RK_DMAW < kPairs ? MINER_RK_DMAW : kPairs;
#pragma unroll
            for (int jj = 0; jj < kJ; ++jj)
              if (jj * kWin / kJ == s * NR + t && pre) dma_block(jj, (q + PD) % RING);
          }
        }
        if (pre) advance();
      }
      if (nchunk == 1 && sl > 0) __syncthreads();   // (one chunk per step: the merge above is done)
      // ---- epilogue: click score of (user uu, news) for this wave's 64 news ----
      if (MINER_RK_ABL & 4) {            // every accumulator stays live (no MFMA is dead code)
        float z = 0.f;
#pragma unroll
        for (int t = 0; t < NR; ++t)
#pragma unroll
          for (int e = 0; e < 16; ++e) z += acc[t][0][e] + acc[t][1][e];
        if (z == 1234.5f) p.top_s[0] = z;
      } else {
        const int lane = fresh_lane();
        const int r = lane & 31, h = lane >> 5;
        const int user = ti * kUT + uu;
        const float th_s = cnt[uu] < p.topk ? -INFINITY : list_s[uu * kMaxTopk + p.topk - 1];
        const int th_i = cnt[uu] < p.topk ? 0x7fffffff : list_i[uu * kMaxTopk + p.topk - 1];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int n = st * kNT + 64 * nsub + 32 * nt + r;
          float score;
          if constexpr (kW) {
            // 4 independent max / sum chains per lane (a 32-long dependent chain each otherwise)
            float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
            for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
              for (int e = 0; e < 16; ++e)
                if (32 * kt + 16 * h + e < K) m4[e & 3] = fmaxf(m4[e & 3], acc[NKT + kt][nt][e]);
            const float mx = xor32_max(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
            float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
            // 16-bit: exp(x - mx) as exp2(x·log2 e - mx·log2 e), one fma + v_exp_f32 per interest
            const float mxl = mx * 1.44269504088896340736f;
#pragma unroll
            for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
              for (int e = 0; e < 16; ++e)
                if (32 * kt + 16 * h + e < K) {
                  const float lg = acc[NKT + kt][nt][e];
                  const float ex = sizeof(T) == 2 ? __builtin_amdgcn_exp2f(__builtin_fmaf(lg, 1.44269504088896340736f, -mxl))
                                                  : expf(lg - mx);
                  s0[e & 3] += ex;
                  s1[e & 3] = __builtin_fmaf(ex, acc[kt][nt][e], s1[e & 3]);
                }
            const float t0 = (s0[0] + s0[1]) + (s0[2] + s0[3]), t1 = (s1[0] + s1[1]) + (s1[2] + s1[3]);
            score = xor32_sum(t1) / xor32_sum(t0);       // Σ softmax_k(Lg) · M  (model.py:213-214)
          } else if constexpr (SCORE == MINER_SCORE_MAX) {
            float mx = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
              for (int e = 0; e < 16; ++e)
                if (32 * kt + 16 * h + e < K) mx = fmaxf(mx, acc[kt][nt][e]);
            score = xor32_max(mx);                       // model.py:128-129
          } else {
            float sm = 0.f;
#pragma unroll
            for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
              for (int e = 0; e < 16; ++e)
                if (32 * kt + 16 * h + e < K) sm += acc[kt][nt][e];
            score = xor32_sum(sm) / (float)K;            // model.py:130-131
          }
          const bool cand = h == 0 && n < N && user < p.U && better(score, n, th_s, th_i);
          const unsigned long long bal = __ballot(cand);
          if (bal) {
            const int buf = sl & 1;
            int b0 = 0;
            if (lane == 0) b0 = atomicAdd(&cnt[kUT + buf * kUT + uu], __popcll(bal));
            b0 = __builtin_amdgcn_readfirstlane(b0);
            if (cand) {
              const int slot = b0 + __popcll(bal & ((1ull << lane) - 1));
              stg_s[(buf * kUT + uu) * kNT + slot] = score;
              stg_i[(buf * kUT + uu) * kNT + slot] = n;
            }
          }
        }
      }
      // the staged candidates are merged at the next step's first chunk (merge, above), the last
      // step's below
    }
    // ---- this tile's users are done: merge the last step, write their top-k ----
    {
      __syncthreads();
      if (merger && !(MINER_RK_ABL & 4)) merge((nsteps - 1) & 1);
      __syncthreads();
      const int user = ti * kUT + uu;
      if (merger && user < p.U) {
        const int lane = fresh_lane();
        const size_t o = ((size_t)user * S + slice) * p.topk;
        float* ds = S == 1 ? p.top_s : p.ws_s;
        int32_t* di = S == 1 ? p.top_i : p.ws_i;
        for (int i = lane; i < p.topk; i += 64) {
          const bool ok = i < cnt[uu];
          ds[o + i] = ok ? list_s[uu * kMaxTopk + i] : -INFINITY;
          di[o + i] = ok ? list_i[uu * kMaxTopk + i] : -1;
        }
      }
      __syncthreads();
      if (threadIdx.x < kUT) cnt[threadIdx.x] = 0;
    }
  }
}

// the S per-slice lists of a user (each best first, valid entries (id >= 0) first; the slices hold
// disjoint news, so no two entries tie in the total order) -> its top-k: an entry's rank is its
// position in its own list plus, per other list, the count of entries better than it (binary
// search); ranks < topk are written. One wave per user, its lists staged in LDS.
constexpr int kMergeUsers = 4;
__global__ __launch_bounds__(256) void rk_merge(const float* __restrict__ ws_s, const int32_t* __restrict__ ws_i, int U,
                                                int topk, float* __restrict__ top_s, int32_t* __restrict__ top_i) {
  __shared__ float ms[kMergeUsers][kSplit * kMaxTopk];
  __shared__ int mi[kMergeUsers][kSplit * kMaxTopk];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int user = blockIdx.x * kMergeUsers + w;
  if (user >= U) return;                   // wave-uniform; no block barrier below
  const size_t base = (size_t)user * kSplit * topk;
  for (int e = lane; e < kSplit * topk; e += 64) {
    ms[w][e] = ws_s[base + e];
    mi[w][e] = ws_i[base + e];
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  int cnt[kSplit];
  int V = 0;
#pragma unroll
  for (int a = 0; a < kSplit; ++a) {
    int c = 0;
    for (int i0 = 0; i0 < topk; i0 += 64) c += __popcll(__ballot(i0 + lane < topk && mi[w][a * topk + i0 + lane] >= 0));
    cnt[a] = c;
    V += c;
  }
#pragma unroll
  for (int a = 0; a < kSplit; ++a) {
    for (int j = lane; j < cnt[a]; j += 64) {
      const float s = ms[w][a * topk + j];
      const int id = mi[w][a * topk + j];
      int rank = j;
#pragma unroll
      for (int o = 0; o < kSplit; ++o) {
        if (o == a) continue;
        int lo = 0, hi = cnt[o];
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (better(ms[w][o * topk + mid], mi[w][o * topk + mid], s, id)) lo = mid + 1; else hi = mid;
        }
        rank += lo;
      }
      if (rank < topk) {
        top_s[(size_t)user * topk + rank] = s;
        top_i[(size_t)user * topk + rank] = id;
      }
    }
  }
  for (int i = min(V, topk) + lane; i < topk; i += 64) {
    top_s[(size_t)user * topk + i] = -INFINITY;
    top_i[(size_t)user * topk + i] = -1;
  }
}

// ================================================================================================
// host side
// ================================================================================================
bool dtype_ok(int dt) { return dt == MINER_DTYPE_F32 || dt == MINER_DTYPE_BF16 || dt == MINER_DTYPE_F16; }
size_t esize(int dt) { return dt == MINER_DTYPE_F32 ? 4 : 2; }

template <class T, int NKT, bool G>
int ue_launch(void* stream, const UeParams& prm) {
  auto kern = ue_fused<T, NKT, G>;
  const int lds = kUeLds<T>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return (int)e;
  int grid = num_cus();
  if (grid > prm.U) grid = prm.U;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, static_cast<hipStream_t>(stream), prm);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

template <class T>
int ue_dispatch(void* stream, const UeParams& prm) {
  const bool g = prm.his_ids != nullptr;
  if (prm.K <= 32) return g ? ue_launch<T, 1, true>(stream, prm) : ue_launch<T, 1, false>(stream, prm);
  return g ? ue_launch<T, 2, true>(stream, prm) : ue_launch<T, 2, false>(stream, prm);
}

// the split form (S = kSplit news slices, rk_merge) when the caller gave a workspace, the device has
// the 256 CUs its tile-to-XCD map assumes, and the users are too few to fill the CUs with 2-user
// tiles (< 256 two-user tiles, i.e. U <= 510): at U = 2,048 it measured 90.5 vs 85.9 ms per config-5 step (each slice's
// top-k warms up on its own; its L2 hit rate is higher, 69 vs 45 %, but the stream is not what
// bounds it). The caller chooses by passing a workspace (miner_rank_topk_split_recommended says
// which form the library would take). Fewer than 256 two-user tiles means U <= 510.
bool rk_split_wanted(int U) { return num_cus() == 256 && (U + kUT - 1) / kUT < num_cus(); }
size_t rk_ws_bytes(int U, int topk) { return (size_t)U * kSplit * topk * 8; }
// the split form runs only on a workspace whose stated size covers it (the launch never trusts an
// earlier size query), on the 256-CU device its tile-to-XCD map assumes
bool rk_split(const RkParams& prm) {
  if (prm.ws_s == nullptr || prm.ws_i == nullptr || prm.ws_bytes < rk_ws_bytes(prm.U, prm.topk)) return false;
  return num_cus() == 256;
}

template <class T, int NKT, int S, int GEO>
int rk_launch_geo(void* stream, const RkParams& prm, bool split) {
  // d = 768 in 16-bit (config 5): the chunk count compile-time
  void (*kern)(RkParams) = split ? rk_fused<T, NKT, S, 0, kSplit, GEO> : rk_fused<T, NKT, S, 0, 1, GEO>;
  if constexpr (sizeof(T) == 2) {
    // config 5's d = 768 and K = 64 compile-time (the masked interest loops of the epilogue compile
    // away; the top-k equals the oracle's at the 16-bit bar, tests/test_gpu_corpus.py)
    constexpr int kN768 = 768 * 2 / kRB<GEO>;
    if (prm.d == 768) {
      if (NKT == 2 && prm.K == 64)
        kern = split ? rk_fused<T, NKT, S, kN768, kSplit, GEO, 64> : rk_fused<T, NKT, S, kN768, 1, GEO, 64>;
      else
        kern = split ? rk_fused<T, NKT, S, kN768, kSplit, GEO> : rk_fused<T, NKT, S, kN768, 1, GEO>;
    }
  }
  constexpr int NR = S == MINER_SCORE_WEIGHTED ? 2 * NKT : NKT;
  const int lds = RkLds<NR, GEO>::kTotal;
  static_assert(RkLds<NR, GEO>::kTotal <= 160 * 1024, "ranker LDS");
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return (int)e;
  const int ntiles = (prm.U + kUT - 1) / kUT;
  int grid = num_cus();
  if (!split && grid > ntiles) grid = ntiles;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, s, prm);
  e = hipGetLastError();
  if (e != hipSuccess || !split) return e == hipSuccess ? MINER_OK : (int)e;
  hipLaunchKernelGGL(rk_merge, dim3((prm.U + kMergeUsers - 1) / kMergeUsers), dim3(64 * kMergeUsers), 0, s, prm.ws_s,
                     prm.ws_i, prm.U, prm.topk, prm.top_s, prm.top_i);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

template <class T, int NKT, int S>
int rk_launch(void* stream, const RkParams& prm) {
  const bool split = rk_split(prm);
  // (GEO 1 — 64-byte rows through a 4-stage ring, three chunks in flight instead of one — measured
  // slower: 95.9 vs 89.7 ms per config-5 step, twice the barriers for no gain in the gather rate;
  // diagnostic builds with -DMINER_RK_GEO1 launch it)
#ifdef MINER_RK_GEO1
  constexpr int NR = S == MINER_SCORE_WEIGHTED ? 2 * NKT : NKT;
  if constexpr (sizeof(T) == 2 && NR >= 2) return rk_launch_geo<T, NKT, S, 1>(stream, prm, split);
#endif
  return rk_launch_geo<T, NKT, S, 0>(stream, prm, split);
}

template <class T>
int rk_dispatch(void* stream, const RkParams& prm) {
  const int st = prm.score_type;
  if (prm.K <= 32) {
    if (st == MINER_SCORE_WEIGHTED) return rk_launch<T, 1, MINER_SCORE_WEIGHTED>(stream, prm);
    if (st == MINER_SCORE_MAX) return rk_launch<T, 1, MINER_SCORE_MAX>(stream, prm);
    return rk_launch<T, 1, MINER_SCORE_MEAN>(stream, prm);
  }
  if (st == MINER_SCORE_WEIGHTED) return rk_launch<T, 2, MINER_SCORE_WEIGHTED>(stream, prm);
  if (st == MINER_SCORE_MAX) return rk_launch<T, 2, MINER_SCORE_MAX>(stream, prm);
  return rk_launch<T, 2, MINER_SCORE_MEAN>(stream, prm);
}

int check_dims(int dtype, int d, int Dc, int K) {
  if (!dtype_ok(dtype) || d <= 0 || K <= 0 || Dc <= 0) return MINER_EINVAL;
  if (K > kMaxK || Dc > 32 * kDcT || d > kMaxD) return MINER_ESHAPE;
  if (d % (dtype == MINER_DTYPE_F32 ? 32 : 64)) return MINER_ESHAPE;
  return MINER_OK;
}

}  // namespace

extern "C" {

size_t miner_encoder_packed_bytes(int dtype, int d, int Dc, int K) {
  if (check_dims(dtype, d, Dc, K) != MINER_OK) return 0;
  return (ue_w1_elems(d) + ue_q_elems(K) + ue_w2_elems(d)) * esize(dtype);
}

int miner_encoder_pack(void* stream, int dtype, const void* w_poly, const void* context_codes, const void* w_target,
                       int d, int Dc, int K, void* packed) {
  const int ck = check_dims(dtype, d, Dc, K);
  if (ck != MINER_OK) return ck;
  if (!w_poly || !context_codes || !packed) return MINER_EINVAL;
  if (!aligned16(packed)) return MINER_EALIGN;
  const size_t n = ue_w1_elems(d) + ue_q_elems(K) + (w_target ? ue_w2_elems(d) : 0);
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dtype == MINER_DTYPE_BF16)
    hipLaunchKernelGGL(ue_pack_kernel<__bf16>, dim3(grid), dim3(256), 0, s, static_cast<const __bf16*>(w_poly),
                       static_cast<const __bf16*>(context_codes), static_cast<const __bf16*>(w_target), d, Dc, K,
                       static_cast<__bf16*>(packed));
  else if (dtype == MINER_DTYPE_F16)
    hipLaunchKernelGGL(ue_pack_kernel<_Float16>, dim3(grid), dim3(256), 0, s, static_cast<const _Float16*>(w_poly),
                       static_cast<const _Float16*>(context_codes), static_cast<const _Float16*>(w_target), d, Dc, K,
                       static_cast<_Float16*>(packed));
  else
    hipLaunchKernelGGL(ue_pack_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<const float*>(w_poly),
                       static_cast<const float*>(context_codes), static_cast<const float*>(w_target), d, Dc, K,
                       static_cast<float*>(packed));
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

int miner_encode_users(void* stream, int dtype, const void* history, const int32_t* his_ids, int n_news,
                       const uint8_t* his_mask, const float* his_bias, const void* packed, int U, int L, int d,
                       int Dc, int K, float* mui_f32, void* user_mui, void* user_proj) {
  const int ck = check_dims(dtype, d, Dc, K);
  if (ck != MINER_OK) return ck;
  if (U < 0 || L <= 0) return MINER_EINVAL;
  if (L > kMaxL) return MINER_ESHAPE;
  if (!history || !his_mask || !packed || !user_mui) return MINER_EINVAL;
  if (his_ids && n_news <= 0) return MINER_EINVAL;
  if (!aligned16(history) || !aligned16(packed) || !aligned16(user_mui) || !aligned16(user_proj) || !aligned16(mui_f32))
    return MINER_EALIGN;
  if (U == 0) return MINER_OK;
  UeParams prm{};
  prm.hist = history; prm.his_ids = his_ids; prm.n_news = n_news; prm.mask = his_mask; prm.bias = his_bias;
  prm.wp = packed; prm.mui_f32 = mui_f32; prm.user_mui = user_mui; prm.user_proj = user_proj;
  prm.U = U; prm.L = L; prm.d = d; prm.Dc = Dc; prm.K = K;
  if (dtype == MINER_DTYPE_BF16) return ue_dispatch<__bf16>(stream, prm);
  if (dtype == MINER_DTYPE_F16) return ue_dispatch<_Float16>(stream, prm);
  return ue_dispatch<float>(stream, prm);
}

size_t miner_rank_topk_workspace_bytes(int U, int topk) {
  if (U <= 0 || topk <= 0 || topk > kMaxTopk || num_cus() != 256) return 0;
  return rk_ws_bytes(U, topk);
}

int miner_rank_topk_split_recommended(int U) { return U > 0 && rk_split_wanted(U) ? 1 : 0; }

int miner_rank_topk(void* stream, int dtype, int score_type, const void* user_mui, const void* user_proj,
                    const void* news, int U, int N, int d, int K, int topk, float* top_scores, int32_t* top_ids) {
  return miner_rank_topk_ws(stream, dtype, score_type, user_mui, user_proj, news, U, N, d, K, topk, top_scores, top_ids,
                            nullptr, 0);
}

int miner_rank_topk_ws(void* stream, int dtype, int score_type, const void* user_mui, const void* user_proj,
                       const void* news, int U, int N, int d, int K, int topk, float* top_scores, int32_t* top_ids,
                       void* workspace, size_t workspace_bytes) {
  const int ck = check_dims(dtype, d, 1, K);
  if (ck != MINER_OK) return ck;
  if (score_type < MINER_SCORE_WEIGHTED || score_type > MINER_SCORE_MEAN) return MINER_EINVAL;
  if (U < 0 || N <= 0 || topk <= 0) return MINER_EINVAL;
  if (topk > kMaxTopk) return MINER_ESHAPE;
  if (!user_mui || !news || !top_scores || !top_ids) return MINER_EINVAL;
  if (score_type == MINER_SCORE_WEIGHTED && !user_proj) return MINER_EINVAL;
  if (!aligned16(user_mui) || !aligned16(user_proj) || !aligned16(news)) return MINER_EALIGN;
  if (U == 0) return MINER_OK;
  RkParams prm{};
  if (!aligned16(workspace)) return MINER_EALIGN;
  prm.mui = user_mui; prm.proj = user_proj; prm.news = news; prm.top_s = top_scores; prm.top_i = top_ids;
  if (workspace) {
    prm.ws_bytes = workspace_bytes;
    prm.ws_s = static_cast<float*>(workspace);
    prm.ws_i = reinterpret_cast<int32_t*>(static_cast<char*>(workspace) + (size_t)U * kSplit * topk * 4);
  }
  prm.U = U; prm.N = N; prm.d = d; prm.K = K; prm.topk = topk; prm.score_type = score_type;
  if (dtype == MINER_DTYPE_BF16) return rk_dispatch<__bf16>(stream, prm);
  if (dtype == MINER_DTYPE_F16) return rk_dispatch<_Float16>(stream, prm);
  return rk_dispatch<float>(stream, prm);
}

}  // extern "C"
