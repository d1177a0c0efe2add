// cdna4_common.h — device helpers shared by the HIP kernels of libminer_hip.so (gfx950 / CDNA4):
// slab fragments and the 32x32 MFMA step over them, the pi row order of packed weight tiles,
// DPP row reductions, bf16-mode transcendental approximations, LDS-DMA from inline asm.
//
// Slab layout (both dtypes): a "slab" is 32 consecutive contraction indices; lane l = 32h + r
// (h = l>>5, r = l&31) holds 16 contiguous elements [16h, 16h+16) of row r of the slab. bf16: two
// v_mfma_f32_32x32x16_bf16 steps (8 elements each); fp32: sixteen v_mfma_f32_32x32x2_f32 steps
// (one element each, an exact fp32 fma chain). A 32x32 accumulator keeps row (e&3)+8(e>>2)+4h of
// column r in register e; with the A-operand rows taken in the order pi(r) register e of lane half
// h holds row 16h+e, so an accumulator IS a slab fragment of a following contraction over its rows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
typedef __attribute__((address_space(3))) char lds_char;


__host__ __device__ inline int pi_row(int r) { return 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3); }

// ---------------------------------------------------------------------------------------------
// element helpers
// ---------------------------------------------------------------------------------------------
template <class T> struct Frag;            // one lane's 16-element slab fragment
template <> struct Frag<__bf16> { u32x4 q[2]; };
template <> struct Frag<_Float16> { u32x4 q[2]; };
template <> struct Frag<float> { u32x4 q[4]; };
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <class T> constexpr bool kIsF16 = __is_same(T, _Float16);
template <class T> constexpr int kNQ = sizeof(T);   // u32x4 per fragment (bf16: 2, fp32: 4)

template <class T>
__device__ __forceinline__ void frag_zero(Frag<T>& f) {
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i) f.q[i] = u32x4{0u, 0u, 0u, 0u};
}

// 16 contiguous elements from a 16-byte-aligned address (global or LDS)
template <class T>
__device__ __forceinline__ void frag_load(Frag<T>& f, const T* p) {
  const u32x4* s = reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i) f.q[i] = s[i];
}

// streamed-once data (candidate rows): non-temporal, so it does not evict the weights from L2
#ifndef MINER_STREAM_NT
#define MINER_STREAM_NT 1
#endif
template <class T>
__device__ __forceinline__ void frag_load_stream(Frag<T>& f, const T* p) {
  const u32x4* s = reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i) f.q[i] = MINER_STREAM_NT ? __builtin_nontemporal_load(s + i) : s[i];
}

// slab fragment of a packed weight block (fragment-major, see the packed layout)
template <class T>
__device__ __forceinline__ void frag_load_tile(Frag<T>& f, const T* block, int lane) {
  const u32x4* s = reinterpret_cast<const u32x4*>(block) + lane;
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i) f.q[i] = s[64 * i];
}

template <class T>
__device__ __forceinline__ void frag_store(T* p, const Frag<T>& f) {
  u32x4* s = reinterpret_cast<u32x4*>(p);
#pragma unroll
  for (int i = 0; i < kNQ<T>; ++i) s[i] = f.q[i];
}

template <class T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

// two fp32 -> one dword of 16-bit values (RNE), as a vector conversion: one v_cvt_pk_f16_f32 /
// v_cvt_pk_bf16_f32 (gfx950); converting the halves one by one costs 3-4 VALU (two converts, a
// shift and an OR) for the same bits
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
#ifndef MINER_PK_CVT
#define MINER_PK_CVT 1   // A/B: 0 = the per-half conversions
#endif
__device__ __forceinline__ unsigned pack_f16x2(float lo, float hi) {
#if MINER_PK_CVT
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){lo, hi}, f16x2v));
#else
  _Float16 a = (_Float16)lo, b = (_Float16)hi;
  return (unsigned)__builtin_bit_cast(unsigned short, a) | ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
#endif
}
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
#if MINER_PK_CVT
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){lo, hi}, bf16x2v));
#else
  __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (unsigned)__builtin_bit_cast(unsigned short, a) | ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
#endif
}

// accumulator tile (rows taken in pi order) -> 16 contiguous elements / slab fragment
template <class T>
__device__ __forceinline__ void acc_to_frag(Frag<T>& f, const f32x16& x) {
  if constexpr (kIsF16<T>) {
#pragma unroll
    for (int m = 0; m < 8; ++m) f.q[m >> 2][m & 3] = pack_f16x2(x[2 * m], x[2 * m + 1]);
  } else if constexpr (sizeof(T) == 2) {
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
  if constexpr (kIsF16<T>) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a.q[s]),
                                                   __builtin_bit_cast(f16x8, b.q[s]), acc, 0, 0, 0);
  } else if constexpr (sizeof(T) == 2) {
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

__device__ __forceinline__ int acc_row(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

// all-reduce over the 16 lanes of a DPP row: quad_perm xor1, xor2, row_half_mirror, row_mirror
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row16_max(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));
  x = fmaxf(x, dpp_f<0x4E>(x));
  x = fmaxf(x, dpp_f<0x141>(x));
  return fmaxf(x, dpp_f<0x140>(x));
}
__device__ __forceinline__ float row16_sum(float x) {
  x += dpp_f<0xB1>(x);
  x += dpp_f<0x4E>(x);
  x += dpp_f<0x141>(x);
  return x + dpp_f<0x140>(x);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  return z;
}

// torch.nn.functional.gelu(approximate='none')
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

// The same GELU branch-free for the fp32 parity kernels: x·Φ(x) with Φ from the Chebyshev erfc of
// Numerical Recipes (erfc(z) = t·exp(-z² + P(t)), t = 1/(1 + z/2), fractional error < 1.2e-7 for
// every z >= 0, tails included): Φ(x) = erfc(|x|/√2)/2 for x < 0, 1 - erfc(|x|/√2)/2 otherwise.
// |Δgelu| <= 1.6e-7·max(1, |x|) against float64 (tools/gelu_error.py; hardware rcp / exp2 add ~1 ulp)
// — about the rounding of Φ itself — in ~16 VALU with one v_rcp and one v_exp, where libm erff
// runs two divergent polynomial branches (~40 VALU + exec-mask SALU). The fp32 MFMA does not
// co-issue with VALU on gfx950, so every VALU instruction of the GELU is paid in MFMA time.
__device__ __forceinline__ float gelu_erfc_nr(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.5f, z, 1.0f));
  float q = 0.17087277f;
  q = __builtin_fmaf(q, t, -0.82215223f);
  q = __builtin_fmaf(q, t, 1.48851587f);
  q = __builtin_fmaf(q, t, -1.13520398f);
  q = __builtin_fmaf(q, t, 0.27886807f);
  q = __builtin_fmaf(q, t, -0.18628806f);
  q = __builtin_fmaf(q, t, 0.09678418f);
  q = __builtin_fmaf(q, t, 0.37409196f);
  q = __builtin_fmaf(q, t, 1.00002368f);
  q = __builtin_fmaf(q, t, -1.26551223f);
  const float y = __builtin_fmaf(-z, z, q);
  const float ec = t * __builtin_amdgcn_exp2f(y * 1.4426950408889634f);   // erfc(z)
  const float phi = x < 0.f ? 0.5f * ec : __builtin_fmaf(-0.5f, ec, 1.0f);
  return x * phi;
}

// ---------------------------------------------------------------------------------------------
// fp32 contractions on the bf16 matrix cores (bf16x6): an fp32 value is cut into three bf16 terms
// by truncation, x = hi + mid + lo EXACTLY (hi takes the top 8 significand bits, mid the top 8 of
// the exact remainder x - hi, and the remainder after that has at most 8 significant bits, so lo
// holds it exactly). A product a·b is then the six partial products whose order is at most 2^-16
// (al·bh, ah·bl, am·bm, am·bh, ah·bm, ah·bh — every product of two bf16 values is exact in fp32);
// what is dropped (am·bl, al·bm, al·bl) is below 2^-23·|a·b|, under the rounding of the fp32 sum.
// Six v_mfma_f32_16x16x32_bf16 (16 cycles each) replace the fp32 MFMA work of one contraction at
// 1/16 of the bf16 rate: 2.67x the fp32 rate, and unlike the fp32 MFMA they co-issue with VALU.
// ---------------------------------------------------------------------------------------------
struct Split8 { u32x4 hi, mid, lo; };       // 8 fp32 elements as three bf16x8 operands
#ifndef MINER_SPLIT3_INF
#define MINER_SPLIT3_INF 2   // residual of a non-finite x: 0 none (inf - inf = NaN), 1 compare + select, 2 med3 clamp
#endif

__device__ __forceinline__ unsigned hi16_pack(unsigned a, unsigned b) {   // (a >> 16) | (b & 0xffff0000)
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
}
// SAFE: the operand may hold ±inf (activations: history rows, mui); the weight operands of the
// dense kernel's S1 / S5 take the plain form (an infinite weight gives NaN in the reference too)
template <bool SAFE = true>
__device__ __forceinline__ void split3_pair(float x0, float x1, unsigned& hi, unsigned& mid, unsigned& lo) {
  const unsigned u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
  hi = hi16_pack(u0, u1);
  if constexpr (!SAFE) {
    const float r0 = x0 - __uint_as_float(u0 & 0xffff0000u), r1 = x1 - __uint_as_float(u1 & 0xffff0000u);
    const unsigned v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
    mid = hi16_pack(v0, v1);
    const float q0 = r0 - __uint_as_float(v0 & 0xffff0000u), q1 = r1 - __uint_as_float(v1 & 0xffff0000u);
    lo = hi16_pack(__float_as_uint(q0), __float_as_uint(q1));
    return;
  }
#if MINER_SPLIT3_INF == 1
  // an infinite x truncates to itself: its residual is 0, not inf - inf (a NaN x stays NaN in mid)
  const float h0 = __uint_as_float(u0 & 0xffff0000u), h1 = __uint_as_float(u1 & 0xffff0000u);
  const float r0 = x0 == h0 ? 0.f : x0 - h0, r1 = x1 == h1 ? 0.f : x1 - h1;
#elif MINER_SPLIT3_INF == 2
  // the residual of x clamped to the finite range (one v_med3 per element): an infinite x keeps hi =
  // ±inf and finite mid / lo (FLT_MAX's low bits, absorbed by the infinite product), not the NaN of
  // inf - inf; a NaN x stays NaN (med3 passes it through to r, and so to mid)
  const float c0 = __builtin_amdgcn_fmed3f(x0, -3.40282347e38f, 3.40282347e38f);
  const float c1 = __builtin_amdgcn_fmed3f(x1, -3.40282347e38f, 3.40282347e38f);
  const float r0 = c0 - __uint_as_float(__float_as_uint(c0) & 0xffff0000u);
  const float r1 = c1 - __uint_as_float(__float_as_uint(c1) & 0xffff0000u);
#else
  const float r0 = x0 - __uint_as_float(u0 & 0xffff0000u), r1 = x1 - __uint_as_float(u1 & 0xffff0000u);
#endif
  const unsigned v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
  mid = hi16_pack(v0, v1);
  const float q0 = r0 - __uint_as_float(v0 & 0xffff0000u), q1 = r1 - __uint_as_float(v1 & 0xffff0000u);
  lo = hi16_pack(__float_as_uint(q0), __float_as_uint(q1));
}
__device__ __forceinline__ Split8 split8(const float* x) {
  Split8 s;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    unsigned h, md, l;
    split3_pair(x[2 * m], x[2 * m + 1], h, md, l);
    s.hi[m] = h;
    s.mid[m] = md;
    s.lo[m] = l;
  }
  return s;
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16_bf16(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// c += A·B over 32 contraction indices at fp32 accuracy; A-operand lane map A[row l&15][k 8(l>>4)+e],
// B-operand B[k 8(l>>4)+e][col l&15], smallest terms first
__device__ __forceinline__ f32x4 mma_x6(f32x4 c, const Split8& a, const Split8& b) {
  c = mfma16_bf16(a.lo, b.hi, c);
  c = mfma16_bf16(a.hi, b.lo, c);
  c = mfma16_bf16(a.mid, b.mid, c);
  c = mfma16_bf16(a.mid, b.hi, c);
  c = mfma16_bf16(a.hi, b.mid, c);
  return mfma16_bf16(a.hi, b.hi, c);
}

// The same on 32x32 slab fragments (miner_fused<fp32> with X6): a Frag<float> (16 contraction
// elements per lane) cut into three bf16 terms, the six partial products smallest first —
// 12 v_mfma_f32_32x32x16_bf16 (384 cycles) for the 1024 cycles of the 16 v_mfma_f32_32x32x2_f32
// of one slab product.
// One 16-element step at a time (8 contraction elements per lane), so only 2 x 3 bf16 operand
// registers quads are live beside the fp32 fragments.
template <bool SAFE = true>
__device__ __forceinline__ void split8_step(const Frag<float>& f, int st, u32x4& h, u32x4& m, u32x4& l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {               // elements 8st + 2i, 8st + 2i + 1 -> dword i
    const int e = 8 * st + 2 * i;
    unsigned hh, mm, ll;
    split3_pair<SAFE>(__uint_as_float(f.q[e >> 2][e & 3]), __uint_as_float(f.q[(e + 1) >> 2][(e + 1) & 3]), hh, mm, ll);
    h[i] = hh;
    m[i] = mm;
    l[i] = ll;
  }
}
__device__ __forceinline__ f32x16 mfma32_bf16(const u32x4& a, const u32x4& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// the six partial products of one 8-element step, smallest first (the order of mma_slab_x6)
__device__ __forceinline__ void mma6_step(f32x16& acc, const u32x4& ah, const u32x4& am, const u32x4& al,
                                          const u32x4& bh, const u32x4& bm, const u32x4& bl) {
  acc = mfma32_bf16(al, bh, acc);
  acc = mfma32_bf16(ah, bl, acc);
  acc = mfma32_bf16(am, bm, acc);
  acc = mfma32_bf16(am, bh, acc);
  acc = mfma32_bf16(ah, bm, acc);
  acc = mfma32_bf16(ah, bh, acc);
}
__device__ __forceinline__ void mma_slab_x6(f32x16& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    u32x4 ah, am, al, bh, bm, bl;
    split8_step<false>(a, st, ah, am, al);     // the weights (S1 W1, S5 W2)
    split8_step<true>(b, st, bh, bm, bl);      // the activations (E, mui): ±inf kept

    acc = mfma32_bf16(al, bh, acc);            // smallest terms first
    acc = mfma32_bf16(ah, bl, acc);
    acc = mfma32_bf16(am, bm, acc);
    acc = mfma32_bf16(am, bh, acc);
    acc = mfma32_bf16(ah, bm, acc);
    acc = mfma32_bf16(ah, bh, acc);
  }
}

// The fp32 kernels' GELU at fewer VALU: Abramowitz & Stegun 7.1.26, erf(z) = 1 - t·P5(t)·e^{-z²},
// t = 1/(1 + 0.3275911 z), |Δerf| <= 1.5e-7 for every z >= 0, so |Δgelu| <= 0.75e-7·|x| plus the
// fp32 rounding: <= 2.2e-7·max(1, |x|) against float64 (tools/gelu_error.py), the accuracy class of
// gelu_erfc_nr in ~13 VALU + rcp + exp instead of ~19 + rcp + exp.
__device__ __forceinline__ float gelu_as_f32(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, z, 1.0f));
  float q = __builtin_fmaf(1.061405429f, t, -1.453152027f);
  q = __builtin_fmaf(q, t, 1.421413741f);
  q = __builtin_fmaf(q, t, -0.284496736f);
  q = __builtin_fmaf(q, t, 0.254829592f);
  q *= t;
  const float e = __builtin_amdgcn_exp2f(-1.4426950408889634f * (z * z));
  const float erfz = __builtin_fmaf(-q, e, 1.0f);
  const float hx = 0.5f * x;
  return __builtin_fmaf(hx, copysignf(erfz, x), hx);
}

// gelu_as_f32 on two values at once in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two results per
// lane per VALU issue). Per pair 14 full-rate VALU + 2 rcp + 2 exp instead of 22 + 4: the fp32 MFMA
// excludes VALU on its SIMD, so the GELU's issue cycles add to the MFMA time one for one. The
// 1/sqrt(2) is folded into the denominator's coefficient and the exponent's (tools/gelu_error.py
// gelu_as_pk: <= 2.2e-7·max(1, |x|) against float64, the accuracy class of gelu_as_f32).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_as_f32x2(f32x2 x) {
  constexpr float kA = 0.3275911f * 0.70710678118654752440f;
  const f32x2 t = {__builtin_amdgcn_rcpf(__builtin_fmaf(kA, fabsf(x[0]), 1.0f)),
                   __builtin_amdgcn_rcpf(__builtin_fmaf(kA, fabsf(x[1]), 1.0f))};
  // nq = -t·P5(t): the Horner coefficients negated (exact), so erf needs no negation instruction
  f32x2 nq = __builtin_elementwise_fma((f32x2)(-1.061405429f), t, (f32x2)(1.453152027f));
  nq = __builtin_elementwise_fma(nq, t, (f32x2)(-1.421413741f));
  nq = __builtin_elementwise_fma(nq, t, (f32x2)(0.284496736f));
  nq = __builtin_elementwise_fma(nq, t, (f32x2)(-0.254829592f));
  nq = nq * t;
  const f32x2 y = (x * x) * (f32x2)(-0.72134752044448170368f);       // -z²·log2(e), z = |x|/sqrt(2)
  const f32x2 e = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
  f32x2 erfz = __builtin_elementwise_fma(nq, e, (f32x2)(1.0f));
  erfz[0] = copysignf(erfz[0], x[0]);
  erfz[1] = copysignf(erfz[1], x[1]);
  const f32x2 hx = x * (f32x2)(0.5f);
  return __builtin_elementwise_fma(hx, erfz, hx);
}
template <class V> __device__ __forceinline__ void gelu_as_pairs(V& x, int n) {   // n even, compile-time
#pragma unroll
  for (int e = 0; e < n; e += 2) {
    const f32x2 r = gelu_as_f32x2(f32x2{x[e], x[e + 1]});
    x[e] = r[0];
    x[e + 1] = r[1];
  }
}

// bf16-mode transcendentals: branch-free, a handful of VALU ops each.  Their error (tanh: a few
// fp32 ulp of 1; erf: <= 1.5e-7 absolute, Abramowitz & Stegun 7.1.26) is far below the bf16
// operand rounding of that mode.  The fp32 parity mode uses the libm tanhf / erff / expf.
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(fminf(2.8853900817779268f * fabsf(x), 126.f));  // e^{2|x|}
  return copysignf(1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f), x);
}
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float erfz = 1.0f - poly * __builtin_amdgcn_exp2f(-1.4426950408889634f * z * z);
  return 0.5f * x * (1.0f + copysignf(erfz, x));
}
// bf16-mode GELU without transcendentals, two values per packed-fp32 instruction (v_pk_fma_f32):
// Φ(x) = 0.5 + x·P(x²) on |x| <= 4 (x clamped there), P the degree-7 weighted least-squares fit of
// 0.5·erf(x/√2)/x: |ΔΦ| <= 5e-5, so |Δgelu(x)| <= 5e-5·|x| — far below bf16 operand rounding.
__device__ __forceinline__ f32x2 gelu_poly2(f32x2 x) {
  f32x2 xc;
  xc.x = __builtin_amdgcn_fmed3f(x.x, -4.0f, 4.0f);
  xc.y = __builtin_amdgcn_fmed3f(x.y, -4.0f, 4.0f);
  const f32x2 u = xc * xc;
  f32x2 q = f32x2{-1.5762298e-09f, -1.5762298e-09f};
  q = __builtin_elementwise_fma(q, u, f32x2{1.2146164e-07f, 1.2146164e-07f});
  q = __builtin_elementwise_fma(q, u, f32x2{-4.095486e-06f, -4.095486e-06f});
  q = __builtin_elementwise_fma(q, u, f32x2{8.060949e-05f, 8.060949e-05f});
  q = __builtin_elementwise_fma(q, u, f32x2{-0.0010478799f, -0.0010478799f});
  q = __builtin_elementwise_fma(q, u, f32x2{0.0096639795f, 0.0096639795f});
  q = __builtin_elementwise_fma(q, u, f32x2{-0.066174366f, -0.066174366f});
  q = __builtin_elementwise_fma(q, u, f32x2{0.39884722f, 0.39884722f});
  const f32x2 phi = __builtin_elementwise_fma(xc, q, f32x2{0.5f, 0.5f});
  return x * phi;
}
// GELU over a whole accumulator tile: packed polynomial (bf16 mode) or exact erf (fp32 parity)
template <class T>
__device__ __forceinline__ void gelu_tile(f32x16& a) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const f32x2 g = gelu_poly2(f32x2{a[e], a[e + 1]});
      a[e] = g.x;
      a[e + 1] = g.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = gelu_erf(a[e]);
  }
}


__device__ __forceinline__ unsigned lds_offset(const void* p) { return (unsigned)(uintptr_t)(const lds_char*)p; }

// LDS-DMA from inline asm.  hipcc tracks its own global_load_lds and then waits vmcnt(0) before
// every later LDS access it cannot prove disjoint; an asm DMA is invisible to that analysis.  Its
// completion is the consumer's business: an explicit `s_waitcnt vmcnt(0)` before the barrier that
// publishes the data (vm_wait_all).  hipcc's own vmcnt(N) waits stay correct — an older untracked
// load only makes the in-order counter wait for one more.  M0 (the LDS base of the DMA) is saved
// and restored around the instruction.  `lds` must be wave-uniform; lane i writes lds + i·size.
__device__ __forceinline__ void dma_b128(const void* g, unsigned lds) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(g), "s"(lds) : "memory");
}
// the same with the default cache policy (lines meant to stay in L2 for other CUs to re-read)
__device__ __forceinline__ void dma_b128_rt(const void* g, unsigned lds) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma_b32(const void* g, unsigned lds) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Lane ids re-derived from an opaque copy of threadIdx.x at the top of every stage (see header).
#define FRESH_LANE_IDS()                                              \
  int tid_o_ = threadIdx.x;                                           \
  asm volatile("" : "+v"(tid_o_));                                    \
  const int tid = tid_o_;                                             \
  const int lane = tid & 63;                                          \
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);          \
  const int r = lane & 31;                                            \
  const int h = lane >> 5;                                            \
  (void)tid; (void)lane; (void)wave; (void)r; (void)h


// element x (0..1023) of a fragment-major block -> (tile row rr, column cc)
template <class T>
__device__ __forceinline__ void block_pos(int x, int& rr, int& cc) {
  constexpr int epp = 16 / (int)sizeof(T);      // elements per 16-byte piece
  const int piece = x / epp, t = x % epp;
  const int q = piece >> 6, l = piece & 63;     // piece q of lane l
  rr = l & 31;
  cc = 16 * (l >> 5) + q * epp + t;
}

// history image in LDS (16-bit rows of a row-major matrix, one LDS-DMA 1 KiB block per wave-instruction)
// Rows of 2d bytes packed back to back — the LDS-DMA (global_load_lds_dwordx4) writes each
// wave's 1 KiB linearly — with 16-byte chunk c of row `row` stored at chunk c ^ eswz(row).  The
// XOR is applied on the DMA's per-lane SOURCE address and again on every read: the 16 rows of a
// ds_read_b128 lane group land in 16 different 16-byte slots (S1) and the 4 rows of a
// ds_read_b64_tr_b16 block in 4 different 64-byte groups (S4), both conflict-free.
// (g16: 16 chunks per 256 B) low 2 bits from the row's quad, (q + 2·(q>>2)) & 3, so that 16
// consecutive rows AND 16 rows taken in pi order (quads 0,1,4,5 / 2,3,6,7: S1's operand rows) hit
// 16 different slots
__device__ __forceinline__ int eswz(int row, int g16) {
  return g16 ? (((row & 3) << 2) | (((row >> 2) + ((row >> 4) << 1)) & 3)) : (((row & 1) << 2) | ((row >> 1) & 3));
}

}  // namespace
