// wide.hip — the scoring tail for reference-legal shapes past the fused kernels' limits
// (include/miner_wide.h): K up to 64 interests, any number of candidates, with the user side from
// miner_encode_users (corpus.hip: PolyAttention for L <= 256, K <= 64, and proj = gelu(mui·W2ᵀ)).
//
// wide_score<T, ST>: one workgroup (4 waves) per impression, candidates in passes of 64. The
// contraction over d runs in 32-column chunks staged through LDS (register prefetch of the next
// chunk behind the current chunk's MFMAs, two LDS buffers): the chunk's user rows mui / proj
// [K <= 64 x 32] and candidate rows [64 x 32]. Wave w owns candidates [16w, 16w + 16) of the pass
// and all interest tiles:
//   M [16 cands x 16 interests]  += Cand · muiᵀ   (model.py:127)
//   Lg[16 cands x 16 interests]  += Cand · projᵀ  (model.py:213, weighted only)
// fp32: v_mfma_f32_16x16x4_f32 (an exact fp32 fma chain), lane (j, g) feeding element 8g + s of
// candidate row j / interest row j to step s; 16-bit: one v_mfma_f32_16x16x32_{bf16,f16} per tile.
// The aggregation over K (model.py:128-136, :214) is an in-register epilogue: lane (j, g) holds
// candidates 4g + e for interests 16 kt + j, reduced over j by DPP within the 16-lane row.
//
// wide_proj<T>: out = gelu(x · W2ᵀ) (model.py:212) as a 64 x 64-tiled GEMM on the same chunk
// staging, for TargetAwareAttention.forward alone at K > 32.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "miner_wide.h"
#include "cdna4_common.h"

namespace {

constexpr int kWThreads = 256;        // 4 waves
constexpr int kWRows = 64;            // rows of a staged matrix: candidates of a pass / interests
constexpr int kWCols = 32;            // columns of a staged chunk

template <class T> struct WCfg {
  static constexpr int RB = kWCols * (int)sizeof(T);     // bytes of one chunk row
  static constexpr int RS = RB + 16;                     // LDS row stride (16-byte skew per row)
  static constexpr int MAT = kWRows * RS;                // one staged matrix
  static constexpr int PPR = RB / 16;                    // 16-byte pieces per chunk row
  static constexpr int PPT = kWRows * PPR / kWThreads;   // pieces per thread per matrix (2 / 1)
};

typedef float f32x4w __attribute__((ext_vector_type(4)));

// one MFMA step over a 32-column chunk: acc += A(row j, cols 8g..8g+7) · B(row j, cols 8g..8g+7)ᵀ
template <class T>
__device__ __forceinline__ f32x4w wide_mma(f32x4w acc, const char* arow, const char* brow, int g) {
  if constexpr (sizeof(T) == 4) {
    const float4 a0 = *reinterpret_cast<const float4*>(arow + 32 * g);
    const float4 a1 = *reinterpret_cast<const float4*>(arow + 32 * g + 16);
    const float4 b0 = *reinterpret_cast<const float4*>(brow + 32 * g);
    const float4 b1 = *reinterpret_cast<const float4*>(brow + 32 * g + 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc, 0, 0, 0);
  } else {
    const u32x4 a = *reinterpret_cast<const u32x4*>(arow + 16 * g);
    const u32x4 b = *reinterpret_cast<const u32x4*>(brow + 16 * g);
    if constexpr (kIsF16<T>)
      return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0,
                                                    0, 0);
    else
      return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                     0, 0, 0);
  }
}

// the pieces this thread stages of one matrix: rows (piece / PPR), 16-byte piece (piece % PPR)
template <class T, class RowPtr>
__device__ __forceinline__ void stage_load(u32x4* r, RowPtr row_ptr, int col0) {
  using Cf = WCfg<T>;
#pragma unroll
  for (int i = 0; i < Cf::PPT; ++i) {
    const int pc = (int)threadIdx.x + i * kWThreads;
    const int row = pc / Cf::PPR, piece = pc % Cf::PPR;
    const char* src = row_ptr(row);
    r[i] = src ? *reinterpret_cast<const u32x4*>(src + (size_t)col0 * sizeof(T) + 16 * piece)
               : u32x4{0u, 0u, 0u, 0u};
  }
}
template <class T>
__device__ __forceinline__ void stage_store(char* mat, const u32x4* r) {
  using Cf = WCfg<T>;
#pragma unroll
  for (int i = 0; i < Cf::PPT; ++i) {
    const int pc = (int)threadIdx.x + i * kWThreads;
    *reinterpret_cast<u32x4*>(mat + (pc / Cf::PPR) * Cf::RS + 16 * (pc % Cf::PPR)) = r[i];
  }
}

struct WideParams {
  const void* mui;
  const void* proj;
  const void* cand;
  const int32_t* cand_ids;
  const int32_t* offs;
  const float* value;
  float* scores;
  int n_news, B, C, d, K;
};

template <class T, int ST>
__global__ __launch_bounds__(kWThreads) void wide_score(WideParams p) {
  using Cf = WCfg<T>;
  constexpr bool WEIGHTED = ST == MINER_SCORE_WEIGHTED;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int K = p.K, d = p.d, KT = (K + 15) >> 4;
  const bool given = p.value != nullptr;               // TargetAwareAttention alone: M from the caller
  int off, cnt;
  if (p.offs) {
    off = p.offs[b];
    cnt = p.offs[b + 1] - off;
  } else {
    off = b * p.C;
    cnt = p.C;
  }
  const char* muiB = static_cast<const char*>(p.mui) + (size_t)b * K * d * sizeof(T);
  const char* prjB = WEIGHTED ? static_cast<const char*>(p.proj) + (size_t)b * K * d * sizeof(T) : nullptr;
  const char* candB = static_cast<const char*>(p.cand);
  const int nch = d / kWCols;
  constexpr int NM = WEIGHTED ? 3 : 2;                  // staged matrices: cand, mui[, proj]
  for (int c0 = 0; c0 < cnt; c0 += kWRows) {
    const int cp = min(kWRows, cnt - c0);
    auto cand_row = [&](int r) -> const char* {
      if (r >= cp) return nullptr;
      const int gi = off + c0 + r;
      if (p.cand_ids) {
        const int id = min(max(p.cand_ids[gi], 0), p.n_news - 1);
        return candB + (size_t)id * d * sizeof(T);
      }
      return candB + (size_t)gi * d * sizeof(T);
    };
    auto mui_row = [&](int r) -> const char* { return (!given && r < K) ? muiB + (size_t)r * d * sizeof(T) : nullptr; };
    auto prj_row = [&](int r) -> const char* { return r < K ? prjB + (size_t)r * d * sizeof(T) : nullptr; };
    f32x4w M[4], Lg[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) M[kt] = Lg[kt] = f32x4w{0.f, 0.f, 0.f, 0.f};
    u32x4 rc[Cf::PPT], rm[Cf::PPT], rp[Cf::PPT];
    auto load = [&](int ch) {
      stage_load<T>(rc, cand_row, ch * kWCols);
      if (!given) stage_load<T>(rm, mui_row, ch * kWCols);
      if (WEIGHTED) stage_load<T>(rp, prj_row, ch * kWCols);
    };
    auto store = [&](int buf) {
      char* base = smem + buf * NM * Cf::MAT;
      stage_store<T>(base, rc);
      if (!given) stage_store<T>(base + Cf::MAT, rm);
      if (WEIGHTED) stage_store<T>(base + (NM - 1) * Cf::MAT, rp);
    };
    load(0);
    store(0);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      if (ch + 1 < nch) load(ch + 1);                  // in flight behind this chunk's MFMAs
      const char* base = smem + (ch & 1) * NM * Cf::MAT;
      const char* arow = base + (16 * wave + j) * Cf::RS;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        if (kt < KT) {
          if (!given) M[kt] = wide_mma<T>(M[kt], arow, base + Cf::MAT + (16 * kt + j) * Cf::RS, g);
          if (WEIGHTED) Lg[kt] = wide_mma<T>(Lg[kt], arow, base + (NM - 1) * Cf::MAT + (16 * kt + j) * Cf::RS, g);
        }
      }
      if (ch + 1 < nch) store((ch + 1) & 1);
      __syncthreads();
    }
    // aggregation over the K interests: lane (j, g) holds candidates 16 wave + 4g + e
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 16 * wave + 4 * g + e;
      float m[4], l[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const int k = 16 * kt + j;
        m[kt] = M[kt][e];
        l[kt] = Lg[kt][e];
        if (given) m[kt] = (kt < KT && k < K && c < cp) ? p.value[(size_t)(off + c0 + c) * K + k] : 0.f;
      }
      float sc;
      if constexpr (WEIGHTED) {                        // softmax over K of Lg, weights on M (model.py:213-214)
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          if (kt < KT && 16 * kt + j < K) mx = fmaxf(mx, l[kt]);
        mx = row16_max(mx);
        float s = 0.f, num = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          if (kt < KT && 16 * kt + j < K) {
            const float pe = expf(l[kt] - mx);
            s += pe;
            num = __builtin_fmaf(pe, m[kt], num);
          }
        }
        s = row16_sum(s);
        num = row16_sum(num);
        sc = num / s;
      } else if constexpr (ST == MINER_SCORE_MAX) {    // model.py:128-129
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          if (kt < KT && 16 * kt + j < K) mx = fmaxf(mx, m[kt]);
        sc = row16_max(mx);
      } else {                                         // mean, model.py:130-131
        float s = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          if (kt < KT && 16 * kt + j < K) s += m[kt];
        sc = row16_sum(s) / (float)K;
      }
      if (j == 0 && c < cp) p.scores[off + c0 + c] = sc;
    }
  }
}

template <class T>
__global__ __launch_bounds__(kWThreads) void wide_proj(const T* x, const T* w2, int R, int d, T* out) {
  using Cf = WCfg<T>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int r0 = blockIdx.x * kWRows, n0 = blockIdx.y * kWRows;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto x_row = [&](int r) -> const char* {
    return r0 + r < R ? reinterpret_cast<const char*>(x + (size_t)(r0 + r) * d) : nullptr;
  };
  auto w_row = [&](int r) -> const char* { return reinterpret_cast<const char*>(w2 + (size_t)(n0 + r) * d); };
  f32x4w acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4w{0.f, 0.f, 0.f, 0.f};
  u32x4 rx[Cf::PPT], rw[Cf::PPT];
  const int nch = d / kWCols;
  stage_load<T>(rx, x_row, 0);
  stage_load<T>(rw, w_row, 0);
  stage_store<T>(smem, rx);
  stage_store<T>(smem + Cf::MAT, rw);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) {
      stage_load<T>(rx, x_row, (ch + 1) * kWCols);
      stage_load<T>(rw, w_row, (ch + 1) * kWCols);
    }
    const char* base = smem + (ch & 1) * 2 * Cf::MAT;
    const char* arow = base + (16 * wave + j) * Cf::RS;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = wide_mma<T>(acc[t], arow, base + Cf::MAT + (16 * t + j) * Cf::RS, g);
    if (ch + 1 < nch) {
      char* nb = smem + ((ch + 1) & 1) * 2 * Cf::MAT;
      stage_store<T>(nb, rx);
      stage_store<T>(nb + Cf::MAT, rw);
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = r0 + 16 * wave + 4 * g + e;
      if (r < R) out[(size_t)r * d + n0 + 16 * t + j] = (T)gelu_erf(acc[t][e]);   // model.py:212
    }
  }
}

bool dtype_ok(int dtype) { return dtype == MINER_DTYPE_F32 || dtype == MINER_DTYPE_BF16 || dtype == MINER_DTYPE_F16; }
bool al16(const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15u) == 0; }

template <class T, int ST>
int launch_score(void* stream, const WideParams& prm) {
  constexpr int NM = ST == MINER_SCORE_WEIGHTED ? 3 : 2;
  const int lds = 2 * NM * WCfg<T>::MAT;
  hipLaunchKernelGGL((wide_score<T, ST>), dim3(prm.B), dim3(kWThreads), lds, static_cast<hipStream_t>(stream), prm);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

template <class T>
int dispatch_score(void* stream, int st, const WideParams& prm) {
  if (st == MINER_SCORE_WEIGHTED) return launch_score<T, MINER_SCORE_WEIGHTED>(stream, prm);
  if (st == MINER_SCORE_MAX) return launch_score<T, MINER_SCORE_MAX>(stream, prm);
  return launch_score<T, MINER_SCORE_MEAN>(stream, prm);
}

template <class T>
int launch_proj(void* stream, const void* x, const void* w2, int R, int d, void* out) {
  const dim3 grid((R + kWRows - 1) / kWRows, d / kWRows);
  hipLaunchKernelGGL(wide_proj<T>, grid, dim3(kWThreads), 4 * WCfg<T>::MAT, static_cast<hipStream_t>(stream),
                     static_cast<const T*>(x), static_cast<const T*>(w2), R, d, static_cast<T*>(out));
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

}  // namespace

extern "C" {

int miner_wide_supported(int dtype, int L, int d, int Dc, int K) {
  if (!dtype_ok(dtype) || L <= 0 || d <= 0 || Dc <= 0 || K <= 0) return MINER_EINVAL;
  // the user side is miner_encode_users (corpus.h: L <= 256, K <= 64, Dc <= 256, d <= 768)
  if (L > 256 || K > MINER_WIDE_MAX_K || Dc > 256 || d > 768) return MINER_ESHAPE;
  if (d % (dtype == MINER_DTYPE_F32 ? 32 : 64)) return MINER_ESHAPE;
  return MINER_OK;
}

int miner_score_wide(void* stream, int dtype, int score_type, const void* user_mui, const void* user_proj,
                     const void* cand, const int32_t* cand_ids, int n_news, const int32_t* cand_offsets,
                     const float* value, int B, int C, int d, int K, float* scores) {
  if (!dtype_ok(dtype) || score_type < MINER_SCORE_WEIGHTED || score_type > MINER_SCORE_MEAN) return MINER_EINVAL;
  if (B < 0 || d <= 0 || K <= 0 || (!cand_offsets && C < 0)) return MINER_EINVAL;
  if (K > MINER_WIDE_MAX_K || d % (dtype == MINER_DTYPE_F32 ? 32 : 64)) return MINER_ESHAPE;
  if (!cand || !scores || (!value && !user_mui)) return MINER_EINVAL;
  if (score_type == MINER_SCORE_WEIGHTED && !user_proj) return MINER_EINVAL;
  if (value && score_type != MINER_SCORE_WEIGHTED) return MINER_EINVAL;
  if (cand_ids && n_news <= 0) return MINER_EINVAL;
  if (!al16(user_mui) || !al16(user_proj) || !al16(cand)) return MINER_EALIGN;
  if (B == 0 || (!cand_offsets && C == 0)) return MINER_OK;
  WideParams prm{};
  prm.mui = user_mui; prm.proj = user_proj; prm.cand = cand; prm.cand_ids = cand_ids; prm.offs = cand_offsets;
  prm.value = value; prm.scores = scores; prm.n_news = n_news; prm.B = B; prm.C = C; prm.d = d; prm.K = K;
  if (dtype == MINER_DTYPE_BF16) return dispatch_score<__bf16>(stream, score_type, prm);
  if (dtype == MINER_DTYPE_F16) return dispatch_score<_Float16>(stream, score_type, prm);
  return dispatch_score<float>(stream, score_type, prm);
}

int miner_wide_proj(void* stream, int dtype, const void* x, const void* w_target, int R, int d, void* out) {
  if (!dtype_ok(dtype) || R < 0 || d <= 0 || !x || !w_target || !out) return MINER_EINVAL;
  if (d % 64) return MINER_ESHAPE;
  if (!al16(x) || !al16(w_target) || !al16(out)) return MINER_EALIGN;
  if (R == 0) return MINER_OK;
  if (dtype == MINER_DTYPE_BF16) return launch_proj<__bf16>(stream, x, w_target, R, d, out);
  if (dtype == MINER_DTYPE_F16) return launch_proj<_Float16>(stream, x, w_target, R, d, out);
  return launch_proj<float>(stream, x, w_target, R, d, out);
}

}  // extern "C"
