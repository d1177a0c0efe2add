// miner_auc.hip — exact global ROC AUC on the device, MI355X (gfx950).
//
// The reference's `auc` is scikit-learn's roc_auc_score over ALL flattened (label, probability)
// pairs (src/evaluation.py:53-55): not decomposable over impressions or ranks, and at config 3 it
// is 120M pairs.  Here it is a rank sum with ties counted one half, in exact integer arithmetic:
//
//   keys   = the fp32 scores mapped to order-preserving uint32 (+0 and -0 one key)
//   sort   (key, label) pairs by key (rocPRIM radix sort, AMD's native device primitives)
//   groups = runs of equal keys: (pos_g, neg_g) by a reduce-by-key over (label ? 2^32 : 1)
//   N2     = Σ_g pos_g · (2·negbelow_g + neg_g)      (negbelow = exclusive scan of neg_g)
//   AUC    = N2 / (2·npos·nneg)                        (NaN when one class is absent)
//
// N2 is the Mann-Whitney statistic doubled, so every count is an integer until the final
// division; sklearn's trapezoid over the ROC curve is the same quantity.  The workspace is
// caller-owned device memory (miner_auc_workspace_bytes); nothing synchronises.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>
#include <math.h>

#include "../../include/miner_score.h"
#include "../../include/miner_metrics.h"

namespace {

// grid-stride loops in size_t: n is up to 2^31 - 1, so a 32-bit index + stride could wrap
#define AUC_FOR(i, n) for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)(n); i += (size_t)gridDim.x * blockDim.x)

__global__ void auc_keys(const float* __restrict__ s, uint32_t* __restrict__ key, int n) {
  AUC_FOR(i, n) {
    uint32_t b = __float_as_uint(s[i]);
    if (b == 0x80000000u) b = 0u;                       // -0 == +0
    key[i] = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  }
}

__global__ void auc_vals(const uint8_t* __restrict__ lab, unsigned long long* __restrict__ v, int n) {
  AUC_FOR(i, n)
    v[i] = lab[i] ? (1ull << 32) : 1ull;
}

__global__ void auc_negs(const unsigned long long* __restrict__ agg, unsigned long long* __restrict__ neg,
                         const int* __restrict__ nruns, int n) {
  const size_t G = (size_t)*nruns;
  AUC_FOR(i, n)
    neg[i] = i < G ? (agg[i] & 0xffffffffull) : 0ull;
}

__global__ void auc_terms(const unsigned long long* __restrict__ agg, const unsigned long long* __restrict__ below,
                          unsigned long long* __restrict__ term, const int* __restrict__ nruns, int n) {
  const size_t G = (size_t)*nruns;
  AUC_FOR(i, n) {
    unsigned long long t = 0ull;
    if (i < G) {
      const unsigned long long a = agg[i];
      t = (a >> 32) * (2ull * below[i] + (a & 0xffffffffull));
    }
    term[i] = t;
  }
}

__global__ void auc_final(const unsigned long long* __restrict__ n2, const unsigned long long* __restrict__ tot,
                          double* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const double npos = (double)(*tot >> 32), nneg = (double)(*tot & 0xffffffffull);
    out[0] = (npos == 0.0 || nneg == 0.0) ? (double)NAN : (double)(*n2) / (2.0 * npos * nneg);
  }
}

struct AucWs {
  size_t keys_in, keys_out, lab_out, v, agg, below, nruns, n2, tot, temp, temp_bytes, total;
};

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

typedef unsigned long long u64;

hipError_t temp_bytes(int n, size_t& bytes) {
  const size_t N = (size_t)n;
  bytes = 0;
  size_t b = 0;
  hipError_t e = rocprim::radix_sort_pairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const uint8_t*)nullptr, (uint8_t*)nullptr, N, 0, 32);
  if (e != hipSuccess) return e;
  bytes = b > bytes ? b : bytes;
  b = 0;
  e = rocprim::reduce_by_key(nullptr, b, (const uint32_t*)nullptr, (const u64*)nullptr, N, (uint32_t*)nullptr,
                             (u64*)nullptr, (int*)nullptr, rocprim::plus<u64>(), rocprim::equal_to<uint32_t>());
  if (e != hipSuccess) return e;
  bytes = b > bytes ? b : bytes;
  b = 0;
  e = rocprim::exclusive_scan(nullptr, b, (const u64*)nullptr, (u64*)nullptr, (u64)0, N, rocprim::plus<u64>());
  if (e != hipSuccess) return e;
  bytes = b > bytes ? b : bytes;
  b = 0;
  e = rocprim::reduce(nullptr, b, (const u64*)nullptr, (u64*)nullptr, (u64)0, N, rocprim::plus<u64>());
  if (e != hipSuccess) return e;
  bytes = b > bytes ? b : bytes;
  return hipSuccess;
}

bool layout(int64_t n, AucWs& w) {
  size_t tb = 0;
  if (temp_bytes((int)n, tb) != hipSuccess) return false;
  const size_t N = (size_t)n;
  size_t o = 0;
  w.keys_in = o;  o = al256(o + 4 * N);
  w.keys_out = o; o = al256(o + 4 * N);
  w.lab_out = o;  o = al256(o + N);
  w.v = o;        o = al256(o + 8 * N);
  w.agg = o;      o = al256(o + 8 * N);
  w.below = o;    o = al256(o + 8 * N);
  w.nruns = o;    o = al256(o + 16);
  w.n2 = o;       o = al256(o + 16);
  w.tot = o;      o = al256(o + 16);
  w.temp = o;     o = al256(o + tb);
  w.temp_bytes = tb;
  w.total = o;
  return true;
}

}  // namespace

extern "C" {

size_t miner_auc_workspace_bytes(int64_t n) {
  if (n <= 0 || n > 0x7fffffffLL) return 0;
  AucWs w;
  return layout(n, w) ? w.total : 0;
}

int miner_global_auc(void* stream, const float* scores, const uint8_t* labels, int64_t n, void* workspace,
                     size_t workspace_bytes, double* auc_out) {
  if (!scores || !labels || !workspace || !auc_out || n <= 0) return MINER_EINVAL;
  if (n > 0x7fffffffLL) return MINER_ESHAPE;
  AucWs w;
  if (!layout(n, w)) return MINER_EINVAL;
  if (workspace_bytes < w.total) return MINER_EINVAL;
  const int N = (int)n;
  hipStream_t st = static_cast<hipStream_t>(stream);
  char* ws = static_cast<char*>(workspace);
  uint32_t* keys_in = reinterpret_cast<uint32_t*>(ws + w.keys_in);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(ws + w.keys_out);
  uint8_t* lab_out = reinterpret_cast<uint8_t*>(ws + w.lab_out);
  unsigned long long* v = reinterpret_cast<unsigned long long*>(ws + w.v);
  unsigned long long* agg = reinterpret_cast<unsigned long long*>(ws + w.agg);
  unsigned long long* below = reinterpret_cast<unsigned long long*>(ws + w.below);
  int* nruns = reinterpret_cast<int*>(ws + w.nruns);
  unsigned long long* n2 = reinterpret_cast<unsigned long long*>(ws + w.n2);
  unsigned long long* tot = reinterpret_cast<unsigned long long*>(ws + w.tot);
  void* temp = ws + w.temp;
  const int grid = (int)(((size_t)N + 255) / 256 < 8192 ? ((size_t)N + 255) / 256 : 8192);
  size_t tb = w.temp_bytes;
  hipError_t e;

  const size_t NN = (size_t)N;
  hipLaunchKernelGGL(auc_keys, dim3(grid), dim3(256), 0, st, scores, keys_in, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = rocprim::radix_sort_pairs(temp, tb, keys_in, keys_out, labels, lab_out, NN, 0, 32, st)) != hipSuccess)
    return (int)e;
  hipLaunchKernelGGL(auc_vals, dim3(grid), dim3(256), 0, st, lab_out, v, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = rocprim::reduce(temp, tb, v, tot, (u64)0, NN, rocprim::plus<u64>(), st)) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = rocprim::reduce_by_key(temp, tb, keys_out, v, NN, keys_in, agg, nruns, rocprim::plus<u64>(),
                                  rocprim::equal_to<uint32_t>(), st)) != hipSuccess)
    return (int)e;
  hipLaunchKernelGGL(auc_negs, dim3(grid), dim3(256), 0, st, agg, v, nruns, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = rocprim::exclusive_scan(temp, tb, v, below, (u64)0, NN, rocprim::plus<u64>(), st)) != hipSuccess)
    return (int)e;
  hipLaunchKernelGGL(auc_terms, dim3(grid), dim3(256), 0, st, agg, below, v, nruns, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = rocprim::reduce(temp, tb, v, n2, (u64)0, NN, rocprim::plus<u64>(), st)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(auc_final, dim3(1), dim3(64), 0, st, n2, tot, auc_out);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

}  // extern "C"
