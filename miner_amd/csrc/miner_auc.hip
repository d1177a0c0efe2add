// miner_auc.hip — exact global ROC AUC on the device, MI355X (gfx950).
//
// The reference's `auc` is scikit-learn's roc_auc_score over ALL flattened (label, probability)
// pairs (src/evaluation.py:53-55): not decomposable over impressions or ranks, and at config 3 it
// is 120M pairs.  Here it is a rank sum with ties counted one half, in exact integer arithmetic:
//
//   keys   = the fp32 scores mapped to order-preserving uint32 (+0 and -0 one key)
//   sort   (key, label) pairs by key (hipCUB radix sort, 4 passes of 8 bits)
//   groups = runs of equal keys: (pos_g, neg_g) by a reduce-by-key over (label ? 2^32 : 1)
//   N2     = Σ_g pos_g · (2·negbelow_g + neg_g)      (negbelow = exclusive scan of neg_g)
//   AUC    = N2 / (2·npos·nneg)                        (NaN when one class is absent)
//
// N2 is the Mann-Whitney statistic doubled, so every count is an integer until the final
// division; sklearn's trapezoid over the ROC curve is the same quantity.  The workspace is
// caller-owned device memory (miner_auc_workspace_bytes); nothing synchronises.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <math.h>

#include "../../include/miner_score.h"
#include "../../include/miner_metrics.h"

namespace {

__global__ void auc_keys(const float* __restrict__ s, uint32_t* __restrict__ key, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t b = __float_as_uint(s[i]);
    if (b == 0x80000000u) b = 0u;                       // -0 == +0
    key[i] = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  }
}

__global__ void auc_vals(const uint8_t* __restrict__ lab, unsigned long long* __restrict__ v, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    v[i] = lab[i] ? (1ull << 32) : 1ull;
}

__global__ void auc_negs(const unsigned long long* __restrict__ agg, unsigned long long* __restrict__ neg,
                         const int* __restrict__ nruns, int n) {
  const int G = *nruns;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    neg[i] = i < G ? (agg[i] & 0xffffffffull) : 0ull;
}

__global__ void auc_terms(const unsigned long long* __restrict__ agg, const unsigned long long* __restrict__ below,
                          unsigned long long* __restrict__ term, const int* __restrict__ nruns, int n) {
  const int G = *nruns;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
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

hipError_t temp_bytes(int n, size_t& bytes) {
  bytes = 0;
  size_t b = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                    (const uint8_t*)nullptr, (uint8_t*)nullptr, n);
  if (e != hipSuccess) return e;
  bytes = b > bytes ? b : bytes;
  b = 0;
  e = hipcub::DeviceReduce::ReduceByKey(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                        (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                        (int*)nullptr, hipcub::Sum(), n);
  if (e != hipSuccess) return e;
  bytes = b > bytes ? b : bytes;
  b = 0;
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const unsigned long long*)nullptr, (unsigned long long*)nullptr, n);
  if (e != hipSuccess) return e;
  bytes = b > bytes ? b : bytes;
  b = 0;
  e = hipcub::DeviceReduce::Sum(nullptr, b, (const unsigned long long*)nullptr, (unsigned long long*)nullptr, n);
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
  const int grid = (int)((N + 255) / 256 < 8192 ? (N + 255) / 256 : 8192);
  size_t tb = w.temp_bytes;
  hipError_t e;

  hipLaunchKernelGGL(auc_keys, dim3(grid), dim3(256), 0, st, scores, keys_in, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = hipcub::DeviceRadixSort::SortPairs(temp, tb, keys_in, keys_out, labels, lab_out, N, 0, 32, st)) != hipSuccess)
    return (int)e;
  hipLaunchKernelGGL(auc_vals, dim3(grid), dim3(256), 0, st, lab_out, v, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = hipcub::DeviceReduce::Sum(temp, tb, v, tot, N, st)) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = hipcub::DeviceReduce::ReduceByKey(temp, tb, keys_out, keys_in, v, agg, nruns, hipcub::Sum(), N, st)) != hipSuccess)
    return (int)e;
  hipLaunchKernelGGL(auc_negs, dim3(grid), dim3(256), 0, st, agg, v, nruns, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = hipcub::DeviceScan::ExclusiveSum(temp, tb, v, below, N, st)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(auc_terms, dim3(grid), dim3(256), 0, st, agg, below, v, nruns, N);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  tb = w.temp_bytes;
  if ((e = hipcub::DeviceReduce::Sum(temp, tb, v, n2, N, st)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(auc_final, dim3(1), dim3(64), 0, st, n2, tot, auc_out);
  e = hipGetLastError();
  return e == hipSuccess ? MINER_OK : (int)e;
}

}  // extern "C"
