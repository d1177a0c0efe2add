// MFMA issue rate on one SIMD: v_mfma_f32_16x16x16_bf16 vs _16x16x32_bf16 vs _16x16x4_f32,
// one wave per SIMD, 4 independent accumulators, cycles per MFMA from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int KIND>
__global__ void k(float* out, unsigned long long* cyc, int iters) {
  f32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  bf16x4 x4; bf16x8 x8;
  for (int i = 0; i < 4; ++i) x4[i] = (__bf16)(threadIdx.x * 0.001f + i);
  for (int i = 0; i < 8; ++i) x8[i] = (__bf16)(threadIdx.x * 0.001f + i);
  float f = threadIdx.x * 0.01f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (KIND == 0) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a2, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a3, 0, 0, 0);
      } else if constexpr (KIND == 1) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a2, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a3, 0, 0, 0);
      } else {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(f, f, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(f, f, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(f, f, a2, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_16x16x4f32(f, f, a3, 0, 0, 0);
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  f32x4 s = a0 + a1 + a2 + a3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  float* out; unsigned long long* cyc;
  hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 8);
  const char* names[3] = {"16x16x16_bf16", "16x16x32_bf16", "16x16x4_f32"};
  for (int kind = 0; kind < 3; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      const int iters = 1000;
      if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      hipDeviceSynchronize();
      unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%s: %.2f memtime ticks per MFMA\n", names[kind], (double)c / (iters * 32.0));
    }
  }
  return 0;
}
