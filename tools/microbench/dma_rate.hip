// LDS-DMA (global_load_lds_dwordx4) issue / completion rate vs plain 16 B/lane loads, per CU.
// One 512-thread workgroup per CU; each wave moves NBLK 1 KiB blocks of distinct HBM lines.
//   hipcc --offload-arch=gfx950 -O3 dma_rate.hip -o dma_rate && ./dma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned lds_off(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void dma16(const void* g, unsigned lds) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(g), "s"(lds) : "memory");
}

template <int MODE, int NBLK>
__global__ __launch_bounds__(512) void k(const char* src, unsigned long long* out, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* base = src + ((size_t)blockIdx.x * 8 + wave) * NBLK * 1024;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < NBLK; ++i)
      dma16(base + i * 1024 + lane * 16, __builtin_amdgcn_readfirstlane(lds_off(sm + (wave * NBLK + i) * 1024 % (150 * 1024))));
  } else {
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 v[NBLK];
#pragma unroll
    for (int i = 0; i < NBLK; ++i) v[i] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(base + i * 1024) + lane);
    const unsigned long long ti = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[(blockIdx.x * 8 + wave) * 2] = ti - t0;
#pragma unroll
    for (int i = 0; i < NBLK; ++i) acc += v[i].x + v[i].w;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
  if (MODE == 0 && lane == 0) out[(blockIdx.x * 8 + wave) * 2] = t1 - t0;
  if (lane == 0) out[(blockIdx.x * 8 + wave) * 2 + 1] = t2 - t0;
  if (acc == 12345.f) sink[0] = acc + sm[lane];
}

template <int MODE, int NBLK>
void run(const char* src, unsigned long long* dout, float* sink, int cus, const char* name) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((k<MODE, NBLK>), dim3(cus), dim3(512), 150 * 1024, 0, src, dout, sink);
  }
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(cus * 16);
  hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost);
  double iss = 0, done = 0;
  for (int i = 0; i < cus * 8; ++i) { iss += h[2 * i]; done += h[2 * i + 1]; }
  iss /= cus * 8; done /= cus * 8;
  printf("%-28s NBLK=%3d per wave: issue %8.0f cyc, complete %8.0f cyc; CU moves %6.1f KB -> %6.1f B/clk/CU\n",
         name, NBLK, iss, done, NBLK * 8.0, NBLK * 8 * 1024.0 / done);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipFuncSetAttribute((const void*)k<0, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  hipFuncSetAttribute((const void*)k<0, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  hipFuncSetAttribute((const void*)k<1, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  hipFuncSetAttribute((const void*)k<1, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  const size_t bytes = (size_t)cus * 8 * 16 * 1024;
  char* src; unsigned long long* dout; float* sink;
  hipMalloc(&src, bytes); hipMalloc(&dout, cus * 16 * 8); hipMalloc(&sink, 64);
  hipMemset(src, 1, bytes);
  run<0, 8>(src, dout, sink, cus, "LDS-DMA, all CUs");
  run<0, 16>(src, dout, sink, cus, "LDS-DMA, all CUs");
  run<1, 8>(src, dout, sink, cus, "load->VGPR, all CUs");
  run<1, 16>(src, dout, sink, cus, "load->VGPR, all CUs");
  run<0, 16>(src, dout, sink, 8, "LDS-DMA, 8 CUs");
  run<1, 16>(src, dout, sink, 8, "load->VGPR, 8 CUs");
  return 0;
}
