// Random-row gather bandwidth by access pattern (the news kernels' row DMAs), one 512-thread
// workgroup per CU, persistent over "impressions" of R = 92 random rows of 3 KiB (a 640 MB table:
// the two fp16-pair planes of config 3).  Each step moves 24 KiB per CU (24 LDS-DMA wave-
// instructions of 1 KiB), then vmcnt(0) + barrier, like one chunk interval of news_score_x2:
//   piece   step c of an impression: the 256-byte piece c of every row (4 rows per instruction)
//   rows    the same bytes as whole rows: step c moves rows 8c .. 8c + 7 entirely (3 instr/row)
//   piece+pf  piece, plus whole-row prefetches of the NEXT impression's rows into a junk LDS area
//             (3 more instructions per wave per step)
//   piece2  piece with two steps in flight (step c + 2 issued at step c into a 3-slot ring, then
//           vmcnt(issued this step): the wait covers step c + 1 only)
//   +work   the same with ~WORK dependent VALU cycles per wave per step (a compute interval)
//   hipcc --offload-arch=gfx950 -O3 tools/mb/gather_pattern.hip -o tools/mb/gather_pattern && tools/mb/gather_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int R = 92, NCH = 12, ROWB = 3072;

__device__ __forceinline__ unsigned lds_off(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void dma16(const void* g, unsigned lds) {
  unsigned t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(t) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}

__device__ __forceinline__ float work(float x, int n) {
  for (int k = 0; k < n; ++k) x = __builtin_fmaf(x, 0.999f, 0.001f);
  return x;
}

// two steps in flight: global step g = i * NCH + c of this workgroup's impression sequence
__device__ __forceinline__ int issue_piece(const char* tab, const int* ids, int n_imp, int i0, int g, char* sm, int wave, int lane) {
  const int i = i0 + (g / NCH) * (int)gridDim.x, c = g % NCH;
  if (i >= n_imp) return 0;
  const int* id = ids + (size_t)i * R;
  char* slot = sm + (g % 3) * 24 * 1024;
  int n = 0;
  for (int b = wave; b < R / 4; b += 8, ++n) {
    const int row = 4 * b + (lane >> 4);
    dma16(tab + (size_t)id[row] * ROWB + c * 256 + (lane & 15) * 16, lds_off(slot + b * 1024));
  }
  return n;
}

template <int MODE, int WORK>
__global__ __launch_bounds__(512) void gather2(const char* __restrict__ tab, const int* __restrict__ ids, int n_imp, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n_mine = (n_imp - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  float x = (float)lane;
  if (MODE == 3) {
    issue_piece(tab, ids, n_imp, blockIdx.x, 0, sm, wave, lane);
    issue_piece(tab, ids, n_imp, blockIdx.x, 1, sm, wave, lane);
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");     // step 0 (<= 3 DMAs of step 1 may remain)
    __syncthreads();
    for (int g = 0; g < n_mine * NCH; ++g) {
      const int n = issue_piece(tab, ids, n_imp, blockIdx.x, g + 2, sm, wave, lane);
      if (WORK) x = work(x + sm[(g % 3) * 24 * 1024 + lane * 4], WORK);
      if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    for (int g = 0; g < n_mine * NCH; ++g) {
      if (g == 0 && MODE != 9) {
        issue_piece(tab, ids, n_imp, blockIdx.x, 0, sm, wave, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      if (MODE != 9) issue_piece(tab, ids, n_imp, blockIdx.x, g + 1, sm, wave, lane);
      if (WORK) x = work(x + sm[(g % 3) * 24 * 1024 + lane * 4], WORK);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if (x == 1234.5f) sink[0] = x;
}

template <int MODE>
__global__ __launch_bounds__(512) void gather(const char* __restrict__ tab, const int* __restrict__ ids, int n_imp) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = blockIdx.x; i < n_imp; i += gridDim.x) {
    const int* id = ids + (size_t)i * R;
    const int* idn = ids + (size_t)min(i + (int)gridDim.x, n_imp - 1) * R;
    for (int c = 0; c < NCH; ++c) {
      char* slot = sm + (c & 1) * 48 * 1024;
      if (MODE == 0 || MODE == 2) {
        // 23 blocks of 4 rows: block b -> rows 4b .. 4b + 3, piece c
        for (int b = wave; b < R / 4; b += 8) {
          const int row = 4 * b + (lane >> 4);
          const char* g = tab + (size_t)id[row] * ROWB + c * 256 + (lane & 15) * 16;
          dma16(g, lds_off(slot + b * 1024));
        }
      }
      if (MODE == 1) {
        // rows 8c' .. : 92 rows over 12 steps (8 rows a step, the last steps 7 or 8), 3 KiB each
        const int r0 = (c * R) / NCH, r1 = ((c + 1) * R) / NCH;
        for (int k = wave; k < 3 * (r1 - r0); k += 8) {
          const int row = r0 + k / 3, part = k % 3;
          const char* g = tab + (size_t)id[row] * ROWB + part * 1024 + lane * 16;
          dma16(g, lds_off(slot + (k % 24) * 1024));
        }
      }
      if (MODE == 2) {
        const int r0 = (c * R) / NCH, r1 = ((c + 1) * R) / NCH;
        for (int k = wave; k < 3 * (r1 - r0); k += 8) {
          const int row = r0 + k / 3, part = k % 3;
          const char* g = tab + (size_t)idn[row] * ROWB + part * 1024 + lane * 16;
          dma16(g, lds_off(sm + 96 * 1024 + wave * 1024));
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
}

int main() {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t n_rows = 208000;
  const int n_imp = 400000;
  char* tab;
  int* ids;
  hipMalloc(&tab, n_rows * ROWB);
  hipMemset(tab, 1, n_rows * ROWB);
  std::vector<int> h((size_t)n_imp * R);
  srand(7);
  for (auto& x : h) x = (int)(((unsigned)rand() * 2654435761u) % n_rows);
  hipMalloc(&ids, h.size() * 4);
  hipMemcpy(ids, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)gather<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 104 * 1024);
  hipFuncSetAttribute((const void*)gather<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 104 * 1024);
  hipFuncSetAttribute((const void*)gather<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 104 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float* sink;
  hipMalloc(&sink, 64);
  const double bytes = (double)n_imp * R * ROWB;
  auto t2 = [&](const char* nm, auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 104 * 1024);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(kern, dim3(cus), dim3(512), 104 * 1024, 0, tab, ids, n_imp, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      printf("%-16s %8.3f ms  %7.1f GB/s  (%.2f us per step)\n", nm, ms, bytes / ms / 1e6,
             ms * 1e3 / ((double)n_imp / cus * NCH));
    }
  };
  t2("piece1", gather2<0, 0>);
  t2("piece2", gather2<3, 0>);
  t2("piece1+work500", gather2<0, 500>);
  t2("piece2+work500", gather2<3, 500>);
  t2("piece1+work1000", gather2<0, 1000>);
  t2("piece2+work1000", gather2<3, 1000>);
  t2("work500 only", gather2<9, 500>);
  t2("work1000 only", gather2<9, 1000>);
  const char* names[3] = {"piece", "rows", "piece+pf"};
  for (int rep = 0; rep < 1; ++rep) {
    for (int m = 0; m < 3; ++m) {
      hipEventRecord(a);
      if (m == 0) hipLaunchKernelGGL(gather<0>, dim3(cus), dim3(512), 104 * 1024, 0, tab, ids, n_imp);
      if (m == 1) hipLaunchKernelGGL(gather<1>, dim3(cus), dim3(512), 104 * 1024, 0, tab, ids, n_imp);
      if (m == 2) hipLaunchKernelGGL(gather<2>, dim3(cus), dim3(512), 104 * 1024, 0, tab, ids, n_imp);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      const double bytes = (double)n_imp * R * ROWB;
      printf("%-9s %8.3f ms  %7.1f GB/s (row bytes moved once; piece+pf moves them twice)\n", names[m], ms, bytes / ms / 1e6);
    }
  }
  return 0;
}
