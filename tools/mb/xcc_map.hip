// Which XCD does workgroup b of a 256 x 512-thread, 160 KiB-LDS grid (the ranker's launch shape)
// land on? Prints, per b % 8, the XCC ids seen (speed-only placement check for rk_fused's split).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(512) void who(int* out) {
  extern __shared__ char smem[];
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = (int)(x & 0xf);
  smem[threadIdx.x] = 0;
}

int main() {
  int* d;
  const int G = 256, lds = 150 * 1024;
  hipMalloc(&d, G * sizeof(int));
  hipFuncSetAttribute((const void*)who, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(who, dim3(G), dim3(512), lds, 0, d);
    int h[G];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int cnt[8][8] = {};
    for (int b = 0; b < G; ++b) cnt[b & 7][h[b] & 7]++;
    printf("rep %d:", rep);
    for (int r = 0; r < 8; ++r) {
      printf(" b%%8=%d:", r);
      for (int x = 0; x < 8; ++x) if (cnt[r][x]) printf("x%d*%d", x, cnt[r][x]);
    }
    printf("\n");
  }
  return 0;
}
