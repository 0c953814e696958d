// Which in-kernel clocks tick on this device (diagnostic): s_memrealtime / s_memtime read twice
// around a short spin, from one lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long* o) {
  if (threadIdx.x) return;
  unsigned long long a = __builtin_amdgcn_s_memrealtime();
  unsigned long long b = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1000; ++i) __builtin_amdgcn_s_sleep(10);
  unsigned long long c = __builtin_amdgcn_s_memrealtime();
  unsigned long long d = __builtin_amdgcn_s_memtime();
  o[0] = a; o[1] = b; o[2] = c; o[3] = d; o[4] = clock64(); o[5] = wall_clock64();
}
int main() {
  unsigned long long* d; unsigned long long h[6];
  hipMalloc(&d, 64);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 48, hipMemcpyDeviceToHost);
  printf("realtime %llu -> %llu (d %llu)\nmemtime %llu -> %llu (d %llu)\nclock64 %llu wall_clock64 %llu\n", h[0], h[2], h[2]-h[0], h[1], h[3], h[3]-h[1], h[4], h[5]);
  int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
  printf("wall clock rate %d kHz\n", rate);
  return 0;
}
