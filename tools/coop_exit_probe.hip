// Diagnostic: does a process that made one cooperative launch exit cleanly under rocprofv3?
// Build: hipcc --offload-arch=gfx950 -O2 tools/coop_exit_probe.hip -o tools/coop_exit_probe
// Run:   rocprofv3 --kernel-trace --stats -d <dir> -o run -- tools/coop_exit_probe [0|1]   (1 = cooperative)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void probe_kernel(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = blockIdx.x;
}

int main(int argc, char** argv) {
  const bool coop = argc > 1 && atoi(argv[1]) != 0;
  int* d = nullptr;
  if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 2;
  void* args[] = {&d};
  hipError_t e = coop ? hipLaunchCooperativeKernel(reinterpret_cast<const void*>(probe_kernel), dim3(256), dim3(256), args, 0, nullptr)
                      : hipLaunchKernel(reinterpret_cast<const void*>(probe_kernel), dim3(256), dim3(256), args, 0, nullptr);
  if (e != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(e)); return 3; }
  if (hipDeviceSynchronize() != hipSuccess) return 4;
  int h[256];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 5;
  (void)hipFree(d);
  printf("coop_exit_probe coop=%d ok=%d\n", (int)coop, h[255] == 255);
  return 0;
}
