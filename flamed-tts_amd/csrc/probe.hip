// Diagnostic probes (no reference counterpart): per-launch device time of GEMM tile variants and of
// an empty kernel, measured as graph replays of `reps` back-to-back launches (what a captured Euler
// step sees), to separate the fixed per-node cost from the K-chain and epilogue costs.
#include "flamed_hip.h"
#include "gemm.hpp"
#include "gemm_dma.hpp"

namespace fl {

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *p = 0;
}

template <int BM, int BN, int NS>
static int probe_launch(const bf16* A, const bf16* W, bf16* C, int M, int N, int K, hipStream_t st) {
  return launch_gemm_cfg<BM, BN, NS, bf16>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
}

static int probe_variant(int v, const bf16* A, const bf16* W, bf16* C, int M, int N, int K, hipStream_t st) {
  switch (v) {
    case 0: return probe_launch<32, 64, 3>(A, W, C, M, N, K, st);
    case 1: return probe_launch<64, 64, 3>(A, W, C, M, N, K, st);
    case 2: return probe_launch<32, 64, 2>(A, W, C, M, N, K, st);
    case 3: return probe_launch<128, 128, 3>(A, W, C, M, N, K, st);
    case 4: return probe_launch<64, 128, 3>(A, W, C, M, N, K, st);
    case 5: return probe_launch<128, 64, 3>(A, W, C, M, N, K, st);
    case 6: return probe_launch<32, 64, 5>(A, W, C, M, N, K, st);
    case 7: return probe_launch<32, 64, 7>(A, W, C, M, N, K, st);
    case 8: return probe_launch<64, 64, 5>(A, W, C, M, N, K, st);
    case 9: return probe_launch<32, 32, 3>(A, W, C, M, N, K, st);
    case 10: return launch_gemm_dma<32, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 11: return launch_gemm_dma<32, 32>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 12: return launch_gemm_dma_fixed<128, 128, 3, true>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 13: return launch_gemm_dma_fixed<128, 128, 2, true>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 14: return launch_gemm_dma_fixed<256, 128, 3, true>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 15: return launch_gemm_dma_fixed<256, 128, 2, true>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 16: return launch_gemm_dma_fixed<128, 128, 3, false>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 17: return launch_gemm_dma_fixed<256, 128, 4, true>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 18: return launch_gemm_dma_fixed<128, 128, 4, true, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 32>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 19: return launch_gemm_dma_fixed<128, 128, 3, true, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 32>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 21: return launch_gemm_dma_fixed<128, 128, 2, true, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 32>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 20: return launch_gemm_dma_fixed<256, 128, 4, true, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 32>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    default: set_error("probe: unknown variant %d", v); return kBadArg;
  }
}

template <class F>
static int time_graph(F body, int reps, hipStream_t st, float* us_out) {
  hipStream_t cap;
  FL_HIP(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  FL_HIP(hipStreamBeginCapture(cap, hipStreamCaptureModeRelaxed));
  int rc = kOk;
  for (int i = 0; i < reps && rc == kOk; ++i) rc = body(cap);
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(cap, &g);
  (void)hipStreamDestroy(cap);
  if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
  FL_HIP(e);
  hipGraphExec_t ex;
  FL_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  (void)hipGraphDestroy(g);
  hipEvent_t a, b;
  FL_HIP(hipEventCreate(&a));
  FL_HIP(hipEventCreate(&b));
  FL_HIP(hipGraphLaunch(ex, st));  // warm
  FL_HIP(hipEventRecord(a, st));
  constexpr int kReplays = 5;
  for (int i = 0; i < kReplays; ++i) FL_HIP(hipGraphLaunch(ex, st));
  FL_HIP(hipEventRecord(b, st));
  FL_HIP(hipEventSynchronize(b));
  float ms = 0.f;
  FL_HIP(hipEventElapsedTime(&ms, a, b));
  *us_out = ms * 1e3f / (float)(kReplays * reps);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipGraphExecDestroy(ex);
  return kOk;
}


// Per-CU ingest probe: each block streams `kb` KB of its own slice of `src` into LDS (mode 1: LDS-DMA,
// 16 KB per K-step, 7 steps in flight) or registers (mode 0: 8 x 16-B loads in flight per thread), and
// writes one word so nothing is dead code.
__global__ __launch_bounds__(256) void stream_probe_kernel(const char* __restrict__ src, int kb, int mode, float* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const char* base = src + (size_t)blockIdx.x * kb * 1024;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int steps = kb / 16;
  float acc = 0.f;
  if (mode == 1) {
    constexpr int NS = 8;
    auto issue = [&](int s) {
      char* st = smem + (s % NS) * 16384;
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(base + (size_t)s * 16384 + (wave * 4 + j) * 1024 + lane * 16, st + (wave * 4 + j) * 1024);
    };
    for (int s = 0; s < NS - 1 && s < steps; ++s) issue(s);
    for (int s = 0; s < steps; ++s) {
      const int ahead = (steps - 1 - s) < (NS - 2) ? (steps - 1 - s) : (NS - 2);
      wait_vm<4, NS - 2>(ahead);
      lds_barrier();
      if (s + NS - 1 < steps) issue(s + NS - 1);
      acc += reinterpret_cast<const float*>(smem + (s % NS) * 16384)[tid];
    }
  } else {
    const u32x4* p = reinterpret_cast<const u32x4*>(base);
    const int n = kb * 1024 / 16;
    for (int i = tid; i < n; i += 256 * 8) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (i + j * 256 < n) ? p[i + j * 256] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += __uint_as_float(v[j].x);
    }
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;
}
}  // namespace fl

using namespace fl;

extern "C" {

FLAMED_API int flamed_probe_gemm(int variant, int M, int N, int K, int reps, int wbufs, const void* A, const void* W,
                                 void* C, float* us_out, hipStream_t st) {
  FL_REQUIRE(A && W && C && us_out && reps > 0 && wbufs > 0 && M > 0 && N > 0 && K > 0, "flamed_probe_gemm: bad args");
  int i = 0;
  auto body = [&](hipStream_t s) {  // launch i reads weight buffer i % wbufs (cold-ish weights when wbufs is large)
    const bf16* w = (const bf16*)W + (size_t)(i++ % wbufs) * N * K;
    return probe_variant(variant, (const bf16*)A, w, (bf16*)C, M, N, K, s);
  };
  return time_graph(body, reps, st, us_out);
}

FLAMED_API int flamed_probe_empty(int blocks, int reps, float* us_out, hipStream_t st) {
  FL_REQUIRE(us_out && reps > 0 && blocks > 0, "flamed_probe_empty: bad args");
  auto body = [&](hipStream_t s) -> int {
    hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, s, nullptr);
    FL_LAUNCH_CHECK();
    return kOk;
  };
  return time_graph(body, reps, st, us_out);
}


FLAMED_API int flamed_probe_stream(int blocks, int kb, int mode, int reps, const void* src, float* us_out, hipStream_t st) {
  FL_REQUIRE(src && us_out && blocks > 0 && kb > 0 && kb % 16 == 0 && reps > 0, "flamed_probe_stream: bad args");
  auto body = [&](hipStream_t s) -> int {
    hipLaunchKernelGGL(stream_probe_kernel, dim3(blocks), dim3(256), mode == 1 ? 8 * 16384 : 0, s, (const char*)src, kb, mode, nullptr);
    FL_LAUNCH_CHECK();
    return kOk;
  };
  FL_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(stream_probe_kernel), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  return time_graph(body, reps, st, us_out);
}
}  // extern "C"
