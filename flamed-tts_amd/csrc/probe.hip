// Diagnostic probes (no reference counterpart): per-launch device time of GEMM tile variants and of
// an empty kernel, measured as graph replays of `reps` back-to-back launches (what a captured Euler
// step sees), to separate the fixed per-node cost from the K-chain and epilogue costs.
#include "flamed_diag.h"
#include "gemm.hpp"
#include "gemm_dma.hpp"
#include "gemm_8p.hpp"

#include <vector>

namespace fl {

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *p = 0;
}

template <int BM, int BN, int NS>
static int probe_launch(const bf16* A, const bf16* W, bf16* C, int M, int N, int K, hipStream_t st) {
  return launch_gemm_cfg<BM, BN, NS, bf16>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
}

// Wave-split-K tile (probe): NW waves share one BM x BN output tile, wave w owning K slice
// [w*K/NW, (w+1)*K/NW).  MFMA operands are loaded straight from global memory into registers (lane
// (fr, fq) of a 16x16x32 fragment reads the 16 B at row fr, k + 8 fq), every load of the slice is
// issued before the first MFMA, and the NW partial tiles are summed through LDS.  No LDS staging of
// operands and no barrier inside the K loop: the whole K chain is one memory round trip deep.
template <int BM, int BN, int NW, int KS>
__global__ __launch_bounds__(NW * 64) void gemm_wsk_probe_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                                 bf16* __restrict__ C, int M, int N, int K) {
  constexpr int FM = BM / 16, FN = BN / 16, LDR = BN + 4;
  __shared__ float red[NW * BM * LDR];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  const int bm = blockIdx.y * BM, bn = blockIdx.x * BN;
  const int k0 = w * KS * 32 + fq * 8;
  u32x4 a[KS][FM], b[KS][FN];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      int m = bm + i * 16 + fr;
      m = m < M ? m : M - 1;
      a[s][i] = *reinterpret_cast<const u32x4*>(A + (size_t)m * K + k0 + s * 32);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j)
      b[s][j] = *reinterpret_cast<const u32x4*>(W + (size_t)(bn + j * 16 + fr) * K + k0 + s * 32);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every load of the slice ahead of the first MFMA
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[s][i]),
                                                            __builtin_bit_cast(bf16x8, b[s][j]), acc[i][j], 0, 0, 0);
  float* rw = red + w * BM * LDR;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) rw[(i * 16 + fq * 4 + r) * LDR + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  for (int e = threadIdx.x; e < BM * BN / 4; e += NW * 64) {
    const int r = e / (BN / 4), c4 = (e % (BN / 4)) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const float4 p = *reinterpret_cast<const float4*>(red + q * BM * LDR + r * LDR + c4);
      v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
    }
    if (bm + r < M) store_val4<bf16>(C + (size_t)(bm + r) * N + bn + c4, v);
  }
}

template <int BM, int BN, int NW>
static int probe_wsk(const bf16* A, const bf16* W, bf16* C, int M, int N, int K, hipStream_t st) {
  FL_REQUIRE(K == 1024 && N % BN == 0, "probe wsk: K must be 1024, N %% %d", BN);
  constexpr int KS = 1024 / 32 / NW;
  hipLaunchKernelGGL((gemm_wsk_probe_kernel<BM, BN, NW, KS>), dim3(N / BN, (M + BM - 1) / BM), dim3(NW * 64), 0, st, A, W, C, M, N, K);
  FL_LAUNCH_CHECK();
  return kOk;
}

// Split-K over workgroups with the register-staged template (slab hand-off, last arriver reduces):
// a bigger tile cuts the total operand bytes pulled into the CUs, the split spreads them over more CUs.
template <int BM, int BN, int SPLIT>
static int probe_split(const bf16* A, const bf16* W, bf16* C, int M, int N, int K, hipStream_t st) {
  static float* slab = nullptr;
  static int* cnt = nullptr;
  constexpr size_t kSlab = (size_t)16 << 20, kCnt = 1 << 16;
  if (!slab) {
    FL_HIP(hipMalloc(&slab, kSlab * 4));
    FL_HIP(hipMalloc(&cnt, kCnt * 4));
    FL_HIP(hipMemset(cnt, 0, kCnt * 4));
    FL_HIP(hipDeviceSynchronize());
  }
  SplitCtx c;
  c.slab = slab; c.slab_floats = kSlab; c.cnt = cnt; c.cnt_n = (int)kCnt;
  c.target = 1 << 30; c.max_split = SPLIT;
  SplitScope scope(&c);
  return launch_gemm_cfg<BM, BN, 3, bf16>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
}

static int probe_variant(int v, const bf16* A, const bf16* W, bf16* C, int M, int N, int K, hipStream_t st) {
  switch (v) {
    case 36: return launch_gemm_dma<64, 32>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 37: return launch_gemm_dma_fixed<32, 32, 4, false, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 40: return launch_gemm_dma_fixed<32, 32, 8, true, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 41: return launch_gemm_dma_fixed<64, 32, 4, false, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 42: return launch_gemm_dma_fixed<32, 32, 2, false, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 43: return launch_gemm_dma_fixed<32, 32, 8, 2, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 44: return launch_gemm_dma_fixed<32, 32, 4, 2, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 45: return launch_gemm_dma_fixed<32, 64, 4, 2, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 46: return launch_gemm_dma_fixed<32, 64, 4, 0, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 47: return launch_gemm_dma_fixed<32, 32, 3, 0, LoadPlain<bf16>, EpiBiasAct<bf16, 0>, 64>(LoadPlain<bf16>{A, K}, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
    case 30: return probe_split<64, 64, 2>(A, W, C, M, N, K, st);
    case 31: return probe_split<64, 64, 4>(A, W, C, M, N, K, st);
    case 32: return probe_split<128, 64, 2>(A, W, C, M, N, K, st);
    case 33: return probe_split<128, 64, 4>(A, W, C, M, N, K, st);
    case 34: return probe_split<32, 64, 2>(A, W, C, M, N, K, st);
    case 35: return probe_split<32, 64, 4>(A, W, C, M, N, K, st);
    case 22: return probe_wsk<32, 32, 4>(A, W, C, M, N, K, st);
    case 23: return probe_wsk<32, 32, 8>(A, W, C, M, N, K, st);
    case 24: return probe_wsk<32, 64, 8>(A, W, C, M, N, K, st);
    case 25: return probe_wsk<64, 32, 8>(A, W, C, M, N, K, st);
    case 26: return probe_wsk<64, 64, 8>(A, W, C, M, N, K, st);
    case 27: return probe_wsk<16, 64, 8>(A, W, C, M, N, K, st);
    case 28: return probe_wsk<32, 32, 16>(A, W, C, M, N, K, st);
    case 29: return probe_wsk<16, 32, 8>(A, W, C, M, N, K, st);
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
    case 50: return launch_gemm8p(A, K, W, K, EpiBiasAct<bf16, 0>{nullptr, C, N}, M, N, K, st);
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
// L2 warm-up of the NEXT GEMM's weights (probe): `gridDim.x` workgroups, those of XCD x (dispatch id
// mod 8) together read all `bytes` of w, so every XCD's L2 ends up holding the whole matrix.
__global__ __launch_bounds__(256) void l2_prefetch_kernel(const char* __restrict__ w, size_t bytes, float* sink) {
  const int per = gridDim.x >> 3, j = blockIdx.x >> 3;
  const size_t slice = (bytes / per + 4095) & ~(size_t)4095;
  const size_t b0 = (size_t)j * slice, b1 = b0 + slice < bytes ? b0 + slice : bytes;
  float acc = 0.f;
  for (size_t o = b0 + (size_t)threadIdx.x * 16; o < b1; o += 256 * 16 * 4) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t q = o + (size_t)u * 256 * 16;
      v[u] = q < b1 ? *reinterpret_cast<const u32x4*>(w + q) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += __uint_as_float(v[u].x);
  }
  if (acc == 12345.678f && sink) sink[blockIdx.x] = acc;
}
}  // namespace fl

using namespace fl;

typedef float f32x4v __attribute__((ext_vector_type(4)));
// STREAM-style copy for the measured HBM peak (bench.py measured_peaks): each thread moves 4 float4 per grid-stride
// iteration (mode 1: non-temporal loads and stores, 0: plain), the 4 loads in flight before the 4 stores.
template <bool NT>
__global__ __launch_bounds__(256) void copy_probe_kernel(const f32x4v* __restrict__ src, f32x4v* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * 1024;
  for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
    f32x4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t j = i + (size_t)k * 256;
      if (j < n) v[k] = NT ? __builtin_nontemporal_load(src + j) : src[j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t j = i + (size_t)k * 256;
      if (j < n) {
        if (NT) __builtin_nontemporal_store(v[k], dst + j);
        else dst[j] = v[k];
      }
    }
  }
}

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

// GEMM chain with a concurrent L2 warm-up of the next launch's weights on a second captured stream
// (pf_blocks workgroups; 0 = no warm-up, same graph shape otherwise).
FLAMED_API int flamed_probe_gemm_pf(int variant, int M, int N, int K, int reps, int wbufs, int pf_blocks, const void* A,
                                    const void* W, void* C, float* us_out, hipStream_t st) {
  FL_REQUIRE(A && W && C && us_out && reps > 1 && wbufs > 0 && pf_blocks >= 0 && pf_blocks % 8 == 0, "flamed_probe_gemm_pf: bad args");
  hipStream_t s1;
  FL_HIP(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  std::vector<hipEvent_t> evs;
  auto mk = [&]() { hipEvent_t e; (void)hipEventCreateWithFlags(&e, hipEventDisableTiming); evs.push_back(e); return e; };
  std::vector<hipEvent_t> done(reps, nullptr);
  int i = 0;
  const size_t wbytes = (size_t)N * K * 2;
  auto body = [&](hipStream_t cap) -> int {
    const int k = i++;
    if (pf_blocks && k + 1 < reps) {  // warm W[k+1] while GEMM k runs (starts when GEMM k-1 has finished)
      hipEvent_t e0 = mk();
      FL_HIP(hipEventRecord(e0, cap));
      FL_HIP(hipStreamWaitEvent(s1, e0, 0));
      const char* wn = (const char*)W + (size_t)((k + 1) % wbufs) * wbytes;
      hipLaunchKernelGGL(l2_prefetch_kernel, dim3(pf_blocks), dim3(256), 0, s1, wn, wbytes, nullptr);
      FL_LAUNCH_CHECK();
      done[k + 1] = mk();
      FL_HIP(hipEventRecord(done[k + 1], s1));
    }
    if (done[k]) FL_HIP(hipStreamWaitEvent(cap, done[k], 0));
    const bf16* w = (const bf16*)W + (size_t)(k % wbufs) * N * K;
    return probe_variant(variant, (const bf16*)A, w, (bf16*)C, M, N, K, cap);
  };
  const int rc = time_graph(body, reps, st, us_out);
  for (hipEvent_t e : evs) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(s1);
  return rc;
}

// One v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) on a 16 x 128 A, 16 x 128 B (row n = output
// column), e8m0 scales sa / sb [16][4]: lane l holds row l % 16 and the 32 bytes of "lane group" l / 16;
// mode 0: bytes [32 g, 32 g + 32) of the row, mode 1: chunks g and 4 + g (K [16 g, 16 g + 16) and
// [64 + 16 g, ...)); the lane passes the scale byte sa[row][g].  C[16][16] (row m, column n).
__global__ void mx_probe_kernel(const unsigned char* A, const unsigned char* B, const unsigned char* sa,
                                const unsigned char* sb, float* C, int mode) {
  typedef int i32x8 __attribute__((ext_vector_type(8)));
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  const int c0 = mode == 0 ? 2 * g : g, c1 = mode == 0 ? 2 * g + 1 : 4 + g;
  const u32x4 a0 = *reinterpret_cast<const u32x4*>(A + r * 128 + c0 * 16), a1 = *reinterpret_cast<const u32x4*>(A + r * 128 + c1 * 16);
  const u32x4 b0 = *reinterpret_cast<const u32x4*>(B + r * 128 + c0 * 16), b1 = *reinterpret_cast<const u32x4*>(B + r * 128 + c1 * 16);
  const i32x8 av = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
  const i32x8 bv = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
  const int sca = sa[r * 4 + g], scb = sb[r * 4 + g];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sca, 0, scb);
#pragma unroll
  for (int e = 0; e < 4; ++e) C[(g * 4 + e) * 16 + r] = acc[e];
}

FLAMED_API int flamed_probe_mx(const void* A, const void* B, const void* sa, const void* sb, float* C, int mode, hipStream_t st) {
  FL_REQUIRE(A && B && sa && sb && C, "flamed_probe_mx: null args");
  hipLaunchKernelGGL(mx_probe_kernel, dim3(1), dim3(64), 0, st, (const unsigned char*)A, (const unsigned char*)B,
                     (const unsigned char*)sa, (const unsigned char*)sb, C, mode);
  FL_LAUNCH_CHECK();
  return kOk;
}

// fp32 rows -> MX-fp8 A operand through the product's producer path (store_f8x8).
__global__ void quant_a_f8_probe_kernel(const float* A, int M, int K, unsigned char* dst, unsigned char* sc) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int K8 = K / 8;
  if (i >= (size_t)M * K8) return;
  const int m = i / K8, k = (int)(i - (size_t)m * K8) * 8;
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = A[(size_t)m * K + k + j];
  store_f8x8(o, dst, sc, m, k, K);
}

FLAMED_API int flamed_probe_mx_gemm(const float* A, const float* W, int M, int N, int K, float* C, hipStream_t st) {
  FL_REQUIRE(A && W && C && M > 0 && N % 256 == 0 && K % 512 == 0 && K <= kMxMaxK, "flamed_probe_mx_gemm: bad args");
  const size_t a8 = (size_t)M * K, as = mx_scale_bytes(M, K), w8 = (size_t)N * K, wsb = mx_scale_bytes(N, K);
  unsigned char* buf = nullptr;
  FL_HIP(hipMalloc(&buf, a8 + as + w8 + wsb));
  unsigned char *A8 = buf, *AS = buf + a8, *W8 = AS + as, *WS = W8 + w8;
  FL_HIP(hipMemsetAsync(AS, 0, as, st));  // padded rows: unused scales stay finite
  const size_t na = (size_t)M * (K / 8);
  hipLaunchKernelGGL(quant_a_f8_probe_kernel, dim3((na + 255) / 256), dim3(256), 0, st, A, M, K, A8, AS);
  const int nb = N * (K / 32);
  hipLaunchKernelGGL(quant_w_f8_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, W, N, K, W8, WS);
  int rc = launch_gemm8p_f8(A8, AS, K, W8, WS, K, EpiBiasAct<float, 0>{nullptr, C, N}, M, N, K, st);
  (void)hipStreamSynchronize(st);
  (void)hipFree(buf);
  return rc;
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


FLAMED_API int flamed_probe_copy(const void* src, void* dst, size_t bytes, int blocks, int mode, int reps, float* us_out,
                                 hipStream_t st) {
  FL_REQUIRE(src && dst && us_out && bytes % 16 == 0 && blocks > 0 && reps > 0, "flamed_probe_copy: bad args");
  const size_t n = bytes / 16;
  auto body = [&](hipStream_t s) -> int {
    if (mode == 1)
      hipLaunchKernelGGL(copy_probe_kernel<true>, dim3(blocks), dim3(256), 0, s, (const f32x4v*)src, (f32x4v*)dst, n);
    else
      hipLaunchKernelGGL(copy_probe_kernel<false>, dim3(blocks), dim3(256), 0, s, (const f32x4v*)src, (f32x4v*)dst, n);
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
  FL_HIP(set_max_lds(reinterpret_cast<const void*>(stream_probe_kernel)));
  return time_graph(body, reps, st, us_out);
}
}  // extern "C"
