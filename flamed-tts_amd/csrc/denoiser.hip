// SimpleMLPAdaLN denoiser + Euler ODE loop on gfx950 (reference: flamed/models/synthesizer/
// prob_generator.py:7-164 (modulate, TimestepEmbedder, ConvNeXtBlock, ResBlock), :208-365
// (FinalLayer, SimpleMLPAdaLN), :434-447 (ProbGenerator.sample Euler loop)).
//
// Per Euler step (M = B*T frame rows, H hidden, C latent):
//   P    proj_in GEMM  xt(f32)->X(f32) + LN partials
//   per ResBlock: K2a dwconv_gn (LN+AdaLN modulate -> depthwise k31 -> GroupNorm over T) -> G
//                 G1 conv_2 GEMM + GELU -> U;  G2 conv_3 GEMM, epilogue X += gate*(h + .) + partials
//                 G3 LN+modulate prologue -> mlp.0 GEMM + SiLU -> U;  G4 mlp.2 GEMM, X += gate*(.)
//   FinalLayer:   K2a, G1, G2 as above (no-affine LN), then conv_out k3 GEMM with the LN+modulate
//                 gather prologue and the Euler update xt += dt*v fused in the epilogue.
// AdaLN (depends only on t and the speaker) is precomputed for every (step, utterance) at once.
#include "flamed_hip.h"
#include "gemm.hpp"

#include <vector>

namespace fl {

// ------------------------------ denoiser loaders / epilogues ------------------------------

struct ModRef {  // AdaLN modulation vectors: row = m / div, stride `ms` floats
  const float* __restrict__ sh;
  const float* __restrict__ sc;
  int ms;
  int div;
};

template <typename DT, bool AFF>
struct LoadLNMod {
  const float* __restrict__ x;
  int ld;
  const float* __restrict__ S;
  int NT, tw;
  float eps;
  ModRef mod;
  const float* __restrict__ lnw;
  const float* __restrict__ lnb;
  static constexpr int EPC = DTraits<DT>::EPC;
  struct Raw { float v[EPC], s[EPC], h[EPC], w[AFF ? EPC : 1], b[AFF ? EPC : 1]; };
  static constexpr int stat_rows(int BM) { return BM; }
  __device__ void prologue(int bm, int BM, int M, float* st) const {
    for (int r = threadIdx.x; r < BM; r += blockDim.x) {
      int m = bm + r;
      m = m < M ? m : M - 1;
      row_stats_from_partials(S, m, NT, tw, eps, st[2 * r], st[2 * r + 1]);
    }
  }
  __device__ Raw issue(int m, int k) const {
    Raw r;
    const float* px = x + (size_t)m * ld + k;
    size_t mo = (size_t)(m / mod.div) * mod.ms + k;
#pragma unroll
    for (int j = 0; j < EPC; j += 4) {
      float4 a = ld4(px + j), s = ld4(mod.sc + mo + j), h = ld4(mod.sh + mo + j);
      r.v[j] = a.x; r.v[j + 1] = a.y; r.v[j + 2] = a.z; r.v[j + 3] = a.w;
      r.s[j] = s.x; r.s[j + 1] = s.y; r.s[j + 2] = s.z; r.s[j + 3] = s.w;
      r.h[j] = h.x; r.h[j + 1] = h.y; r.h[j + 2] = h.z; r.h[j + 3] = h.w;
      if constexpr (AFF) {
        float4 w = ld4(lnw + k + j), b = ld4(lnb + k + j);
        r.w[j] = w.x; r.w[j + 1] = w.y; r.w[j + 2] = w.z; r.w[j + 3] = w.w;
        r.b[j] = b.x; r.b[j + 1] = b.y; r.b[j + 2] = b.z; r.b[j + 3] = b.w;
      }
    }
    return r;
  }
  template <typename D>
  __device__ uint4 finish(const Raw& r, int m, int, const float* st, int bm) const {
    const float mean = st[2 * (m - bm)], rstd = st[2 * (m - bm) + 1];
    float o[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) {
      float xh = (r.v[j] - mean) * rstd;
      if constexpr (AFF) xh = xh * r.w[j] + r.b[j];
      o[j] = xh * (1.0f + r.s[j]) + r.h[j];
    }
    return pack_chunk<D>(o);
  }
};

// FinalLayer conv_out: k=3, pad=1 over T of each utterance; source rows LN(no affine)+modulated.
// K index = tap*H + c (weights re-ordered tap-major at load).
template <typename DT>
struct LoadConv3LN {
  const float* __restrict__ x;
  int H;
  const float* __restrict__ S;
  int NT, tw;
  float eps;
  ModRef mod;
  int T;
  static constexpr int EPC = DTraits<DT>::EPC;
  struct Raw { float v[EPC], s[EPC], h[EPC]; int src; };
  static constexpr int stat_rows(int BM) { return BM + 2; }
  __device__ void prologue(int bm, int BM, int M, float* st) const {
    for (int r = threadIdx.x; r < BM + 2; r += blockDim.x) {
      int m = bm - 1 + r;
      m = m < 0 ? 0 : (m < M ? m : M - 1);
      row_stats_from_partials(S, m, NT, tw, eps, st[2 * r], st[2 * r + 1]);
    }
  }
  __device__ Raw issue(int m, int k) const {
    Raw r;
    int tap = k / H, c = k - tap * H;
    int t = m % T + tap - 1;
    r.src = (t >= 0 && t < T) ? m + tap - 1 : -1;
    if (r.src >= 0) {
      const float* px = x + (size_t)r.src * H + c;
      size_t mo = (size_t)(r.src / mod.div) * mod.ms + c;
#pragma unroll
      for (int j = 0; j < EPC; j += 4) {
        float4 a = ld4(px + j), s = ld4(mod.sc + mo + j), h = ld4(mod.sh + mo + j);
        r.v[j] = a.x; r.v[j + 1] = a.y; r.v[j + 2] = a.z; r.v[j + 3] = a.w;
        r.s[j] = s.x; r.s[j + 1] = s.y; r.s[j + 2] = s.z; r.s[j + 3] = s.w;
        r.h[j] = h.x; r.h[j + 1] = h.y; r.h[j + 2] = h.z; r.h[j + 3] = h.w;
      }
    }
    return r;
  }
  template <typename D>
  __device__ uint4 finish(const Raw& r, int, int, const float* st, int bm) const {
    float o[EPC];
    if (r.src < 0) {
#pragma unroll
      for (int j = 0; j < EPC; ++j) o[j] = 0.f;
    } else {
      int i = r.src - (bm - 1);
      const float mean = st[2 * i], rstd = st[2 * i + 1];
#pragma unroll
      for (int j = 0; j < EPC; ++j) o[j] = ((r.v[j] - mean) * rstd) * (1.0f + r.s[j]) + r.h[j];
    }
    return pack_chunk<D>(o);
  }
};

// AdaLN input: A[r][k] = SiLU(TE[tidx[r]][k] + CE[sidx[r]][k])   (fp32 path)
struct LoadAdaY {
  const float* __restrict__ te;
  const float* __restrict__ ce;
  const int* __restrict__ tidx;
  const int* __restrict__ sidx;
  int H;
  struct Raw { float v[4]; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    float4 a = ld4(te + (size_t)tidx[m] * H + k), b = ld4(ce + (size_t)sidx[m] * H + k);
    return Raw{{silu(a.x + b.x), silu(a.y + b.y), silu(a.z + b.z), silu(a.w + b.w)}};
  }
  template <typename D> __device__ uint4 finish(const Raw& r, int, int, const float*, int) const { return pack_chunk<D>(r.v); }
};

// X = X + gate * (h + acc + b3), h = LN(X)(+affine) * (1 + sc) + sh recomputed from the same
// stats the dwconv_gn prologue used; emits LN partials of the new X.
template <bool AFF>
struct EpiConvNeXtResid {
  const float* __restrict__ b3;
  float* X;
  int ld;
  const float* __restrict__ Sin;
  int NTin, twin;
  float eps;
  ModRef mod;
  const float* __restrict__ gate;
  const float* __restrict__ lnw;
  const float* __restrict__ lnb;
  float* __restrict__ Sout;
  int NTout;
  static constexpr bool kRowStats = true;
  static constexpr int stat_rows(int BM) { return BM; }
  __device__ void prologue(int bm, int BM, int M, float* st) const {
    for (int r = threadIdx.x; r < BM; r += blockDim.x) {
      int m = bm + r;
      m = m < M ? m : M - 1;
      row_stats_from_partials(Sin, m, NTin, twin, eps, st[2 * r], st[2 * r + 1]);
    }
  }
  __device__ float value(int m, int n, float acc, const float* st, int bm) const {
    float x = X[(size_t)m * ld + n];
    size_t mo = (size_t)(m / mod.div) * mod.ms + n;
    float xh = (x - st[2 * (m - bm)]) * st[2 * (m - bm) + 1];
    if constexpr (AFF) xh = xh * lnw[n] + lnb[n];
    float h = xh * (1.0f + mod.sc[mo]) + mod.sh[mo];
    return x + gate[mo] * (h + (acc + b3[n]));
  }
  __device__ void store(int m, int n, float v) const { X[(size_t)m * ld + n] = v; }
  __device__ void store_stats(int m, int nt, float mean, float m2) const {
    reinterpret_cast<float2*>(Sout)[(size_t)m * NTout + nt] = make_float2(mean, m2);
  }
};

struct EpiGatedResid {  // X = X + gate * (acc + b)
  const float* __restrict__ b;
  float* X;
  int ld;
  const float* __restrict__ gate;
  int ms, div;
  float* __restrict__ Sout;
  int NTout;
  static constexpr bool kRowStats = true;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int m, int n, float acc, const float*, int) const {
    return X[(size_t)m * ld + n] + gate[(size_t)(m / div) * ms + n] * (acc + b[n]);
  }
  __device__ void store(int m, int n, float v) const { X[(size_t)m * ld + n] = v; }
  __device__ void store_stats(int m, int nt, float mean, float m2) const {
    reinterpret_cast<float2*>(Sout)[(size_t)m * NTout + nt] = make_float2(mean, m2);
  }
};

struct EpiEuler {  // xt = xt + dt * (acc + b)   (prob_generator.py:445)
  const float* __restrict__ b;
  float* xt;
  int ld;
  float dt;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int, int n, float acc, const float*, int) const { return acc + b[n]; }
  __device__ void store(int m, int n, float v) const {
    float* p = xt + (size_t)m * ld + n;
    *p = __fadd_rn(*p, __fmul_rn(dt, v));
  }
  __device__ void store_stats(int, int, float, float) const {}
};

// ------------------------------ K2a: LN+mod -> depthwise conv -> GroupNorm(T) ------------------------------
// grid (H/CG, B); one workgroup owns CG channels of one utterance for ALL T frames, so the GroupNorm
// statistics over T (prob_generator.py:89, GroupNorm(H,H)) are exact in-workgroup reductions and the
// conv output never leaves LDS.
constexpr int kDwTC = 64;  // frames per staging chunk

template <int CG, int KS>
struct DwSmem {
  static constexpr int HALO = KS / 2;
  static constexpr int RG = 256 / CG;
  static size_t bytes(int T) {
    return (size_t)T * CG * 4 + (size_t)(kDwTC + 2 * HALO) * CG * 4 + (kDwTC + 2 * HALO) * 8 + (size_t)RG * CG * 12 + CG * 8;
  }
};

template <typename DT, bool AFF, int CG, int KS>
__global__ __launch_bounds__(256) void dwconv_gn_kernel(const float* __restrict__ X, int H, const float* __restrict__ S,
                                                        int NT, int tw, float eps_ln, ModRef mod,
                                                        const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                        const float* __restrict__ dww, const float* __restrict__ dwb,
                                                        const float* __restrict__ gnw, const float* __restrict__ gnb,
                                                        float eps_gn, DT* __restrict__ G, int T) {
  using SMD = DwSmem<CG, KS>;
  constexpr int HALO = SMD::HALO, RG = SMD::RG, RPT = kDwTC / RG, SR = kDwTC + 2 * HALO;
  static_assert(kDwTC % RG == 0, "chunk/rowgroup mismatch");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* dbuf = reinterpret_cast<float*>(smem);            // T x CG
  float* hs = dbuf + (size_t)T * CG;                         // SR x CG
  float* rs = hs + SR * CG;                                  // SR x 2
  float* red = rs + SR * 2;                                  // RG x CG x 3
  float* gnp = red + RG * CG * 3;                            // CG x 2

  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * CG;
  const int b = blockIdx.y;
  const int cl = tid % CG, rg = tid / CG;
  const int c = c0 + cl;

  float w[KS];
#pragma unroll
  for (int j = 0; j < KS; ++j) w[j] = dww[(size_t)c * KS + j];
  const float bias = dwb[c];

  float n_run = 0.f, mean_run = 0.f, m2_run = 0.f;
  for (int t0 = 0; t0 < T; t0 += kDwTC) {
    for (int r = tid; r < SR; r += 256) {
      int t = t0 - HALO + r;
      if (t >= 0 && t < T) row_stats_from_partials(S, b * T + t, NT, tw, eps_ln, rs[2 * r], rs[2 * r + 1]);
    }
    __syncthreads();
    for (int idx = tid; idx < SR * CG; idx += 256) {
      int r = idx / CG, cc = idx - r * CG;
      int t = t0 - HALO + r;
      float v = 0.f;
      if (t >= 0 && t < T) {
        size_t m = (size_t)b * T + t;
        float xh = (X[m * H + c0 + cc] - rs[2 * r]) * rs[2 * r + 1];
        size_t mo = (m / mod.div) * mod.ms + c0 + cc;
        if constexpr (AFF) xh = xh * lnw[c0 + cc] + lnb[c0 + cc];
        v = xh * (1.0f + mod.sc[mo]) + mod.sh[mo];
      }
      hs[idx] = v;
    }
    __syncthreads();
    float vals[RPT];
    float cn = 0.f, cs = 0.f;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      int tl = rg * RPT + q;
      float a = bias;
#pragma unroll
      for (int j = 0; j < KS; ++j) a += w[j] * hs[(tl + j) * CG + cl];
      vals[q] = a;
      if (t0 + tl < T) {
        dbuf[(size_t)(t0 + tl) * CG + cl] = a;
        cn += 1.f;
        cs += a;
      }
    }
    if (cn > 0.f) {
      float cm = cs / cn, c2 = 0.f;
#pragma unroll
      for (int q = 0; q < RPT; ++q)
        if (t0 + rg * RPT + q < T) {
          float d = vals[q] - cm;
          c2 += d * d;
        }
      chan_combine(n_run, mean_run, m2_run, cn, cm, c2);
    }
    __syncthreads();
  }
  red[(rg * CG + cl) * 3 + 0] = n_run;
  red[(rg * CG + cl) * 3 + 1] = mean_run;
  red[(rg * CG + cl) * 3 + 2] = m2_run;
  __syncthreads();
  if (tid < CG) {
    float n = 0.f, mu = 0.f, m2 = 0.f;
    for (int g = 0; g < RG; ++g) chan_combine(n, mu, m2, red[(g * CG + tid) * 3], red[(g * CG + tid) * 3 + 1], red[(g * CG + tid) * 3 + 2]);
    gnp[2 * tid] = mu;
    gnp[2 * tid + 1] = 1.0f / sqrtf(m2 / (float)T + eps_gn);
  }
  __syncthreads();
  for (int idx = tid; idx < T * CG; idx += 256) {
    int t = idx / CG, cc = idx - t * CG;
    float g = ((dbuf[idx] - gnp[2 * cc]) * gnp[2 * cc + 1]) * gnw[c0 + cc] + gnb[c0 + cc];
    store_val<DT>(G + ((size_t)b * T + t) * H + c0 + cc, g);
  }
}

template <typename DT, bool AFF, int KS>
static int launch_dwconv_gn(const float* X, int H, const float* S, int NT, int tw, ModRef mod, const float* lnw,
                            const float* lnb, const float* dww, const float* dwb, const float* gnw, const float* gnb,
                            DT* G, int B, int T, hipStream_t st) {
  const size_t budget = 150 * 1024;
  auto go = [&](auto cgc) -> int {
    constexpr int CG = decltype(cgc)::value;
    size_t bytes = DwSmem<CG, KS>::bytes(T);
    auto kern = dwconv_gn_kernel<DT, AFF, CG, KS>;
    static bool attr = false;
    if (!attr) {
      FL_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(H / CG, B), dim3(256), bytes, st, X, H, S, NT, tw, 1e-6f, mod, lnw, lnb, dww, dwb, gnw, gnb, 1e-5f, G, T);
    FL_LAUNCH_CHECK();
    return kOk;
  };
  FL_REQUIRE(H % 32 == 0, "dwconv_gn: H=%d must be a multiple of 32", H);
  if (DwSmem<32, KS>::bytes(T) <= budget && B * (H / 32) >= 128) return go(std::integral_constant<int, 32>());
  if (DwSmem<16, KS>::bytes(T) <= budget) return go(std::integral_constant<int, 16>());
  if (DwSmem<8, KS>::bytes(T) <= budget) return go(std::integral_constant<int, 8>());
  FL_REQUIRE(false, "dwconv_gn: T=%d frames too long for the LDS-resident GroupNorm (max ~4500)", T);
}

// ------------------------------ AdaLN helpers ------------------------------

// TimestepEmbedder.timestep_embedding (prob_generator.py:49-67): F[r] = [cos(t f), sin(t f)]
__global__ void tfreq_kernel(const float* __restrict__ t, int R, int dim, float* __restrict__ F) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  int half = dim / 2;
  if (idx >= R * dim) return;
  int r = idx / dim, j = idx - r * dim;
  int jj = j < half ? j : j - half;
  const float nl = -9.210340371976184f;  // -ln(10000) as fp32
  float f = expf((nl * (float)jj) / (float)half);
  float a = t[r] * f;
  F[idx] = j < half ? cosf(a) : sinf(a);
}

__global__ void cast_kernel_bf16(const float* __restrict__ src, bf16* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (bf16)src[i];
}
__global__ void copy_kernel_f32(const float* __restrict__ src, float* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}
// conv weight (N, Cin, KT) -> (N, KT, Cin) in DT
template <typename DT>
__global__ void reorder_taps_kernel(const float* __restrict__ src, DT* __restrict__ dst, int N, int Cin, int KT) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)N * Cin * KT;
  if (i >= total) return;
  int k = i % KT;
  size_t t = i / KT;
  int c = t % Cin;
  int n = t / Cin;
  store_val<DT>(dst + ((size_t)n * KT + k) * Cin + c, src[i]);
}

// ------------------------------ handle ------------------------------

struct DenBlockW {
  const void* w2; const void* w3; const void* m0; const void* m2;  // DT (H x H)
  const float *b2, *b3, *mb0, *mb2, *lnw, *lnb, *lnmw, *lnmb, *dww, *dwb, *gnw, *gnb;
};

struct Den {
  int C, H, NB, KS, S, dt;  // dt: 0 f32, 1 bf16
  int MS;                   // mods row stride = (6 NB + 5) H
  char* dev = nullptr;      // packed weight arena
  size_t dev_bytes = 0;
  // fp32 AdaLN path
  float *t0w, *t0b, *t2w, *t2b, *cw, *cb, *adaw, *adab;
  // DT
  void* win; const float* bin;
  std::vector<DenBlockW> blk;
  DenBlockW fin;  // m0/m2/lnmw.. unused
  void* wout; const float* bout;
  // graph cache
  hipGraphExec_t gexec = nullptr;
  hipStream_t cap_stream = nullptr;
  int g_B = -1, g_T = -1, g_nfe = -1;
  const void *g_xt = nullptr, *g_mods = nullptr, *g_ws = nullptr;
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace fl

using namespace fl;

extern "C" {

FLAMED_API int flamed_den_create(int C, int H, int n_blocks, int kernel, int spk_dim, int dtype, flamed_den_t* out) {
  FL_REQUIRE(out, "flamed_den_create: null out");
  FL_REQUIRE(C > 0 && C % 32 == 0 && H % 128 == 0 && n_blocks >= 1 && spk_dim % 32 == 0, "flamed_den_create: unsupported dims C=%d H=%d S=%d", C, H, spk_dim);
  FL_REQUIRE(kernel == 31, "flamed_den_create: only convnext kernel_size=31 is specialised (got %d)", kernel);
  FL_REQUIRE(dtype == FLAMED_F32 || dtype == FLAMED_BF16, "flamed_den_create: dtype must be FLAMED_F32 or FLAMED_BF16");
  Den* d = new Den();
  d->C = C; d->H = H; d->NB = n_blocks; d->KS = kernel; d->S = spk_dim; d->dt = dtype;
  d->MS = (6 * n_blocks + 5) * H;
  *out = reinterpret_cast<flamed_den_t>(d);
  return kOk;
}

FLAMED_API int flamed_den_destroy(flamed_den_t h) {
  Den* d = reinterpret_cast<Den*>(h);
  if (!d) return kOk;
  if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
  if (d->cap_stream) (void)hipStreamDestroy(d->cap_stream);
  if (d->dev) (void)hipFree(d->dev);
  delete d;
  return kOk;
}

FLAMED_API int flamed_den_num_weights(flamed_den_t h) {
  Den* d = reinterpret_cast<Den*>(h);
  return d ? FLAMED_DEN_HEAD_W + FLAMED_DEN_BLOCK_W * d->NB + FLAMED_DEN_FINAL_W : -1;
}

FLAMED_API int flamed_den_load(flamed_den_t h, const float* const* w, int n, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && w, "flamed_den_load: null handle/weights");
  FL_REQUIRE(n == flamed_den_num_weights(h), "flamed_den_load: expected %d weight pointers, got %d", flamed_den_num_weights(h), n);
  for (int i = 0; i < n; ++i) FL_REQUIRE(w[i], "flamed_den_load: weight %d is null", i);
  const int H = d->H, C = d->C, S = d->S, NB = d->NB, KS = d->KS;
  const size_t es = d->dt == FLAMED_BF16 ? 2 : 4;
  // arena layout
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
  size_t o_t0w = take(4ull * H * 256), o_t0b = take(4ull * H), o_t2w = take(4ull * H * H), o_t2b = take(4ull * H);
  size_t o_cw = take(4ull * H * S), o_cb = take(4ull * H);
  size_t o_adaw = take(4ull * d->MS * H), o_adab = take(4ull * d->MS);
  size_t o_win = take(es * H * C);
  std::vector<size_t> o_blk(NB);
  for (int i = 0; i < NB; ++i) o_blk[i] = take(es * 4ull * H * H);
  size_t o_fin = take(es * 2ull * H * H);
  size_t o_out = take(es * (size_t)C * 3 * H);
  if (d->dev) { FL_HIP(hipFree(d->dev)); d->dev = nullptr; }
  FL_HIP(hipMalloc(&d->dev, off));
  d->dev_bytes = off;
  char* base = d->dev;
  auto cpy = [&](size_t o, const float* src, size_t n) -> int {
    hipLaunchKernelGGL(copy_kernel_f32, dim3((n + 255) / 256), dim3(256), 0, st, src, reinterpret_cast<float*>(base + o), n);
    FL_LAUNCH_CHECK();
    return kOk;
  };
  auto cast = [&](size_t o, const float* src, size_t n) -> int {
    if (d->dt == FLAMED_BF16) {
      hipLaunchKernelGGL(cast_kernel_bf16, dim3((n + 255) / 256), dim3(256), 0, st, src, reinterpret_cast<bf16*>(base + o), n);
      FL_LAUNCH_CHECK();
      return kOk;
    }
    return cpy(o, src, n);
  };
  int rc;
#define TRY(x) do { if ((rc = (x)) != kOk) return rc; } while (0)
  TRY(cpy(o_t0w, w[0], (size_t)H * 256)); TRY(cpy(o_t0b, w[1], H));
  TRY(cpy(o_t2w, w[2], (size_t)H * H)); TRY(cpy(o_t2b, w[3], H));
  TRY(cpy(o_cw, w[4], (size_t)H * S)); TRY(cpy(o_cb, w[5], H));
  TRY(cast(o_win, w[6], (size_t)H * C));
  d->t0w = (float*)(base + o_t0w); d->t0b = (float*)(base + o_t0b); d->t2w = (float*)(base + o_t2w); d->t2b = (float*)(base + o_t2b);
  d->cw = (float*)(base + o_cw); d->cb = (float*)(base + o_cb); d->adaw = (float*)(base + o_adaw); d->adab = (float*)(base + o_adab);
  d->win = base + o_win; d->bin = w[7];
  d->blk.resize(NB);
  for (int i = 0; i < NB; ++i) {
    const float* const* bw = w + FLAMED_DEN_HEAD_W + FLAMED_DEN_BLOCK_W * i;
    TRY(cpy(o_adaw + 4ull * (size_t)i * 6 * H * H, bw[0], 6ull * H * H));
    TRY(cpy(o_adab + 4ull * (size_t)i * 6 * H, bw[1], 6ull * H));
    DenBlockW& B = d->blk[i];
    size_t ob = o_blk[i];
    TRY(cast(ob, bw[8], (size_t)H * H));
    TRY(cast(ob + es * H * H, bw[10], (size_t)H * H));
    TRY(cast(ob + 2 * es * H * H, bw[14], (size_t)H * H));
    TRY(cast(ob + 3 * es * H * H, bw[16], (size_t)H * H));
    B.w2 = base + ob; B.w3 = base + ob + es * H * H; B.m0 = base + ob + 2 * es * H * H; B.m2 = base + ob + 3 * es * H * H;
    B.lnw = bw[2]; B.lnb = bw[3]; B.dww = bw[4]; B.dwb = bw[5]; B.gnw = bw[6]; B.gnb = bw[7];
    B.b2 = bw[9]; B.b3 = bw[11]; B.lnmw = bw[12]; B.lnmb = bw[13]; B.mb0 = bw[15]; B.mb2 = bw[17];
  }
  {
    const float* const* fw = w + FLAMED_DEN_HEAD_W + FLAMED_DEN_BLOCK_W * NB;
    TRY(cpy(o_adaw + 4ull * (size_t)NB * 6 * H * H, fw[0], 5ull * H * H));
    TRY(cpy(o_adab + 4ull * (size_t)NB * 6 * H, fw[1], 5ull * H));
    DenBlockW& F = d->fin;
    F.dww = fw[2]; F.dwb = fw[3]; F.gnw = fw[4]; F.gnb = fw[5];
    TRY(cast(o_fin, fw[6], (size_t)H * H)); F.b2 = fw[7];
    TRY(cast(o_fin + es * H * H, fw[8], (size_t)H * H)); F.b3 = fw[9];
    F.w2 = base + o_fin; F.w3 = base + o_fin + es * H * H;
    size_t n = (size_t)C * H * 3;
    if (d->dt == FLAMED_BF16)
      hipLaunchKernelGGL(reorder_taps_kernel<bf16>, dim3((n + 255) / 256), dim3(256), 0, st, fw[10], reinterpret_cast<bf16*>(base + o_out), C, H, 3);
    else
      hipLaunchKernelGGL(reorder_taps_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, st, fw[10], reinterpret_cast<float*>(base + o_out), C, H, 3);
    FL_LAUNCH_CHECK();
    d->wout = base + o_out; d->bout = fw[11];
  }
#undef TRY
  (void)KS;
  if (d->gexec) { (void)hipGraphExecDestroy(d->gexec); d->gexec = nullptr; }
  return kOk;
}

FLAMED_API size_t flamed_den_adaln_workspace_size(flamed_den_t h, int n_t, int n_spk) {
  Den* d = reinterpret_cast<Den*>(h);
  if (!d) return 0;
  return align256(4ull * n_t * 256) + 2 * align256(4ull * n_t * d->H) + align256(4ull * n_spk * d->H);
}

FLAMED_API int flamed_den_adaln(flamed_den_t h, const float* t_vals, int n_t, const float* spk, int n_spk,
                                const int* tidx, const int* sidx, int R, float* mods, void* ws, size_t ws_bytes,
                                hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev, "flamed_den_adaln: handle not loaded");
  FL_REQUIRE(t_vals && spk && tidx && sidx && mods && ws && n_t > 0 && n_spk > 0 && R > 0, "flamed_den_adaln: bad args");
  if (ws_bytes < flamed_den_adaln_workspace_size(h, n_t, n_spk)) {
    set_error("flamed_den_adaln: workspace too small");
    return kNoWorkspace;
  }
  const int H = d->H;
  char* p = (char*)ws;
  float* F = (float*)p; p += align256(4ull * n_t * 256);
  float* T1 = (float*)p; p += align256(4ull * n_t * H);
  float* TE = (float*)p; p += align256(4ull * n_t * H);
  float* CE = (float*)p;
  hipLaunchKernelGGL(tfreq_kernel, dim3((n_t * 256 + 255) / 256), dim3(256), 0, st, t_vals, n_t, 256, F);
  FL_LAUNCH_CHECK();
  int rc;
  if ((rc = launch_gemm<64, 64, 4, float>(LoadF32<float>{F, 256}, d->t0w, 256, EpiBiasAct<float, 2>{d->t0b, T1, H}, n_t, H, 256, st))) return rc;
  if ((rc = launch_gemm<64, 64, 4, float>(LoadF32<float>{T1, H}, d->t2w, H, EpiBiasAct<float, 0>{d->t2b, TE, H}, n_t, H, H, st))) return rc;
  if ((rc = launch_gemm<64, 64, 4, float>(LoadF32<float>{spk, d->S}, d->cw, d->S, EpiBiasAct<float, 0>{d->cb, CE, H}, n_spk, H, d->S, st))) return rc;
  if ((rc = launch_gemm<64, 64, 4, float>(LoadAdaY{TE, CE, tidx, sidx, H}, d->adaw, H, EpiBiasAct<float, 0>{d->adab, mods, d->MS}, R, d->MS, H, st))) return rc;
  return kOk;
}

FLAMED_API size_t flamed_den_workspace_size(flamed_den_t h, int B, int T) {
  Den* d = reinterpret_cast<Den*>(h);
  if (!d) return 0;
  size_t M = (size_t)B * T;
  size_t es = d->dt == FLAMED_BF16 ? 2 : 4;
  size_t NTmax = d->H / 64;
  return align256(4 * M * d->H) + 2 * align256(8 * M * NTmax) + 2 * align256(es * M * d->H);
}

}  // extern "C"

namespace fl {

struct DenWs {
  float* X;
  float* S0;
  float* S1;
  void* G;
  void* U;
};

static DenWs carve(Den* d, void* ws, int B, int T) {
  size_t M = (size_t)B * T;
  size_t es = d->dt == FLAMED_BF16 ? 2 : 4;
  size_t NTmax = d->H / 64;
  char* p = (char*)ws;
  DenWs w;
  w.X = (float*)p; p += align256(4 * M * d->H);
  w.S0 = (float*)p; p += align256(8 * M * NTmax);
  w.S1 = (float*)p; p += align256(8 * M * NTmax);
  w.G = p; p += align256(es * M * d->H);
  w.U = p;
  return w;
}

// One velocity evaluation (+ Euler update when vout == nullptr).
template <typename DT, int BM, int BN, int KCH>
static int den_step_impl(Den* d, float* xt, const float* mods, int mod_div, int B, int T, float dt, float* vout,
                         const DenWs& w, hipStream_t st, int only = -1) {
  const int M = B * T, H = d->H, C = d->C, MS = d->MS;
  const int NT = H / BN;
  DT* G = reinterpret_cast<DT*>(w.G);
  DT* U = reinterpret_cast<DT*>(w.U);
  int rc;
#define TRY(x) do { if ((rc = (x)) != kOk) return rc; } while (0)
#define K_(cls) if (only < 0 || only == (cls))
  K_(0) TRY((launch_gemm<BM, BN, KCH, DT>(LoadF32<DT>{xt, C}, (const DT*)d->win, C, EpiBiasStats{d->bin, w.X, H, w.S0, NT}, M, H, C, st)));
  for (int i = 0; i < (only < 0 ? d->NB : 1); ++i) {
    const DenBlockW& Bw = d->blk[i];
    const float* md = mods + (size_t)i * 6 * H;
    ModRef mc{md, md + H, MS, mod_div};
    ModRef mm{md + 3 * H, md + 4 * H, MS, mod_div};
    K_(1) TRY((launch_dwconv_gn<DT, true, 31>(w.X, H, w.S0, NT, BN, mc, Bw.lnw, Bw.lnb, Bw.dww, Bw.dwb, Bw.gnw, Bw.gnb, G, B, T, st)));
    K_(2) TRY((launch_gemm<BM, BN, KCH, DT>(LoadPlain<DT>{G, H}, (const DT*)Bw.w2, H, EpiBiasAct<DT, 1>{Bw.b2, U, H}, M, H, H, st)));
    K_(3) TRY((launch_gemm<BM, BN, KCH, DT>(LoadPlain<DT>{U, H}, (const DT*)Bw.w3, H,
                                      EpiConvNeXtResid<true>{Bw.b3, w.X, H, w.S0, NT, BN, 1e-6f, mc, md + 2 * H, Bw.lnw, Bw.lnb, w.S1, NT},
                                      M, H, H, st)));
    K_(4) TRY((launch_gemm<BM, BN, KCH, DT>(LoadLNMod<DT, true>{w.X, H, w.S1, NT, BN, 1e-6f, mm, Bw.lnmw, Bw.lnmb}, (const DT*)Bw.m0, H,
                                      EpiBiasAct<DT, 2>{Bw.mb0, U, H}, M, H, H, st)));
    K_(5) TRY((launch_gemm<BM, BN, KCH, DT>(LoadPlain<DT>{U, H}, (const DT*)Bw.m2, H,
                                      EpiGatedResid{Bw.mb2, w.X, H, md + 5 * H, MS, mod_div, w.S0, NT}, M, H, H, st)));
  }
  const float* mf = mods + (size_t)d->NB * 6 * H;
  ModRef mc{mf, mf + H, MS, mod_div};
  ModRef mo{mf + 3 * H, mf + 4 * H, MS, mod_div};
  const DenBlockW& F = d->fin;
  if (only >= 0 && only != 6) return kOk;
  if (only < 0) {
  TRY((launch_dwconv_gn<DT, false, 31>(w.X, H, w.S0, NT, BN, mc, nullptr, nullptr, F.dww, F.dwb, F.gnw, F.gnb, G, B, T, st)));
  TRY((launch_gemm<BM, BN, KCH, DT>(LoadPlain<DT>{G, H}, (const DT*)F.w2, H, EpiBiasAct<DT, 1>{F.b2, U, H}, M, H, H, st)));
  TRY((launch_gemm<BM, BN, KCH, DT>(LoadPlain<DT>{U, H}, (const DT*)F.w3, H,
                                    EpiConvNeXtResid<false>{F.b3, w.X, H, w.S0, NT, BN, 1e-6f, mc, mf + 2 * H, nullptr, nullptr, w.S1, NT},
                                    M, H, H, st)));
  }
  LoadConv3LN<DT> lo{w.X, H, w.S1, NT, BN, 1e-6f, mo, T};
  if (vout) {
    TRY((launch_gemm<BM, BN, KCH, DT>(lo, (const DT*)d->wout, 3 * H, EpiBiasAct<float, 0>{d->bout, vout, C}, M, C, 3 * H, st)));
  } else {
    TRY((launch_gemm<BM, BN, KCH, DT>(lo, (const DT*)d->wout, 3 * H, EpiEuler{d->bout, xt, C, dt}, M, C, 3 * H, st)));
  }
#undef K_
#undef TRY
  return kOk;
}

static int den_step(Den* d, float* xt, const float* mods, int mod_div, int B, int T, float dt, float* vout, void* ws,
                    hipStream_t st, int only = -1) {
  DenWs w = carve(d, ws, B, T);
  const int M = B * T;
  const bool big = M >= 4096;
  if (d->dt == FLAMED_BF16) {
    return big ? den_step_impl<bf16, 128, 128, 4>(d, xt, mods, mod_div, B, T, dt, vout, w, st, only)
               : den_step_impl<bf16, 64, 64, 4>(d, xt, mods, mod_div, B, T, dt, vout, w, st, only);
  }
  return big ? den_step_impl<float, 128, 128, 4>(d, xt, mods, mod_div, B, T, dt, vout, w, st, only)
             : den_step_impl<float, 64, 64, 4>(d, xt, mods, mod_div, B, T, dt, vout, w, st, only);
}

}  // namespace fl

extern "C" {

FLAMED_API int flamed_den_velocity(flamed_den_t h, const float* x, const float* mods, int mod_div, int B, int T,
                                   float* v_out, void* ws, size_t ws_bytes, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev, "flamed_den_velocity: handle not loaded");
  FL_REQUIRE(x && mods && v_out && ws && B > 0 && T > 0 && mod_div > 0, "flamed_den_velocity: bad args");
  if (ws_bytes < flamed_den_workspace_size(h, B, T)) {
    set_error("flamed_den_velocity: workspace too small (%zu < %zu)", ws_bytes, flamed_den_workspace_size(h, B, T));
    return kNoWorkspace;
  }
  return den_step(d, const_cast<float*>(x), mods, mod_div, B, T, 0.f, v_out, ws, st);
}

FLAMED_API int flamed_den_step(flamed_den_t h, float* xt, const float* mods, int mod_div, int B, int T, float dt,
                               void* ws, size_t ws_bytes, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev, "flamed_den_step: handle not loaded");
  FL_REQUIRE(xt && mods && ws && B > 0 && T > 0 && mod_div > 0, "flamed_den_step: bad args");
  if (ws_bytes < flamed_den_workspace_size(h, B, T)) {
    set_error("flamed_den_step: workspace too small");
    return kNoWorkspace;
  }
  return den_step(d, xt, mods, mod_div, B, T, dt, nullptr, ws, st);
}

FLAMED_API int flamed_den_solve(flamed_den_t h, float* xt, const float* mods, int nfe, int B, int T, void* ws,
                                size_t ws_bytes, int use_graph, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev, "flamed_den_solve: handle not loaded");
  FL_REQUIRE(xt && mods && ws && B > 0 && T > 0 && nfe > 0, "flamed_den_solve: bad args");
  if (ws_bytes < flamed_den_workspace_size(h, B, T)) {
    set_error("flamed_den_solve: workspace too small");
    return kNoWorkspace;
  }
  // delta_t = 1 / nfe as a python float, applied in fp32 (prob_generator.py:441,445)
  const float dt = (float)(1.0 / (double)nfe);
  const size_t step_stride = (size_t)B * d->MS;
  if (!use_graph) {
    for (int s = 0; s < nfe; ++s) {
      int rc = den_step(d, xt, mods + s * step_stride, T, B, T, dt, nullptr, ws, st);
      if (rc) return rc;
    }
    return kOk;
  }
  const bool hit = d->gexec && d->g_B == B && d->g_T == T && d->g_nfe == nfe && d->g_xt == xt && d->g_mods == mods && d->g_ws == ws;
  if (!hit) {
    if (d->gexec) { FL_HIP(hipGraphExecDestroy(d->gexec)); d->gexec = nullptr; }
    if (!d->cap_stream) FL_HIP(hipStreamCreateWithFlags(&d->cap_stream, hipStreamNonBlocking));
    FL_HIP(hipStreamBeginCapture(d->cap_stream, hipStreamCaptureModeRelaxed));
    int rc = kOk;
    for (int s = 0; s < nfe && rc == kOk; ++s) rc = den_step(d, xt, mods + s * step_stride, T, B, T, dt, nullptr, ws, d->cap_stream);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(d->cap_stream, &g);
    if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
    FL_HIP(e);
    hipError_t ie = hipGraphInstantiate(&d->gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    FL_HIP(ie);
    d->g_B = B; d->g_T = T; d->g_nfe = nfe; d->g_xt = xt; d->g_mods = mods; d->g_ws = ws;
  }
  FL_HIP(hipGraphLaunch(d->gexec, st));
  return kOk;
}

}  // extern "C"

extern "C" {

FLAMED_API int flamed_den_time_kernels(flamed_den_t h, float* xt, const float* mods, int B, int T, void* ws,
                                       size_t ws_bytes, int iters, float* ms_out, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev && xt && mods && ws && ms_out && iters > 0, "flamed_den_time_kernels: bad args");
  if (ws_bytes < flamed_den_workspace_size(h, B, T)) {
    set_error("flamed_den_time_kernels: workspace too small");
    return kNoWorkspace;
  }
  hipEvent_t e0, e1;
  FL_HIP(hipEventCreate(&e0));
  FL_HIP(hipEventCreate(&e1));
  int rc = kOk;
  for (int cls = 0; cls < FLAMED_DEN_KERNEL_CLASSES && rc == kOk; ++cls) {
    rc = den_step(d, xt, mods, T, B, T, 0.f, nullptr, ws, st, cls);  // warm
    if (rc) break;
    FL_HIP(hipEventRecord(e0, st));
    for (int i = 0; i < iters && rc == kOk; ++i) rc = den_step(d, xt, mods, T, B, T, 0.f, nullptr, ws, st, cls);
    FL_HIP(hipEventRecord(e1, st));
    FL_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    FL_HIP(hipEventElapsedTime(&ms, e0, e1));
    ms_out[cls] = ms / iters;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return rc;
}

}  // extern "C"
