// Condition fold of ProbGenerator.sample, run once per utterance before the Euler
// loop (reference flamed/models/synthesizer/prob_generator.py:435-436):
//   QuantizerEncoding  (:368-381)  x = (cond[b][q][t] + emb[q]) folded to (B, T, Q*D)
//   ConditionDownSampler (:167-205), n_stages = 1 (prob.yaml downsampling_stages):
//     ResnetBlock1D  (:25-32)      x = x + Mish(GroupNorm8(conv1x1(x * mask))) * mask
//     downblock                    h = ReLU(GroupNorm8(conv1x1 C -> C/2 (x)))
//     proj_out                     out = ReLU(Linear(C/2 -> out)(h))
// Frames are channels-last rows (M = B*T).  Five launches: GEMM1 (loader = quantizer encoding + mask,
// stored H1) -> GroupNorm(8) statistics over (channels of a group x every frame, padding included, as
// F.group_norm) -> GEMM2 (loader = the residual x + Mish(GN(H1)) * mask, recomputing x from cond) ->
// statistics -> GEMM3 (loader = ReLU(GN(H2)), epilogue bias + ReLU).  GEMM operands are exact fp32
// (default; the folded condition is added straight into the solve's start point) or bf16.
#include "flamed_hip.h"
#include "gemm.hpp"

#include <mutex>

namespace fl {

// A[m][k] = (cond[b][q][t][d] + emb[q][d]) * mask[m]   (m = b*T + t, k = q*D + d; EPC | D)
template <typename DT>
struct LoadQEnc {
  const float* __restrict__ cond;
  const float* __restrict__ emb;
  const float* __restrict__ mask;
  int T, Q, D;
  static constexpr int EPC = DTraits<DT>::EPC;
  struct Raw { float v[EPC]; float e[EPC]; float mk; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    Raw r;
    const int b = m / T, t = m - b * T, q = k / D, d = k - q * D;
    const float* p = cond + (((size_t)b * Q + q) * T + t) * D + d;
    const float* e = emb + (size_t)q * D + d;
#pragma unroll
    for (int j = 0; j < EPC; j += 4) {
      const float4 a = ld4(p + j), c = ld4(e + j);
      r.v[j] = a.x; r.v[j + 1] = a.y; r.v[j + 2] = a.z; r.v[j + 3] = a.w;
      r.e[j] = c.x; r.e[j + 1] = c.y; r.e[j + 2] = c.z; r.e[j + 3] = c.w;
    }
    r.mk = mask[m];
    return r;
  }
  __device__ float raw(const Raw& r, int j) const { return r.v[j] + r.e[j]; }          // x (unmasked)
  __device__ float value(const Raw& r, int j) const { return (r.v[j] + r.e[j]) * r.mk; }  // x * mask
  template <typename D_> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const {
    float o[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) o[j] = value(r, j);
    return pack_chunk<D_>(o);
  }
};

__device__ __forceinline__ float mish(float x) {  // x * tanh(softplus(x)), softplus threshold 20 (F.mish)
  const float sp = x > 20.f ? x : log1pf(expf(x));
  return x * tanhf(sp);
}

// A[m][k] = x[m][k] + Mish(GN(H1)[m][k]) * mask[m], x (unmasked, :31) recomputed by the quantizer-encoding loader
template <typename DT>
struct LoadResMish {
  LoadQEnc<DT> xq;
  const float* __restrict__ h;      // H1, M x C
  const float* __restrict__ gs;     // (B, G, 2) = (mean, rstd)
  const float* __restrict__ gw;
  const float* __restrict__ gb;
  int C, CG;                        // channels, channels per group
  static constexpr int EPC = DTraits<DT>::EPC;
  struct Raw { typename LoadQEnc<DT>::Raw x; float h[EPC]; float w[EPC]; float bb[EPC]; float mean, rstd; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    Raw r;
    r.x = xq.issue(m, k);
    const float* p = h + (size_t)m * C + k;
#pragma unroll
    for (int j = 0; j < EPC; j += 4) {
      const float4 a = ld4(p + j), w = ld4(gw + k + j), c = ld4(gb + k + j);
      r.h[j] = a.x; r.h[j + 1] = a.y; r.h[j + 2] = a.z; r.h[j + 3] = a.w;
      r.w[j] = w.x; r.w[j + 1] = w.y; r.w[j + 2] = w.z; r.w[j + 3] = w.w;
      r.bb[j] = c.x; r.bb[j + 1] = c.y; r.bb[j + 2] = c.z; r.bb[j + 3] = c.w;
    }
    const int G = C / CG;
    const float2 s = reinterpret_cast<const float2*>(gs)[(size_t)(m / xq.T) * G + k / CG];  // EPC | CG
    r.mean = s.x; r.rstd = s.y;
    return r;
  }
  template <typename D_> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const {
    float o[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) {
      const float g = (r.h[j] - r.mean) * r.rstd * r.w[j] + r.bb[j];
      o[j] = xq.raw(r.x, j) + mish(g) * r.x.mk;  // ResnetBlock1D: x + block(x, mask), x itself unmasked
    }
    return pack_chunk<D_>(o);
  }
};

// A[m][k] = ReLU(GN(H2)[m][k])
template <typename DT>
struct LoadGNRelu {
  const float* __restrict__ h;
  const float* __restrict__ gs;
  const float* __restrict__ gw;
  const float* __restrict__ gb;
  int C, CG, T;
  static constexpr int EPC = DTraits<DT>::EPC;
  struct Raw { float h[EPC]; float w[EPC]; float bb[EPC]; float mean, rstd; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    Raw r;
    const float* p = h + (size_t)m * C + k;
#pragma unroll
    for (int j = 0; j < EPC; j += 4) {
      const float4 a = ld4(p + j), w = ld4(gw + k + j), c = ld4(gb + k + j);
      r.h[j] = a.x; r.h[j + 1] = a.y; r.h[j + 2] = a.z; r.h[j + 3] = a.w;
      r.w[j] = w.x; r.w[j + 1] = w.y; r.w[j + 2] = w.z; r.w[j + 3] = w.w;
      r.bb[j] = c.x; r.bb[j + 1] = c.y; r.bb[j + 2] = c.z; r.bb[j + 3] = c.w;
    }
    const float2 s = reinterpret_cast<const float2*>(gs)[(size_t)(m / T) * (C / CG) + k / CG];
    r.mean = s.x; r.rstd = s.y;
    return r;
  }
  template <typename D_> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const {
    float o[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) o[j] = fmaxf((r.h[j] - r.mean) * r.rstd * r.w[j] + r.bb[j], 0.f);
    return pack_chunk<D_>(o);
  }
};

// GroupNorm statistics (F.group_norm, biased variance, eps) of H (B*T x C) for G groups of CG channels
// over every frame of an utterance: one workgroup per (group, utterance); per-thread Chan partials over
// a strided slice, combined through LDS in a fixed order (deterministic).
__global__ __launch_bounds__(256) void group_stats_kernel(const float* __restrict__ H, int T, int C, int CG, float eps,
                                                          float* __restrict__ gs) {
  const int g = blockIdx.x, b = blockIdx.y, G = gridDim.x;
  const int tid = threadIdx.x;
  const int c4 = CG / 4;  // float4 chunks per frame (CG % 4 == 0)
  float n = 0.f, mu = 0.f, m2 = 0.f;
  const size_t total = (size_t)T * c4;
  for (size_t i = tid; i < total; i += 256) {
    const int t = i / c4, c = (int)(i - (size_t)t * c4) * 4;
    const float4 v = ld4(H + ((size_t)b * T + t) * C + (size_t)g * CG + c);
    const float s = v.x + v.y + v.z + v.w;
    const float mb = s * 0.25f;
    const float d0 = v.x - mb, d1 = v.y - mb, d2 = v.z - mb, d3 = v.w - mb;
    chan_combine(n, mu, m2, 4.f, mb, d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
  }
  __shared__ float red[256 * 3];
  red[tid * 3] = n; red[tid * 3 + 1] = mu; red[tid * 3 + 2] = m2;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      float a = red[tid * 3], am = red[tid * 3 + 1], a2 = red[tid * 3 + 2];
      chan_combine(a, am, a2, red[(tid + s) * 3], red[(tid + s) * 3 + 1], red[(tid + s) * 3 + 2]);
      red[tid * 3] = a; red[tid * 3 + 1] = am; red[tid * 3 + 2] = a2;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float cnt = red[0];
    gs[((size_t)b * G + g) * 2] = red[1];
    gs[((size_t)b * G + g) * 2 + 1] = 1.0f / sqrtf(red[2] / cnt + eps);
  }
}

struct CondFold {
  int Q, D, C, C2, OUT, G, dt;
  int device = -1;
  std::mutex mu;
  char* dev = nullptr;
  void *w1, *w2, *w3;       // packed GEMM weights (DT): C x C, C2 x C, OUT x C2
  const float *emb, *b1, *g1w, *g1b, *b2, *g2w, *g2b, *b3;
};

static size_t cf_a256(size_t x) { return (x + 255) & ~(size_t)255; }

struct CondWs { float *H1, *H2, *S1, *S2; };
static size_t cond_ws_layout(const CondFold* f, int B, int T, void* base, CondWs* w) {
  const size_t M = (size_t)B * T;
  const size_t sizes[4] = {4 * M * f->C, 4 * M * f->C2, 8ull * B * f->G, 8ull * B * f->G};
  size_t off = 0;
  char* p[4];
  for (int i = 0; i < 4; ++i) {
    p[i] = base ? (char*)base + off : nullptr;
    off += cf_a256(sizes[i]);
  }
  if (w) *w = CondWs{(float*)p[0], (float*)p[1], (float*)p[2], (float*)p[3]};
  return off;
}

__global__ void cf_cast_kernel(const float* __restrict__ src, void* __restrict__ dst, size_t n, int bf) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (bf) reinterpret_cast<bf16*>(dst)[i] = (bf16)src[i];
  else reinterpret_cast<float*>(dst)[i] = src[i];
}

template <typename DT>
static int cond_fold_impl(CondFold* f, const float* cond, const float* mask, int B, int T, float* out, const CondWs& w,
                          hipStream_t st) {
  const int M = B * T;
  int rc;
  const LoadQEnc<DT> xq{cond, f->emb, mask, T, f->Q, f->D};
  if ((rc = launch_gemm<DT>(xq, (const DT*)f->w1, f->C, EpiBiasAct<float, 0>{f->b1, w.H1, f->C}, M, f->C, f->C, st))) return rc;
  hipLaunchKernelGGL(group_stats_kernel, dim3(f->G, B), dim3(256), 0, st, w.H1, T, f->C, f->C / f->G, 1e-5f, w.S1);
  FL_LAUNCH_CHECK();
  const LoadResMish<DT> lr{xq, w.H1, w.S1, f->g1w, f->g1b, f->C, f->C / f->G};
  if ((rc = launch_gemm<DT>(lr, (const DT*)f->w2, f->C, EpiBiasAct<float, 0>{f->b2, w.H2, f->C2}, M, f->C2, f->C, st))) return rc;
  hipLaunchKernelGGL(group_stats_kernel, dim3(f->G, B), dim3(256), 0, st, w.H2, T, f->C2, f->C2 / f->G, 1e-5f, w.S2);
  FL_LAUNCH_CHECK();
  const LoadGNRelu<DT> lg{w.H2, w.S2, f->g2w, f->g2b, f->C2, f->C2 / f->G, T};
  return launch_gemm<DT>(lg, (const DT*)f->w3, f->C2, EpiBiasAct<float, 3>{f->b3, out, f->OUT}, M, f->OUT, f->C2, st);
}

}  // namespace fl

using namespace fl;

extern "C" {

FLAMED_API int flamed_cond_create(int n_quantizers, int cond_dim, int out_dim, int n_stages, int dtype, flamed_cond_t* out) {
  FL_REQUIRE(out, "flamed_cond_create: null out");
  FL_REQUIRE(n_stages == 1, "flamed_cond_create: only downsampling_stages = 1 is specialised (got %d)", n_stages);
  FL_REQUIRE(dtype == FLAMED_F32 || dtype == FLAMED_BF16, "flamed_cond_create: bad dtype");
  const int C = n_quantizers * cond_dim;
  FL_REQUIRE(n_quantizers > 0 && cond_dim % 8 == 0 && C % 128 == 0 && (C / 2) % 64 == 0 && out_dim % 64 == 0 &&
                 (C / 8) % 8 == 0 && (C / 16) % 8 == 0,
             "flamed_cond_create: unsupported dims Q=%d D=%d out=%d", n_quantizers, cond_dim, out_dim);
  CondFold* f = new CondFold();
  f->Q = n_quantizers; f->D = cond_dim; f->C = C; f->C2 = C / 2; f->OUT = out_dim; f->G = 8; f->dt = dtype;
  *out = reinterpret_cast<flamed_cond_t>(f);
  return kOk;
}

FLAMED_API int flamed_cond_destroy(flamed_cond_t h) {
  CondFold* f = reinterpret_cast<CondFold*>(h);
  if (!f) return kOk;
  {
    std::lock_guard<std::mutex> lk(f->mu);
    DeviceGuard dg(f->device);
    if (f->dev) (void)hipFree(f->dev);
  }
  delete f;
  return kOk;
}

FLAMED_API int flamed_cond_load(flamed_cond_t h, const float* const* w, int nw, hipStream_t st) {
  CondFold* f = reinterpret_cast<CondFold*>(h);
  FL_REQUIRE(f && w && nw == FLAMED_COND_W, "flamed_cond_load: expected %d weights", FLAMED_COND_W);
  for (int i = 0; i < nw; ++i) FL_REQUIRE(w[i], "flamed_cond_load: weight %d is null", i);
  int wdev = -1;
  FL_REQUIRE(device_of(w[0], &wdev) == kOk, "flamed_cond_load: weights must be device memory");
  for (int i = 1; i < nw; ++i) FL_REQUIRE_ON(w[i], wdev, "flamed_cond_load");
  std::lock_guard<std::mutex> lk(f->mu);
  if (f->device >= 0 && f->device != wdev && f->dev) {
    DeviceGuard og(f->device);
    (void)hipFree(f->dev);
    f->dev = nullptr;
  }
  f->device = wdev;
  FL_ON_DEVICE(wdev);
  const size_t es = f->dt == FLAMED_BF16 ? 2 : 4;
  const size_t n1 = (size_t)f->C * f->C, n2 = (size_t)f->C2 * f->C, n3 = (size_t)f->OUT * f->C2;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = cf_a256(off + bytes); return o; };
  const size_t o1 = take(es * n1), o2 = take(es * n2), o3 = take(es * n3);
  VecCopies vc;
  vc.add(w[0], (size_t)f->Q * f->D, &f->emb);
  vc.add(w[2], f->C, &f->b1); vc.add(w[3], f->C, &f->g1w); vc.add(w[4], f->C, &f->g1b);
  vc.add(w[6], f->C2, &f->b2); vc.add(w[7], f->C2, &f->g2w); vc.add(w[8], f->C2, &f->g2b);
  vc.add(w[10], f->OUT, &f->b3);
  const size_t ov = take(vc.bytes);
  if (f->dev) { FL_HIP(hipFree(f->dev)); f->dev = nullptr; }
  FL_HIP(hipMalloc(&f->dev, off));
  const int bf = f->dt == FLAMED_BF16;
  auto cast = [&](size_t o, const float* src, size_t n) -> int {
    hipLaunchKernelGGL(cf_cast_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, (void*)(f->dev + o), n, bf);
    FL_LAUNCH_CHECK();
    return kOk;
  };
  int rc;
  if ((rc = cast(o1, w[1], n1)) || (rc = cast(o2, w[5], n2)) || (rc = cast(o3, w[9], n3))) return rc;
  if ((rc = vc.commit(f->dev + ov, st))) return rc;
  f->w1 = f->dev + o1; f->w2 = f->dev + o2; f->w3 = f->dev + o3;
  return kOk;
}

FLAMED_API size_t flamed_cond_workspace_size(flamed_cond_t h, int B, int T) {
  CondFold* f = reinterpret_cast<CondFold*>(h);
  return f ? cond_ws_layout(f, B, T, nullptr, nullptr) : 0;
}

FLAMED_API int flamed_cond_fold(flamed_cond_t h, const float* cond, const float* mask, int B, int T, float* out, void* ws,
                                size_t ws_bytes, hipStream_t st) {
  CondFold* f = reinterpret_cast<CondFold*>(h);
  FL_REQUIRE(f && f->dev, "flamed_cond_fold: handle not loaded");
  FL_REQUIRE(cond && mask && out && ws && B > 0 && T > 0, "flamed_cond_fold: bad args");
  if (ws_bytes < cond_ws_layout(f, B, T, nullptr, nullptr)) {
    set_error("flamed_cond_fold: workspace too small");
    return kNoWorkspace;
  }
  std::lock_guard<std::mutex> lk(f->mu);
  FL_ON_DEVICE(f->device);
  FL_REQUIRE_ON(cond, f->device, "flamed_cond_fold");
  const Tune tsnap = tune_snapshot(nullptr);
  TuneScope ts_(&tsnap);
  CondWs w;
  cond_ws_layout(f, B, T, ws, &w);
  return f->dt == FLAMED_BF16 ? cond_fold_impl<bf16>(f, cond, mask, B, T, out, w, st)
                              : cond_fold_impl<float>(f, cond, mask, B, T, out, w, st);
}

}  // extern "C"
