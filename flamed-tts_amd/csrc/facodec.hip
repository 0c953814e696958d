// FaCodec decoder (inference) and encoder (prompt path) on gfx950.  Reference:
// flamed/models/facodec/facodec.py:136-244 (EncoderBlock, FACodecEncoder), :27-32
// (WNConv1d / WNConvTranspose1d), :57-118 (SnakeBeta), :121-133 (ResidualUnit), :246-265
// (DecoderBlock), :398-415 (model stack), :630-638 (FACodecDecoder.inference);
// alias_free_torch/act.py:7-29, resample.py:9-57, filter.py:27-96 (Activation1d).
//
// Layout: channels-last rows (B*n, C) fp32 residual stream; every conv is an implicit GEMM on the
// MFMA template (K = tap*Cin + c), weight norm folded at load.  ConvTranspose(k=2s, stride s) is
// s polyphase GEMMs with 2 taps each: output o = q*s + r - p takes W[:,:,r] x[q] + W[:,:,r+s] x[q-1].
// Activation1d (replicate-pad, 12-tap kaiser-sinc x2 upsample, SnakeBeta, 12-tap lowpass /2) is one
// LDS-tiled stencil kernel: fp32 in, GEMM-operand dtype out.
#include "flamed_hip.h"
#include "gemm.hpp"

#include <vector>

namespace fl {

// ------------------------------ weight packing ------------------------------

// weight_norm(dim=0): w[i] = g[i] * v[i] / ||v[i]||  (one workgroup per dim-0 slice of `inner` values)
__global__ __launch_bounds__(256) void wn_fold_kernel(const float* __restrict__ g, const float* __restrict__ v, int inner,
                                                      float* __restrict__ w) {
  __shared__ float red[4];
  const int i = blockIdx.x;
  const float* vi = v + (size_t)i * inner;
  float s = 0.f;
  for (int k = threadIdx.x; k < inner; k += 256) s += vi[k] * vi[k];
  s = wave_sum64(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float nrm = sqrtf(red[0] + red[1] + red[2] + red[3]);
  const float sc = g[i] / nrm;
  for (int k = threadIdx.x; k < inner; k += 256) w[(size_t)i * inner + k] = vi[k] * sc;
}

// conv (N, Cin, KT) -> rows of (KT, Cin) in DT with row stride ldk >= KT*Cin (pad pre-zeroed)
template <typename DT>
__global__ void pack_conv_kernel(const float* __restrict__ src, DT* __restrict__ dst, int N, int Cin, int KT, int ldk) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)N * Cin * KT) return;
  int k = i % KT;
  size_t t = i / KT;
  int c = t % Cin;
  int n = t / Cin;
  store_val<DT>(dst + (size_t)n * ldk + (size_t)k * Cin + c, src[i]);
}

// convT (Cin, Cout, 2s) -> per phase r: (Cout, 2, Cin) with tap 0 = kernel index r, tap 1 = r + s
template <typename DT>
__global__ void pack_convt_kernel(const float* __restrict__ src, DT* __restrict__ dst, int Cin, int Cout, int s) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int KT = 2 * s;
  if (i >= (size_t)Cin * Cout * KT) return;
  int k = i % KT;
  size_t t = i / KT;
  int oc = t % Cout;
  int ic = t / Cout;
  int r = k % s, tap = k / s;
  store_val<DT>(dst + (size_t)r * Cout * 2 * Cin + ((size_t)oc * 2 + tap) * Cin + ic, src[i]);
}

// ------------------------------ fused Activation1d ------------------------------
constexpr int kActA = 64;  // output samples per workgroup

// kActCG channels per workgroup (64, or 32 for the encoder's first stage)
template <typename OT, int kActCG>
__global__ __launch_bounds__(256) void act1d_kernel(const float* __restrict__ x, int C, int n,
                                                    const float* __restrict__ alpha, const float* __restrict__ beta,
                                                    const float* __restrict__ fu, const float* __restrict__ fd,
                                                    OT* __restrict__ out) {
  constexpr int XR = kActA + 13;      // x rows a0-6 .. a0+A+6
  constexpr int SR = 2 * kActA + 12;  // snake samples j = 2a0-5 .. 2a0+2A+6
  constexpr int RGS = 256 / kActCG;   // row groups
  __shared__ float xs[XR * kActCG];
  __shared__ float ss[SR * kActCG];
  __shared__ float filt[24];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * kActCG, a0 = blockIdx.y * kActA, b = blockIdx.z;
  if (tid < 12) filt[tid] = fu[tid];
  else if (tid < 24) filt[tid] = fd[tid - 12];
  const float* xb = x + (size_t)b * n * C;
  for (int idx = tid; idx < XR * kActCG; idx += 256) {
    int r = idx / kActCG, cc = idx - r * kActCG;
    int a = a0 - 6 + r;
    a = a < 0 ? 0 : (a >= n ? n - 1 : a);
    xs[idx] = xb[(size_t)a * C + c0 + cc];
  }
  __syncthreads();
  const int cc = tid % kActCG, rg = tid / kActCG;
  const float ea = expf(alpha[c0 + cc]);
  const float ib = 1.0f / (expf(beta[c0 + cc]) + 1e-9f);
  const int n2 = 2 * n;
  for (int jj = rg; jj < SR; jj += RGS) {
    int j = 2 * a0 - 5 + jj;
    j = j < 0 ? 0 : (j >= n2 ? n2 - 1 : j);
    const int ap = j >> 1;
    const int base = ap - (a0 - 6);  // xs row of x[ap]
    float u = 0.f;
    if (j & 1) {
#pragma unroll
      for (int m = -2; m <= 3; ++m) u += filt[6 - 2 * m] * xs[(base + m) * kActCG + cc];
    } else {
#pragma unroll
      for (int m = -3; m <= 2; ++m) u += filt[5 - 2 * m] * xs[(base + m) * kActCG + cc];
    }
    u = 2.0f * u;
    float sn = sinf(u * ea);
    ss[jj * kActCG + cc] = u + ib * (sn * sn);
  }
  __syncthreads();
  OT* ob = out + (size_t)b * n * C;
  for (int q = rg; q < kActA; q += RGS) {
    int a = a0 + q;
    if (a >= n) break;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 12; ++k) acc += filt[12 + k] * ss[(2 * q + k) * kActCG + cc];
    store_val<OT>(ob + (size_t)a * C + c0 + cc, acc);
  }
}

// ------------------------------ prep: LayerNorm over C + timbre affine + transpose ------------------------------
// lat (B, C, T) channels-first -> h0 (B*T, C): LN(eps 1e-5, no affine) then x*gamma + beta (facodec.py:631-636)
__global__ __launch_bounds__(256) void fac_prep_kernel(const float* __restrict__ lat, const float* __restrict__ style,
                                                       int C, int T, float* __restrict__ h0) {
  extern __shared__ float tile[];  // C x 33
  const int b = blockIdx.y, t0 = blockIdx.x * 32, tid = threadIdx.x;
  for (int idx = tid; idx < C * 32; idx += 256) {
    int c = idx >> 5, t = idx & 31;
    tile[c * 33 + t] = (t0 + t < T) ? lat[((size_t)b * C + c) * T + t0 + t] : 0.f;
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  const int per = C / 64;
  for (int t = wave; t < 32; t += 4) {
    if (t0 + t >= T) break;
    float v[8];
    float s = 0.f;
    for (int j = 0; j < per; ++j) {
      v[j] = tile[(lane + 64 * j) * 33 + t];
      s += v[j];
    }
    float mean = wave_sum64(s) / (float)C;
    float q = 0.f;
    for (int j = 0; j < per; ++j) {
      float d = v[j] - mean;
      q += d * d;
    }
    float rstd = 1.0f / sqrtf(wave_sum64(q) / (float)C + 1e-5f);
    for (int j = 0; j < per; ++j) {
      int c = lane + 64 * j;
      float y = (v[j] - mean) * rstd;
      h0[((size_t)b * T + t0 + t) * C + c] = y * style[(size_t)b * 2 * C + c] + style[(size_t)b * 2 * C + C + c];
    }
  }
}

// ------------------------------ final Conv1d(64 -> 1, k7, pad 3) + tanh ------------------------------
template <typename IT>
__global__ __launch_bounds__(128) void fac_out_kernel(const IT* __restrict__ act, int C, int n, const float* __restrict__ w,
                                                      const float* __restrict__ bias, float* __restrict__ wav) {
  constexpr int TS = 128, HALO = 3;
  extern __shared__ float sm[];
  float* rows = sm;                      // (TS + 6) x (C + 1)
  float* ws = sm + (TS + 2 * HALO) * (C + 1);  // C x 7
  const int b = blockIdx.y, t0 = blockIdx.x * TS, tid = threadIdx.x;
  for (int i = tid; i < C * 7; i += TS) ws[i] = w[i];
  const IT* ab = act + (size_t)b * n * C;
  for (int idx = tid; idx < (TS + 2 * HALO) * C; idx += TS) {
    int r = idx / C, c = idx - r * C;
    int t = t0 - HALO + r;
    rows[r * (C + 1) + c] = (t >= 0 && t < n) ? (float)ab[(size_t)t * C + c] : 0.f;
  }
  __syncthreads();
  const int t = t0 + tid;
  if (t >= n) return;
  float acc = bias[0];
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int k = 0; k < 7; ++k) acc += ws[c * 7 + k] * rows[(tid + k) * (C + 1) + c];
  wav[(size_t)b * n + t] = tanhf(acc);
}

// ------------------------------ GEMM loaders / epilogues ------------------------------

// ConvTranspose phase GEMM A operand: row m -> (b, q), q in [0, n]; tap 0 = x[q], tap 1 = x[q-1].
template <typename DT>
struct LoadConvT {
  const DT* __restrict__ x;
  int Cin;
  int n;
  struct Raw { u32x4 v; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    int b = m / (n + 1), q = m - b * (n + 1);
    int tap = k / Cin, c = k - tap * Cin;
    int i = q - tap;
    if (i < 0 || i >= n) return Raw{u32x4{0u, 0u, 0u, 0u}};
    return Raw{*reinterpret_cast<const u32x4*>(x + ((size_t)b * n + i) * Cin + c)};
  }
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return r.v; }
};

struct EpiConvTStore {
  const float* __restrict__ bias;
  float* __restrict__ out;
  int Cout, n, s, r, p;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int, int col, float acc, const float*, int) const { return acc + bias[col]; }
  __device__ void store(int m, int col, float v) const {
    int b = m / (n + 1), q = m - b * (n + 1);
    int o = q * s + r - p;
    if (o >= 0 && o < s * n) out[((size_t)b * s * n + o) * Cout + col] = v;
  }
  __device__ void store_stats(int, int, float, float) const {}
};

struct EpiResAdd {  // X += acc + bias  (ResidualUnit skip, facodec.py:132-133)
  const float* __restrict__ bias;
  float* X;
  int ld;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int m, int col, float acc, const float*, int) const { return X[(size_t)m * ld + col] + (acc + bias[col]); }
  __device__ void store(int m, int col, float v) const { X[(size_t)m * ld + col] = v; }
  __device__ void store_stats(int, int, float, float) const {}
};

template <typename DT, class AL, class EP>
static int gemm_auto(const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  return launch_gemm<DT>(al, W, ldw, ep, M, N, K, st);
}

// ------------------------------ handle ------------------------------
struct FacAct { const float *alpha, *beta, *fu, *fd; };
struct FacRU { FacAct a1, a2; void* w7; const float* b7; void* w1; const float* b1; int dil; };
struct FacBlk { FacAct a; void* wt; const float* bt; int s, cin, cout; FacRU ru[3]; };

struct Fac {
  int C0, CI, NUP, dt;
  int ups[8];
  const float *tlw, *tlb;
  void* win; const float* bin;
  FacBlk blk[8];
  FacAct afin;
  float* wout; const float* bout;
  int cfin;
  char* dev = nullptr;
  int device = -1;  // device of the arena (from the loaded weights)
  std::mutex mu;    // one call at a time per handle
  hipGraphExec_t gexec = nullptr;
  hipStream_t cap = nullptr;
  std::vector<const void*> gkey;
  void release() {
    retire_graph(gexec);
    if (cap) (void)hipStreamDestroy(cap);
    if (dev) (void)hipFree(dev);
    gexec = nullptr; cap = nullptr; dev = nullptr;
    gkey.clear();
  }
};

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct FacWs { float* style; float* h0; float* X; float* Z; void* A; };
static size_t fac_ws_layout(const Fac* f, int B, int T, void* base, FacWs* w) {
  size_t maxcn = (size_t)f->CI * T;
  size_t n = T;
  int c = f->CI;
  for (int i = 0; i < f->NUP; ++i) {
    n *= f->ups[i];
    c /= 2;
    maxcn = maxcn > (size_t)c * n ? maxcn : (size_t)c * n;
  }
  size_t es = f->dt == FLAMED_BF16 ? 2 : 4;
  size_t sizes[5] = {4ull * B * 2 * f->C0, 4ull * B * T * f->C0, 4 * B * maxcn, 4 * B * maxcn, es * B * maxcn};
  size_t off = 0;
  char* p[5];
  for (int i = 0; i < 5; ++i) {
    p[i] = base ? (char*)base + off : nullptr;
    off += al256(sizes[i]);
  }
  if (w) *w = FacWs{(float*)p[0], (float*)p[1], (float*)p[2], (float*)p[3], p[4]};
  return off;
}

template <typename DT>
static int launch_act(const FacAct& a, const float* x, int C, int n, int B, DT* out, hipStream_t st) {
  FL_REQUIRE(C % 32 == 0, "act1d: C=%d must be a multiple of 32", C);
  const int na = (n + kActA - 1) / kActA;
  if (C % 64 == 0)
    hipLaunchKernelGGL((act1d_kernel<DT, 64>), dim3(C / 64, na, B), dim3(256), 0, st, x, C, n, a.alpha, a.beta, a.fu, a.fd, out);
  else
    hipLaunchKernelGGL((act1d_kernel<DT, 32>), dim3(C / 32, na, B), dim3(256), 0, st, x, C, n, a.alpha, a.beta, a.fu, a.fd, out);
  FL_LAUNCH_CHECK();
  return kOk;
}

template <typename DT>
static int fac_decode_impl(Fac* f, const float* lat, const float* spk, int B, int T, float* wav, const FacWs& w,
                           hipStream_t st) {
  int rc;
#define TRY(x) do { if ((rc = (x)) != kOk) return rc; } while (0)
  const int C0 = f->C0;
  DT* A = reinterpret_cast<DT*>(w.A);
  TRY((launch_gemm<float>(LoadF32<float>{spk, C0}, f->tlw, C0, EpiBiasAct<float, 0>{f->tlb, w.style, 2 * C0}, B, 2 * C0, C0, st)));
  hipLaunchKernelGGL(fac_prep_kernel, dim3((T + 31) / 32, B), dim3(256), (size_t)C0 * 33 * 4, st, lat, w.style, C0, T, w.h0);
  FL_LAUNCH_CHECK();
  TRY((gemm_auto<DT>(LoadConvRows<DT, false>{w.h0, C0, T, 7, 1, nullptr, 0, 0, 0.f, nullptr, nullptr}, (const DT*)f->win, 7 * C0,
                     EpiBiasAct<float, 0>{f->bin, w.X, f->CI}, B * T, f->CI, 7 * C0, st)));
  int n = T;
  for (int i = 0; i < f->NUP; ++i) {
    const FacBlk& bk = f->blk[i];
    const int s = bk.s, Cin = bk.cin, Cout = bk.cout, p = s / 2 + s % 2;
    TRY(launch_act<DT>(bk.a, w.X, Cin, n, B, A, st));
    for (int r = 0; r < s; ++r) {
      const DT* Wr = (const DT*)bk.wt + (size_t)r * Cout * 2 * Cin;
      TRY((gemm_auto<DT>(LoadConvT<DT>{A, Cin, n}, Wr, 2 * Cin, EpiConvTStore{bk.bt, w.X, Cout, n, s, r, p}, B * (n + 1), Cout,
                         2 * Cin, st)));
    }
    n *= s;
    for (int j = 0; j < 3; ++j) {
      const FacRU& ru = bk.ru[j];
      TRY(launch_act<DT>(ru.a1, w.X, Cout, n, B, A, st));
      TRY((gemm_auto<DT>(LoadConvPlain<DT>{A, Cout, n, 7, ru.dil}, (const DT*)ru.w7, 7 * Cout,
                         EpiBiasAct<float, 0>{ru.b7, w.Z, Cout}, B * n, Cout, 7 * Cout, st)));
      TRY(launch_act<DT>(ru.a2, w.Z, Cout, n, B, A, st));
      TRY((gemm_auto<DT>(LoadPlain<DT>{A, Cout}, (const DT*)ru.w1, Cout, EpiResAdd{ru.b1, w.X, Cout}, B * n, Cout, Cout, st)));
    }
  }
  const int cf = f->cfin;
  TRY(launch_act<DT>(f->afin, w.X, cf, n, B, A, st));
  size_t smem = ((128 + 6) * (cf + 1) + cf * 7) * 4;
  hipLaunchKernelGGL(fac_out_kernel<DT>, dim3((n + 127) / 128, B), dim3(128), smem, st, A, cf, n, f->wout, f->bout, wav);
  FL_LAUNCH_CHECK();
#undef TRY
  return kOk;
}

}  // namespace fl

using namespace fl;

extern "C" {

FLAMED_API int flamed_fac_create(int in_channels, int upsample_initial_channel, int n_up, const int* up_ratios, int dtype,
                                 flamed_fac_t* out) {
  FL_REQUIRE(out && up_ratios, "flamed_fac_create: null args");
  FL_REQUIRE(n_up >= 1 && n_up <= 8, "flamed_fac_create: n_up=%d unsupported", n_up);
  FL_REQUIRE(dtype == FLAMED_F32 || dtype == FLAMED_BF16, "flamed_fac_create: bad dtype");
  FL_REQUIRE(in_channels % 64 == 0 && in_channels <= 512, "flamed_fac_create: in_channels=%d unsupported", in_channels);
  FL_REQUIRE((upsample_initial_channel >> n_up) >= 64 && (upsample_initial_channel >> n_up) % 64 == 0,
             "flamed_fac_create: unsupported dims (channels %d over %d stages)", upsample_initial_channel, n_up);
  Fac* f = new Fac();
  f->C0 = in_channels; f->CI = upsample_initial_channel; f->NUP = n_up; f->dt = dtype;
  for (int i = 0; i < n_up; ++i) {
    FL_REQUIRE(up_ratios[i] >= 1 && up_ratios[i] <= 8, "flamed_fac_create: up ratio %d unsupported", up_ratios[i]);
    f->ups[i] = up_ratios[i];
  }
  *out = reinterpret_cast<flamed_fac_t>(f);
  return kOk;
}

FLAMED_API int flamed_fac_destroy(flamed_fac_t h) {
  Fac* f = reinterpret_cast<Fac*>(h);
  if (!f) return kOk;
  {
    std::lock_guard<std::mutex> lk(f->mu);
    DeviceGuard dg(f->device);
    f->release();
  }
  delete f;
  return kOk;
}

FLAMED_API int flamed_fac_num_weights(flamed_fac_t h) {
  Fac* f = reinterpret_cast<Fac*>(h);
  return f ? 5 + FLAMED_FAC_BLOCK_W * f->NUP + 7 : -1;
}

FLAMED_API int flamed_fac_load(flamed_fac_t h, const float* const* w, int nw, hipStream_t st) {
  Fac* f = reinterpret_cast<Fac*>(h);
  FL_REQUIRE(f && w, "flamed_fac_load: null args");
  FL_REQUIRE(nw == flamed_fac_num_weights(h), "flamed_fac_load: expected %d weights, got %d", flamed_fac_num_weights(h), nw);
  for (int i = 0; i < nw; ++i) FL_REQUIRE(w[i], "flamed_fac_load: weight %d is null", i);
  int wdev = -1;
  FL_REQUIRE(device_of(w[0], &wdev) == kOk, "flamed_fac_load: weights must be device memory");
  for (int i = 1; i < nw; ++i) FL_REQUIRE_ON(w[i], wdev, "flamed_fac_load");
  std::lock_guard<std::mutex> lk(f->mu);
  if (f->device >= 0 && f->device != wdev) {
    DeviceGuard og(f->device);
    f->release();
  }
  f->device = wdev;
  FL_ON_DEVICE(wdev);
  const size_t es = f->dt == FLAMED_BF16 ? 2 : 4;
  VecCopies vc;  // every vector is copied into the arena (the caller may free its tensors)
  auto act = [&](FacAct& a, const float* const* p, int ch) {
    vc.add(p[0], ch, &a.alpha); vc.add(p[1], ch, &a.beta); vc.add(p[2], 12, &a.fu); vc.add(p[3], 12, &a.fd);
  };
  // ---- arena layout
  struct Conv { const float *g, *v, *b; int dim0, inner, kind, N, Cin, KT, s; size_t off; };  // kind 0 conv, 1 convT
  std::vector<Conv> convs;
  size_t off = 0, maxfold = 0;
  auto add = [&](const float* g, const float* v, const float* b, int kind, int N, int Cin, int KT, int s) -> int {
    Conv c{g, v, b, kind == 0 ? N : Cin, kind == 0 ? Cin * KT : N * KT, kind, N, Cin, KT, s, off};
    off = al256(off + es * (size_t)N * Cin * KT);
    maxfold = maxfold > (size_t)N * Cin * KT ? maxfold : (size_t)N * Cin * KT;
    convs.push_back(c);
    return (int)convs.size() - 1;
  };
  vc.add(w[0], 2ull * f->C0 * f->C0, &f->tlw); vc.add(w[1], 2ull * f->C0, &f->tlb);
  int ci = add(w[2], w[3], w[4], 0, f->CI, f->C0, 7, 0);
  vc.add(w[4], f->CI, &f->bin);
  std::vector<int> idx_t(f->NUP), idx7(f->NUP * 3), idx1(f->NUP * 3);
  int c = f->CI;
  for (int i = 0; i < f->NUP; ++i) {
    const float* const* bw = w + 5 + FLAMED_FAC_BLOCK_W * i;
    FacBlk& bk = f->blk[i];
    bk.s = f->ups[i]; bk.cin = c; bk.cout = c / 2;
    act(bk.a, bw, bk.cin);
    idx_t[i] = add(bw[4], bw[5], bw[6], 1, bk.cout, bk.cin, 2 * bk.s, bk.s);
    vc.add(bw[6], bk.cout, &bk.bt);
    const int dils[3] = {1, 3, 9};
    for (int j = 0; j < 3; ++j) {
      const float* const* rw = bw + 7 + 14 * j;
      FacRU& ru = bk.ru[j];
      ru.dil = dils[j];
      act(ru.a1, rw, bk.cout);
      idx7[i * 3 + j] = add(rw[4], rw[5], rw[6], 0, bk.cout, bk.cout, 7, 0);
      vc.add(rw[6], bk.cout, &ru.b7);
      act(ru.a2, rw + 7, bk.cout);
      idx1[i * 3 + j] = add(rw[11], rw[12], rw[13], 0, bk.cout, bk.cout, 1, 0);
      vc.add(rw[13], bk.cout, &ru.b1);
    }
    c /= 2;
  }
  f->cfin = c;
  const float* const* fw = w + 5 + FLAMED_FAC_BLOCK_W * f->NUP;
  act(f->afin, fw, c);
  vc.add(fw[6], 1, &f->bout);
  size_t o_out = off;
  off = al256(off + 4ull * c * 7);
  size_t o_tmp = off;
  off = al256(off + 4 * maxfold);
  const size_t o_vec = off;
  off = al256(off + vc.bytes);
  f->release();
  FL_HIP(hipMalloc(&f->dev, off));
  {
    const int rc = vc.commit(f->dev + o_vec, st);
    if (rc) return rc;
  }
  float* tmp = reinterpret_cast<float*>(f->dev + o_tmp);
  for (const Conv& cv : convs) {
    hipLaunchKernelGGL(wn_fold_kernel, dim3(cv.dim0), dim3(256), 0, st, cv.g, cv.v, cv.inner, tmp);
    FL_LAUNCH_CHECK();
    size_t total = (size_t)cv.N * cv.Cin * cv.KT;
    dim3 grid((total + 255) / 256);
    if (cv.kind == 0) {
      if (f->dt == FLAMED_BF16) hipLaunchKernelGGL(pack_conv_kernel<bf16>, grid, dim3(256), 0, st, tmp, (bf16*)(f->dev + cv.off), cv.N, cv.Cin, cv.KT, cv.Cin * cv.KT);
      else hipLaunchKernelGGL(pack_conv_kernel<float>, grid, dim3(256), 0, st, tmp, (float*)(f->dev + cv.off), cv.N, cv.Cin, cv.KT, cv.Cin * cv.KT);
    } else {
      if (f->dt == FLAMED_BF16) hipLaunchKernelGGL(pack_convt_kernel<bf16>, grid, dim3(256), 0, st, tmp, (bf16*)(f->dev + cv.off), cv.Cin, cv.N, cv.s);
      else hipLaunchKernelGGL(pack_convt_kernel<float>, grid, dim3(256), 0, st, tmp, (float*)(f->dev + cv.off), cv.Cin, cv.N, cv.s);
    }
    FL_LAUNCH_CHECK();
  }
  // final conv (1, c, 7): folded fp32, kept as (c, 7)
  hipLaunchKernelGGL(wn_fold_kernel, dim3(1), dim3(256), 0, st, fw[4], fw[5], c * 7, reinterpret_cast<float*>(f->dev + o_out));
  FL_LAUNCH_CHECK();
  f->wout = reinterpret_cast<float*>(f->dev + o_out);
  f->win = f->dev + convs[ci].off;
  for (int i = 0; i < f->NUP; ++i) {
    f->blk[i].wt = f->dev + convs[idx_t[i]].off;
    for (int j = 0; j < 3; ++j) {
      f->blk[i].ru[j].w7 = f->dev + convs[idx7[i * 3 + j]].off;
      f->blk[i].ru[j].w1 = f->dev + convs[idx1[i * 3 + j]].off;
    }
  }
  FL_HIP(hipStreamSynchronize(st));  // the fold scratch is reused per conv on the same stream; drain before returning
  retire_graph(f->gexec);
  return kOk;
}

FLAMED_API size_t flamed_fac_workspace_size(flamed_fac_t h, int B, int T) {
  Fac* f = reinterpret_cast<Fac*>(h);
  return f ? fac_ws_layout(f, B, T, nullptr, nullptr) : 0;
}

FLAMED_API int flamed_fac_decode(flamed_fac_t h, const float* latents, const float* spk, int B, int T, float* wav,
                                 void* ws, size_t ws_bytes, int use_graph, hipStream_t st) {
  Fac* f = reinterpret_cast<Fac*>(h);
  FL_REQUIRE(f && f->dev, "flamed_fac_decode: handle not loaded");
  FL_REQUIRE(latents && spk && wav && ws && B > 0 && T > 0, "flamed_fac_decode: bad args");
  std::lock_guard<std::mutex> lk(f->mu);
  FL_ON_DEVICE(f->device);
  FL_REQUIRE_ON(latents, f->device, "flamed_fac_decode");
  const Tune tsnap = tune_snapshot(nullptr);
  TuneScope ts_(&tsnap);
  if (ws_bytes < fac_ws_layout(f, B, T, nullptr, nullptr)) {
    set_error("flamed_fac_decode: workspace too small");
    return kNoWorkspace;
  }
  FacWs w;
  fac_ws_layout(f, B, T, ws, &w);
  auto run = [&](hipStream_t s) -> int {
    return f->dt == FLAMED_BF16 ? fac_decode_impl<bf16>(f, latents, spk, B, T, wav, w, s)
                                : fac_decode_impl<float>(f, latents, spk, B, T, wav, w, s);
  };
  if (!use_graph) return run(st);
  std::vector<const void*> key = {latents, spk, wav, ws, (const void*)(intptr_t)B, (const void*)(intptr_t)T, f->dev};
  if (!f->gexec || f->gkey != key) {
    retire_graph(f->gexec);
    if (!f->cap) FL_HIP(hipStreamCreateWithFlags(&f->cap, hipStreamNonBlocking));
    FL_HIP(hipStreamBeginCapture(f->cap, hipStreamCaptureModeRelaxed));
    int r = run(f->cap);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(f->cap, &g);
    if (r) { if (g) (void)hipGraphDestroy(g); return r; }
    FL_HIP(e);
    hipError_t ie = hipGraphInstantiate(&f->gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    FL_HIP(ie);
    f->gkey = key;
  }
  FL_HIP(hipGraphLaunch(f->gexec, st));
  note_graph_use(f->gexec, st);
  return kOk;
}

}  // extern "C"

// ======================================================================================
// FaCodec encoder (prompt encoding): facodec.py:136-244.
//   conv_in WNConv1d(1 -> ngf, k7, p3)                       -> enc_in_kernel (direct, fp32)
//   per EncoderBlock(d, s): 3 x ResidualUnit(d/2, dil 1/3/9)  -> act1d + K-padded conv GEMMs + EpiResAdd
//                           Activation1d + WNConv1d(d/2 -> d, k=2s, stride s, pad ceil(s/2))
//                                                             -> strided-gather GEMM (LoadConvStride)
//   Activation1d + WNConv1d(d -> out, k3, p1)                 -> GEMM, channels-first store (B, out, T)
// Lengths follow Conv1d: n_out = floor((n + 2p - k) / s) + 1 at every stride.
// ======================================================================================
namespace fl {

// Direct Conv1d(1 -> C, k7, pad 3): X[(b*n + t)*C + c] = bias[c] + sum_k w[c][k] wav[b][t + k - 3]
__global__ __launch_bounds__(256) void enc_in_kernel(const float* __restrict__ wav, int n, int C, const float* __restrict__ w,
                                                     const float* __restrict__ bias, float* __restrict__ X, size_t total) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % C;
  const size_t bt = i / C;
  const int t = bt % n;
  const float* wb = wav + (bt - t);
  float acc = bias[c];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int src = t + k - 3;
    if (src >= 0 && src < n) acc += w[c * 7 + k] * wb[src];
  }
  X[i] = acc;
}

// Dilated conv tap gather over a DT activation with K zero-padded to the GEMM K-step: k >= kreal -> 0.
template <typename DT>
struct LoadConvPad {
  const DT* __restrict__ x;
  int Cin, L, KT, dil, kreal;
  struct Raw { u32x4 v; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    if (k >= kreal) return Raw{u32x4{0u, 0u, 0u, 0u}};
    int tap = k / Cin, c = k - tap * Cin;
    int off = (tap - KT / 2) * dil;
    int l = m % L + off;
    if (l < 0 || l >= L) return Raw{u32x4{0u, 0u, 0u, 0u}};
    return Raw{*reinterpret_cast<const u32x4*>(x + (size_t)(m + off) * Cin + c)};
  }
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return r.v; }
};

// Strided conv gather: output row m = (b, o), o < nout; tap t reads x[b][o*s + t - p] (zero outside).
template <typename DT>
struct LoadConvStride {
  const DT* __restrict__ x;
  int Cin, nin, nout, s, p;
  struct Raw { u32x4 v; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    const int b = m / nout, o = m - b * nout;
    const int tap = k / Cin, c = k - tap * Cin;
    const int i = o * s + tap - p;
    if (i < 0 || i >= nin) return Raw{u32x4{0u, 0u, 0u, 0u}};
    return Raw{*reinterpret_cast<const u32x4*>(x + ((size_t)b * nin + i) * Cin + c)};
  }
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return r.v; }
};

// out (B, N, T) channels-first = acc + bias (the encoder's (B, C, T) output layout)
struct EpiStoreCF {
  const float* __restrict__ bias;
  float* __restrict__ out;
  int N, T;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int, int col, float acc, const float*, int) const { return acc + bias[col]; }
  __device__ void store(int m, int col, float v) const {
    const int b = m / T, t = m - b * T;
    out[((size_t)b * N + col) * T + t] = v;
  }
  __device__ void store_stats(int, int, float, float) const {}
};

// N = 32 (the encoder's first stage) runs a 64 x 32 tile; every other width the shape-driven configs.
template <typename DT, class AL, class EP>
static int enc_gemm(const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  if (N % 64 != 0) return launch_gemm_cfg<64, 32, 3, DT>(al, W, ldw, ep, M, N, K, st);
  return launch_gemm<DT>(al, W, ldw, ep, M, N, K, st);
}

struct EncRU { FacAct a1, a2; void* w7; const float* b7; int k7; void* w1; const float* b1; int k1; int dil; };
struct EncBlk { EncRU ru[3]; FacAct a; void* wc; const float* bc; int s, cin, cout; };

struct Enc {
  int ngf, NDN, cout, dt;
  int ratios[8];
  float* w_in = nullptr; const float* b_in = nullptr;
  EncBlk blk[8];
  FacAct afin;
  void* wfin = nullptr; const float* bfin = nullptr;
  int cfin;
  char* dev = nullptr;
  int device = -1;  // device of the arena (from the loaded weights)
  std::mutex mu;    // one call at a time per handle
  hipGraphExec_t gexec = nullptr;
  hipStream_t cap = nullptr;
  std::vector<const void*> gkey;
  void release() {
    retire_graph(gexec);
    if (cap) (void)hipStreamDestroy(cap);
    if (dev) (void)hipFree(dev);
    gexec = nullptr; cap = nullptr; dev = nullptr;
    gkey.clear();
  }
};

static int kpad64(int k) { return (k + 63) / 64 * 64; }

static int enc_len_after(const Enc* e, int n, int upto) {  // sequence length after `upto` blocks
  for (int i = 0; i < upto; ++i) {
    const int s = e->ratios[i], p = s / 2 + s % 2;
    n = (n + 2 * p - 2 * s) / s + 1;
  }
  return n;
}

struct EncWs { float* X; float* Z; void* A; };
static size_t enc_ws_layout(const Enc* e, int B, int n, void* base, EncWs* w) {
  // largest (length x channels) over the stages (block i runs at ngf * 2^i / 2 channels ... d)
  size_t maxcn = (size_t)n * e->ngf;
  int len = n, d = e->ngf;
  for (int i = 0; i < e->NDN; ++i) {
    maxcn = maxcn > (size_t)len * d ? maxcn : (size_t)len * d;
    const int s = e->ratios[i], p = s / 2 + s % 2;
    len = (len + 2 * p - 2 * s) / s + 1;
    d *= 2;
    maxcn = maxcn > (size_t)len * d ? maxcn : (size_t)len * d;
  }
  const size_t es = e->dt == FLAMED_BF16 ? 2 : 4;
  const size_t sizes[3] = {4 * B * maxcn, 4 * B * maxcn, es * B * maxcn};
  size_t off = 0;
  char* p[3];
  for (int i = 0; i < 3; ++i) {
    p[i] = base ? (char*)base + off : nullptr;
    off += al256(sizes[i]);
  }
  if (w) *w = EncWs{(float*)p[0], (float*)p[1], p[2]};
  return off;
}

template <typename DT>
static int enc_impl(Enc* e, const float* wav, int B, int n, float* out, const EncWs& w, hipStream_t st) {
  int rc;
#define TRY(x) do { if ((rc = (x)) != kOk) return rc; } while (0)
  DT* A = reinterpret_cast<DT*>(w.A);
  {
    const size_t total = (size_t)B * n * e->ngf;
    hipLaunchKernelGGL(enc_in_kernel, dim3((total + 255) / 256), dim3(256), 0, st, wav, n, e->ngf, e->w_in, e->b_in, w.X, total);
    FL_LAUNCH_CHECK();
  }
  int len = n;
  for (int i = 0; i < e->NDN; ++i) {
    const EncBlk& bk = e->blk[i];
    const int C = bk.cin;
    for (int j = 0; j < 3; ++j) {
      const EncRU& ru = bk.ru[j];
      TRY(launch_act<DT>(ru.a1, w.X, C, len, B, A, st));
      TRY((enc_gemm<DT>(LoadConvPad<DT>{A, C, len, 7, ru.dil, 7 * C}, (const DT*)ru.w7, ru.k7, EpiBiasAct<float, 0>{ru.b7, w.Z, C},
                        B * len, C, ru.k7, st)));
      TRY(launch_act<DT>(ru.a2, w.Z, C, len, B, A, st));
      TRY((enc_gemm<DT>(LoadConvPad<DT>{A, C, len, 1, 1, C}, (const DT*)ru.w1, ru.k1, EpiResAdd{ru.b1, w.X, C}, B * len, C, ru.k1, st)));
    }
    TRY(launch_act<DT>(bk.a, w.X, C, len, B, A, st));
    const int s = bk.s, p = s / 2 + s % 2;
    const int nout = (len + 2 * p - 2 * s) / s + 1;
    FL_REQUIRE(nout > 0, "flamed_enc_encode: input too short for the stride-%d stage", s);
    TRY((enc_gemm<DT>(LoadConvStride<DT>{A, C, len, nout, s, p}, (const DT*)bk.wc, 2 * s * C, EpiBiasAct<float, 0>{bk.bc, w.X, bk.cout},
                      B * nout, bk.cout, 2 * s * C, st)));
    len = nout;
  }
  const int cf = e->cfin;
  TRY(launch_act<DT>(e->afin, w.X, cf, len, B, A, st));
  TRY((enc_gemm<DT>(LoadConvPad<DT>{A, cf, len, 3, 1, 3 * cf}, (const DT*)e->wfin, kpad64(3 * cf), EpiStoreCF{e->bfin, out, e->cout, len},
                    B * len, e->cout, kpad64(3 * cf), st)));
#undef TRY
  return kOk;
}

}  // namespace fl

extern "C" {

FLAMED_API int flamed_enc_create(int ngf, int n_down, const int* ratios, int out_channels, int dtype, flamed_enc_t* out) {
  FL_REQUIRE(out && ratios, "flamed_enc_create: null args");
  FL_REQUIRE(n_down >= 1 && n_down <= 8, "flamed_enc_create: n_down=%d unsupported", n_down);
  FL_REQUIRE(dtype == FLAMED_F32 || dtype == FLAMED_BF16, "flamed_enc_create: bad dtype");
  FL_REQUIRE(ngf % 32 == 0 && ngf <= 256, "flamed_enc_create: ngf=%d must be a multiple of 32", ngf);
  FL_REQUIRE(out_channels % 64 == 0, "flamed_enc_create: out_channels=%d must be a multiple of 64", out_channels);
  Enc* e = new Enc();
  e->ngf = ngf; e->NDN = n_down; e->cout = out_channels; e->dt = dtype;
  for (int i = 0; i < n_down; ++i) {
    FL_REQUIRE(ratios[i] >= 1 && ratios[i] <= 8, "flamed_enc_create: ratio %d unsupported", ratios[i]);
    e->ratios[i] = ratios[i];
  }
  *out = reinterpret_cast<flamed_enc_t>(e);
  return kOk;
}

FLAMED_API int flamed_enc_destroy(flamed_enc_t h) {
  Enc* e = reinterpret_cast<Enc*>(h);
  if (!e) return kOk;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    DeviceGuard dg(e->device);
    e->release();
  }
  delete e;
  return kOk;
}

FLAMED_API int flamed_enc_num_weights(flamed_enc_t h) {
  Enc* e = reinterpret_cast<Enc*>(h);
  return e ? 3 + FLAMED_ENC_BLOCK_W * e->NDN + 7 : -1;
}

FLAMED_API int flamed_enc_out_len(flamed_enc_t h, int n) {
  Enc* e = reinterpret_cast<Enc*>(h);
  return e ? enc_len_after(e, n, e->NDN) : -1;
}

FLAMED_API int flamed_enc_load(flamed_enc_t h, const float* const* w, int nw, hipStream_t st) {
  Enc* e = reinterpret_cast<Enc*>(h);
  FL_REQUIRE(e && w, "flamed_enc_load: null args");
  FL_REQUIRE(nw == flamed_enc_num_weights(h), "flamed_enc_load: expected %d weights, got %d", flamed_enc_num_weights(h), nw);
  for (int i = 0; i < nw; ++i) FL_REQUIRE(w[i], "flamed_enc_load: weight %d is null", i);
  int wdev = -1;
  FL_REQUIRE(device_of(w[0], &wdev) == kOk, "flamed_enc_load: weights must be device memory");
  for (int i = 1; i < nw; ++i) FL_REQUIRE_ON(w[i], wdev, "flamed_enc_load");
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->device >= 0 && e->device != wdev) {
    DeviceGuard og(e->device);
    e->release();
  }
  e->device = wdev;
  FL_ON_DEVICE(wdev);
  const size_t es = e->dt == FLAMED_BF16 ? 2 : 4;
  VecCopies vc;  // every vector is copied into the arena (the caller may free its tensors)
  auto act = [&](FacAct& a, const float* const* p, int ch) {
    vc.add(p[0], ch, &a.alpha); vc.add(p[1], ch, &a.beta); vc.add(p[2], 12, &a.fu); vc.add(p[3], 12, &a.fd);
  };
  struct Conv { const float *g, *v; int N, Cin, KT, ldk; size_t off; };
  std::vector<Conv> convs;
  size_t off = 0, maxfold = 0;
  auto add = [&](const float* g, const float* v, int N, int Cin, int KT, int ldk) -> int {
    convs.push_back(Conv{g, v, N, Cin, KT, ldk, off});
    off = al256(off + es * (size_t)N * ldk);
    maxfold = maxfold > (size_t)N * Cin * KT ? maxfold : (size_t)N * Cin * KT;
    return (int)convs.size() - 1;
  };
  // conv_in (ngf, 1, 7): folded fp32 for the direct kernel
  const size_t o_in = off;
  off = al256(off + 4ull * e->ngf * 7);
  vc.add(w[2], e->ngf, &e->b_in);
  std::vector<int> i7(e->NDN * 3), i1(e->NDN * 3), ic(e->NDN);
  int d = e->ngf;
  for (int i = 0; i < e->NDN; ++i) {
    const float* const* bw = w + 3 + FLAMED_ENC_BLOCK_W * i;
    EncBlk& bk = e->blk[i];
    bk.cin = d; bk.cout = 2 * d; bk.s = e->ratios[i];
    const int dils[3] = {1, 3, 9};
    for (int j = 0; j < 3; ++j) {
      const float* const* rw = bw + 14 * j;
      EncRU& ru = bk.ru[j];
      ru.dil = dils[j];
      act(ru.a1, rw, d);
      ru.k7 = kpad64(7 * d);
      i7[i * 3 + j] = add(rw[4], rw[5], d, d, 7, ru.k7);
      vc.add(rw[6], d, &ru.b7);
      act(ru.a2, rw + 7, d);
      ru.k1 = kpad64(d);
      i1[i * 3 + j] = add(rw[11], rw[12], d, d, 1, ru.k1);
      vc.add(rw[13], d, &ru.b1);
    }
    act(bk.a, bw + 42, d);
    ic[i] = add(bw[46], bw[47], 2 * d, d, 2 * bk.s, 2 * bk.s * d);
    vc.add(bw[48], 2 * d, &bk.bc);
    d *= 2;
  }
  e->cfin = d;
  const float* const* fw = w + 3 + FLAMED_ENC_BLOCK_W * e->NDN;
  act(e->afin, fw, d);
  const int ifin = add(fw[4], fw[5], e->cout, d, 3, kpad64(3 * d));
  vc.add(fw[6], e->cout, &e->bfin);
  const size_t o_tmp = off;
  off = al256(off + 4 * maxfold);
  const size_t o_vec = off;
  off = al256(off + vc.bytes);
  e->release();
  FL_HIP(hipMalloc(&e->dev, off));
  {
    const int rc = vc.commit(e->dev + o_vec, st);
    if (rc) return rc;
  }
  FL_HIP(hipMemsetAsync(e->dev, 0, o_tmp, st));  // zero K padding of the packed weights
  float* tmp = reinterpret_cast<float*>(e->dev + o_tmp);
  hipLaunchKernelGGL(wn_fold_kernel, dim3(e->ngf), dim3(256), 0, st, w[0], w[1], 7, reinterpret_cast<float*>(e->dev + o_in));
  FL_LAUNCH_CHECK();
  e->w_in = reinterpret_cast<float*>(e->dev + o_in);
  for (const Conv& cv : convs) {
    hipLaunchKernelGGL(wn_fold_kernel, dim3(cv.N), dim3(256), 0, st, cv.g, cv.v, cv.Cin * cv.KT, tmp);
    FL_LAUNCH_CHECK();
    const size_t total = (size_t)cv.N * cv.Cin * cv.KT;
    const dim3 grid((total + 255) / 256);
    if (e->dt == FLAMED_BF16) hipLaunchKernelGGL(pack_conv_kernel<bf16>, grid, dim3(256), 0, st, tmp, (bf16*)(e->dev + cv.off), cv.N, cv.Cin, cv.KT, cv.ldk);
    else hipLaunchKernelGGL(pack_conv_kernel<float>, grid, dim3(256), 0, st, tmp, (float*)(e->dev + cv.off), cv.N, cv.Cin, cv.KT, cv.ldk);
    FL_LAUNCH_CHECK();
  }
  for (int i = 0; i < e->NDN; ++i) {
    for (int j = 0; j < 3; ++j) {
      e->blk[i].ru[j].w7 = e->dev + convs[i7[i * 3 + j]].off;
      e->blk[i].ru[j].w1 = e->dev + convs[i1[i * 3 + j]].off;
    }
    e->blk[i].wc = e->dev + convs[ic[i]].off;
  }
  e->wfin = e->dev + convs[ifin].off;
  FL_HIP(hipStreamSynchronize(st));  // fold scratch reused per conv
  retire_graph(e->gexec);
  return kOk;
}

FLAMED_API size_t flamed_enc_workspace_size(flamed_enc_t h, int B, int n) {
  Enc* e = reinterpret_cast<Enc*>(h);
  return e ? enc_ws_layout(e, B, n, nullptr, nullptr) : 0;
}

FLAMED_API int flamed_enc_encode(flamed_enc_t h, const float* wav, int B, int n, float* out, void* ws, size_t ws_bytes,
                                 int use_graph, hipStream_t st) {
  Enc* e = reinterpret_cast<Enc*>(h);
  FL_REQUIRE(e && e->dev, "flamed_enc_encode: handle not loaded");
  FL_REQUIRE(wav && out && ws && B > 0 && n > 0, "flamed_enc_encode: bad args");
  FL_REQUIRE(enc_len_after(e, n, e->NDN) > 0, "flamed_enc_encode: n=%d too short", n);
  std::lock_guard<std::mutex> lk(e->mu);
  FL_ON_DEVICE(e->device);
  FL_REQUIRE_ON(wav, e->device, "flamed_enc_encode");
  const Tune tsnap = tune_snapshot(nullptr);
  TuneScope ts_(&tsnap);
  if (ws_bytes < enc_ws_layout(e, B, n, nullptr, nullptr)) {
    set_error("flamed_enc_encode: workspace too small");
    return kNoWorkspace;
  }
  EncWs w;
  enc_ws_layout(e, B, n, ws, &w);
  auto run = [&](hipStream_t s) -> int {
    return e->dt == FLAMED_BF16 ? enc_impl<bf16>(e, wav, B, n, out, w, s) : enc_impl<float>(e, wav, B, n, out, w, s);
  };
  if (!use_graph) return run(st);
  std::vector<const void*> key = {wav, out, ws, (const void*)(intptr_t)B, (const void*)(intptr_t)n, e->dev};
  if (!e->gexec || e->gkey != key) {
    retire_graph(e->gexec);
    if (!e->cap) FL_HIP(hipStreamCreateWithFlags(&e->cap, hipStreamNonBlocking));
    FL_HIP(hipStreamBeginCapture(e->cap, hipStreamCaptureModeRelaxed));
    int r = run(e->cap);
    hipGraph_t g = nullptr;
    hipError_t er = hipStreamEndCapture(e->cap, &g);
    if (r) { if (g) (void)hipGraphDestroy(g); return r; }
    FL_HIP(er);
    hipError_t ie = hipGraphInstantiate(&e->gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    FL_HIP(ie);
    e->gkey = key;
  }
  FL_HIP(hipGraphLaunch(e->gexec, st));
  note_graph_use(e->gexec, st);
  return kOk;
}

}  // extern "C"
