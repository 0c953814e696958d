// Prompt-side FaCodec quantizers + timbre encoder on gfx950 (the part after the
// encoder conv stack): FACodecDecoder.forward(vq=True) (reference facodec.py:470-533).
//   * the three residual VQs (prosody, content on x; residual on x - (prosody + content)), each layer a
//     FactorizedVectorQuantize (quantize/fvq.py:35-116): weight-norm in_proj (C -> codebook_dim), L2
//     normalise, nearest normalised code by |e|^2 - 2 e.c + |c|^2 (first index on ties, as max(1)),
//     raw code row, straight-through z_e + (z_q - z_e), weight-norm out_proj, residual update
//     (quantize/rvq.py:27-73) -> one workgroup per frame runs all layers of all groups;
//   * the timbre TransformerEncoder (facodec/transformer.py:154-234; pre-LN layers :86-151, FFN
//     Conv1d(k) -> ReLU -> Linear :54-83), `x + pe[:B]` (the batch index selects the position vector,
//     :49-51), last LayerNorm, mean over time (facodec.py:530-532).
// Exact fp32 (codes must match the reference's argmax; f32 MFMA GEMMs are fp32 FMA chains).
#include "flamed_hip.h"
#include "gemm.hpp"
#include "xfmr.hpp"

#include <mutex>
#include <vector>

namespace fl {

// torch._weight_norm(v, g, dim=0) of a Linear weight: w[o][i] = v[o][i] * (g[o] / ||v[o]||_2).
__global__ void wn_rows_kernel(const float* __restrict__ g, const float* __restrict__ v, float* __restrict__ w, int rows,
                               int cols) {
  int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= rows) return;
  const float* vr = v + (size_t)o * cols;
  float s = 0.f;
  for (int i = 0; i < cols; ++i) s += vr[i] * vr[i];
  const float f = g[o] / sqrtf(s);
  for (int i = 0; i < cols; ++i) w[(size_t)o * cols + i] = vr[i] * f;
}

// F.normalize(codebook) (fvq.py:106) and the row sums of squares of the normalised codes (:110-112).
__global__ void cb_norm_kernel(const float* __restrict__ cb, float* __restrict__ cbn, float* __restrict__ cbsq, int K, int cd) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const float* r = cb + (size_t)k * cd;
  float s = 0.f;
  for (int j = 0; j < cd; ++j) s += r[j] * r[j];
  const float den = fmaxf(sqrtf(s), 1e-12f);
  float q = 0.f;
  for (int j = 0; j < cd; ++j) {
    float e = r[j] / den;
    cbn[(size_t)k * cd + j] = e;
    q += e * e;
  }
  cbsq[k] = q;
}

struct VqLayer {
  const float *win, *bin, *wout, *bout, *cb, *cbn, *cbsq;
  int K;
};
constexpr int kMaxVqLayers = 16;
struct VqParams {
  VqLayer l[kMaxVqLayers];
  int G;
  int nl[4];
};

// One workgroup (C = 256 threads, thread c = channel c) per frame (b, t); CD = codebook_dim.
template <int CD>
__global__ __launch_bounds__(256) void rvq_kernel(VqParams P, const float* __restrict__ x, int B, int T,
                                                  float* __restrict__ outs, int64_t* __restrict__ codes,
                                                  float* __restrict__ qbuf) {
  constexpr int C = 256;
  __shared__ float red[4][CD];
  __shared__ float ze_s[CD];
  __shared__ float bv[4];
  __shared__ int bi[4];
  const int c = threadIdx.x, lane = c & 63, w = c >> 6;
  const int b = blockIdx.x / T, t = blockIdx.x - b * T;
  const size_t at = ((size_t)b * C + c) * T + t;  // (B, C, T) layouts
  const float xv = x[at];
  float gsum[4] = {0.f, 0.f, 0.f, 0.f};  // per-group quantized sums (qbuf)
  int li = 0;
  for (int g = 0; g < P.G; ++g) {
    float r = g < 2 ? xv : xv - (gsum[0] + gsum[1]);  // facodec.py:495-497
    for (int l = 0; l < P.nl[g]; ++l, ++li) {
      const VqLayer& L = P.l[li];
      // z_e = in_proj(r)
      float p[CD];
#pragma unroll
      for (int j = 0; j < CD; ++j) p[j] = wave_sum64(L.win[(size_t)j * C + c] * r);
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < CD; ++j) red[w][j] = p[j];
      }
      __syncthreads();
      if (c < CD) ze_s[c] = ((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) + L.bin[c];
      __syncthreads();
      float ze[CD], nrm = 0.f;
#pragma unroll
      for (int j = 0; j < CD; ++j) {
        ze[j] = ze_s[j];
        nrm += ze[j] * ze[j];
      }
      const float den = fmaxf(sqrtf(nrm), 1e-12f);
      float enc[CD], esq = 0.f;
#pragma unroll
      for (int j = 0; j < CD; ++j) {
        enc[j] = ze[j] / den;
        esq += enc[j] * enc[j];
      }
      // nearest normalised code: max of -dist, lowest index on ties
      float best = -INFINITY;
      int bidx = 0x7fffffff;
      for (int k = c; k < L.K; k += C) {
        const float* cr = L.cbn + (size_t)k * CD;
        float dot = 0.f;
#pragma unroll
        for (int j = 0; j < CD; ++j) dot = fmaf(enc[j], cr[j], dot);
        const float nd = -((esq - 2.f * dot) + L.cbsq[k]);
        if (nd > best) { best = nd; bidx = k; }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        float ov = __shfl_xor(best, o);
        int oi = __shfl_xor(bidx, o);
        if (ov > best || (ov == best && oi < bidx)) { best = ov; bidx = oi; }
      }
      if (lane == 0) { bv[w] = best; bi[w] = bidx; }
      __syncthreads();
      best = bv[0]; bidx = bi[0];
#pragma unroll
      for (int u = 1; u < 4; ++u)
        if (bv[u] > best || (bv[u] == best && bi[u] < bidx)) { best = bv[u]; bidx = bi[u]; }
      // straight-through value z_e + (z_q - z_e) (fvq.py:76-77), then out_proj for channel c
      const float* zq = L.cb + (size_t)bidx * CD;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < CD; ++j) q = fmaf(L.wout[(size_t)c * CD + j], ze[j] + (zq[j] - ze[j]), q);
      q += L.bout[c];
      r = r - q;                                     // rvq.py:60
      gsum[g] = l == 0 ? q : gsum[g] + q;            // rvq.py:62 (0.0 + q is q)
      if (c == 0) codes[((size_t)li * B + b) * T + t] = bidx;
      __syncthreads();  // red / ze_s / bv reuse by the next layer
    }
    qbuf[(size_t)g * B * C * T + at] = gsum[g];
  }
  float o = gsum[0];
  for (int g = 1; g < P.G; ++g) o = o + gsum[g];  // facodec.py:503 outs accumulation
  outs[at] = o;
}

// Timbre encoder input: x (B, C, T) -> rows (B*T, C) + pe[b] (transformer.py:49-51: pe[:x.size(0)]).
__global__ void timbre_in_kernel(const float* __restrict__ x, const float* __restrict__ pe, int B, int C, int T,
                                 float* __restrict__ X) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C * T) return;
  int t = i % T;
  int bc = i / T;
  int c = bc % C, b = bc / C;
  X[((size_t)b * T + t) * C + c] = x[i] + pe[(size_t)b * C + c];
}

// mean over time of the last-LayerNorm rows (facodec.py:531-532): spk[b][c] = sum_t Y[b][t][c] / T.
__global__ void mean_t_kernel(const float* __restrict__ Y, int B, int T, int C, float* __restrict__ spk) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  int b = i / C, c = i - b * C;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += Y[((size_t)b * T + t) * C + c];
  spk[i] = s / (float)T;
}

__global__ void vq_taps_kernel(const float* __restrict__ src, float* __restrict__ dst, int N, int Cin, int KT) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)N * Cin * KT;
  if (i >= total) return;
  int k = i % KT;
  size_t t = i / KT;
  int c = t % Cin;
  int n = t / Cin;
  dst[((size_t)n * KT + k) * Cin + c] = src[i];
}

struct TimbreLayer {
  const float *g1, *b1, *wqkv, *bqkv, *wo, *bo, *g2, *b2, *w1, *c1b, *w2, *c2b;
};

struct PromptVq {
  int C = 0, cd = 0, G = 0, nl[4] = {0, 0, 0, 0}, K[4] = {0, 0, 0, 0};
  int d = 0, heads = 0, F = 0, k = 0, pe_len = 0;
  int device = -1;
  std::mutex mu;
  char* dev = nullptr;
  VqParams vp;
  const float* pe = nullptr;
  std::vector<TimbreLayer> tl;
  const float *lg = nullptr, *lb = nullptr;
  CapGraph graph;
  int n_vq_layers() const { int s = 0; for (int g = 0; g < G; ++g) s += nl[g]; return s; }
};

static size_t a256p(size_t x) { return (x + 255) & ~(size_t)255; }

struct VqWs {
  float *X, *R, *H, *QKV, *O, *Hf;
};
static size_t vq_ws_layout(const PromptVq* p, int B, int T, void* base, VqWs* w) {
  const size_t M = (size_t)B * T;
  size_t sizes[6] = {4 * M * p->d, 4 * M * p->d, 4 * M * p->d, 12 * M * p->d, 4 * M * p->d, 4 * M * p->F};
  size_t off = 0;
  float* q[6];
  for (int i = 0; i < 6; ++i) {
    q[i] = base ? (float*)((char*)base + off) : nullptr;
    off += a256p(sizes[i]);
  }
  if (w) *w = VqWs{q[0], q[1], q[2], q[3], q[4], q[5]};
  return off;
}

static int run_vq(PromptVq* p, const float* x, int B, int T, float* outs, int64_t* codes, float* qbuf, float* spk,
                  const VqWs& w, hipStream_t st) {
  hipLaunchKernelGGL(rvq_kernel<8>, dim3(B * T), dim3(256), 0, st, p->vp, x, B, T, outs, codes, qbuf);
  FL_LAUNCH_CHECK();
  const int M = B * T, d = p->d, F = p->F;
  hipLaunchKernelGGL(timbre_in_kernel, dim3((B * d * T + 255) / 256), dim3(256), 0, st, x, p->pe, B, d, T, w.X);
  FL_LAUNCH_CHECK();
  float* X = w.X;
  float* R = w.R;
  int rc;
  for (const TimbreLayer& L : p->tl) {  // pre-LN layer, transformer.py:122-151
    if ((rc = ln_mask(d, X, L.g1, L.b1, nullptr, w.H, M, T, nullptr, 0, 0, 0, 0, st))) return rc;
    if ((rc = xf_gemm(LoadF32<float>{w.H, d}, L.wqkv, d, EpiBiasAct<float, 0>{L.bqkv, w.QKV, 3 * d}, M, 3 * d, d, st))) return rc;
    if ((rc = attention(d / p->heads, w.QKV, nullptr, B, T, d, p->heads, w.O, st))) return rc;
    if ((rc = xf_gemm(LoadF32<float>{w.O, d}, L.wo, d, EpiBiasRes{L.bo, X, R, d}, M, d, d, st))) return rc;
    std::swap(X, R);
    if ((rc = ln_mask(d, X, L.g2, L.b2, nullptr, w.H, M, T, nullptr, 0, 0, 0, 0, st))) return rc;
    if ((rc = xf_gemm(LoadConvRows<float, false>{w.H, d, T, p->k, 1, nullptr, 0, 0, 0.f, nullptr, nullptr}, L.w1,
                                 p->k * d, EpiBiasAct<float, 3>{L.c1b, w.Hf, F}, M, F, p->k * d, st)))
      return rc;
    if ((rc = xf_gemm(LoadF32<float>{w.Hf, F}, L.w2, F, EpiBiasRes{L.c2b, X, R, d}, M, d, F, st))) return rc;
    std::swap(X, R);
  }
  if ((rc = ln_mask(d, X, p->lg, p->lb, nullptr, w.H, M, T, nullptr, 0, 0, 0, 0, st))) return rc;
  hipLaunchKernelGGL(mean_t_kernel, dim3((B * d + 255) / 256), dim3(256), 0, st, w.H, B, T, d, spk);
  FL_LAUNCH_CHECK();
  return kOk;
}

}  // namespace fl

using namespace fl;

extern "C" {

FLAMED_API int flamed_vq_create(const int* d, int nd, flamed_vq_t* out) {
  FL_REQUIRE(out && d && nd >= 3, "flamed_vq_create: bad dims");
  const int G = d[2];
  FL_REQUIRE(G >= 1 && G <= 4 && nd == 3 + 2 * G + 6, "flamed_vq_create: expected %d dims", 3 + 2 * G + 6);
  PromptVq* p = new PromptVq();
  p->C = d[0]; p->cd = d[1]; p->G = G;
  for (int g = 0; g < G; ++g) { p->nl[g] = d[3 + g]; p->K[g] = d[3 + G + g]; }
  const int* t = d + 3 + 2 * G;
  p->d = t[0]; p->heads = t[1]; p->F = t[2]; p->k = t[3]; p->pe_len = t[5];
  p->tl.resize(t[4] > 0 ? t[4] : 0);
  bool ok = p->C == 256 && p->cd == 8 && p->d == p->C && p->heads > 0 && p->d % p->heads == 0 &&
            (p->d / p->heads == 32 || p->d / p->heads == 48 || p->d / p->heads == 64) && p->F % 64 == 0 && (p->k & 1) &&
            p->pe_len > 0 && p->n_vq_layers() <= kMaxVqLayers && t[4] >= 0;
  for (int g = 0; g < G; ++g) ok = ok && p->nl[g] >= 1 && p->K[g] >= 1;
  if (!ok) {
    delete p;
    FL_REQUIRE(false, "flamed_vq_create: unsupported dims (C=256, codebook_dim=8, timbre hidden = C, head width 32/48/64)");
  }
  p->vp.G = G;
  for (int g = 0; g < G; ++g) p->vp.nl[g] = p->nl[g];
  *out = reinterpret_cast<flamed_vq_t>(p);
  return kOk;
}

FLAMED_API int flamed_vq_destroy(flamed_vq_t h) {
  PromptVq* p = reinterpret_cast<PromptVq*>(h);
  if (!p) return kOk;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceGuard dg(p->device);
    p->graph.release();
    if (p->dev) (void)hipFree(p->dev);
  }
  delete p;
  return kOk;
}

FLAMED_API int flamed_vq_num_weights(flamed_vq_t h) {
  PromptVq* p = reinterpret_cast<PromptVq*>(h);
  return p ? 7 * p->n_vq_layers() + 1 + 12 * (int)p->tl.size() + 2 : -1;
}

FLAMED_API int flamed_vq_load(flamed_vq_t h, const float* const* w, int nw, hipStream_t st) {
  PromptVq* p = reinterpret_cast<PromptVq*>(h);
  FL_REQUIRE(p && w, "flamed_vq_load: null handle / weights");
  FL_REQUIRE(nw == flamed_vq_num_weights(h), "flamed_vq_load: expected %d weights, got %d", flamed_vq_num_weights(h), nw);
  for (int i = 0; i < nw; ++i) FL_REQUIRE(w[i], "flamed_vq_load: weight %d is null", i);
  int wdev = -1;
  FL_REQUIRE(device_of(w[0], &wdev) == kOk, "flamed_vq_load: weights must be device memory");
  for (int i = 1; i < nw; ++i) FL_REQUIRE_ON(w[i], wdev, "flamed_vq_load");
  std::lock_guard<std::mutex> lk(p->mu);
  if (p->device >= 0 && p->device != wdev) {
    DeviceGuard og(p->device);
    p->graph.release();
    if (p->dev) { (void)hipFree(p->dev); p->dev = nullptr; }
  }
  p->device = wdev;
  FL_ON_DEVICE(wdev);
  p->graph.release();
  if (p->dev) { FL_HIP(hipFree(p->dev)); p->dev = nullptr; }
  const int C = p->C, cd = p->cd, d = p->d, F = p->F, k = p->k;
  // packed region: per VQ layer folded in/out weights, normalised codebook, code norms; per timbre layer
  // the tap-major conv weight
  size_t off = 0;
  std::vector<size_t> o_win, o_wout, o_cbn, o_cbsq, o_w1;
  for (int g = 0, li = 0; g < p->G; ++g)
    for (int l = 0; l < p->nl[g]; ++l, ++li) {
      o_win.push_back(off); off += a256p(4ull * cd * C);
      o_wout.push_back(off); off += a256p(4ull * C * cd);
      o_cbn.push_back(off); off += a256p(4ull * p->K[g] * cd);
      o_cbsq.push_back(off); off += a256p(4ull * p->K[g]);
    }
  for (size_t i = 0; i < p->tl.size(); ++i) { o_w1.push_back(off); off += a256p(4ull * F * k * d); }
  VecCopies vc;
  int i = 0;
  for (int g = 0, li = 0; g < p->G; ++g)
    for (int l = 0; l < p->nl[g]; ++l, ++li) {
      VqLayer& L = p->vp.l[li];
      L.K = p->K[g];
      vc.add(w[i + 2], cd, &L.bin);
      vc.add(w[i + 5], C, &L.bout);
      vc.add(w[i + 6], (size_t)p->K[g] * cd, &L.cb);
      i += 7;
    }
  vc.add(w[i++], (size_t)p->pe_len * d, &p->pe);
  for (TimbreLayer& L : p->tl) {
    vc.add(w[i + 0], d, &L.g1); vc.add(w[i + 1], d, &L.b1);
    vc.add(w[i + 2], 3ull * d * d, &L.wqkv); vc.add(w[i + 3], 3ull * d, &L.bqkv);
    vc.add(w[i + 4], (size_t)d * d, &L.wo); vc.add(w[i + 5], d, &L.bo);
    vc.add(w[i + 6], d, &L.g2); vc.add(w[i + 7], d, &L.b2);
    vc.add(w[i + 9], F, &L.c1b);
    vc.add(w[i + 10], (size_t)d * F, &L.w2); vc.add(w[i + 11], d, &L.c2b);
    i += 12;
  }
  vc.add(w[i], d, &p->lg);
  vc.add(w[i + 1], d, &p->lb);
  FL_HIP(hipMalloc(&p->dev, a256p(off) + a256p(vc.bytes)));
  char* base = p->dev;
  i = 0;
  for (int g = 0, li = 0; g < p->G; ++g)
    for (int l = 0; l < p->nl[g]; ++l, ++li) {
      VqLayer& L = p->vp.l[li];
      float* win = (float*)(base + o_win[li]);
      float* wout = (float*)(base + o_wout[li]);
      float* cbn = (float*)(base + o_cbn[li]);
      float* cbsq = (float*)(base + o_cbsq[li]);
      hipLaunchKernelGGL(wn_rows_kernel, dim3(1), dim3(64), 0, st, w[i + 0], w[i + 1], win, cd, C);
      hipLaunchKernelGGL(wn_rows_kernel, dim3((C + 63) / 64), dim3(64), 0, st, w[i + 3], w[i + 4], wout, C, cd);
      hipLaunchKernelGGL(cb_norm_kernel, dim3((p->K[g] + 255) / 256), dim3(256), 0, st, w[i + 6], cbn, cbsq, p->K[g], cd);
      FL_LAUNCH_CHECK();
      L.win = win; L.wout = wout; L.cbn = cbn; L.cbsq = cbsq;
      i += 7;
    }
  i += 1;
  for (size_t li = 0; li < p->tl.size(); ++li) {
    float* w1 = (float*)(base + o_w1[li]);
    const size_t n = (size_t)F * d * k;
    hipLaunchKernelGGL(vq_taps_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w[i + 8], w1, F, d, k);
    FL_LAUNCH_CHECK();
    p->tl[li].w1 = w1;
    i += 12;
  }
  return vc.commit(base + a256p(off), st);
}

FLAMED_API size_t flamed_vq_workspace_size(flamed_vq_t h, int B, int T) {
  PromptVq* p = reinterpret_cast<PromptVq*>(h);
  return p ? vq_ws_layout(p, B, T, nullptr, nullptr) : 0;
}

FLAMED_API int flamed_vq_encode(flamed_vq_t h, const float* x, int B, int T, float* outs, int64_t* codes, float* qbuf,
                                float* spk, void* ws, size_t ws_bytes, int use_graph, hipStream_t st) {
  PromptVq* p = reinterpret_cast<PromptVq*>(h);
  FL_REQUIRE(p && p->dev, "flamed_vq_encode: handle not loaded");
  FL_REQUIRE(x && outs && codes && qbuf && spk && ws && B > 0 && T > 0, "flamed_vq_encode: bad args");
  FL_REQUIRE(B <= p->pe_len, "flamed_vq_encode: B=%d exceeds the position table (%d rows)", B, p->pe_len);
  std::lock_guard<std::mutex> lk(p->mu);
  FL_ON_DEVICE(p->device);
  FL_REQUIRE_ON(x, p->device, "flamed_vq_encode");
  const Tune tsnap = tune_snapshot(nullptr);
  TuneScope ts_(&tsnap);
  if (ws_bytes < vq_ws_layout(p, B, T, nullptr, nullptr)) {
    set_error("flamed_vq_encode: workspace too small");
    return kNoWorkspace;
  }
  VqWs w;
  vq_ws_layout(p, B, T, ws, &w);
  std::vector<const void*> key = {x, outs, codes, qbuf, spk, ws, (const void*)(intptr_t)B, (const void*)(intptr_t)T, p->dev};
  return with_graph(p->graph, key, use_graph != 0, st,
                    [&](hipStream_t s) { return run_vq(p, x, B, T, outs, codes, qbuf, spk, w, s); });
}

}  // extern "C"
