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
#include <cstring>
#include "flamed_hip.h"
#include "flamed_diag.h"
#include "gemm.hpp"
#include "gemm_dma.hpp"
#include "gemm_8p.hpp"
#include "persist.hpp"

#include <mutex>
#include <string>
#include <vector>

namespace fl {

// Below kTinyRows rows (tune bn32 1, default) the denoiser GEMMs use 32 x 32 tiles: measured at B = 1
// (profiles/r01_dma_ab.txt) 34.6 vs 37.5 ms/solve at T = 131, but 41.9 vs 40.5 at T = 400.
constexpr int kTinyRows = 320;
// Knob notes (values live in Tune, common.hpp; set by flamed_tune / flamed_den_tune):
//   use_dma 1: small-M bf16 GEMMs whose A operand is bf16 run on the LDS-DMA pipeline (gemm_dma.hpp),
//     2 also those with fp32 (transforming) A loaders; in-graph per-launch costs at B = 1
//     (profiles/r01_dma_ab.txt): no gain for 2.
//   dma_ns: at M = 400, K = 1024 with the step's weights streaming from MALL (tools/probe_gemm.py, 24
//     weight buffers) 3 stages 6.48 us, 4: 6.70, 8: 7.14, 2: 8.36 per launch.

// Diagnostic stamps (FL_STAMPS builds): kernels of class tn().stamp_class point fl_stamp_buf at g_stamp_dev.
#ifdef FL_STAMPS
static unsigned long long* g_stamp_dev = nullptr;
static void stamp_select(int cls, hipStream_t st) {
  unsigned long long* p = (cls == tn().stamp_class) ? g_stamp_dev : nullptr;
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(fl_stamp_buf), &p, sizeof(p), 0, hipMemcpyHostToDevice, st);
}
#else
static void stamp_select(int, hipStream_t) {}
#endif

// ------------------------------ denoiser loaders / epilogues ------------------------------

// Device-side Euler step index (graph replay of a few captured steps, see flamed_den_solve): the
// modulation rows of step s live at mods + s * stride; a null `step` means offset 0.
struct StepOff {
  const int* __restrict__ step;
  long long stride;
  __device__ __forceinline__ long long get() const { return step ? (long long)(*step) * stride : 0; }
};

struct ModRef {  // AdaLN modulation vectors: row = m / div, stride `ms` floats
  const float* __restrict__ sh;
  const float* __restrict__ sc;
  int ms;
  int div;
  StepOff so;
  __device__ __forceinline__ ModRef at() const {  // pointers advanced to the current step
    const long long o = so.get();
    return ModRef{sh + o, sc + o, ms, div, StepOff{nullptr, 0}};
  }
};

// LayerNorm (+ optional affine) + AdaLN modulate of fp32 rows, converted to DT (A-operand loader).
// Row stats come from the producer's partials; the per-column modulation vectors
// alpha = w (1 + scale), beta = b (1 + scale) + shift are staged once per workgroup in LDS for the
// (at most two) modulation rows the tile touches; otherwise (per-frame t, or T < tile) each chunk
// is transformed straight from global memory.
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
  int kdim;  // K: columns staged per vector
  const bf16* x16 = nullptr;  // large-M x16 path: the bf16 residual rows (normalise pass only; x unused)
  static constexpr int EPC = DTraits<DT>::EPC;
  static constexpr int kSrcBytes = 4;
  __device__ const char* src_row(int m) const { return reinterpret_cast<const char*>(x + (size_t)m * ld); }
  // DMA-path transform: row statistics and the vector slot are per-thread constants of the K loop;
  // per K-step only alpha/beta (two float4 pairs from LDS) change.
  struct XRow { float mean, rstd; int voff, m; bool use; };
  __device__ XRow xrow(int m, const float* st, const float*, bool use, int bm) const {
    const int slot = use ? m / mod.div - bm / mod.div : 0;
    return XRow{st[2 * (m - bm)], st[2 * (m - bm) + 1], 2 * slot * kdim, m, use};
  }
  template <typename D, typename R>
  __device__ u32x4 xform(const XRow& xr, const R& r, int k, const float* st, const float* vec, int bm) const {
    if (!xr.use) return finish_v<D>(r, xr.m, k, st, vec, false, bm);
    const float* va = vec + xr.voff + k;
    const float* vb = va + kdim;
    const float4 a0 = ld4(va), a1 = ld4(va + 4), b0 = ld4(vb), b1 = ld4(vb + 4);
    const float al[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float be[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    float o[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) o[j] = ((r.v[j] - xr.mean) * xr.rstd) * al[j] + be[j];
    return pack_chunk<D>(o);
  }
  static constexpr int kVec = 4;  // 2 slots x (alpha, beta)
  struct Raw { float v[EPC]; };
  static constexpr int stat_rows(int BM) { return BM; }
  // Staging loads (float4, two passes kept in registers) are issued before the row statistics' loads
  // so both groups are in flight together.
  __device__ bool prologue_v(int bm, int BM, int M, int K, float* st, float* vec) const {
    const int last = (bm + BM - 1 < M ? bm + BM - 1 : M - 1);
    const int r0 = bm / mod.div, r1 = last / mod.div;
    const bool ok = r1 - r0 <= 1;
    const int K4 = K / 4, n4 = ok ? (r1 - r0 + 1) * K4 : 0;
    const ModRef md = mod.at();
    constexpr int P = 2;
    float4 sc[P], sh[P], w[P], b[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int q = threadIdx.x + p * blockDim.x;
      if (q < n4) {
        const int slot = q / K4, k = (q - slot * K4) * 4;
        const size_t mo = (size_t)(r0 + slot) * md.ms + k;
        sc[p] = ld4(md.sc + mo);
        sh[p] = ld4(md.sh + mo);
        w[p] = AFF ? ld4(lnw + k) : make_float4(1.f, 1.f, 1.f, 1.f);
        b[p] = AFF ? ld4(lnb + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    for (int r = threadIdx.x; r < BM; r += blockDim.x) {
      int m = bm + r;
      m = m < M ? m : M - 1;
      row_stats_from_partials(S, m, NT, tw, eps, st[2 * r], st[2 * r + 1]);
    }
    auto put = [&](int q, float4 c, float4 h, float4 ww, float4 bb) {
      const int slot = q / K4, k = (q - slot * K4) * 4;
      const float4 s1 = make_float4(1.f + c.x, 1.f + c.y, 1.f + c.z, 1.f + c.w);
      *reinterpret_cast<float4*>(vec + (size_t)(2 * slot) * K + k) = make_float4(ww.x * s1.x, ww.y * s1.y, ww.z * s1.z, ww.w * s1.w);
      *reinterpret_cast<float4*>(vec + (size_t)(2 * slot + 1) * K + k) =
          make_float4(bb.x * s1.x + h.x, bb.y * s1.y + h.y, bb.z * s1.z + h.z, bb.w * s1.w + h.w);
    };
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int q = threadIdx.x + p * blockDim.x;
      if (q < n4) put(q, sc[p], sh[p], w[p], b[p]);
    }
    for (int q = threadIdx.x + P * blockDim.x; q < n4; q += blockDim.x) {  // K > 2 * 4 * blockDim / slots
      const int slot = q / K4, k = (q - slot * K4) * 4;
      const size_t mo = (size_t)(r0 + slot) * md.ms + k;
      put(q, ld4(md.sc + mo), ld4(md.sh + mo), AFF ? ld4(lnw + k) : make_float4(1.f, 1.f, 1.f, 1.f),
          AFF ? ld4(lnb + k) : make_float4(0.f, 0.f, 0.f, 0.f));
    }
    return ok;
  }
  __device__ Raw issue_v(int m, int k) const {
    Raw r;
    const float* px = x + (size_t)m * ld + k;
#pragma unroll
    for (int j = 0; j < EPC; j += 4) {
      float4 a = ld4(px + j);
      r.v[j] = a.x; r.v[j + 1] = a.y; r.v[j + 2] = a.z; r.v[j + 3] = a.w;
    }
    return r;
  }
  template <typename D>
  __device__ u32x4 finish_v(const Raw& r, int m, int k, const float* st, const float* vec, bool use, int bm) const {
    const float mean = st[2 * (m - bm)], rstd = st[2 * (m - bm) + 1];
    float o[EPC];
    if (use) {
      const int slot = m / mod.div - bm / mod.div;
      const float* va = vec + (size_t)(2 * slot) * kdim + k;
      const float* vb = vec + (size_t)(2 * slot + 1) * kdim + k;
#pragma unroll
      for (int j = 0; j < EPC; ++j) o[j] = ((r.v[j] - mean) * rstd) * va[j] + vb[j];
    } else {  // rare path (per-frame t or tiles spanning > 2 modulation rows): vectors from global
      const ModRef md = mod.at();
      size_t mo = (size_t)(m / md.div) * md.ms + k;
#pragma unroll
      for (int j = 0; j < EPC; ++j) {
        float sc1 = 1.0f + md.sc[mo + j];
        float w = AFF ? lnw[k + j] : 1.0f, b = AFF ? lnb[k + j] : 0.0f;
        o[j] = ((r.v[j] - mean) * rstd) * (w * sc1) + (b * sc1 + md.sh[mo + j]);
      }
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
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return pack_chunk<D>(r.v); }
};

// X = X + gate * (h + acc + b3), h = LN(X)(+affine) * (1 + sc) + sh recomputed from the same
// stats the dwconv prologue used; emits LN partials of the new X.  Per-column vectors
// [alpha, beta, gate] x 2 modulation rows + b3 are staged in LDS (kEVec = 8 floats per column).
template <bool AFF, typename XT = float>  // XT: residual stream type (bf16 on the large-M x16 path)
struct EpiConvNeXtResid {
  const float* __restrict__ b3;
  XT* X;
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
  // LayerNorm fold of the consumer (bf16 handles, else ya = null): ya = bf16(X_new * alpha_next),
  // alpha_next = yw (1 + ysc) of the next LayerNorm + modulation (rows as `mod`)
  bf16* __restrict__ ya = nullptr;
  const float* __restrict__ yw = nullptr;
  const float* __restrict__ ysc = nullptr;
  static constexpr bool kRowStats = true;
  static constexpr bool kPre = true;  // X[m][n] prefetched before the main loop
  static constexpr int kEVec = 9;  // fields x kEVecStride floats in LDS
  static constexpr int stat_rows(int BM) { return BM; }
  __device__ float pre(int m, int n) const { return (float)X[(size_t)m * ld + n]; }
  __device__ void pre4(int m, int n, float* x) const {
    const float4 v = ldx4<XT>(X + (size_t)m * ld + n);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
  __device__ bool prologue_v(int bm, int bn, int BM, int BN, int M, float* st, float* vec) const {
    const int last = (bm + BM - 1 < M ? bm + BM - 1 : M - 1);
    const int r0 = bm / mod.div, r1 = last / mod.div;
    const bool ok = r1 - r0 <= 1;
    const int cnt = ok ? (r1 - r0 + 1) * BN : 0;
    const long long so = mod.so.get();
    const ModRef md = mod.at();
    // this thread's staging values (one pass: cnt <= 2 * BN <= blockDim) load before the row statistics
    const int idx = threadIdx.x;
    float sc1 = 0.f, shv = 0.f, gv = 0.f, w = 1.f, b = 0.f, b3v = 0.f, al = 1.f;
    int slot = 0, c = 0;
    if (idx < cnt) {
      slot = idx / BN; c = idx - slot * BN;
      const int n = bn + c;
      const size_t mo = (size_t)(r0 + slot) * md.ms + n;
      sc1 = 1.0f + md.sc[mo];
      shv = md.sh[mo];
      gv = gate[so + mo];
      if (AFF) { w = lnw[n]; b = lnb[n]; }
      b3v = b3[n];
      if (ya) al = (yw ? yw[n] : 1.0f) * (1.0f + ysc[so + mo]);
    }
    for (int r = threadIdx.x; r < BM; r += blockDim.x) {
      int m = bm + r;
      m = m < M ? m : M - 1;
      row_stats_from_partials(Sin, m, NTin, twin, eps, st[2 * r], st[2 * r + 1]);
    }
    constexpr int S = kEVecStride;  // field-major (structure of arrays): a row's lanes read consecutive columns
    if (idx < cnt) {
      vec[(slot * 3 + 0) * S + c] = w * sc1;
      vec[(slot * 3 + 1) * S + c] = __builtin_fmaf(b, sc1, shv);
      vec[(slot * 3 + 2) * S + c] = gv;
      if (slot == 0) vec[6 * S + c] = b3v;
      vec[(7 + slot) * S + c] = al;
    }
    for (int q = idx + blockDim.x; q < cnt; q += blockDim.x) {  // BN > blockDim / 2 (not used by the tile configs)
      const int sl = q / BN, cc = q - sl * BN, n = bn + cc;
      const size_t mo = (size_t)(r0 + sl) * md.ms + n;
      const float s1 = 1.0f + md.sc[mo];
      vec[(sl * 3 + 0) * S + cc] = (AFF ? lnw[n] : 1.0f) * s1;
      vec[(sl * 3 + 1) * S + cc] = __builtin_fmaf(AFF ? lnb[n] : 0.0f, s1, md.sh[mo]);
      vec[(sl * 3 + 2) * S + cc] = gate[so + mo];
      if (sl == 0) vec[6 * S + cc] = b3[n];
      vec[(7 + sl) * S + cc] = ya ? (yw ? yw[n] : 1.0f) * (1.0f + ysc[so + mo]) : 1.0f;
    }
    return ok;
  }
  // Every rounding is explicit (no contraction left to the compiler), so the staged path (`use`: the tile spans <= 2
  // modulation rows) and the direct path give the same bits, whichever GEMM tile family a batch split selects:
  //   va = w sc1, vb = fma(b, sc1, sh), h = fma(xh, va, vb), out = fma(gate, h + (acc + b3), x)
  static __device__ __forceinline__ float cnx_out(float x, float xh, float va, float vb, float g, float acc, float b3v) {
#pragma clang fp contract(off)
    const float h = __builtin_fmaf(xh, va, vb);
    return __builtin_fmaf(g, h + (acc + b3v), x);
  }
  __device__ float value_v(int m, int n, float acc, const float* st, const float* vec, bool use, int bm, int bn, float x) const {
#pragma clang fp contract(off)
    float xh = (x - st[2 * (m - bm)]) * st[2 * (m - bm) + 1];
    if (use) {
      constexpr int S = kEVecStride;
      const int slot = m / mod.div - bm / mod.div;
      const float* v = vec + slot * 3 * S + (n - bn);
      return cnx_out(x, xh, v[0], v[S], v[2 * S], acc, vec[6 * S + (n - bn)]);
    }
    const long long so = mod.so.get();
    const ModRef md = mod.at();
    size_t mo = (size_t)(m / md.div) * md.ms + n;
    float sc1 = 1.0f + md.sc[mo];
    float w = AFF ? lnw[n] : 1.0f, b = AFF ? lnb[n] : 0.0f;
    return cnx_out(x, xh, w * sc1, __builtin_fmaf(b, sc1, md.sh[mo]), gate[so + mo], acc, b3[n]);
  }
  // four consecutive columns (n % 4 == 0), the staged vectors read as float4 (gemm_dma.hpp value4_pre); value_v's
  // expression per column
  __device__ void value4_v(int m, int n, const float* acc, const float* st, const float* vec, bool use, int bm, int bn,
                           const float* x, float* out) const {
    if (!use) {
#pragma unroll
      for (int e = 0; e < 4; ++e) out[e] = value_v(m, n + e, acc[e], st, vec, use, bm, bn, x[e]);
      return;
    }
    constexpr int S = kEVecStride;
    const float mean = st[2 * (m - bm)], rstd = st[2 * (m - bm) + 1];
    const int slot = m / mod.div - bm / mod.div;
    const float* v = vec + slot * 3 * S + (n - bn);
    const float4 va = *reinterpret_cast<const float4*>(v), vb = *reinterpret_cast<const float4*>(v + S);
    const float4 vg = *reinterpret_cast<const float4*>(v + 2 * S), v3 = *reinterpret_cast<const float4*>(vec + 6 * S + (n - bn));
    const float a4[4] = {va.x, va.y, va.z, va.w}, b4[4] = {vb.x, vb.y, vb.z, vb.w};
    const float g4[4] = {vg.x, vg.y, vg.z, vg.w}, c4[4] = {v3.x, v3.y, v3.z, v3.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma clang fp contract(off)
      const float xh = (x[e] - mean) * rstd;
      out[e] = cnx_out(x[e], xh, a4[e], b4[e], g4[e], acc[e], c4[e]);
    }
  }
  // alpha_next of column n for row m (staged, or from the mods table)
  __device__ float alpha_next(int m, int n, const float* vec, bool use, int bm, int bn) const {
    if (use) return vec[(7 + m / mod.div - bm / mod.div) * kEVecStride + (n - bn)];
    const size_t mo = (size_t)(m / mod.div) * mod.ms + n;
    return (yw ? yw[n] : 1.0f) * (1.0f + ysc[mod.so.get() + mo]);
  }
  static constexpr bool kStoreV = true;
  __device__ void store_v(int m, int n, float v, const float* vec, bool use, int bm, int bn) const {
    store_val<XT>(X + (size_t)m * ld + n, v);
    if (ya) ya[(size_t)m * ld + n] = (bf16)(v * alpha_next(m, n, vec, use, bm, bn));
  }
  __device__ void store4_v(int m, int n, const float* v, const float* vec, bool use, int bm, int bn) const {
    store_val4<XT>(X + (size_t)m * ld + n, v);
    if (ya) {
      float y[4];
      if (use && (n - bn) % 4 == 0) {  // the staged alpha row as one float4
        const float4 a = *reinterpret_cast<const float4*>(vec + (7 + m / mod.div - bm / mod.div) * kEVecStride + (n - bn));
        y[0] = v[0] * a.x; y[1] = v[1] * a.y; y[2] = v[2] * a.z; y[3] = v[3] * a.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = v[e] * alpha_next(m, n + e, vec, use, bm, bn);
      }
      store_val4<bf16>(ya + (size_t)m * ld + n, y);
    }
  }
  __device__ void store(int m, int n, float v) const { store_val<XT>(X + (size_t)m * ld + n, v); }
  __device__ void store4(int m, int n, const float* v) const { store_val4<XT>(X + (size_t)m * ld + n, v); }
  __device__ void store_stats(int m, int nt, float mean, float m2) const {
    reinterpret_cast<float2*>(Sout)[(size_t)m * NTout + nt] = make_float2(mean, m2);
  }
};

template <typename XT = float>
struct EpiGatedResidT {  // X = X + gate * (acc + b); [gate x 2 rows, b] staged per column
  const float* __restrict__ b;
  XT* X;
  int ld;
  const float* __restrict__ gate;
  int ms, div;
  float* __restrict__ Sout;
  int NTout;
  StepOff so;
  static constexpr bool kRowStats = true;
  static constexpr bool kPre = true;  // X[m][n] prefetched before the main loop
  static constexpr int kEVec = 4;
  static constexpr int stat_rows(int) { return 0; }
  __device__ float pre(int m, int n) const { return (float)X[(size_t)m * ld + n]; }
  __device__ void pre4(int m, int n, float* x) const {
    const float4 v = ldx4<XT>(X + (size_t)m * ld + n);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
  __device__ bool prologue_v(int bm, int bn, int BM, int BN, int M, float*, float* vec) const {
    const int last = (bm + BM - 1 < M ? bm + BM - 1 : M - 1);
    const int r0 = bm / div, r1 = last / div;
    if (r1 - r0 > 1) return false;
    const float* g = gate + so.get();
    for (int idx = threadIdx.x; idx < (r1 - r0 + 1) * BN; idx += blockDim.x) {  // field-major, as EpiConvNeXtResid
      int slot = idx / BN, c = idx - slot * BN, n = bn + c;
      vec[slot * kEVecStride + c] = g[(size_t)(r0 + slot) * ms + n];
      if (slot == 0) vec[2 * kEVecStride + c] = b[n];
    }
    return true;
  }
  __device__ float value_v(int m, int n, float acc, const float*, const float* vec, bool use, int bm, int bn, float x) const {
    // out = fma(gate, acc + b, x) with explicit roundings: the staged and direct paths give the same bits
    if (use) {
      return __builtin_fmaf(vec[(m / div - bm / div) * kEVecStride + (n - bn)], acc + vec[2 * kEVecStride + (n - bn)], x);
    }
    return __builtin_fmaf(gate[so.get() + (size_t)(m / div) * ms + n], acc + b[n], x);
  }
  // four consecutive columns (n % 4 == 0), the staged gate and bias read as float4; value_v's expression per column
  __device__ void value4_v(int m, int n, const float* acc, const float* st, const float* vec, bool use, int bm, int bn,
                           const float* x, float* out) const {
    if (!use) {
#pragma unroll
      for (int e = 0; e < 4; ++e) out[e] = value_v(m, n + e, acc[e], st, vec, use, bm, bn, x[e]);
      return;
    }
    const float4 g = *reinterpret_cast<const float4*>(vec + (m / div - bm / div) * kEVecStride + (n - bn));
    const float4 bb = *reinterpret_cast<const float4*>(vec + 2 * kEVecStride + (n - bn));
    const float g4[4] = {g.x, g.y, g.z, g.w}, b4[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = __builtin_fmaf(g4[e], acc[e] + b4[e], x[e]);
  }
  __device__ void store(int m, int n, float v) const { store_val<XT>(X + (size_t)m * ld + n, v); }
  __device__ void store4(int m, int n, const float* v) const { store_val4<XT>(X + (size_t)m * ld + n, v); }
  __device__ void store_stats(int m, int nt, float mean, float m2) const {
    reinterpret_cast<float2*>(Sout)[(size_t)m * NTout + nt] = make_float2(mean, m2);
  }
};

// ---- LayerNorm fold (bf16 handles): a GEMM whose A operand is LN(x)*alpha + beta (mlp.0 :151-152,
// conv_out :238-245), alpha = w (1 + scale), beta = b (1 + scale) + shift per column k, is computed as
//   out[m][n] = rstd_m * (sum_k W[n][k] (x[m][k] alpha_k) - mean_m * wa[n]) + wb[n]
// with wa = W alpha, wb = W beta (+ bias) precomputed for every modulation row by flamed_den_adaln
// (LoadFold) and x*alpha written in bf16 by the producer's epilogue (EpiConvNeXtResid::ya) — so the
// GEMM runs on a plain bf16 operand (LDS-DMA main loop) with no A-side transform, and the row
// statistics enter only the epilogue.

// A[r][k] = alpha (WHICH 0) or beta (WHICH 1) of modulation row r, from the mods table.
template <int WHICH>
struct LoadFold {
  const float* __restrict__ sc;
  const float* __restrict__ sh;
  int ms;
  const float* __restrict__ lw;  // LN weight / bias (null: elementwise_affine=False)
  const float* __restrict__ lb;
  struct Raw { float s[8]; float h[WHICH ? 8 : 1]; };
  static constexpr int kSrcBytes = 4;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    Raw r;
    const float* q = sc + (size_t)m * ms + k;
    const float4 a = ld4(q), b = ld4(q + 4);
    r.s[0] = a.x; r.s[1] = a.y; r.s[2] = a.z; r.s[3] = a.w; r.s[4] = b.x; r.s[5] = b.y; r.s[6] = b.z; r.s[7] = b.w;
    if constexpr (WHICH == 1) {
      const float* p = sh + (size_t)m * ms + k;
      const float4 c = ld4(p), d = ld4(p + 4);
      r.h[0] = c.x; r.h[1] = c.y; r.h[2] = c.z; r.h[3] = c.w; r.h[4] = d.x; r.h[5] = d.y; r.h[6] = d.z; r.h[7] = d.w;
    }
    return r;
  }
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int k, const float*, int) const {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s1 = 1.0f + r.s[j];
      if constexpr (WHICH == 0) v[j] = (lw ? lw[k + j] : 1.0f) * s1;
      else v[j] = (lb ? lb[k + j] : 0.0f) * s1 + r.h[j];
    }
    return pack_chunk<D>(v);
  }
};

// Consumer epilogue: out = act(rstd_m (acc - mean_m wa[n]) + wb[n]) with (mean, rstd) from the
// producer's row partials and [wa, wb] of the (at most two) modulation rows of the tile staged in LDS.
template <typename OT, int ACT>
struct EpiLNFold {
  OT* __restrict__ out;
  int ldo;
  const float* __restrict__ Sin;
  int NTin, twin;
  float eps;
  const float* __restrict__ fold;  // wa at fold[row * ms + n], wb at fold[row * ms + N + n]
  int N, ms, div;
  StepOff so;
  static constexpr bool kRowStats = false;
  static constexpr int kEVec = 4;
  static constexpr int stat_rows(int BM) { return BM; }
  __device__ bool prologue_v(int bm, int bn, int BM, int BN, int M, float* st, float* vec) const {
    const int last = (bm + BM - 1 < M ? bm + BM - 1 : M - 1);
    const int r0 = bm / div, r1 = last / div;
    const bool ok = r1 - r0 <= 1;
    const float* f = fold + so.get();
    const int cnt = ok ? (r1 - r0 + 1) * BN : 0;
    for (int idx = threadIdx.x; idx < cnt; idx += blockDim.x) {
      const int slot = idx / BN, c = idx - slot * BN;
      const size_t o = (size_t)(r0 + slot) * ms + bn + c;
      vec[(2 * slot) * kEVecStride + c] = f[o];
      vec[(2 * slot + 1) * kEVecStride + c] = f[o + N];
    }
    for (int r = threadIdx.x; r < BM; r += blockDim.x) {
      int m = bm + r;
      m = m < M ? m : M - 1;
      row_stats_from_partials(Sin, m, NTin, twin, eps, st[2 * r], st[2 * r + 1]);
    }
    return ok;
  }
  __device__ float value_v(int m, int n, float acc, const float* st, const float* vec, bool use, int bm, int bn) const {
    const float mean = st[2 * (m - bm)], rstd = st[2 * (m - bm) + 1];
    float wa, wb;
    if (use) {
      const float* v = vec + 2 * (m / div - bm / div) * kEVecStride + (n - bn);
      wa = v[0];
      wb = v[kEVecStride];
    } else {
      const float* f = fold + so.get() + (size_t)(m / div) * ms + n;
      wa = f[0];
      wb = f[N];
    }
    return fold_out(acc, mean, rstd, wa, wb);
  }
  // out = act(fma(rstd, fma(-mean, wa, acc), wb)): explicit roundings (staged and direct paths agree bitwise)
  static __device__ __forceinline__ float fold_out(float acc, float mean, float rstd, float wa, float wb) {
    float v = __builtin_fmaf(rstd, __builtin_fmaf(-mean, wa, acc), wb);
    if constexpr (ACT == 2) v = silu(v);
    return v;
  }
  // four consecutive columns (n % 4 == 0): the staged wa / wb rows read as float4
  __device__ void value4_v(int m, int n, const float* acc, const float* st, const float* vec, bool use, int bm, int bn,
                           const float*, float* out) const {
    if (!use) {
#pragma unroll
      for (int e = 0; e < 4; ++e) out[e] = value_v(m, n + e, acc[e], st, vec, use, bm, bn);
      return;
    }
    const float mean = st[2 * (m - bm)], rstd = st[2 * (m - bm) + 1];
    const float* v = vec + 2 * (m / div - bm / div) * kEVecStride + (n - bn);
    const float4 a = *reinterpret_cast<const float4*>(v), b = *reinterpret_cast<const float4*>(v + kEVecStride);
    const float a4[4] = {a.x, a.y, a.z, a.w}, b4[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = fold_out(acc[e], mean, rstd, a4[e], b4[e]);
  }
  __device__ void store(int m, int n, float v) const { store_val<OT>(out + (size_t)m * ldo + n, v); }
  __device__ void store4(int m, int n, const float* v) const { store_val4<OT>(out + (size_t)m * ldo + n, v); }
  __device__ void store_stats(int, int, float, float) const {}
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

// ------------------------------ K2a: LN+mod -> depthwise conv (+ GroupNorm partials) ------------------------------
// grid (H/64, ceil(T/64), B): one workgroup = 64 frames x 64 channels of one utterance.  It stages the
// LN+AdaLN-modulated input rows (64 + 2*15 halo) in LDS, runs the depthwise k31 conv (reference
// prob_generator.py:81-88, zero padding at the utterance edges), writes the raw conv output D (fp32)
// and per-channel (count, mean, M2) partials of this frame chunk.  GroupNorm(H,H) statistics over the
// whole T axis (:89) are finished by gn_finalize; the normalisation itself is applied in the conv_2
// GEMM's A-operand loader (LoadGN).
constexpr int kDwCG = 64, kDwTC = 64;
// T-chunk of the depthwise-conv workgroups at large M (B*T >= 8192): tn().dw_tc_big 64 | 128 (128: half
// the workgroups, half the halo re-read; measured slower at B = 64, 97 vs 82 us per launch,
// profiles/r01_b64_bigpath.txt).  Below tn().dw_cg32_rows rows: narrow tn().dw_cg_small-channel groups.

template <bool AFF, int KS, int TC, int CG = kDwCG, typename XT = float>  // XT: X and D type (bf16 on the x16 path)
__global__ __launch_bounds__(256) void dwconv_stats_kernel(const XT* __restrict__ X, int H, const float* __restrict__ S,
                                                           int NT, int tw, float eps_ln, ModRef mod,
                                                           const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                           const float* __restrict__ dww, const float* __restrict__ dwb,
                                                           XT* __restrict__ D, float* __restrict__ GP, int T, int TS,
                                                           int* __restrict__ gcnt, float* __restrict__ GNS) {
  constexpr int HALO = KS / 2, SR = TC + 2 * HALO, RG = 256 / CG, RPT = TC / RG, WIN = RPT + KS - 1;
  constexpr int C4 = CG / 4;                      // float4 chunks per staged row
  constexpr int NX = (SR * C4 + 255) / 256;          // float4 loads per thread for the X tile
  FL_STAMP(0);
  __shared__ float hs[SR * CG];
  __shared__ float rs[SR * 2];
  __shared__ float red[RG * CG * 3 + 1];  // + "last arriver" flag
  __shared__ float va[CG], vb[CG];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * CG, ts = blockIdx.y, b = blockIdx.z;
  const int t0 = ts * TC;
  const int cl = tid % CG, rg = tid / CG, c = c0 + cl;
  mod = mod.at();
  // every independent global load is issued up front: X tile (float4), conv taps, LN stats, alpha/beta
  float4 xv[NX];
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    const int q = tid + j * 256;
    const int r = q / C4, c4 = q - r * C4;
    const int t = t0 - HALO + r;
    xv[j] = (q < SR * C4 && t >= 0 && t < T) ? ldx4<XT>(X + ((size_t)b * T + t) * H + c0 + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float w[KS];
#pragma unroll
  for (int j = 0; j < KS; ++j) w[j] = dww[(size_t)j * H + c];  // tap-major (KS, H) copy: coalesced
  const float bias = dwb[c];
  // one modulation row for the whole utterance (sampling path): stage alpha/beta once
  const bool uni = ((size_t)b * T) / mod.div == ((size_t)b * T + T - 1) / mod.div;
  if (uni && tid < CG) {
    size_t mo = (((size_t)b * T) / mod.div) * mod.ms + c0 + tid;
    float sc1 = 1.0f + mod.sc[mo];
    float lw = AFF ? lnw[c0 + tid] : 1.0f, lb = AFF ? lnb[c0 + tid] : 0.0f;
    va[tid] = lw * sc1;
    vb[tid] = lb * sc1 + mod.sh[mo];
  }
  if (tid < SR) {
    int t = t0 - HALO + tid;
    if (t >= 0 && t < T) row_stats_from_partials(S, b * T + t, NT, tw, eps_ln, rs[2 * tid], rs[2 * tid + 1]);
  }
  __syncthreads();
  FL_STAMP(1);
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    const int q = tid + j * 256;
    if (q >= SR * C4) break;
    const int r = q / C4, c4 = q - r * C4;
    const int t = t0 - HALO + r;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    if (t >= 0 && t < T) {
      const float xs[4] = {xv[j].x, xv[j].y, xv[j].z, xv[j].w};
      const float mean = rs[2 * r], rstd = rs[2 * r + 1];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cc = 4 * c4 + e;
        const float xh = (xs[e] - mean) * rstd;
        if (uni) {
          o[e] = xh * va[cc] + vb[cc];
        } else {
          size_t m = (size_t)b * T + t;
          size_t mo = (m / mod.div) * mod.ms + c0 + cc;
          float sc1 = 1.0f + mod.sc[mo];
          float lw = AFF ? lnw[c0 + cc] : 1.0f, lb = AFF ? lnb[c0 + cc] : 0.0f;
          o[e] = xh * (lw * sc1) + (lb * sc1 + mod.sh[mo]);
        }
      }
    }
    *reinterpret_cast<float4*>(hs + r * CG + 4 * c4) = make_float4(o[0], o[1], o[2], o[3]);
  }
  __syncthreads();
  FL_STAMP(2);
  float win[WIN];
#pragma unroll
  for (int j = 0; j < WIN; ++j) win[j] = hs[(rg * RPT + j) * CG + cl];
  float vals[RPT];
  float cn = 0.f, cs = 0.f;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    float a = bias;
#pragma unroll
    for (int j = 0; j < KS; ++j) a += w[j] * win[q + j];
    vals[q] = a;
    if (t0 + rg * RPT + q < T) {
      cn += 1.f;
      cs += a;
    }
  }
  // D is written after the chunk partials are published (below): with the GroupNorm hand-off its
  // stores then drain alongside the ticket round trip instead of ahead of the partials' drain.
  auto store_d = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int t = t0 + rg * RPT + q;
      if (t < T) store_val<XT>(D + ((size_t)b * T + t) * H + c, vals[q]);
    }
  };
  float cm = cn > 0.f ? cs / cn : 0.f, c2 = 0.f;
#pragma unroll
  for (int q = 0; q < RPT; ++q)
    if (t0 + rg * RPT + q < T) {
      float d = vals[q] - cm;
      c2 += d * d;
    }
  red[(rg * CG + cl) * 3 + 0] = cn;
  red[(rg * CG + cl) * 3 + 1] = cm;
  red[(rg * CG + cl) * 3 + 2] = c2;
  FL_STAMP(3);
  lds_barrier();
  if (tid < CG) {
    float n = 0.f, mu = 0.f, m2 = 0.f;
#pragma unroll
    for (int g = 0; g < RG; ++g) chan_combine(n, mu, m2, red[(g * CG + tid) * 3], red[(g * CG + tid) * 3 + 1], red[(g * CG + tid) * 3 + 2]);
    float* o = GP + (((size_t)b * TS + ts) * H + c0 + tid) * 3;
    if (gcnt) {  // handed to another workgroup: write-through (sc1) stores, no release fence needed
      __hip_atomic_store(o, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 1, mu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 2, m2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      o[0] = n; o[1] = mu; o[2] = m2;
    }
  }
  FL_STAMP(4);
  if (!gcnt) {
    store_d();
    return;
  }
  // GroupNorm finalize fused: the last T-chunk block of this (utterance, channel group) combines the
  // TS chunk partials in chunk order (as gn_finalize_kernel) and writes GNS = (mean, rstd).
  // Hand-off (cdna_hip_programming.md §6 Guideline 16, sc1 form): partials stored write-through and
  // drained, one relaxed agent-scope ticket; the last arriver reads them with sc1 (agent atomic) loads.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  store_d();
  int* flag = reinterpret_cast<int*>(red + RG * CG * 3);
  if (tid == 0) {
    int* cnt = gcnt + (size_t)b * gridDim.x + blockIdx.x;
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == TS - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    *flag = last;
  }
  __syncthreads();
  if (!*flag || tid >= CG) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 loads below the ticket
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int t0c = 0; t0c < TS; t0c += 8) {
    float q[8][3];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float* p = GP + (((size_t)b * TS + (t0c + i < TS ? t0c + i : TS - 1)) * H + c0 + tid) * 3;
      q[i][0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      q[i][1] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      q[i][2] = __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (t0c + i < TS) chan_combine(n, mu, m2, q[i][0], q[i][1], q[i][2]);
  }
  GNS[((size_t)b * H + c0 + tid) * 2] = mu;
  GNS[((size_t)b * H + c0 + tid) * 2 + 1] = 1.0f / sqrtf(m2 / (float)T + 1e-5f);
  FL_STAMP(5);
}

// GroupNorm(H,H) statistics over all T frames of each (utterance, channel): GNS[b][c] = (mean, rstd).
__global__ void gn_finalize_kernel(const float* __restrict__ GP, float* __restrict__ GNS, int H, int T, int TS, float eps) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  int b = blockIdx.y;
  if (c >= H) return;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int t0 = 0; t0 < TS; t0 += 8) {  // batches of 8 chunk partials loaded together
    float q[8][3];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float* p = GP + (((size_t)b * TS + (t0 + i < TS ? t0 + i : TS - 1)) * H + c) * 3;
      q[i][0] = p[0]; q[i][1] = p[1]; q[i][2] = p[2];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (t0 + i < TS) chan_combine(n, mu, m2, q[i][0], q[i][1], q[i][2]);
  }
  GNS[((size_t)b * H + c) * 2] = mu;
  GNS[((size_t)b * H + c) * 2 + 1] = 1.0f / sqrtf(m2 / (float)T + eps);
}

template <bool AFF, typename XT = float>
// part 1: conv + partials (+ GroupNorm finalize fused in when gcnt is given); part 2: standalone
// finalize (used only without counters).  XT: type of X and D (bf16 on the large-M x16 path, which
// always uses the 64-channel workgroups).
static int launch_dwconv_stats(const XT* X, int H, const float* S, int NT, int tw, ModRef mod, const float* lnw,
                               const float* lnb, const float* dww, const float* dwb, XT* D, float* GP, float* GNS,
                               int B, int T, hipStream_t st, int part, int* gcnt) {
  FL_REQUIRE(H % kDwCG == 0 && H % 256 == 0, "dwconv: H=%d must be a multiple of 256", H);
  const int TC = ((size_t)B * T >= 8192 && tn().dw_tc_big == 128) ? 128 : kDwTC;
  const int TS = (T + TC - 1) / TC;
  // fewer than dw_cg32_rows frames: 32-channel workgroups (twice the workgroups, half the serial work each)
  const bool cg32 = std::is_same<XT, float>::value && (size_t)B * T < (size_t)tn().dw_cg32_rows;
  if (part != 2) {
    if (TC == 128)
      hipLaunchKernelGGL((dwconv_stats_kernel<AFF, 31, 128, kDwCG, XT>), dim3(H / kDwCG, TS, B), dim3(256), 0, st, X, H, S, NT, tw,
                         1e-6f, mod, lnw, lnb, dww, dwb, D, GP, T, TS, gcnt, GNS);
    else if (cg32 && tn().dw_cg_small == 16)
      hipLaunchKernelGGL((dwconv_stats_kernel<AFF, 31, kDwTC, 16, XT>), dim3(H / 16, TS, B), dim3(256), 0, st, X, H, S, NT, tw,
                         1e-6f, mod, lnw, lnb, dww, dwb, D, GP, T, TS, gcnt, GNS);
    else if (cg32)
      hipLaunchKernelGGL((dwconv_stats_kernel<AFF, 31, kDwTC, 32, XT>), dim3(H / 32, TS, B), dim3(256), 0, st, X, H, S, NT, tw,
                         1e-6f, mod, lnw, lnb, dww, dwb, D, GP, T, TS, gcnt, GNS);
    else
      hipLaunchKernelGGL((dwconv_stats_kernel<AFF, 31, kDwTC, kDwCG, XT>), dim3(H / kDwCG, TS, B), dim3(256), 0, st, X, H, S, NT,
                         tw, 1e-6f, mod, lnw, lnb, dww, dwb, D, GP, T, TS, gcnt, GNS);
    FL_LAUNCH_CHECK();
  }
  if (part != 1 && !gcnt) {
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(H / 256, B), dim3(256), 0, st, GP, GNS, H, T, TS, 1e-5f);
    FL_LAUNCH_CHECK();
  }
  return kOk;
}

// Large-M path, one modulation row per utterance (sampling): the whole depthwise-conv + GroupNorm
// sub-block (reference prob_generator.py:81-89) in one kernel per (utterance, 32 channels), writing
// the normalised conv_2 A operand in bf16 directly (no D round trip, no separate GroupNorm pass).
// grid (H/32, B), 256 threads = 16 channel pairs x 16 row groups; the conv runs on channel pairs in
// packed fp32 (v_pk_fma_f32: two FMAs per lane per instruction, the VALU bound of this kernel).  The
// LN row statistics of the whole utterance are combined into LDS once; the utterance is then walked in
// 64-frame chunks: the LN+AdaLN-modulated rows (+-15 halo, zero padding at the edges) are staged in
// LDS (double buffered, one barrier per chunk, rows padded to 40 floats so the two row groups of a
// 32-lane LDS group hit disjoint banks), the k31 conv of 4 frames x 2 channels per thread is kept in
// registers (NCH chunks: T <= 64 * NCH), each thread keeps shifted sums of its frames and the row
// groups' (count, mean, M2) partials are combined once (Chan) into the GroupNorm(H,H) statistics over
// all T frames.  The output pass applies LoadGN's arithmetic
// (x - mean) * (rstd * gn_w) + gn_b to the register-resident values.  The X tiles of the next two
// chunks are in flight while the current one is convolved.
constexpr int kDgMaxT = 512;  // frames covered by the register-resident path (NCH <= 8)
typedef float dg_f2 __attribute__((ext_vector_type(2)));
// fp32 pair arithmetic.  VAR 1 (the default, every T) does it with scalar fp32 ops kept apart by empty asm
// barriers: on gfx950 a v_pk_*_f32 that consumes a VGPR pair written by a 64-bit LDS read (ds_read_b64)
// was measured to return a wrong low dword for one channel parity of one 64-frame chunk when waves of
// our fp32-MFMA GEMMs were co-resident on the CU (two handles on two streams, tools/conc_dwgn3.py,
// DESIGN.md "dwgn concurrency").  Diagnostic variants (tune dwgn_var, T in (384, 448] only): VAR 0 is
// the packed form that showed it, VAR 2 keeps the packed math and moves the staged window through LDS
// with scalar (volatile) accesses (also clean, 1.3x slower).
template <int VAR>
__device__ __forceinline__ dg_f2 dg_fma(dg_f2 a, dg_f2 b, dg_f2 c) {
  if constexpr (VAR == 1) {
    float x = __builtin_fmaf(a.x, b.x, c.x), y = __builtin_fmaf(a.y, b.y, c.y);
    asm volatile("" : "+v"(x), "+v"(y));  // keep them scalar (no re-pairing into v_pk_fma_f32)
    return dg_f2{x, y};
  } else {
    return __builtin_elementwise_fma(a, b, c);
  }
}
template <int VAR>
__device__ __forceinline__ dg_f2 dg_lnmod(dg_f2 x, dg_f2 mean, dg_f2 rstd, dg_f2 a, dg_f2 b) {
  if constexpr (VAR == 1) {
    float u = (x.x - mean.x) * rstd.x, v = (x.y - mean.y) * rstd.y;
    asm volatile("" : "+v"(u), "+v"(v));
    float o0 = u * a.x + b.x, o1 = v * a.y + b.y;
    asm volatile("" : "+v"(o0), "+v"(o1));
    return dg_f2{o0, o1};
  } else {
    return ((x - mean) * rstd) * a + b;
  }
}
template <int VAR>
__device__ __forceinline__ dg_f2 dg_apply(dg_f2 x, dg_f2 mu, dg_f2 sc, dg_f2 sh) {  // (x - mu) * sc + sh
  if constexpr (VAR == 1) {
    float u = x.x - mu.x, v = x.y - mu.y;
    asm volatile("" : "+v"(u), "+v"(v));
    float o0 = u * sc.x + sh.x, o1 = v * sc.y + sh.y;
    asm volatile("" : "+v"(o0), "+v"(o1));
    return dg_f2{o0, o1};
  } else {
    return (x - mu) * sc + sh;
  }
}
__device__ __forceinline__ dg_f2 dg_add1(dg_f2 a, dg_f2 b) {  // scalar pair add (no v_pk_add_f32)
  float x = a.x + b.x, y = a.y + b.y;
  asm volatile("" : "+v"(x), "+v"(y));
  return dg_f2{x, y};
}
template <bool AFF, int NCH, typename XT, int VAR = 1>
__global__ __launch_bounds__(256) void dwgn_kernel(const XT* __restrict__ X, int H, const float* __restrict__ S, int NT, int tw,
                                                   float eps_ln, ModRef mod, const float* __restrict__ lnw,
                                                   const float* __restrict__ lnb, const float* __restrict__ dww,
                                                   const float* __restrict__ dwb, const float* __restrict__ gnw,
                                                   const float* __restrict__ gnb, bf16* __restrict__ A, int T) {
  constexpr int KS = 31, HALO = KS / 2, CG = 32, NP = CG / 2, TC = 64, SR = TC + 2 * HALO, RG = 16, RPT = TC / RG;
  constexpr int WIN = RPT + KS - 1, LDH = CG + 8;  // padded LDS row
  constexpr int NTH = 256, C4 = CG / 4, NX = (SR * C4 + NTH - 1) / NTH;
  __shared__ float hs[2][SR * LDH];
  __shared__ float rs[NCH * TC * 2];
  __shared__ float red[RG * CG * 3];
  __shared__ float va[CG], vb[CG], gmu[CG], gsc[CG];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * CG, b = blockIdx.y;
  const int pp = tid % NP, rg = tid / NP, c = c0 + 2 * pp;  // channels c, c + 1
  const int nch = (T + TC - 1) / TC;
  mod = mod.at();
  // tiles of chunks ch and ch + 1 in flight, held RAW (bf16 pairs or fp32): converting at load time
  // would make the compiler wait for each prefetch right after issuing it
  using XR = typename std::conditional<std::is_same<XT, bf16>::value, uint2, float4>::type;
  XR xv[2][NX];
  auto cvt = [](const XR& r) __attribute__((always_inline)) -> float4 {
    if constexpr (std::is_same<XT, bf16>::value)
      return make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u), __uint_as_float(r.y << 16),
                         __uint_as_float(r.y & 0xffff0000u));
    else
      return r;
  };
  auto load_x = [&](XR* xs, int t0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int q = tid + j * NTH;
      const int r = q / C4, c4 = q - r * C4;
      const int t = t0 - HALO + r;
      // unconditional load from a clamped row (rows outside the utterance are zeroed when staged): no
      // branches around the loads, so the wait before staging chunk ch leaves chunk ch + 1's in flight
      const int tc = min(max(t, 0), T - 1), c4c = q < SR * C4 ? c4 : 0;
      xs[j] = *reinterpret_cast<const XR*>(X + ((size_t)b * T + tc) * H + c0 + 4 * c4c);
    }
  };
  load_x(xv[0], 0);
  load_x(xv[1], min(TC, (nch - 1) * TC));
  for (int t = tid; t < T; t += NTH) row_stats_from_partials(S, b * T + t, NT, tw, eps_ln, rs[2 * t], rs[2 * t + 1]);
  dg_f2 w[KS];
#pragma unroll
  for (int j = 0; j < KS; ++j) w[j] = *reinterpret_cast<const dg_f2*>(dww + (size_t)j * H + c);  // tap-major (KS, H) copy
  const dg_f2 bias = *reinterpret_cast<const dg_f2*>(dwb + c);
  if (tid < CG) {  // alpha/beta of the utterance's modulation row
    const size_t mo = (((size_t)b * T) / mod.div) * mod.ms + c0 + tid;
    const float sc1 = 1.0f + mod.sc[mo];
    const float lw = AFF ? lnw[c0 + tid] : 1.0f, lb = AFF ? lnb[c0 + tid] : 0.0f;
    va[tid] = lw * sc1;
    vb[tid] = lb * sc1 + mod.sh[mo];
  }
  __syncthreads();
  dg_f2 dv[NCH][RPT];
  // GroupNorm partials of this thread's frames: shifted sums s1 = sum(x - K), s2 = sum((x - K)^2) with
  // K = the thread's first conv output (a value of the data's own range, so no cancellation)
  dg_f2 K = {0.f, 0.f}, s1 = {0.f, 0.f}, s2 = {0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    if (ch >= nch) break;
    const int t0 = ch * TC;
    float* h = hs[ch & 1];
    XR* xr = xv[ch & 1];
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int q = tid + j * NTH;
      if (q < SR * C4) {
        const int r = q / C4, c4 = q - r * C4;
        const int t = t0 - HALO + r;
        dg_f2 lo = {0.f, 0.f}, hi = {0.f, 0.f};
        const float4 xcj = cvt(xr[j]);
        if (t >= 0 && t < T) {
          const dg_f2 mean = rs[2 * t], rstd = rs[2 * t + 1];
          const float4 a4 = *reinterpret_cast<const float4*>(va + 4 * c4), b4 = *reinterpret_cast<const float4*>(vb + 4 * c4);
          lo = dg_lnmod<VAR>(dg_f2{xcj.x, xcj.y}, mean, rstd, dg_f2{a4.x, a4.y}, dg_f2{b4.x, b4.y});
          hi = dg_lnmod<VAR>(dg_f2{xcj.z, xcj.w}, mean, rstd, dg_f2{a4.z, a4.w}, dg_f2{b4.z, b4.w});
        }
        if constexpr (VAR == 2) {
          volatile float* hv = h + r * LDH + 4 * c4;
          hv[0] = lo.x; hv[1] = lo.y; hv[2] = hi.x; hv[3] = hi.y;
        } else {
          *reinterpret_cast<float4*>(h + r * LDH + 4 * c4) = make_float4(lo.x, lo.y, hi.x, hi.y);
        }
      }
    }
    // two chunks ahead, in flight during the next two convs; issued unconditionally (past the end: the
    // last chunk again) so every path has the same loads in flight and the waits stay counted
    load_x(xr, min(t0 + 2 * TC, (nch - 1) * TC));
    __syncthreads();  // h staged; the other buffer (chunk ch-1) is no longer read
    // sliding window: staged row r feeds frames q = r - j of this thread's RPT (each frame's taps still
    // accumulate in tap order j = 0..KS-1), so only a few window rows are live at a time
    dg_f2 acc[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) acc[q] = bias;
#pragma unroll
    for (int r = 0; r < WIN; ++r) {
      dg_f2 row;
      if constexpr (VAR == 2) {
        volatile const float* hv = h + (rg * RPT + r) * LDH + 2 * pp;
        row = dg_f2{hv[0], hv[1]};
      } else {
        row = *reinterpret_cast<const dg_f2*>(h + (rg * RPT + r) * LDH + 2 * pp);
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q)
        if (r - q >= 0 && r - q < KS) acc[q] = dg_fma<VAR>(w[r - q], row, acc[q]);
    }
    const int nv = T - (t0 + rg * RPT);  // valid frames of this thread in the chunk (may be <= 0)
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const dg_f2 a = acc[q];
      dv[ch][q] = a;
      if (ch == 0 && q == 0) K = a;
      if (q < nv) {
        const dg_f2 e = a - K;
        s1 += e;
        s2 = __builtin_elementwise_fma(e, e, s2);
      }
    }
  }
  {
    int n = 0;  // frames this thread covered
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) n += max(0, min(RPT, T - (ch * TC + rg * RPT)));
    const float fn = (float)n, inv = n > 0 ? 1.0f / fn : 0.f;
    const dg_f2 m = K + s1 * inv, m2 = s2 - s1 * s1 * inv;
    red[(rg * CG + 2 * pp) * 3 + 0] = fn;
    red[(rg * CG + 2 * pp) * 3 + 1] = m.x;
    red[(rg * CG + 2 * pp) * 3 + 2] = fmaxf(m2.x, 0.f);
    red[(rg * CG + 2 * pp + 1) * 3 + 0] = fn;
    red[(rg * CG + 2 * pp + 1) * 3 + 1] = m.y;
    red[(rg * CG + 2 * pp + 1) * 3 + 2] = fmaxf(m2.y, 0.f);
  }
  __syncthreads();
  if (tid < CG) {  // the row groups' partials, in order
    float n = 0.f, m = 0.f, m2 = 0.f;
#pragma unroll
    for (int g = 0; g < RG; ++g) chan_combine(n, m, m2, red[(g * CG + tid) * 3], red[(g * CG + tid) * 3 + 1], red[(g * CG + tid) * 3 + 2]);
    gmu[tid] = m;
    gsc[tid] = (1.0f / sqrtf(m2 / (float)T + 1e-5f)) * gnw[c0 + tid];
  }
  __syncthreads();
  const dg_f2 mu = {gmu[2 * pp], gmu[2 * pp + 1]}, sc = {gsc[2 * pp], gsc[2 * pp + 1]};
  const dg_f2 sh = *reinterpret_cast<const dg_f2*>(gnb + c);
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 ob[NCH][RPT];  // all outputs converted first: the stores below then need no register waits
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const dg_f2 o = dg_apply<VAR>(dv[ch][q], mu, sc, sh);
      ob[ch][q] = bf16x2{(bf16)o.x, (bf16)o.y};
    }
  bf16* ap = A + ((size_t)b * T + rg * RPT) * H + c;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
    for (int q = 0; q < RPT; ++q)
      if (ch * TC + rg * RPT + q < T) *reinterpret_cast<bf16x2*>(ap + (size_t)(ch * TC + q) * H) = ob[ch][q];
}

template <bool AFF, typename XT>
static int launch_dwgn(const XT* X, int H, const float* S, int NT, int tw, ModRef mod, const float* lnw, const float* lnb,
                       const float* dww, const float* dwb, const float* gnw, const float* gnb, bf16* A, int B, int T,
                       hipStream_t st) {
  FL_REQUIRE(H % 32 == 0 && T >= 1 && T <= kDgMaxT && mod.div % T == 0, "dwgn: H=%d T=%d div=%d", H, T, mod.div);
  const int nch = (T + 63) / 64;
  const dim3 g(H / 32, B), blk(256);
#define FL_DWGN(N) hipLaunchKernelGGL((dwgn_kernel<AFF, N, XT>), g, blk, 0, st, X, H, S, NT, tw, 1e-6f, mod, lnw, lnb, dww, dwb, gnw, gnb, A, T)
#define FL_DWGN_V(N, V) hipLaunchKernelGGL((dwgn_kernel<AFF, N, XT, V>), g, blk, 0, st, X, H, S, NT, tw, 1e-6f, mod, lnw, lnb, dww, dwb, gnw, gnb, A, T)
  if (tn().dwgn_var == 0 && nch == 7) FL_DWGN_V(7, 0);
  else if (tn().dwgn_var == 2 && nch == 7) FL_DWGN_V(7, 2);
  else if (nch <= 2) FL_DWGN(2);
  else if (nch <= 4) FL_DWGN(4);
  else if (nch <= 6) FL_DWGN(6);
  else if (nch == 7) FL_DWGN(7);
  else FL_DWGN(8);
#undef FL_DWGN
#undef FL_DWGN_V
  FL_LAUNCH_CHECK();
  return kOk;
}

// Small-M path (B*T below the large-M threshold, T <= 576, one modulation row per utterance): the
// depthwise-conv + GroupNorm sub-block (prob_generator.py:81-89) of one utterance and 8 channels in
// one workgroup, so no cross-workgroup hand-off is needed for the GroupNorm statistics.  grid
// (H/8, B), 256 threads = 4 channel pairs x 64 row groups of RPT consecutive frames (RPT odd: the
// row groups of a 32-lane LDS group then hit disjoint banks).  All T (+-15 halo) LN+AdaLN-modulated
// rows are staged in LDS at once, the conv runs in packed fp32 on channel pairs with its outputs in
// registers (X rows and the producer's LN partials of all the thread's staged frames are loaded
// before any is used), the GroupNorm statistics are two exact passes (sum, then sum of squared deviations: wave shuffles
// + one LDS exchange each, fixed order), and the normalised bf16 conv_2 operand is written with
// LoadGN's arithmetic (x - mean) * (rstd * gn_w) + gn_b.  conv_2 then runs as a plain bf16 GEMM on the
// LDS-DMA loop.
template <bool AFF, int RPT>
__global__ __launch_bounds__(256) void dwgn_small_kernel(const float* __restrict__ X, int H, const float* __restrict__ S, int NT,
                                                         int tw, float eps_ln, ModRef mod, const float* __restrict__ lnw,
                                                         const float* __restrict__ lnb, const float* __restrict__ dww,
                                                         const float* __restrict__ dwb, const float* __restrict__ gnw,
                                                         const float* __restrict__ gnb, bf16* __restrict__ A, int T) {
  constexpr int KS = 31, HALO = KS / 2, CG = 8, WIN = RPT + KS - 1, MAXR = 64 * RPT + 2 * HALO;
  static_assert(RPT % 2 == 1, "odd RPT keeps the window reads conflict-free");
  __shared__ float hs[MAXR * CG];
  __shared__ dg_f2 red[2][4][4];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * CG, b = blockIdx.y;
  const int p = tid & 3, rg = tid >> 2, c = c0 + 2 * p;
  FL_STAMP(0);
  mod = mod.at();
  // this thread's staged rows r = tid, tid + 256, ... (frame r - HALO): X loads issued first (clamped
  // rows, zeroed when staged), so they are in flight during the row-statistics pass
  constexpr int NSR = (MAXR + 255) / 256;
  float4 xv[NSR][2];
#pragma unroll
  for (int i = 0; i < NSR; ++i) {
    const int t = min(max(tid + 256 * i - HALO, 0), T - 1);
    const float* xr = X + ((size_t)b * T + t) * H + c0;
    xv[i][0] = ld4(xr);
    xv[i][1] = ld4(xr + 4);
  }
  // LN row statistics of this thread's staged frames, combined from the producer's partials; with
  // NT <= 16 the partials of all its frames are loaded before any is reduced (one latency, not NSR)
  float rmean[NSR], rrstd[NSR];
  if (NT <= 16) {
    float2 q[NSR][16];
#pragma unroll
    for (int i = 0; i < NSR; ++i) {
      const int t = min(max(tid + 256 * i - HALO, 0), T - 1);
      const float2* pp = reinterpret_cast<const float2*>(S) + (size_t)(b * T + t) * NT;
#pragma unroll
      for (int k = 0; k < 16; ++k) q[i][k] = k < NT ? pp[k] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < NSR; ++i) {
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sm += q[i][k].x;
      const float mean = sm / (float)NT;
      float m2 = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < NT) { const float d = q[i][k].x - mean; m2 += q[i][k].y + (float)tw * d * d; }
      rmean[i] = mean;
      rrstd[i] = 1.0f / sqrtf(m2 / (float)(NT * tw) + eps_ln);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NSR; ++i) {
      const int t = min(max(tid + 256 * i - HALO, 0), T - 1);
      row_stats_from_partials(S, b * T + t, NT, tw, eps_ln, rmean[i], rrstd[i]);
    }
  }
  FL_STAMP(1);
  float va[CG], vb[CG];  // per-channel alpha/beta of the 8 staged channels
  {
    const size_t mo = (((size_t)b * T) / mod.div) * mod.ms + c0;
#pragma unroll
    for (int e = 0; e < CG; ++e) {
      const float sc1 = 1.0f + mod.sc[mo + e];
      const float lw = AFF ? lnw[c0 + e] : 1.0f, lb = AFF ? lnb[c0 + e] : 0.0f;
      va[e] = lw * sc1;
      vb[e] = lb * sc1 + mod.sh[mo + e];
    }
  }
#pragma unroll
  for (int i = 0; i < NSR; ++i) {
    const int r = tid + 256 * i, t = r - HALO;
    if (r >= T + 2 * HALO) break;
    float o[CG];
#pragma unroll
    for (int e = 0; e < CG; ++e) o[e] = 0.f;
    if (t >= 0 && t < T) {
      const float mean = rmean[i], rstd = rrstd[i];
      const float xs[CG] = {xv[i][0].x, xv[i][0].y, xv[i][0].z, xv[i][0].w, xv[i][1].x, xv[i][1].y, xv[i][1].z, xv[i][1].w};
#pragma unroll
      for (int e = 0; e < CG; ++e) o[e] = ((xs[e] - mean) * rstd) * va[e] + vb[e];
    }
    *reinterpret_cast<float4*>(hs + r * CG) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(hs + r * CG + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
  dg_f2 w[KS];
#pragma unroll
  for (int j = 0; j < KS; ++j) w[j] = *reinterpret_cast<const dg_f2*>(dww + (size_t)j * H + c);
  const dg_f2 bias = *reinterpret_cast<const dg_f2*>(dwb + c);
  __syncthreads();
  FL_STAMP(2);
  dg_f2 win[WIN];
#pragma unroll
  for (int j = 0; j < WIN; ++j) win[j] = *reinterpret_cast<const dg_f2*>(hs + (rg * RPT + j) * CG + 2 * p);
  dg_f2 dv[RPT];
  const int nv = T - rg * RPT;  // valid frames of this thread (may be <= 0); rows past T are discarded
  dg_f2 s = {0.f, 0.f};
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    dg_f2 a = bias;
#pragma unroll
    for (int j = 0; j < KS; ++j) a = dg_fma<1>(w[j], win[q + j], a);  // scalar: see dg_fma
    dv[q] = a;
    if (q < nv) s += a;
  }
  auto block_sum = [&](dg_f2 v, int slot) __attribute__((always_inline)) -> dg_f2 {
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) {
      v.x += __shfl_xor(v.x, o);
      v.y += __shfl_xor(v.y, o);
    }
    if ((tid & 63) < 4) red[slot][tid >> 6][p] = v;
    __syncthreads();
    return dg_add1(dg_add1(dg_add1(red[slot][0][p], red[slot][1][p]), red[slot][2][p]), red[slot][3][p]);
  };
  FL_STAMP(3);
  const float invT = 1.0f / (float)T;
  const dg_f2 mean = block_sum(s, 0) * invT;
  dg_f2 s2 = {0.f, 0.f};
#pragma unroll
  for (int q = 0; q < RPT; ++q)
    if (q < nv) { const dg_f2 e = dv[q] - mean; s2 = __builtin_elementwise_fma(e, e, s2); }
  const dg_f2 m2 = block_sum(s2, 1);
  const dg_f2 sc = dg_f2{1.0f / sqrtf(m2.x * invT + 1e-5f), 1.0f / sqrtf(m2.y * invT + 1e-5f)} * *reinterpret_cast<const dg_f2*>(gnw + c);
  const dg_f2 sh = *reinterpret_cast<const dg_f2*>(gnb + c);
  FL_STAMP(4);
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 ob[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const dg_f2 o = (dv[q] - mean) * sc + sh;
    ob[q] = bf16x2{(bf16)o.x, (bf16)o.y};
  }
  bf16* ap = A + ((size_t)b * T + rg * RPT) * H + c;
#pragma unroll
  for (int q = 0; q < RPT; ++q)
    if (q < nv) *reinterpret_cast<bf16x2*>(ap + (size_t)q * H) = ob[q];
  FL_STAMP(5);
}

constexpr int kDgSmallMaxT = 576;  // 64 row groups x RPT <= 9
template <bool AFF>
static int launch_dwgn_small(const float* X, int H, const float* S, int NT, int tw, ModRef mod, const float* lnw, const float* lnb,
                             const float* dww, const float* dwb, const float* gnw, const float* gnb, bf16* A, int B, int T,
                             hipStream_t st) {
  FL_REQUIRE(H % 8 == 0 && T >= 1 && T <= kDgSmallMaxT && mod.div % T == 0 && NT <= 32, "dwgn_small: H=%d T=%d div=%d NT=%d", H, T,
             mod.div, NT);
  const dim3 g(H / 8, B), blk(256);
#define FL_DWGNS(R) hipLaunchKernelGGL((dwgn_small_kernel<AFF, R>), g, blk, 0, st, X, H, S, NT, tw, 1e-6f, mod, lnw, lnb, dww, dwb, gnw, gnb, A, T)
  if (T <= 64) FL_DWGNS(1);
  else if (T <= 192) FL_DWGNS(3);
  else if (T <= 320) FL_DWGNS(5);
  else if (T <= 448) FL_DWGNS(7);
  else FL_DWGNS(9);
#undef FL_DWGNS
  FL_LAUNCH_CHECK();
  return kOk;
}

// conv_2 A operand: GroupNorm applied on the fly, A = (D - mean) * (rstd * gn_w) + gn_b, with
// [mean, rstd*gn_w] per (utterance, channel) staged in LDS for the <= 2 utterances of the tile.
template <typename DT>
struct LoadGN {
  const float* __restrict__ D;
  int H;
  const float* __restrict__ gns;  // (B, H, 2) = (mean, rstd)
  const float* __restrict__ gnw;
  const float* __restrict__ gnb;
  int T;
  const bf16* D16 = nullptr;  // large-M x16 path: bf16 depthwise output (normalise pass only; D unused)
  static constexpr int EPC = DTraits<DT>::EPC;
  static constexpr int kSrcBytes = 4;
  __device__ const char* src_row(int m) const { return reinterpret_cast<const char*>(D + (size_t)m * H); }
  struct XRow { int voff, m; bool use; };
  __device__ XRow xrow(int m, const float*, const float*, bool use, int bm) const {
    return XRow{use ? 2 * (m / T - bm / T) * H : 0, m, use};
  }
  template <typename Dt, typename R>
  __device__ u32x4 xform(const XRow& xr, const R& r, int k, const float* st, const float* vec, int bm) const {
    if (!xr.use) return finish_v<Dt>(r, xr.m, k, st, vec, false, bm);
    const float* mu = vec + xr.voff + k;
    const float* sc = mu + H;
    const float* bb = vec + 4 * H + k;
    const float4 m0 = ld4(mu), m1 = ld4(mu + 4), s0 = ld4(sc), s1 = ld4(sc + 4), c0 = ld4(bb), c1 = ld4(bb + 4);
    const float mv[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    float o[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) o[j] = (r.v[j] - mv[j]) * sv[j] + cv[j];
    return pack_chunk<Dt>(o);
  }
  static constexpr int kVec = 5;  // 2 slots x (mean, scale) + bias
  struct Raw { float v[EPC]; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ bool prologue_v(int bm, int BM, int M, int K, float*, float* vec) const {
    const int last = (bm + BM - 1 < M ? bm + BM - 1 : M - 1);
    const int b0 = bm / T, b1 = last / T;
    const bool ok = b1 - b0 <= 1;
    const int K4 = K / 4, n4 = ok ? (b1 - b0 + 1) * K4 : 0;
    constexpr int P = 2;  // passes whose loads are all issued before any use
    float4 g0[P], g1[P], w[P], bb[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int q = threadIdx.x + p * blockDim.x;
      if (q < n4) {
        const int slot = q / K4, k = (q - slot * K4) * 4;
        const float* g = gns + ((size_t)(b0 + slot) * H + k) * 2;
        g0[p] = ld4(g);
        g1[p] = ld4(g + 4);
        w[p] = ld4(gnw + k);
        bb[p] = ld4(gnb + k);
      }
    }
    auto put = [&](int q, float4 a, float4 c, float4 ww, float4 b) {
      const int slot = q / K4, k = (q - slot * K4) * 4;
      *reinterpret_cast<float4*>(vec + (size_t)(2 * slot) * K + k) = make_float4(a.x, a.z, c.x, c.z);
      *reinterpret_cast<float4*>(vec + (size_t)(2 * slot + 1) * K + k) = make_float4(a.y * ww.x, a.w * ww.y, c.y * ww.z, c.w * ww.w);
      if (slot == 0) *reinterpret_cast<float4*>(vec + (size_t)4 * K + k) = b;
    };
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int q = threadIdx.x + p * blockDim.x;
      if (q < n4) put(q, g0[p], g1[p], w[p], bb[p]);
    }
    for (int q = threadIdx.x + P * blockDim.x; q < n4; q += blockDim.x) {
      const int slot = q / K4, k = (q - slot * K4) * 4;
      const float* g = gns + ((size_t)(b0 + slot) * H + k) * 2;
      put(q, ld4(g), ld4(g + 4), ld4(gnw + k), ld4(gnb + k));
    }
    return ok;
  }
  __device__ Raw issue_v(int m, int k) const {
    Raw r;
    const float* pd = D + (size_t)m * H + k;
#pragma unroll
    for (int j = 0; j < EPC; j += 4) {
      float4 a = ld4(pd + j);
      r.v[j] = a.x; r.v[j + 1] = a.y; r.v[j + 2] = a.z; r.v[j + 3] = a.w;
    }
    return r;
  }
  template <typename Dt>
  __device__ u32x4 finish_v(const Raw& r, int m, int k, const float*, const float* vec, bool use, int bm) const {
    float o[EPC];
    if (use) {
      const int slot = m / T - bm / T;
      const float* mu = vec + (size_t)(2 * slot) * H + k;
      const float* sc = vec + (size_t)(2 * slot + 1) * H + k;
      const float* bb = vec + (size_t)4 * H + k;
#pragma unroll
      for (int j = 0; j < EPC; ++j) o[j] = (r.v[j] - mu[j]) * sc[j] + bb[j];
    } else {
      const float* g = gns + ((size_t)(m / T) * H + k) * 2;
#pragma unroll
      for (int j = 0; j < EPC; ++j) o[j] = (r.v[j] - g[2 * j]) * (g[2 * j + 1] * gnw[k + j]) + gnb[k + j];
    }
    return pack_chunk<Dt>(o);
  }
};

// FinalLayer conv_out (k=3, pad=1) from the tap-stacked GEMM Y[m] = [W_0; W_1; W_2] x_mod[m]:
// v[t] = b + Y0[t-1] + Y1[t] + Y2[t+1] within each utterance; then xt += dt*v (or v_out = v).
// `src` (null: xt itself) is the state the update starts from (the fused solve's last step).
__global__ void conv3_combine_kernel(const float* __restrict__ Y, const float* __restrict__ bias, float* xt,
                                     float* __restrict__ vout, int M, int T, int C, float dt, int* step_ctr,
                                     const float* src = nullptr) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (step_ctr && idx == 0) *step_ctr += 1;  // last kernel of the step; nothing in it reads the counter
  if (idx >= (size_t)M * C) return;
  int m = idx / C, n = idx - (size_t)m * C;
  int t = m % T;
  const size_t ld = 3 * (size_t)C;
  float v = bias[n] + Y[m * ld + C + n];
  if (t > 0) v += Y[(m - 1) * ld + n];
  if (t < T - 1) v += Y[(m + 1) * ld + 2 * C + n];
  if (vout) {
    vout[idx] = v;
  } else {
    xt[idx] = __fadd_rn((src ? src : xt)[idx], __fmul_rn(dt, v));
  }
}

// Fused solve (small M, graph path): the conv_out tap combine + Euler update of step s-1 is computed
// inside step s's proj_in A loader, exactly as conv3_combine_kernel does it (same fp32 operation order,
// so the solve stays bitwise equal to the eager one):  x_s = x_{s-1} + dt * (b + Y1[t] + Y0[t-1] +
// Y2[t+1]).  The state ping-pongs between two buffers (src = x_{s-1}, dst = x_s, written once by the
// column-tile-0 workgroups while every column tile reads src); the loader's prologue advances the step
// counter (nothing in proj_in reads it).  Step 0 starts from euler_init_kernel's image: src = x_0,
// Y1 = -b, Y0 = Y2 = 0, so v = b + (-b) = 0 exactly and x_0 passes through.
template <typename DT>
struct LoadEulerIn {
  const float* __restrict__ src;
  float* dst;
  const float* __restrict__ Y;
  const float* __restrict__ bias;
  int* ctr;
  float dt;
  int T, C;
  static constexpr int EPC = DTraits<DT>::EPC;
  static constexpr int kSrcBytes = 4;
  struct Raw { float x[EPC], b[EPC], y1[EPC], y0[EPC], y2[EPC]; int t; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {
    if (ctr && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) *ctr += 1;
  }
  __device__ Raw issue(int m, int k) const {
    Raw r;
    r.t = m % T;
    const size_t ld = 3 * (size_t)C;
#pragma unroll
    for (int j = 0; j < EPC; j += 4) {
      float4 a = ld4(src + (size_t)m * C + k + j), b = ld4(bias + k + j), y1 = ld4(Y + (size_t)m * ld + C + k + j);
      float4 y0 = r.t > 0 ? ld4(Y + (size_t)(m - 1) * ld + k + j) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 y2 = r.t < T - 1 ? ld4(Y + (size_t)(m + 1) * ld + 2 * C + k + j) : make_float4(0.f, 0.f, 0.f, 0.f);
      r.x[j] = a.x; r.x[j + 1] = a.y; r.x[j + 2] = a.z; r.x[j + 3] = a.w;
      r.b[j] = b.x; r.b[j + 1] = b.y; r.b[j + 2] = b.z; r.b[j + 3] = b.w;
      r.y1[j] = y1.x; r.y1[j + 1] = y1.y; r.y1[j + 2] = y1.z; r.y1[j + 3] = y1.w;
      r.y0[j] = y0.x; r.y0[j + 1] = y0.y; r.y0[j + 2] = y0.z; r.y0[j + 3] = y0.w;
      r.y2[j] = y2.x; r.y2[j + 1] = y2.y; r.y2[j + 2] = y2.z; r.y2[j + 3] = y2.w;
    }
    return r;
  }
  template <typename D>
  __device__ u32x4 finish(const Raw& r, int m, int k, const float*, int) const {
    float o[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) {
      float v = r.b[j] + r.y1[j];
      if (r.t > 0) v += r.y0[j];
      if (r.t < T - 1) v += r.y2[j];
      o[j] = __fadd_rn(r.x[j], __fmul_rn(dt, v));
    }
    if (blockIdx.x == 0) {
#pragma unroll
      for (int j = 0; j < EPC; j += 4)
        *reinterpret_cast<float4*>(dst + (size_t)m * C + k + j) = make_float4(o[j], o[j + 1], o[j + 2], o[j + 3]);
    }
    return pack_chunk<D>(o);
  }
};

// Fused solve start: src image x_0 (xs; null on the large-M path, whose update is in place) and a conv_out
// output whose combine is exactly 0 (see LoadEulerIn).
__global__ void euler_init_kernel(const float* __restrict__ xt, const float* __restrict__ bias, float* __restrict__ xs,
                                  float* __restrict__ Y, int M, int C) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)M * C) return;
  int m = idx / C, n = idx - (size_t)m * C;
  if (xs) xs[idx] = xt[idx];
  float* y = Y + (size_t)m * 3 * C;
  y[n] = 0.f;
  y[C + n] = -bias[n];
  y[2 * C + n] = 0.f;
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

// depthwise taps (H, 1, KS) -> tap-major (KS, H), so a wave's 64 channels read one contiguous line per tap
__global__ void taps_t_kernel(const float* __restrict__ src, float* __restrict__ dst, int H, int KS) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)H * KS) return;
  const int c = i / KS, j = i - (size_t)c * KS;
  dst[(size_t)j * H + c] = src[i];
}

__global__ void cast_kernel_bf16(const float* __restrict__ src, bf16* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (bf16)src[i];
}
__global__ void copy_kernel_f32(const float* __restrict__ src, float* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}
// conv weight (N, Cin, KT) -> tap-stacked rows (KT, N, Cin) in DT
template <typename DT>
__global__ void stack_taps_kernel(const float* __restrict__ src, DT* __restrict__ dst, int N, int Cin, int KT) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)N * Cin * KT;
  if (i >= total) return;
  int k = i % KT;
  size_t t = i / KT;
  int c = t % Cin;
  int n = t / Cin;
  store_val<DT>(dst + ((size_t)k * N + n) * Cin + c, src[i]);
}

// ------------------------------ large-M bf16 path ------------------------------
// At B*T >= 8192 rows the GEMMs are MFMA-bound and an A loader that transforms fp32 rows inside the
// GEMM re-does that work for every column tile.  There each transforming A operand is written once as
// bf16 rows (A16) by a streaming pass — LayerNorm + AdaLN modulate, GroupNorm apply or a plain cast,
// the same arithmetic as the fused loaders — and the GEMM runs on 128 x 128 LDS-DMA tiles with
// XCD-aware placement (gemm_dma.hpp).  tn().big 0 keeps the fused register-staged GEMMs;
// tn().big_min_rows: smallest B*T on the large-M path (B=4/8/16 at T=400: 93.6/113.4/188.5 ->
// 80.1/91.2/116.0 ms per solve; B=3 even); tn().big_ns: LDS ring depth of the 128 x 128 tiles (2: two
// workgroups per CU, 635 TF plain at M = 25600; 3: one, 418 TF).
thread_local bf16* g_a16 = nullptr;  // the calling thread's step workspace (set per step, A16Scope)

// Large-M fused Euler step (tune fuse_euler): the previous step's conv_out tap combine + Euler update, in place
// (each thread reads and writes only its own 8 state values), and the bf16 cast of the new state that proj_in
// reads (A16) -- conv3_combine_kernel's arithmetic in its order, then cast_bf16x8_kernel's, so the solve is
// bitwise the unfused one -- in ONE streaming pass instead of a combine launch at the end of the step and a
// cast launch at its start.  Thread 0 advances the step counter (nothing here or in proj_in reads it).
__global__ void euler_cast_kernel(float* xt, const float* __restrict__ Y, const float* __restrict__ bias,
                                  bf16* __restrict__ a16, int M, int T, int C, float dt, int* step_ctr) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (step_ctr && i == 0) *step_ctr += 1;
  const int C8 = C / 8;
  if (i >= (size_t)M * C8) return;
  const int m = i / C8, k = (int)(i - (size_t)m * C8) * 8, t = m % T;
  const size_t ld = 3 * (size_t)C;
  float x[8], o[8];
  {
    const float4 a = ld4(xt + (size_t)m * C + k), b = ld4(xt + (size_t)m * C + k + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  }
#pragma unroll
  for (int h = 0; h < 8; h += 4) {
    const float4 bb = ld4(bias + k + h), y1 = ld4(Y + (size_t)m * ld + C + k + h);
    const float4 y0 = t > 0 ? ld4(Y + (size_t)(m - 1) * ld + k + h) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 y2 = t < T - 1 ? ld4(Y + (size_t)(m + 1) * ld + 2 * C + k + h) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w}, v1[4] = {y1.x, y1.y, y1.z, y1.w};
    const float v0[4] = {y0.x, y0.y, y0.z, y0.w}, v2[4] = {y2.x, y2.y, y2.z, y2.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = bv[e] + v1[e];
      if (t > 0) v += v0[e];
      if (t < T - 1) v += v2[e];
      o[h + e] = __fadd_rn(x[h + e], __fmul_rn(dt, v));
    }
  }
  *reinterpret_cast<float4*>(xt + (size_t)m * C + k) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(xt + (size_t)m * C + k + 4) = make_float4(o[4], o[5], o[6], o[7]);
  *reinterpret_cast<u32x4*>(a16 + (size_t)m * C + k) = pack_chunk<bf16>(o);
}

__global__ void cast_bf16x8_kernel(const float* __restrict__ src, int ld, bf16* __restrict__ dst, int M, int K) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int K8 = K / 8;
  if (i >= (size_t)M * K8) return;
  const int m = i / K8, c = i - (size_t)m * K8;
  const float* p = src + (size_t)m * ld + c * 8;
  const float4 a = ld4(p), b = ld4(p + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  *reinterpret_cast<u32x4*>(dst + (size_t)m * K + c * 8) = pack_chunk<bf16>(v);
}

// A16 = GroupNorm(D) (LoadGN's arithmetic: (x - mean) * (rstd * gn_w) + gn_b); D fp32, or bf16 on the
// x16 path (then written in place: each thread reads its 8 elements before storing them).
template <typename DS>
__global__ void gn_apply_bf16_kernel(LoadGN<bf16> al, const DS* src, bf16* dst, int M) {
  const int H = al.H, K8 = H / 8;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)M * K8) return;
  const int m = i / K8, k = (int)(i - (size_t)m * K8) * 8;
  float xv[8];
  ldx8<DS>(src + (size_t)m * H + k, xv);
  const float* g = al.gns + ((size_t)(m / al.T) * H + k) * 2;
  const float4 g0 = ld4(g), g1 = ld4(g + 4), g2 = ld4(g + 8), g3 = ld4(g + 12);
  const float4 w0 = ld4(al.gnw + k), w1 = ld4(al.gnw + k + 4), b0 = ld4(al.gnb + k), b1 = ld4(al.gnb + k + 4);
  const float mu[8] = {g0.x, g0.z, g1.x, g1.z, g2.x, g2.z, g3.x, g3.z};
  const float rs[8] = {g0.y, g0.w, g1.y, g1.w, g2.y, g2.w, g3.y, g3.w};
  const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
  const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (xv[j] - mu[j]) * (rs[j] * wv[j]) + bv[j];
  *reinterpret_cast<u32x4*>(dst + (size_t)m * H + k) = pack_chunk<bf16>(o);
}

// A16 = LayerNorm(X) (+affine) * (1 + scale) + shift (LoadLNMod's arithmetic); 2 rows per workgroup,
// the row statistics combined once per row from the producer's partials.  X fp32 (al.x) or the x16
// path's bf16 rows (al.x16).
template <bool AFF, typename XT>
__global__ __launch_bounds__(256) void lnmod_apply_bf16_kernel(LoadLNMod<bf16, AFF> al, const XT* xs, bf16* __restrict__ dst,
                                                               int M) {
  __shared__ float st[2][2];
  const int r = threadIdx.x >> 7, lt = threadIdx.x & 127;
  const int m = blockIdx.x * 2 + r;
  if (lt == 0 && m < M) row_stats_from_partials(al.S, m, al.NT, al.tw, al.eps, st[r][0], st[r][1]);
  __syncthreads();
  if (m >= M) return;
  const float mean = st[r][0], rstd = st[r][1];
  const ModRef md = al.mod.at();
  const size_t mo = (size_t)(m / md.div) * md.ms;
  const int K = al.kdim;
  for (int k = lt * 8; k < K; k += 128 * 8) {
    float xv[8];
    ldx8<XT>(xs + (size_t)m * al.ld + k, xv);
    const float4 c0 = ld4(md.sc + mo + k), c1 = ld4(md.sc + mo + k + 4), h0 = ld4(md.sh + mo + k), h1 = ld4(md.sh + mo + k + 4);
    float4 w0 = make_float4(1.f, 1.f, 1.f, 1.f), w1 = w0, b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (AFF) { w0 = ld4(al.lnw + k); w1 = ld4(al.lnw + k + 4); b0 = ld4(al.lnb + k); b1 = ld4(al.lnb + k + 4); }
    const float sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s1 = 1.0f + sc[j];
      o[j] = ((xv[j] - mean) * rstd) * (wv[j] * s1) + (bv[j] * s1 + sh[j]);
    }
    *reinterpret_cast<u32x4*>(dst + (size_t)m * K + k) = pack_chunk<bf16>(o);
  }
}

// ---- MX-fp8 operands (fp8 handles, large M; gemm_8p.hpp): the same normalise passes writing e4m3 rows +
// the scale image through store_f8x8.
template <typename DS>
__global__ void gn_apply_f8_kernel(LoadGN<bf16> al, const DS* src, unsigned char* dst, unsigned char* sc, int M) {
  const int H = al.H, K8 = H / 8;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)M * K8) return;  // M * K8 is a multiple of 64: whole waves leave
  const int m = i / K8, k = (int)(i - (size_t)m * K8) * 8;
  float xv[8];
  ldx8<DS>(src + (size_t)m * H + k, xv);
  const float* g = al.gns + ((size_t)(m / al.T) * H + k) * 2;
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (xv[j] - g[2 * j]) * (g[2 * j + 1] * al.gnw[k + j]) + al.gnb[k + j];
  store_f8x8(o, dst, sc, m, k, H);
}

template <bool AFF, typename XT>
__global__ __launch_bounds__(256) void lnmod_apply_f8_kernel(LoadLNMod<bf16, AFF> al, const XT* xs, unsigned char* dst,
                                                             unsigned char* sc, int M) {
  __shared__ float st[2][2];
  const int r = threadIdx.x >> 7, lt = threadIdx.x & 127;
  const int m = blockIdx.x * 2 + r;
  if (lt == 0 && m < M) row_stats_from_partials(al.S, m, al.NT, al.tw, al.eps, st[r][0], st[r][1]);
  __syncthreads();
  if (m >= M) return;  // a whole 128-lane row half-block (two waves) leaves together
  const float mean = st[r][0], rstd = st[r][1];
  const ModRef md = al.mod.at();
  const size_t mo = (size_t)(m / md.div) * md.ms;
  const int K = al.kdim;
  for (int k = lt * 8; k < K; k += 128 * 8) {
    float xv[8], o[8];
    ldx8<XT>(xs + (size_t)m * al.ld + k, xv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s1 = 1.0f + md.sc[mo + k + j];
      const float wv = AFF ? al.lnw[k + j] : 1.0f, bv = AFF ? al.lnb[k + j] : 0.0f;
      o[j] = ((xv[j] - mean) * rstd) * (wv * s1) + (bv * s1 + md.sh[mo + k + j]);
    }
    store_f8x8(o, dst, sc, m, k, K);
  }
}

static int f8_prep(const LoadGN<bf16>& al, int M, unsigned char* a8, unsigned char* s8, hipStream_t st) {
  const size_t n = (size_t)M * (al.H / 8);
  if (al.D16)
    hipLaunchKernelGGL(gn_apply_f8_kernel<bf16>, dim3((n + 255) / 256), dim3(256), 0, st, al, al.D16, a8, s8, M);
  else
    hipLaunchKernelGGL(gn_apply_f8_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, st, al, al.D, a8, s8, M);
  FL_LAUNCH_CHECK();
  return kOk;
}
template <bool AFF>
static int f8_prep(const LoadLNMod<bf16, AFF>& al, int M, unsigned char* a8, unsigned char* s8, hipStream_t st) {
  FL_REQUIRE(al.kdim % 1024 == 0, "f8_prep(LN): K=%d", al.kdim);
  if (al.x16)
    hipLaunchKernelGGL((lnmod_apply_f8_kernel<AFF, bf16>), dim3((M + 1) / 2), dim3(256), 0, st, al, al.x16, a8, s8, M);
  else
    hipLaunchKernelGGL((lnmod_apply_f8_kernel<AFF, float>), dim3((M + 1) / 2), dim3(256), 0, st, al, al.x, a8, s8, M);
  FL_LAUNCH_CHECK();
  return kOk;
}

static int big_prep(const LoadF32<bf16>& al, int M, int K, bf16* a16, hipStream_t st) {
  const size_t n = (size_t)M * (K / 8);
  hipLaunchKernelGGL(cast_bf16x8_kernel, dim3((n + 255) / 256), dim3(256), 0, st, al.p, al.ld, a16, M, K);
  FL_LAUNCH_CHECK();
  return kOk;
}
static int big_prep(const LoadGN<bf16>& al, int M, int K, bf16* a16, hipStream_t st) {
  FL_REQUIRE(K == al.H && K % 8 == 0, "big_prep(GN): K=%d", K);
  const size_t n = (size_t)M * (K / 8);
  if (al.D16)  // x16 path: bf16 depthwise output
    hipLaunchKernelGGL(gn_apply_bf16_kernel<bf16>, dim3((n + 255) / 256), dim3(256), 0, st, al, al.D16, a16, M);
  else
    hipLaunchKernelGGL(gn_apply_bf16_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, st, al, al.D, a16, M);
  FL_LAUNCH_CHECK();
  return kOk;
}
template <bool AFF>
static int big_prep(const LoadLNMod<bf16, AFF>& al, int M, int K, bf16* a16, hipStream_t st) {
  FL_REQUIRE(K == al.kdim && K % 8 == 0, "big_prep(LN): K=%d", K);
  if (al.x16)
    hipLaunchKernelGGL((lnmod_apply_bf16_kernel<AFF, bf16>), dim3((M + 1) / 2), dim3(256), 0, st, al, al.x16, a16, M);
  else
    hipLaunchKernelGGL((lnmod_apply_bf16_kernel<AFF, float>), dim3((M + 1) / 2), dim3(256), 0, st, al, al.x, a16, M);
  FL_LAUNCH_CHECK();
  return kOk;
}
template <class EP>
static int launch_big(const LoadPlain<bf16>& al, const bf16* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  // 256 x 256 8-phase tiles once there are enough of them to fill the chip (gemm_8p.hpp; M = 25600:
  // 855 vs 774 TF plain for the 128 x 128 ring, tools/probe_gemm.py; M = 6400: 440 vs 643 TF)
  const int g8 = tn().g8p_rows;
  if (g8 > 0 && M >= g8 && N % 256 == 0 && K % 128 == 0) {
    // one 256 x 256 tile per CU at a time: use it only when the last round of tiles is well filled
    // (conv_out's N = 768 at M = 25600 gives 300 tiles = 1.17 rounds: measured slower than the ring)
    const size_t tiles = (size_t)((M + 255) / 256) * (N / 256), rounds = (tiles + 255) / 256;
    if (tiles * 10 >= rounds * 256 * 7) return launch_gemm8p(al.p, al.ld, W, ldw, ep, M, N, K, st);
  }
  if (tn().big_ns == 2) return launch_gemm_dma_fixed<128, 128, 2, true>(al, W, ldw, ep, M, N, K, st);
  return launch_gemm_dma_fixed<128, 128, 3, true>(al, W, ldw, ep, M, N, K, st);
}

// tn().lnfold: 1 (default, bf16 handles) mlp.0 / conv_out run as plain bf16 GEMMs with the
// LayerNorm folded into the epilogue (EpiLNFold); 0: LayerNorm + modulation in the A loader.
// On the large-M path the fold pays only from tn().fold_big_rows rows (default 6144): measured
// (ms/solve, fold vs not) M = 1600: 84.8 vs 81.7, 2400 (nfe 256): 187.1 vs 182.8, 3200: 94.2 vs 93.2,
// 6400: 116.2 vs 118.0, 25600: 409.5 vs 411.1 — with few 128 x 128 tiles the x*alpha stores lengthen
// conv_3 more than the dropped LayerNorm pass saves.

// Denoiser GEMM dispatch: DMA pipeline for bf16 at small/mid M, gemm_kernel otherwise.
template <typename DT, class AL, class EP>
static int den_gemm(GemmCfg c, bool wide_a, const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K,
                    hipStream_t st) {
  if constexpr (std::is_same<DT, bf16>::value) {
    if (c == kCfgLarge && tn().big) {
      if constexpr (AL::kSrcBytes == 2) {
        return launch_big(al, W, ldw, ep, M, N, K, st);
      } else {
        FL_REQUIRE(g_a16, "den_gemm: large-M A16 workspace missing");
        int rc = big_prep(al, M, K, g_a16, st);
        if (rc) return rc;
        return launch_big(LoadPlain<bf16>{g_a16, K}, W, ldw, ep, M, N, K, st);
      }
    }
  }
  if (c == kCfgTiny) {  // row partials are 32 columns wide (cfg_bn): every GEMM of the step uses BN = 32
    if constexpr (std::is_same<DT, bf16>::value) {
      if (tn().use_dma >= 2 || (tn().use_dma == 1 && AL::kSrcBytes == 2)) return launch_gemm_dma<32, 32>(al, W, ldw, ep, M, N, K, st);
    }
    return launch_gemm_cfg<32, 32, 3, DT>(al, W, ldw, ep, M, N, K, st);
  }
  if constexpr (std::is_same<DT, bf16>::value) {
    // measured (B = 1, T = 400, stamps + in-graph dup timing): the DMA ring shortens the K loop of
    // the bf16-A GEMMs; for fp32-A loaders its LDS->LDS transform pass costs more LDS bandwidth than
    // the ring saves, and at mid M its ~150 KB of LDS drops residency to one block per CU
    if (c == kCfgSmall && (tn().use_dma >= 2 || (tn().use_dma == 1 && AL::kSrcBytes == 2)))
      return launch_gemm_dma<32, 64>(al, W, ldw, ep, M, N, K, st);
  }
  return wide_a ? launch_gemm_auto<DT>(c, kWideA, al, W, ldw, ep, M, N, K, st) : launch_gemm_auto<DT>(c, al, W, ldw, ep, M, N, K, st);
}

// ------------------------------ handle ------------------------------

struct DenBlockW {
  const void* w2; const void* w3; const void* m0; const void* m2;  // DT (H x H)
  // fp8 handles: e4m3 copies + W scale images of w2, w3, m0, m2 (the final layer: w2, w3)
  const unsigned char* q[4] = {nullptr, nullptr, nullptr, nullptr};
  const unsigned char* qs[4] = {nullptr, nullptr, nullptr, nullptr};
  const float *b2, *b3, *mb0, *mb2, *lnw, *lnb, *lnmw, *lnmb, *dww, *dwb, *gnw, *gnb;
};

struct Den {
  int C, H, NB, KS, S, dt;  // dt: 0 f32, 1 bf16 (also for fp8 handles)
  bool f8 = false;          // FLAMED_FP8 handle: bf16 everywhere + MX-fp8 conv_2/conv_3/mlp.0/mlp.2 at large M
  int MS;                   // mods row stride: MS0 modulation floats + the LayerNorm-fold tables (bf16)
  int MS0;                  // (6 NB + 5) H: shift/scale/gate vectors of every adaLN_modulation
  int fold = 0;             // row holds fold tables [wa, wb] per LN-consuming GEMM (mlp.0 x NB, conv_out)
  char* dev = nullptr;      // packed weight arena
  size_t dev_bytes = 0;
  // fp32 AdaLN path
  float *t0w, *t0b, *t2w, *t2b, *cw, *cb, *adaw, *adab;
  // DT
  void* win; const float* bin;
  std::vector<DenBlockW> blk;
  DenBlockW fin;  // m0/m2/lnmw.. unused
  void* wout; const float* bout;
  int device = -1;          // device of the weight arena (from the loaded weights' pointers)
  std::recursive_mutex mu;  // one call at a time per handle (single-stream use: counters, graph cache)
  Tune tune;                // knob snapshot of this handle (process defaults unless tune_own)
  int tune_seen = -1;       // process tune epoch of that snapshot
  bool tune_own = false;    // set by flamed_den_tune: this handle keeps its own knobs
  int tune_ver = 0;         // bumped on every change of `tune` (graph cache key)
  int part_epoch = -1;      // tune_ver pinned by the s0 == 0 part of a flamed_den_solve_part sequence
  // graph cache
  hipGraphExec_t gexec = nullptr;
  hipStream_t cap_stream = nullptr;
  static constexpr int kMaxSplit = 4;          // sub-batch chains of a large-M solve (den_split)
  hipStream_t cap_aux[kMaxSplit] = {};         // (unused since round 5: each chain is captured on cap_stream)
  hipEvent_t cap_ev[kMaxSplit] = {};           // fork / join events of the chains' replays
  hipGraphExec_t gexec_c[kMaxSplit] = {};      // graphs of chains 1..S-1 (chain 0's is gexec)
  hipStream_t run_aux[3][kMaxSplit] = {};      // replay streams of the chains per tune split_prio (den_chain_streams)
  static constexpr int kMaxParked = 8;
  hipStream_t parked[kMaxParked] = {};         // streams the queue probe found serialising with a chain's (kept alive)
  int n_parked = 0, qprobe_retries = 0;
  int qprobe_busy = 0;  // probe pairs that neither ran concurrently nor back-to-back (the device was busy): not parked
  int* qprobe = nullptr;                       // probe flag + result words
  int g_B = -1, g_T = -1, g_nfe = -1, g_epoch = -1;
  const void *g_xt = nullptr, *g_mods = nullptr, *g_ws = nullptr;
  int* ctr = nullptr;  // device Euler step counter for graph replay
  int* scnt = nullptr;  // split-K tile counters (zeroed at load; every launch leaves them zero)
  static constexpr int kSplitCounters = 16384;
  int* gcnt = nullptr;  // fused GroupNorm-finalize counters, one per (utterance, 64-channel group)
  static constexpr int kGnCounters = 65536;
  // persistent B = 1 solve (persist.hpp): scratch (counters first), device verdict, failure bookkeeping
  char* pmem = nullptr;
  int* pfail = nullptr;      // device: failed persistent launches so far (sticky, written by the kernel)
  int* pfail_host = nullptr; // pinned copy of it, refreshed asynchronously after every uncaptured launch
  int pfails_seen = 0;       // failures the host has acted on
  static constexpr int kPersistRetry = 3;  // failed launches before the handle gives up the persistent path
  int pdev_ok = -1;          // 1: 256 CUs and one 256-thread workgroup per CU fits; 0: not on this device
  bool pbroken = false;      // kPersistRetry launches failed on this handle: launch path from then on
  int pruns = 0;             // persistent launches enqueued
  int ppath = -1;            // path of the solve whose step 0 ran last: 1 persistent, 0 graph of launches
  int ppath_key[3] = {-1, -1, -1};  // its (B, T, nfe)
  // the most recent uncaptured persistent launches, a ring: HIP events around the kernel ([0], [1]: device time) and
  // behind the async copies that follow it ([2]), and each launch's own error word (pinned; 0 = the launch
  // succeeded), so a caller can ask after one launch without waiting (flamed_den_persist_query)
  static constexpr int kPRing = 64;
  hipEvent_t pring[kPRing][3] = {};
  int* perr_host = nullptr;  // kPRing pinned ints: the error word of the launch in that slot
  long long pring_n = 0;     // launches recorded so far (slot = n % kPRing)
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Wait for the last uncaptured persistent launch of the handle (its end event), then free the persistent
// scratch, the pinned failure word and the timing events (handle destroy / re-load on another device).
static void persist_release(Den* d) {
  if (d->pring_n > 0) {
    hipEvent_t last = d->pring[(d->pring_n - 1) % Den::kPRing][2];
    if (last) (void)hipEventSynchronize(last);
  }
  if (d->pmem) { (void)hipFree(d->pmem); d->pmem = nullptr; }
  d->pfail = nullptr;
  if (d->pfail_host) { (void)hipHostFree(d->pfail_host); d->pfail_host = nullptr; }
  if (d->perr_host) { (void)hipHostFree(d->perr_host); d->perr_host = nullptr; }
  for (auto& pr : d->pring)
    for (hipEvent_t& e : pr)
      if (e) { (void)hipEventDestroy(e); e = nullptr; }
  d->pring_n = 0;
}
static int persist_alloc(Den* d, hipStream_t st);

// Active knobs of a handle call: the process defaults (re-snapshotted when flamed_tune moved the epoch)
// unless flamed_den_tune gave the handle its own.
static const Tune* den_tune_sync(Den* d) {
  if (!d->tune_own) {
    int ep = 0;
    Tune t = tune_snapshot(&ep);
    if (ep != d->tune_seen) {
      d->tune = t;
      d->tune_seen = ep;
      ++d->tune_ver;
    }
  }
  return &d->tune;
}

// Prologue of every compute entry point on a handle: serialise calls on the handle, make its device
// current, and install its knob snapshot for the launches of this call.
struct DenCall {
  std::lock_guard<std::recursive_mutex> lk;
  DeviceGuard dg;
  TuneScope ts;
  explicit DenCall(Den* d) : lk(d->mu), dg(d->device), ts(den_tune_sync(d)) {}
};
#define FL_DEN_CALL(d)                                                                              \
  ::fl::DenCall call_(d);                                                                           \
  do {                                                                                              \
    if (call_.dg.err != hipSuccess) {                                                               \
      ::fl::set_error("hipSetDevice(%d) -> %s", (d)->device, hipGetErrorString(call_.dg.err));     \
      return ::fl::kHip;                                                                            \
    }                                                                                               \
  } while (0)

struct DenWs {
  float* X;    // residual stream, M x H (bf16 rows on the x16 path)
  float* S0;   // LN partials, M x (H/64) x 2
  float* S1;
  float* D;    // depthwise conv output, M x H fp32 (bf16 on the x16 path)
  void* U;     // GEMM intermediate, M x H (DT)
  float* GP;   // GroupNorm chunk partials, B x TS x H x 3
  float* GNS;  // GroupNorm (mean, rstd), B x H x 2
  float* Y;    // conv_out tap-stacked GEMM output, M x 3C
  float* SL;   // split-K slabs (small-M GEMMs), SLn floats
  size_t SLn;
  bf16* A16;   // large-M bf16 path: normalised A operand rows, M x H (null otherwise)
  bf16* XA;    // LayerNorm fold: X * alpha_next rows (bf16 handles), M x H
  float* XP;   // fused solve: second Euler-state buffer, M x C
};

// split-K slab capacity: 32 x 64 tiles of the widest GEMM (max(H, 3C) columns) x 4 slices, small M only
static size_t den_slab_floats(const Den* d, int B, int T) {
  const size_t M = (size_t)B * T;
  if (M >= 2048) return 0;
  const size_t nmax = (size_t)(d->H > 3 * d->C ? d->H : 3 * d->C);
  return ((M + 31) / 32) * (nmax / 64) * 4 * 32 * 64;
}

// Large-M bf16 residual stream (tune x16): X and the depthwise output D are stored as bf16 rows on the
// large-M path (half the HBM bytes of the residual epilogues, the depthwise conv and the GroupNorm pass);
// norms, statistics, GEMM accumulation and the Euler state stay fp32.
static bool den_x16(const Den* d, int B, int T) {
  const Tune& t = tn();
  return d->dt == FLAMED_BF16 && t.x16 && t.big && (size_t)B * T >= (size_t)t.big_min_rows &&
         !(t.bn32 && (size_t)B * T < (size_t)kTinyRows);
}

static size_t den_ws_layout(const Den* d, int B, int T, void* base, DenWs* w) {
  size_t M = (size_t)B * T;
  size_t es = d->dt == FLAMED_BF16 ? 2 : 4;
  const size_t xs = den_x16(d, B, T) ? 2 : 4;  // residual stream / depthwise output element size
  size_t NTmax = d->H / 32;  // LN row partials per row: H / BN, BN >= 32
  size_t TS = (T + 63) / 64;
  const size_t sl = den_slab_floats(d, B, T);
  const size_t a16 = (d->dt == FLAMED_BF16 && M >= (size_t)tn().big_min_rows) ? 2 * M * d->H : 0;  // large-M path range
  const size_t xa = d->fold ? 2 * M * d->H : 0;
  size_t sizes[12] = {xs * M * d->H, 8 * M * NTmax, 8 * M * NTmax, xs * M * d->H, es * M * d->H, 12 * B * TS * d->H,
                      8 * (size_t)B * d->H, 12 * M * d->C, 4 * sl, a16, xa, 4 * M * d->C};
  size_t off = 0;
  void* ptrs[12];
  for (int i = 0; i < 12; ++i) {
    ptrs[i] = base ? (char*)base + off : nullptr;
    off += align256(sizes[i]);
  }
  if (w) {
    w->X = (float*)ptrs[0]; w->S0 = (float*)ptrs[1]; w->S1 = (float*)ptrs[2]; w->D = (float*)ptrs[3];
    w->U = ptrs[4]; w->GP = (float*)ptrs[5]; w->GNS = (float*)ptrs[6]; w->Y = (float*)ptrs[7];
    w->SL = (float*)ptrs[8]; w->SLn = sl;
    w->A16 = a16 ? (bf16*)ptrs[9] : nullptr;
    w->XA = xa ? (bf16*)ptrs[10] : nullptr;
    w->XP = (float*)ptrs[11];
  }
  return off;
}
static size_t den_ws_bytes(const Den* d, int B, int T) { return den_ws_layout(d, B, T, nullptr, nullptr); }

// Large-M solves as concurrent sub-batches (tune split_batch, default 2): utterances are independent in the
// denoiser (GroupNorm statistics and the depthwise halo never cross an utterance: prob_generator.py:81-89),
// so the batch's Euler steps run as S chains of B / S utterances, captured as S parallel branches of one graph.
// One chain's inter-kernel gaps and the partly filled last round of its GEMM tiles are then covered by the
// other chain's kernels (B = 64: 336 -> 295 ms, B = 32: 189 -> 159 ms; S = 4: 307 / 189).  The chains are
// bitwise equal to the single chain (test_cfg2_split_batch_bitwise) since dwgn's pair math is scalar (dg_fma:
// the packed form was perturbed by co-resident fp32-MFMA waves, DESIGN.md "dwgn concurrency").  fp8 handles
// keep one chain (their MX GEMMs need the large tiles of the whole batch).
static int den_split(const Den* d, int B, int T) {
  const Tune& tu = tn();
  const int S = tu.split_batch;
  if (S <= 1 || d->dt != FLAMED_BF16 || d->f8 || !tu.big || B % S != 0) return 1;
  if ((size_t)(B / S) * T < (size_t)tu.split_min_rows) return 1;
  return S;
}
// workspace of one of the S sub-batch chains (each chain has its own; chain k's starts at k * this)
static size_t den_split_ws(const Den* d, int B, int T, int S) { return align256(den_ws_bytes(d, B / S, T)); }
// workspace a solve of B x T needs (the whole-batch layout, or S chain workspaces when it splits)
static size_t den_solve_ws(const Den* d, int B, int T) {
  const size_t one = den_ws_bytes(d, B, T);
  const int S = den_split(d, B, T);
  const size_t split = S > 1 ? (size_t)S * den_split_ws(d, B, T, S) : 0;
  return one > split ? one : split;
}

static bool stream_capturing(hipStream_t st);

}  // namespace fl

using namespace fl;

extern "C" {

static int den_chain_streams(Den* d, int S, hipStream_t st);

FLAMED_API int flamed_den_create(int C, int H, int n_blocks, int kernel, int spk_dim, int dtype, flamed_den_t* out) {
  FL_REQUIRE(out, "flamed_den_create: null out");
  FL_REQUIRE(C > 0 && C % 64 == 0 && H % 256 == 0 && H <= 1024 && n_blocks >= 1 && spk_dim % 64 == 0,
             "flamed_den_create: unsupported dims C=%d H=%d S=%d", C, H, spk_dim);
  FL_REQUIRE(kernel == 31, "flamed_den_create: only convnext kernel_size=31 is specialised (got %d)", kernel);
  FL_REQUIRE(dtype == FLAMED_F32 || dtype == FLAMED_BF16 || dtype == FLAMED_FP8,
             "flamed_den_create: dtype must be FLAMED_F32, FLAMED_BF16 or FLAMED_FP8");
  FL_REQUIRE(dtype != FLAMED_FP8 || (H % 256 == 0 && H <= kMxMaxK), "flamed_den_create: fp8 needs H %% 256 == 0, H <= %d", kMxMaxK);
  Den* d = new Den();
  d->C = C; d->H = H; d->NB = n_blocks; d->KS = kernel; d->S = spk_dim;
  d->dt = dtype == FLAMED_FP8 ? FLAMED_BF16 : dtype;
  d->f8 = dtype == FLAMED_FP8;
  dtype = d->dt;
  d->MS0 = (6 * n_blocks + 5) * H;
  d->fold = dtype == FLAMED_BF16;
  d->MS = d->MS0 + (d->fold ? n_blocks * 2 * H + 2 * 3 * C : 0);
  *out = reinterpret_cast<flamed_den_t>(d);
  return kOk;
}

FLAMED_API int flamed_den_destroy(flamed_den_t h) {
  Den* d = reinterpret_cast<Den*>(h);
  if (!d) return kOk;
  {
    std::lock_guard<std::recursive_mutex> lk(d->mu);
    DeviceGuard dg(d->device);
    retire_graph(d->gexec);
    for (auto& g : d->gexec_c) retire_graph(g);
    if (d->cap_stream) (void)hipStreamDestroy(d->cap_stream);
    for (auto& a : d->cap_aux)
      if (a) (void)hipStreamDestroy(a);
    for (auto& r : d->run_aux)
      for (auto& a : r)
        if (a) (void)hipStreamDestroy(a);
    for (int i = 0; i < d->n_parked; ++i) (void)hipStreamDestroy(d->parked[i]);
    if (d->qprobe) (void)hipFree(d->qprobe);
    for (auto& e : d->cap_ev)
      if (e) (void)hipEventDestroy(e);
    if (d->ctr) (void)hipFree(d->ctr);
    if (d->scnt) (void)hipFree(d->scnt);
    if (d->gcnt) (void)hipFree(d->gcnt);
    persist_release(d);
    if (d->dev) (void)hipFree(d->dev);
  }
  delete d;
  return kOk;
}

FLAMED_API int flamed_den_num_weights(flamed_den_t h) {
  Den* d = reinterpret_cast<Den*>(h);
  return d ? FLAMED_DEN_HEAD_W + FLAMED_DEN_BLOCK_W * d->NB + FLAMED_DEN_FINAL_W : -1;
}

FLAMED_API int flamed_den_device(flamed_den_t h) {
  Den* d = reinterpret_cast<Den*>(h);
  return d ? d->device : -1;
}

FLAMED_API int flamed_den_tune(flamed_den_t h, const char* key, int value) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d, "flamed_den_tune: null handle");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  den_tune_sync(d);
  Tune t = d->tune;
  const int rc = tune_apply(t, key, value);
  if (rc) return rc;
  d->tune = t;
  d->tune_own = true;
  ++d->tune_ver;
  return kOk;
}

FLAMED_API int flamed_den_load(flamed_den_t h, const float* const* w, int n, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && w, "flamed_den_load: null handle/weights");
  FL_REQUIRE(n == flamed_den_num_weights(h), "flamed_den_load: expected %d weight pointers, got %d", flamed_den_num_weights(h), n);
  for (int i = 0; i < n; ++i) FL_REQUIRE(w[i], "flamed_den_load: weight %d is null", i);
  int wdev = -1;
  FL_REQUIRE(device_of(w[0], &wdev) == kOk, "flamed_den_load: weights must be device memory");
  for (int i = 1; i < n; ++i) FL_REQUIRE_ON(w[i], wdev, "flamed_den_load");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  if (d->device >= 0 && d->device != wdev) {  // re-load onto another device: drop the old device's state
    DeviceGuard og(d->device);
    retire_graph(d->gexec);
    for (auto& g : d->gexec_c) retire_graph(g);
    if (d->cap_stream) { (void)hipStreamDestroy(d->cap_stream); d->cap_stream = nullptr; }
    for (auto& a : d->cap_aux)
      if (a) { (void)hipStreamDestroy(a); a = nullptr; }
    for (auto& r : d->run_aux)
      for (auto& a : r)
        if (a) { (void)hipStreamDestroy(a); a = nullptr; }
    for (int i = 0; i < d->n_parked; ++i) (void)hipStreamDestroy(d->parked[i]);
    d->n_parked = 0;
    if (d->qprobe) { (void)hipFree(d->qprobe); d->qprobe = nullptr; }
    for (auto& e : d->cap_ev)
      if (e) { (void)hipEventDestroy(e); e = nullptr; }
    if (d->ctr) { (void)hipFree(d->ctr); d->ctr = nullptr; }
    if (d->scnt) { (void)hipFree(d->scnt); d->scnt = nullptr; }
    if (d->gcnt) { (void)hipFree(d->gcnt); d->gcnt = nullptr; }
    persist_release(d);
    if (d->dev) { (void)hipFree(d->dev); d->dev = nullptr; }
    d->pdev_ok = -1;
  }
  d->device = wdev;
  FL_ON_DEVICE(wdev);
  const int H = d->H, C = d->C, S = d->S, NB = d->NB, KS = d->KS;
  const size_t es = d->dt == FLAMED_BF16 ? 2 : 4;
  // arena layout: packed GEMM weights and copies of every vector (the caller may free its tensors)
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
  size_t o_t0w = take(4ull * H * 256), o_t0b = take(4ull * H), o_t2w = take(4ull * H * H), o_t2b = take(4ull * H);
  size_t o_cw = take(4ull * H * S), o_cb = take(4ull * H);
  size_t o_adaw = take(4ull * d->MS0 * H), o_adab = take(4ull * d->MS0);
  size_t o_win = take(es * H * C);
  std::vector<size_t> o_blk(NB);
  for (int i = 0; i < NB; ++i) o_blk[i] = take(es * 4ull * H * H);
  size_t o_fin = take(es * 2ull * H * H);
  size_t o_out = take(es * (size_t)C * 3 * H);
  std::vector<size_t> o_dw(NB + 1);
  for (int i = 0; i <= NB; ++i) o_dw[i] = take(4ull * KS * H);
  const size_t n_vec = 1 + 11ull * NB + 5;  // H-wide vectors: proj_in bias, 11 per block, 5 final
  const size_t o_vec = take(4ull * (n_vec * H + C));
  const size_t q_bytes = (size_t)H * H + mx_scale_bytes(H, H);  // one fp8 matrix + its scale image
  const size_t o_q = d->f8 ? take(q_bytes * (4ull * NB + 2)) : 0;
  if (d->dev) { FL_HIP(hipFree(d->dev)); d->dev = nullptr; }
  FL_HIP(hipMalloc(&d->dev, off));
  d->dev_bytes = off;
  char* base = d->dev;
  auto cpy = [&](size_t o, const float* src, size_t n) -> int {
    hipLaunchKernelGGL(copy_kernel_f32, dim3((n + 255) / 256), dim3(256), 0, st, src, reinterpret_cast<float*>(base + o), n);
    FL_LAUNCH_CHECK();
    return kOk;
  };
  auto quant = [&](int slot, const float* src, const unsigned char** q, const unsigned char** qs) -> int {
    if (!d->f8) return kOk;
    unsigned char* p = reinterpret_cast<unsigned char*>(base + o_q + (size_t)slot * q_bytes);
    const int nb = H * (H / 32);
    hipLaunchKernelGGL(quant_w_f8_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, src, H, H, p, p + (size_t)H * H);
    FL_LAUNCH_CHECK();
    *q = p;
    *qs = p + (size_t)H * H;
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
  size_t vcur = o_vec;
  auto vec = [&](const float* src, size_t n, const float** dst) -> int {
    TRY(cpy(vcur, src, n));
    *dst = reinterpret_cast<const float*>(base + vcur);
    vcur += 4 * n;
    return kOk;
  };
  TRY(cpy(o_t0w, w[0], (size_t)H * 256)); TRY(cpy(o_t0b, w[1], H));
  TRY(cpy(o_t2w, w[2], (size_t)H * H)); TRY(cpy(o_t2b, w[3], H));
  TRY(cpy(o_cw, w[4], (size_t)H * S)); TRY(cpy(o_cb, w[5], H));
  TRY(cast(o_win, w[6], (size_t)H * C));
  d->t0w = (float*)(base + o_t0w); d->t0b = (float*)(base + o_t0b); d->t2w = (float*)(base + o_t2w); d->t2b = (float*)(base + o_t2b);
  d->cw = (float*)(base + o_cw); d->cb = (float*)(base + o_cb); d->adaw = (float*)(base + o_adaw); d->adab = (float*)(base + o_adab);
  d->win = base + o_win;
  TRY(vec(w[7], H, &d->bin));
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
    TRY(quant(4 * i + 0, bw[8], &B.q[0], &B.qs[0])); TRY(quant(4 * i + 1, bw[10], &B.q[1], &B.qs[1]));
    TRY(quant(4 * i + 2, bw[14], &B.q[2], &B.qs[2])); TRY(quant(4 * i + 3, bw[16], &B.q[3], &B.qs[3]));
    hipLaunchKernelGGL(taps_t_kernel, dim3((H * KS + 255) / 256), dim3(256), 0, st, bw[4], reinterpret_cast<float*>(base + o_dw[i]), H, KS);
    FL_LAUNCH_CHECK();
    B.dww = reinterpret_cast<float*>(base + o_dw[i]);
    TRY(vec(bw[2], H, &B.lnw)); TRY(vec(bw[3], H, &B.lnb)); TRY(vec(bw[5], H, &B.dwb)); TRY(vec(bw[6], H, &B.gnw));
    TRY(vec(bw[7], H, &B.gnb)); TRY(vec(bw[9], H, &B.b2)); TRY(vec(bw[11], H, &B.b3)); TRY(vec(bw[12], H, &B.lnmw));
    TRY(vec(bw[13], H, &B.lnmb)); TRY(vec(bw[15], H, &B.mb0)); TRY(vec(bw[17], H, &B.mb2));
  }
  {
    const float* const* fw = w + FLAMED_DEN_HEAD_W + FLAMED_DEN_BLOCK_W * NB;
    TRY(cpy(o_adaw + 4ull * (size_t)NB * 6 * H * H, fw[0], 5ull * H * H));
    TRY(cpy(o_adab + 4ull * (size_t)NB * 6 * H, fw[1], 5ull * H));
    DenBlockW& F = d->fin;
    hipLaunchKernelGGL(taps_t_kernel, dim3((H * KS + 255) / 256), dim3(256), 0, st, fw[2], reinterpret_cast<float*>(base + o_dw[NB]), H, KS);
    FL_LAUNCH_CHECK();
    F.dww = reinterpret_cast<float*>(base + o_dw[NB]);
    TRY(vec(fw[3], H, &F.dwb)); TRY(vec(fw[4], H, &F.gnw)); TRY(vec(fw[5], H, &F.gnb));
    TRY(cast(o_fin, fw[6], (size_t)H * H)); TRY(vec(fw[7], H, &F.b2));
    TRY(cast(o_fin + es * H * H, fw[8], (size_t)H * H)); TRY(vec(fw[9], H, &F.b3));
    F.w2 = base + o_fin; F.w3 = base + o_fin + es * H * H;
    TRY(quant(4 * NB + 0, fw[6], &F.q[0], &F.qs[0])); TRY(quant(4 * NB + 1, fw[8], &F.q[1], &F.qs[1]));
    size_t n = (size_t)C * H * 3;
    if (d->dt == FLAMED_BF16)
      hipLaunchKernelGGL(stack_taps_kernel<bf16>, dim3((n + 255) / 256), dim3(256), 0, st, fw[10], reinterpret_cast<bf16*>(base + o_out), C, H, 3);
    else
      hipLaunchKernelGGL(stack_taps_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, st, fw[10], reinterpret_cast<float*>(base + o_out), C, H, 3);
    FL_LAUNCH_CHECK();
    d->wout = base + o_out;
    TRY(vec(fw[11], C, &d->bout));
  }
#undef TRY
  if (!d->scnt) FL_HIP(hipMalloc(&d->scnt, sizeof(int) * Den::kSplitCounters));
  FL_HIP(hipMemsetAsync(d->scnt, 0, sizeof(int) * Den::kSplitCounters, st));
  if (!d->gcnt) FL_HIP(hipMalloc(&d->gcnt, sizeof(int) * Den::kGnCounters));
  FL_HIP(hipMemsetAsync(d->gcnt, 0, sizeof(int) * Den::kGnCounters, st));
  if (!d->ctr) FL_HIP(hipMalloc(&d->ctr, 256));  // graph-replay step counter (never allocated inside a capture)
  if (d->dt == FLAMED_BF16 && !d->f8 && H == pk::kH && C == pk::kC && KS == pk::kTaps && NB <= pk::kMaxNB) {
    const int prc = persist_alloc(d, st);
    if (prc) return prc;
  }
  // the split chains' replay streams now, ahead of any persistent (cooperative) launch of this handle: streams
  // created after one replayed the chains with little overlap (B = 64: 334-343 vs 298-312 ms when created
  // before; tools/solve_time.py runs r05t/r05x)
  if (d->dt == FLAMED_BF16 && !d->f8 && !stream_capturing(st)) {
    TuneScope ts(den_tune_sync(d));
    const int crc = den_chain_streams(d, std::max(2, std::min(tn().split_batch, (int)Den::kMaxSplit)), st);
    if (crc) return crc;
  }
  retire_graph(d->gexec);
  for (auto& g : d->gexec_c) retire_graph(g);
  return kOk;
}

FLAMED_API int flamed_den_mods_stride(flamed_den_t h) {
  Den* d = reinterpret_cast<Den*>(h);
  return d ? d->MS : 0;
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
  FL_DEN_CALL(d);
  FL_REQUIRE_ON(mods, d->device, "flamed_den_adaln");
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
  if ((rc = launch_gemm<float>(LoadF32<float>{F, 256}, d->t0w, 256, EpiBiasAct<float, 2>{d->t0b, T1, H}, n_t, H, 256, st))) return rc;
  if ((rc = launch_gemm<float>(LoadF32<float>{T1, H}, d->t2w, H, EpiBiasAct<float, 0>{d->t2b, TE, H}, n_t, H, H, st))) return rc;
  if ((rc = launch_gemm<float>(LoadF32<float>{spk, d->S}, d->cw, d->S, EpiBiasAct<float, 0>{d->cb, CE, H}, n_spk, H, d->S, st))) return rc;
  if ((rc = launch_gemm<float>(LoadAdaY{TE, CE, tidx, sidx, H}, d->adaw, H, EpiBiasAct<float, 0>{d->adab, mods, d->MS}, R, d->MS0, H, st))) return rc;
  if (d->fold) {  // LayerNorm-fold tables of every mlp.0 / conv_out GEMM for these rows (den_fold_gemms)
    for (int i = 0; i <= d->NB; ++i) {
      const bool fin = i == d->NB;
      const float* md = mods + (size_t)i * 6 * H + 3 * H;  // [shift, scale] of the LN feeding this GEMM
      const bf16* W = reinterpret_cast<const bf16*>(fin ? d->wout : d->blk[i].m0);
      const int N = fin ? 3 * d->C : H;
      float* wa = mods + d->MS0 + (size_t)i * 2 * H;
      const float* lw = fin ? nullptr : d->blk[i].lnmw;
      const float* lb = fin ? nullptr : d->blk[i].lnmb;
      const float* bias = fin ? nullptr : d->blk[i].mb0;
      if ((rc = launch_gemm<bf16>(LoadFold<0>{md + H, md, d->MS, lw, lb}, W, H, EpiBiasAct<float, 0>{nullptr, wa, d->MS}, R, N, H, st))) return rc;
      if ((rc = launch_gemm<bf16>(LoadFold<1>{md + H, md, d->MS, lw, lb}, W, H, EpiBiasAct<float, 0>{bias, wa + N, d->MS}, R, N, H, st))) return rc;
    }
  }
  return kOk;
}

FLAMED_API size_t flamed_den_workspace_size(flamed_den_t h, int B, int T) {
  Den* d = reinterpret_cast<Den*>(h);
  if (!d) return 0;
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  TuneScope ts(den_tune_sync(d));  // the layout depends on the handle's large-M threshold
  return den_solve_ws(d, B, T);
}

// Diagnostic (include/flamed_diag.h): byte offsets of the one-chain step workspace's buffers
// X, S0, S1, D, U, GP, GNS, Y, SL, A16, XA, XP (den_ws_layout; SIZE_MAX for an absent buffer).
FLAMED_API int flamed_den_ws_offsets(flamed_den_t h, int B, int T, size_t* off) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && off && B > 0 && T > 0, "flamed_den_ws_offsets: bad args");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  TuneScope ts(den_tune_sync(d));
  char* const base = reinterpret_cast<char*>(4096);  // any non-null base: offsets are relative to it
  DenWs w;
  den_ws_layout(d, B, T, base, &w);
  const void* p[12] = {w.X, w.S0, w.S1, w.D, w.U, w.GP, w.GNS, w.Y, w.SL, w.A16, w.XA, w.XP};
  for (int i = 0; i < 12; ++i) off[i] = p[i] ? (size_t)((const char*)p[i] - base) : SIZE_MAX;
  return kOk;
}

// Diagnostic (include/flamed_diag.h): the split-chain stream probe's record (den_chain_streams).
FLAMED_API int flamed_den_chain_busy(flamed_den_t h, int* busy) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && busy, "flamed_den_chain_busy: bad args");
  *busy = d->qprobe_busy;
  return kOk;
}

FLAMED_API int flamed_den_chain_info(flamed_den_t h, int* parked, int* retries) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && parked && retries, "flamed_den_chain_info: bad args");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  *parked = d->n_parked;
  *retries = d->qprobe_retries;
  return kOk;
}

}  // extern "C"

namespace fl {

// Large-M fused Euler step: euler_cast_kernel (x_{s-1} -> x_s in place, bf16 x_s into A16) + proj_in on A16.
template <typename XT>
static int big_euler_proj_in(Den* d, float* xt, const DenWs& w, XT* X, int* ctr, float dt, int M, int T, hipStream_t st) {
  const int H = d->H, C = d->C;
  FL_REQUIRE(w.A16 && C % 8 == 0, "den_step: large-M fused Euler step needs the A16 buffer");
  const size_t n = (size_t)M * (C / 8);
  hipLaunchKernelGGL(euler_cast_kernel, dim3((n + 255) / 256), dim3(256), 0, st, xt, w.Y, d->bout, w.A16, M, T, C, dt, ctr);
  FL_LAUNCH_CHECK();
  const GemmCfg cfg = kCfgLarge;
  const int NT = H / 128;
  return den_gemm<bf16>(cfg, false, LoadPlain<bf16>{w.A16, C}, (const bf16*)d->win, C,
                        EpiBiasStatsT<false, XT>{d->bin, X, H, w.S0, NT}, M, H, C, st);
}

// One velocity evaluation (+ Euler update when vout == nullptr).
// `ctr` (optional): device step counter; when set the modulation rows are read at
// mods + (*ctr) * B * MS and the last kernel increments it (graph replay of captured steps).
template <typename DT, typename XT>
static int den_step_impl(Den* d, float* xt, const float* mods, int mod_div, int B, int T, float dt, float* vout,
                         const DenWs& w, int* ctr, hipStream_t st, const float* xsrc, int Bs, int chain, int nchains) {
  const int M = B * T, H = d->H, C = d->C, MS = d->MS;
  const Tune& tu = tn();
  // a step's modulation rows are Bs apart (Bs = B, or the whole batch when this is one of its sub-batches)
  const StepOff so{tu.noctr ? nullptr : ctr, (long long)Bs * MS};
  SplitCtx sctx;
  // sub-batch chains (den_split) each own 1/nchains of the split-K and GroupNorm counters
  const int scn = Den::kSplitCounters / nchains, gcn = Den::kGnCounters / nchains;
  sctx.slab = w.SL; sctx.slab_floats = w.SLn; sctx.cnt = d->scnt ? d->scnt + (size_t)chain * scn : nullptr;
  sctx.cnt_n = scn;
  sctx.target = tu.split_target; sctx.max_split = tu.split_max;
  SplitScope split_scope(w.SLn ? &sctx : nullptr);
  // GroupNorm finalize fused into the depthwise-conv kernel when the counters cover B x H/64
  int* gcnt = (d->gcnt && (size_t)B * (H / 16) <= (size_t)gcn) ? d->gcnt + (size_t)chain * gcn : nullptr;  // >= 16-channel groups
  const GemmCfg cfg = (tu.bn32 && M < kTinyRows) ? kCfgTiny
                      : (std::is_same<DT, bf16>::value && tu.big && M >= tu.big_min_rows) ? kCfgLarge : pick_cfg(M);
  const bool big = std::is_same<DT, bf16>::value && cfg == kCfgLarge && tu.big;
  FL_REQUIRE(!big || w.A16, "den_step: large-M workspace without the A16 buffer");
  const int BN = big ? 128 : cfg_bn(cfg);  // LN row-partial width = the N tile of the stats epilogues
  struct A16Scope {
    bf16* prev;
    explicit A16Scope(bf16* p) : prev(g_a16) { g_a16 = p; }
    ~A16Scope() { g_a16 = prev; }
  } a16_scope(w.A16);
  const int NT = H / BN;
  DT* U = reinterpret_cast<DT*>(w.U);
  // residual stream X and depthwise output D: fp32, or bf16 rows on the large-M x16 path
  constexpr bool X16 = std::is_same<XT, bf16>::value;
  FL_REQUIRE(!X16 || big, "den_step: the bf16 residual stream runs on the large-M path only");
  XT* X = reinterpret_cast<XT*>(w.X);
  XT* Dx = reinterpret_cast<XT*>(w.D);
  const bf16* X16p = X16 ? reinterpret_cast<const bf16*>(w.X) : nullptr;
  const bf16* D16p = X16 ? reinterpret_cast<const bf16*>(w.D) : nullptr;
  // fp8 handle at large M: MX-fp8 conv_2 / conv_3 / mlp.0 / mlp.2 on the 256 x 256 tiles, their A operands
  // written as e4m3 + scales by the normalise passes and by the conv_2 / mlp.0 epilogues (no LayerNorm
  // fold, no dwgn: their producers write bf16)
  const bool f8 = std::is_same<DT, bf16>::value && d->f8 && big && tu.g8p_rows > 0 && M >= tu.g8p_rows;
  const bool fold = std::is_same<DT, bf16>::value && d->fold && tu.lnfold && w.XA && (!big || M >= tu.fold_big_rows) && !f8;
  // whole-utterance depthwise conv + GroupNorm (launch_dwgn): large M, one modulation row per utterance
  const bool dwgn = big && tu.dwgn && T <= kDgMaxT && mod_div % T == 0 && H % 64 == 0 && !f8;
  unsigned char* const A8 = reinterpret_cast<unsigned char*>(w.A16);  // fp8 operands: e4m3 rows, then scales
  unsigned char* const A8s = f8 ? A8 + (size_t)M * H : nullptr;
  unsigned char* const U8 = reinterpret_cast<unsigned char*>(w.U);
  unsigned char* const U8s = f8 ? U8 + (size_t)M * H : nullptr;
  // small M (bf16): the same sub-block in one workgroup per (utterance, 8 channels), bf16 operand in D's space
  const bool dwgn_s = std::is_same<DT, bf16>::value && !big && !X16 && tu.dwgn_small && T <= kDgSmallMaxT && mod_div % T == 0;
  bf16* const As = reinterpret_cast<bf16*>(w.D);
  int rc;
#define TRY(x) do { if ((rc = (x)) != kOk) return rc; } while (0)
  int n_launched = 0;  // kernel-class launches so far (diagnostic stop_after)
#define K_(cls, x)                                                  \
  do {                                                              \
    if (tu.stop_after >= 0 && n_launched >= tu.stop_after) return kOk; \
    ++n_launched;                                                   \
    if (tu.stamp_class >= 0) stamp_select(cls, st);                 \
    TRY(x);                                                         \
    if (tu.dup_class == (cls)) TRY(x);                              \
  } while (0)
  // fused solve step (xsrc != null; small M only, den_fused_ok): the previous step's combine + Euler
  // update is proj_in's A loader, and there is no combine launch at the end of the step
  FL_REQUIRE(!xsrc || !vout, "den_step: a fused Euler step has no velocity output");
  FL_REQUIRE(!xsrc || !big || xsrc == xt, "den_step: the large-M fused Euler step updates the state in place");
  if (xsrc && big) {  // large M: the previous step's combine + Euler update and proj_in's bf16 cast in one pass
    if constexpr (std::is_same<DT, bf16>::value) K_(0, big_euler_proj_in<XT>(d, xt, w, X, ctr, dt, M, T, st));
  } else if (xsrc) {
    const LoadEulerIn<DT> le{xsrc, xt, w.Y, d->bout, ctr, dt, T, C};
    const EpiBiasStatsT<false, XT> ep{d->bin, X, H, w.S0, NT};
    if (cfg == kCfgTiny) K_(0, (launch_gemm_cfg<32, 32, 3, DT>(le, (const DT*)d->win, C, ep, M, H, C, st)));
    else K_(0, (launch_gemm_auto<DT>(cfg, le, (const DT*)d->win, C, ep, M, H, C, st)));
  } else {
    K_(0, (den_gemm<DT>(cfg, false, LoadF32<DT>{xt, C}, (const DT*)d->win, C, EpiBiasStatsT<false, XT>{d->bin, X, H, w.S0, NT}, M, H, C, st)));
  }
  for (int i = 0; i < d->NB; ++i) {
    const DenBlockW& Bw = d->blk[i];
    const float* md = mods + (size_t)i * 6 * H;
    ModRef mc{md, md + H, MS, mod_div, so};
    ModRef mm{md + 3 * H, md + 4 * H, MS, mod_div, so};
    if (f8) {
      K_(1, (launch_dwconv_stats<true, XT>(X, H, w.S0, NT, BN, mc, Bw.lnw, Bw.lnb, Bw.dww, Bw.dwb, Dx, w.GP, w.GNS, B, T, st, 1, gcnt)));
      K_(2, (launch_dwconv_stats<true, XT>(X, H, w.S0, NT, BN, mc, Bw.lnw, Bw.lnb, Bw.dww, Bw.dwb, Dx, w.GP, w.GNS, B, T, st, 2, gcnt)));
      K_(3, f8_prep(LoadGN<bf16>{w.D, H, w.GNS, Bw.gnw, Bw.gnb, T, D16p}, M, A8, A8s, st));
      K_(3, launch_gemm8p_f8(A8, A8s, H, Bw.q[0], Bw.qs[0], H, EpiBiasActF8<1>{Bw.b2, U8, U8s, H}, M, H, H, st));
      K_(4, launch_gemm8p_f8(U8, U8s, H, Bw.q[1], Bw.qs[1], H,
                             EpiConvNeXtResid<true, XT>{Bw.b3, X, H, w.S0, NT, BN, 1e-6f, mc, md + 2 * H, Bw.lnw, Bw.lnb, w.S1, NT},
                             M, H, H, st));
      K_(5, f8_prep(LoadLNMod<bf16, true>{w.X, H, w.S1, NT, BN, 1e-6f, mm, Bw.lnmw, Bw.lnmb, H, X16p}, M, A8, A8s, st));
      K_(5, launch_gemm8p_f8(A8, A8s, H, Bw.q[2], Bw.qs[2], H, EpiBiasActF8<2>{Bw.mb0, U8, U8s, H}, M, H, H, st));
      K_(6, launch_gemm8p_f8(U8, U8s, H, Bw.q[3], Bw.qs[3], H,
                             EpiGatedResidT<XT>{Bw.mb2, X, H, md + 5 * H, MS, mod_div, w.S0, NT, so}, M, H, H, st));
      continue;
    }
    if (dwgn) {  // large M: conv + GroupNorm in one kernel, conv_2 on the normalised bf16 rows
      K_(1, (launch_dwgn<true, XT>(X, H, w.S0, NT, BN, mc, Bw.lnw, Bw.lnb, Bw.dww, Bw.dwb, Bw.gnw, Bw.gnb, w.A16, B, T, st)));
      K_(3, (den_gemm<DT>(cfg, false, LoadPlain<DT>{(const DT*)w.A16, H}, (const DT*)Bw.w2, H, EpiBiasAct<DT, 1>{Bw.b2, U, H}, M, H, H, st)));
    } else if (dwgn_s) {
      K_(1, (launch_dwgn_small<true>((const float*)w.X, H, w.S0, NT, BN, mc, Bw.lnw, Bw.lnb, Bw.dww, Bw.dwb, Bw.gnw, Bw.gnb, As, B, T, st)));
      K_(3, (den_gemm<DT>(cfg, false, LoadPlain<DT>{(const DT*)As, H}, (const DT*)Bw.w2, H, EpiBiasAct<DT, 1>{Bw.b2, U, H}, M, H, H, st)));
    } else {
      K_(1, (launch_dwconv_stats<true, XT>(X, H, w.S0, NT, BN, mc, Bw.lnw, Bw.lnb, Bw.dww, Bw.dwb, Dx, w.GP, w.GNS, B, T, st, 1, gcnt)));
      K_(2, (launch_dwconv_stats<true, XT>(X, H, w.S0, NT, BN, mc, Bw.lnw, Bw.lnb, Bw.dww, Bw.dwb, Dx, w.GP, w.GNS, B, T, st, 2, gcnt)));
      K_(3, (den_gemm<DT>(cfg, true, LoadGN<DT>{w.D, H, w.GNS, Bw.gnw, Bw.gnb, T, D16p}, (const DT*)Bw.w2, H,
                                          EpiBiasAct<DT, 1>{Bw.b2, U, H}, M, H, H, st)));
    }
    if (fold) {  // mlp.0 on x * alpha (written by conv_3's epilogue) with the LayerNorm in its epilogue
      K_(4, (den_gemm<DT>(cfg, false, LoadPlain<DT>{U, H}, (const DT*)Bw.w3, H,
                                          EpiConvNeXtResid<true, XT>{Bw.b3, X, H, w.S0, NT, BN, 1e-6f, mc, md + 2 * H, Bw.lnw, Bw.lnb, w.S1, NT,
                                                                 w.XA, Bw.lnmw, md + 4 * H},
                                          M, H, H, st)));
      K_(5, (den_gemm<DT>(cfg, false, LoadPlain<DT>{(const DT*)w.XA, H}, (const DT*)Bw.m0, H,
                                          EpiLNFold<DT, 2>{U, H, w.S1, NT, BN, 1e-6f, mods + d->MS0 + (size_t)i * 2 * H, H, MS, mod_div, so},
                                          M, H, H, st)));
    } else {
      K_(4, (den_gemm<DT>(cfg, false, LoadPlain<DT>{U, H}, (const DT*)Bw.w3, H,
                                          EpiConvNeXtResid<true, XT>{Bw.b3, X, H, w.S0, NT, BN, 1e-6f, mc, md + 2 * H, Bw.lnw, Bw.lnb, w.S1, NT},
                                          M, H, H, st)));
      K_(5, (den_gemm<DT>(cfg, true, LoadLNMod<DT, true>{w.X, H, w.S1, NT, BN, 1e-6f, mm, Bw.lnmw, Bw.lnmb, H, X16p}, (const DT*)Bw.m0, H,
                                          EpiBiasAct<DT, 2>{Bw.mb0, U, H}, M, H, H, st)));
    }
    K_(6, (den_gemm<DT>(cfg, false, LoadPlain<DT>{U, H}, (const DT*)Bw.m2, H,
                                        EpiGatedResidT<XT>{Bw.mb2, X, H, md + 5 * H, MS, mod_div, w.S0, NT, so}, M, H, H, st)));
  }
  const float* mf = mods + (size_t)d->NB * 6 * H;
  ModRef mc{mf, mf + H, MS, mod_div, so};
  ModRef mo{mf + 3 * H, mf + 4 * H, MS, mod_div, so};
  const DenBlockW& F = d->fin;
  if (f8) {
    K_(1, (launch_dwconv_stats<false, XT>(X, H, w.S0, NT, BN, mc, nullptr, nullptr, F.dww, F.dwb, Dx, w.GP, w.GNS, B, T, st, 1, gcnt)));
    K_(2, (launch_dwconv_stats<false, XT>(X, H, w.S0, NT, BN, mc, nullptr, nullptr, F.dww, F.dwb, Dx, w.GP, w.GNS, B, T, st, 2, gcnt)));
    K_(3, f8_prep(LoadGN<bf16>{w.D, H, w.GNS, F.gnw, F.gnb, T, D16p}, M, A8, A8s, st));
    K_(3, launch_gemm8p_f8(A8, A8s, H, F.q[0], F.qs[0], H, EpiBiasActF8<1>{F.b2, U8, U8s, H}, M, H, H, st));
  } else if (dwgn) {
    K_(1, (launch_dwgn<false, XT>(X, H, w.S0, NT, BN, mc, nullptr, nullptr, F.dww, F.dwb, F.gnw, F.gnb, w.A16, B, T, st)));
    K_(3, (den_gemm<DT>(cfg, false, LoadPlain<DT>{(const DT*)w.A16, H}, (const DT*)F.w2, H, EpiBiasAct<DT, 1>{F.b2, U, H}, M, H, H, st)));
  } else if (dwgn_s) {
    K_(1, (launch_dwgn_small<false>((const float*)w.X, H, w.S0, NT, BN, mc, nullptr, nullptr, F.dww, F.dwb, F.gnw, F.gnb, As, B, T, st)));
    K_(3, (den_gemm<DT>(cfg, false, LoadPlain<DT>{(const DT*)As, H}, (const DT*)F.w2, H, EpiBiasAct<DT, 1>{F.b2, U, H}, M, H, H, st)));
  } else {
    K_(1, (launch_dwconv_stats<false, XT>(X, H, w.S0, NT, BN, mc, nullptr, nullptr, F.dww, F.dwb, Dx, w.GP, w.GNS, B, T, st, 1, gcnt)));
    K_(2, (launch_dwconv_stats<false, XT>(X, H, w.S0, NT, BN, mc, nullptr, nullptr, F.dww, F.dwb, Dx, w.GP, w.GNS, B, T, st, 2, gcnt)));
    K_(3, (den_gemm<DT>(cfg, true, LoadGN<DT>{w.D, H, w.GNS, F.gnw, F.gnb, T, D16p}, (const DT*)F.w2, H, EpiBiasAct<DT, 1>{F.b2, U, H}, M, H, H, st)));
  }
  if (f8) {
    K_(4, launch_gemm8p_f8(U8, U8s, H, F.q[1], F.qs[1], H,
                           EpiConvNeXtResid<false, XT>{F.b3, X, H, w.S0, NT, BN, 1e-6f, mc, mf + 2 * H, nullptr, nullptr, w.S1, NT},
                           M, H, H, st));
    K_(7, (den_gemm<DT>(cfg, true, LoadLNMod<DT, false>{w.X, H, w.S1, NT, BN, 1e-6f, mo, nullptr, nullptr, H, X16p}, (const DT*)d->wout, H,
                                        EpiBiasAct<float, 0>{nullptr, w.Y, 3 * C}, M, 3 * C, H, st)));
  } else if (fold) {
    K_(4, (den_gemm<DT>(cfg, false, LoadPlain<DT>{U, H}, (const DT*)F.w3, H,
                                        EpiConvNeXtResid<false, XT>{F.b3, X, H, w.S0, NT, BN, 1e-6f, mc, mf + 2 * H, nullptr, nullptr, w.S1, NT,
                                                                w.XA, nullptr, mf + 4 * H},
                                        M, H, H, st)));
    K_(7, (den_gemm<DT>(cfg, false, LoadPlain<DT>{(const DT*)w.XA, H}, (const DT*)d->wout, H,
                                        EpiLNFold<float, 0>{w.Y, 3 * C, w.S1, NT, BN, 1e-6f, mods + d->MS0 + (size_t)d->NB * 2 * H, 3 * C, MS, mod_div, so},
                                        M, 3 * C, H, st)));
  } else {
    K_(4, (den_gemm<DT>(cfg, false, LoadPlain<DT>{U, H}, (const DT*)F.w3, H,
                                        EpiConvNeXtResid<false, XT>{F.b3, X, H, w.S0, NT, BN, 1e-6f, mc, mf + 2 * H, nullptr, nullptr, w.S1, NT},
                                        M, H, H, st)));
    K_(7, (den_gemm<DT>(cfg, true, LoadLNMod<DT, false>{w.X, H, w.S1, NT, BN, 1e-6f, mo, nullptr, nullptr, H, X16p}, (const DT*)d->wout, H,
                                        EpiBiasAct<float, 0>{nullptr, w.Y, 3 * C}, M, 3 * C, H, st)));
  }
  if (!xsrc) {
    size_t n = (size_t)M * C;
    hipLaunchKernelGGL(conv3_combine_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w.Y, d->bout, xt, vout, M, T, C, dt, ctr, nullptr);
    FL_LAUNCH_CHECK();
    if (tu.dup_class == 8) {  // duplicate without a second counter increment
      hipLaunchKernelGGL(conv3_combine_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w.Y, d->bout, xt, vout, M, T, C, dt, nullptr, nullptr);
      FL_LAUNCH_CHECK();
    }
  }
#undef K_
#undef TRY
  return kOk;
}

static int den_step(Den* d, float* xt, const float* mods, int mod_div, int B, int T, float dt, float* vout, void* ws,
                    hipStream_t st, int* ctr = nullptr, const float* xsrc = nullptr, int Bs = 0, int chain = 0,
                    int nchains = 1) {
  if (Bs <= 0) Bs = B;
  DenWs w;
  den_ws_layout(d, B, T, ws, &w);
  if (d->dt == FLAMED_BF16) {
    if (den_x16(d, B, T)) return den_step_impl<bf16, bf16>(d, xt, mods, mod_div, B, T, dt, vout, w, ctr, st, xsrc, Bs, chain, nchains);
    return den_step_impl<bf16, float>(d, xt, mods, mod_div, B, T, dt, vout, w, ctr, st, xsrc, Bs, chain, nchains);
  }
  return den_step_impl<float, float>(d, xt, mods, mod_div, B, T, dt, vout, w, ctr, st, xsrc, Bs, chain, nchains);
}

// The fused Euler step (LoadEulerIn) runs where proj_in takes the small-M register loop with one
// workgroup column per tile column (no XCD strip remap) and no split-K of its fp32-A GEMM; the large-M
// path fuses differently (den_fused_big).
static bool den_fused_ok(const Den* d, int B, int T) {
  const Tune& tu = tn();
  const int M = B * T;
  const bool big = d->dt == FLAMED_BF16 && tu.big && M >= tu.big_min_rows;
  return tu.fuse_euler && !big && tu.xcd_strips == 0 && !d->f8;
}
// Large-M solves fuse the combine + Euler update into the next step's proj_in cast (euler_cast_kernel, in place:
// no ping-pong); per sub-batch chain when the solve splits.  `B` is the rows' batch of one chain.
static bool den_fused_big(const Den* d, int B, int T) {
  const Tune& tu = tn();
  return tu.fuse_euler && d->dt == FLAMED_BF16 && tu.big && (size_t)B * T >= (size_t)tu.big_min_rows &&
         !(tu.bn32 && (size_t)B * T < (size_t)kTinyRows);
}

// Steps per captured graph: the largest divisor of nfe that is <= tn().graph_steps (default 16; the
// graph is replayed nfe/G times per solve, so a new (B, T) costs one G-step capture instead of an
// nfe-step one).
// ------------------------------ persistent B = 1 solve (persist.hpp) ------------------------------

// Scratch of the persistent solve, sized for T <= pk::kMaxT: the counter block (reset by every launch's own
// prologue), the sticky words (failure count and the prologue's monotonic arrival counters: zeroed once at
// allocation, never again) and the hand-off buffers.
static size_t persist_layout(char* base, pk::Params* P) {
  size_t off = 0;
  auto take = [&](size_t bytes) { char* p = base ? base + off : nullptr; off = align256(off + bytes); return p; };
  const size_t T = pk::kMaxT, H = pk::kH, C = pk::kC;
  char* ctr = take(4 * (size_t)pk::kCtrInts);
  char* sticky = take(4 * (size_t)pk::kStickyInts);
  char* seal = take((size_t)pk::kWGs * 16);
  char* xp0 = take(T * pk::kSlots * 8);
  char* xp1 = take(T * pk::kSlots * 8);
  char* ximg = take(T * H * 4);
  char* a2 = take(T * H * 2);
  char* u = take(T * H * 2);
  char* xa = take(T * H * 2);
  char* xs = take(T * C * 2);
  char* gnp = take((size_t)pk::kGroups * H * 16);
  char* yb = take((size_t)pk::kWGs * 16 * 4);
  if (P) {
    P->ctr = reinterpret_cast<int*>(ctr);
    P->sticky = reinterpret_cast<int*>(sticky);
    P->seal = reinterpret_cast<int*>(seal);
    P->xpart[0] = reinterpret_cast<float2*>(xp0);
    P->xpart[1] = reinterpret_cast<float2*>(xp1);
    P->ximg = reinterpret_cast<float*>(ximg);
    P->a2 = reinterpret_cast<bf16*>(a2);
    P->u = reinterpret_cast<bf16*>(u);
    P->xa = reinterpret_cast<bf16*>(xa);
    P->xs = reinterpret_cast<bf16*>(xs);
    P->gnp = reinterpret_cast<float4*>(gnp);
    P->yb = reinterpret_cast<float*>(yb);
  }
  return off;
}

// Persistent scratch + pinned failure word, allocated once when the handle is loaded (so a solve inside a
// stream capture never allocates); the failure word starts at 0 and only the kernel writes it after that.
static int persist_alloc(Den* d, hipStream_t st) {
  if (d->pmem) return kOk;
  const size_t bytes = persist_layout(nullptr, nullptr);
  FL_HIP(hipMalloc(&d->pmem, bytes));
  FL_HIP(hipMemsetAsync(d->pmem, 0, bytes, st));
  FL_HIP(hipHostMalloc(reinterpret_cast<void**>(&d->pfail_host), 16, hipHostMallocDefault));
  *d->pfail_host = 0;
  FL_HIP(hipHostMalloc(reinterpret_cast<void**>(&d->perr_host), Den::kPRing * sizeof(int), hipHostMallocDefault));
  for (int i = 0; i < Den::kPRing; ++i) d->perr_host[i] = 0;
  d->pfails_seen = 0;
  return kOk;
}

static bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}

// Failed launches the kernel has counted since the handle's last look (the pinned copy is refreshed by an
// async copy behind every uncaptured launch, so this never blocks; it may lag one launch).  After
// kPersistRetry failures the handle stays on the graph-of-launches path.
static void persist_poll_fails(Den* d) {
  if (!d->pfail_host) return;
  const int f = __atomic_load_n(d->pfail_host, __ATOMIC_RELAXED);
  if (f <= d->pfails_seen) return;
  d->pfails_seen = f;
  if (f >= Den::kPersistRetry && !d->pbroken) {
    d->pbroken = true;
    fprintf(stderr, "flamed: %d persistent solves failed (output NaN-poisoned); this handle uses the launch path from now on\n", f);
  } else {
    fprintf(stderr, "flamed: a persistent solve failed (%d of %d allowed); its output was NaN-poisoned\n", f, Den::kPersistRetry);
  }
}

// The persistent solve covers one utterance of 16..512 frames on a bf16 handle with the LayerNorm fold and
// the shipped dims, on a device where all 256 workgroups are resident at once (one per CU: the cooperative
// launch checks it again).  Stream capture is allowed: nothing on the call path waits on the device.
// A batch of 3 or 5..7 utterances runs as the persistent launch of the next supported size (4 / 8) with idle
// zero utterances in the spare row groups (knob persist_pad): the reference's metadata mode batches 4 utterances and
// leaves a trailing batch of 1..3 (synthesize.py:268-291, 344).  Time is set by the most-loaded group, the same as
// for the padded size.
static int persist_batch(int B) {
  if (B == 3) return 4;
  if (B >= 5 && B <= 7) return 8;
  return B;
}

static bool persist_eligible(Den* d, int B, int T) {
  const Tune& tu = tn();
  persist_poll_fails(d);
  if (!tu.persist || d->pbroken || d->dt != FLAMED_BF16 || d->f8 || !d->fold || !tu.lnfold) return false;
  if (d->H != pk::kH || d->C != pk::kC || d->NB > pk::kMaxNB || d->KS != pk::kTaps || T < 16) return false;
  // one utterance, or (knob persist_multi) B in {2, 4, 8}, each utterance's frames split over its 8 / B row groups;
  // a group holds up to kMaxNTW chunks of 64 frames (kernel variant by chunk count; knob persist_ntw caps it)
  const int B0 = B;
  if (B != 1 && tu.persist_multi && tu.persist_pad) B = persist_batch(B);
  if (B != 1 && (!tu.persist_multi || (B != 2 && B != 4 && B != 8))) return false;
  const int ntw = pk::persist_ntw(B, T, tu.persist_opt);
  // padded to at least 1.5x the batch (B = 5 as 8): the idle utterances cost whole chunks, so only up to persist_pad_ntw
  if (B != B0 && 2 * B >= 3 * B0 && ntw > tu.persist_pad_ntw) return false;
  if (ntw > pk::kMaxNTW || ntw > tu.persist_ntw || ((tu.persist_opt & 1024) && ntw != 1)) return false;
  if (B > 1 && ntw > tu.persist_multi_ntw) return false;  // several utterances: the graph path is faster beyond 2 chunks
  if (d->pdev_ok < 0) d->pdev_ok = pk::persist_device_ok(d->device) ? 1 : 0;
  return d->pdev_ok == 1;
}

// Steps [s0, s1) of a B = 1 solve as ONE cooperative launch, enqueued on `st` with no host synchronisation:
// the kernel (it resets its own counter block) and, outside a capture, HIP events around it plus an async
// copy of the sticky failure word.  A failed launch NaN-poisons x and is reported by the next call / persist_info.
static int persist_solve(Den* d, float* xt, const float* mods, int nfe, int B, int T, int s0, int s1, hipStream_t st) {
  const bool cap = stream_capturing(st);
  FL_REQUIRE(d->pmem && d->pfail_host && d->perr_host, "persistent solve: scratch not allocated at load");
  pk::Params P{};
  persist_layout(d->pmem, &P);
  d->pfail = P.sticky + pk::SY_FAILS;
  const int Bp = tn().persist_pad ? persist_batch(B) : B;
  P.T = T; P.B = Bp; P.Bx = Bp != B ? B : 0; P.NB = d->NB; P.s0 = s0; P.s1 = s1;
  P.dt = (float)(1.0 / (double)nfe);
  P.mods = mods; P.MS = d->MS; P.MS0 = d->MS0;
  // the kernel reads modulation rows as 16-B vectors (persist.hip ld_cols)
  FL_REQUIRE(P.MS % 4 == 0 && P.MS0 % 4 == 0 && ((uintptr_t)mods & 15) == 0, "persistent solve: modulation rows not 16-B aligned");
  P.win = reinterpret_cast<const bf16*>(d->win); P.bin = d->bin;
  for (int i = 0; i <= d->NB; ++i) {
    const DenBlockW& b = i < d->NB ? d->blk[i] : d->fin;
    pk::BlockW& o = P.blk[i];
    o.w2 = reinterpret_cast<const bf16*>(b.w2); o.w3 = reinterpret_cast<const bf16*>(b.w3);
    o.m0 = i < d->NB ? reinterpret_cast<const bf16*>(b.m0) : nullptr;
    o.m2 = i < d->NB ? reinterpret_cast<const bf16*>(b.m2) : nullptr;
    o.b2 = b.b2; o.b3 = b.b3; o.dww = b.dww; o.dwb = b.dwb; o.gnw = b.gnw; o.gnb = b.gnb;
    if (i < d->NB) {
      o.mb0 = b.mb0; o.mb2 = b.mb2; o.lnw = b.lnw; o.lnb = b.lnb; o.lnmw = b.lnmw; o.lnmb = b.lnmb;
    }
  }
  P.wout = reinterpret_cast<const bf16*>(d->wout); P.bout = d->bout;
  P.xt = xt;
  P.tmo = 50000000;  // 0.5 s of s_memrealtime (100 MHz) per wait
  P.opt = tn().persist_opt;
  P.ntw = pk::persist_ntw(Bp, T, P.opt);
  P.inject_step = tn().persist_inject;
  P.seal_skip = tn().persist_seal_skip;
  hipEvent_t* ev = nullptr;
  const int slot = (int)(d->pring_n % Den::kPRing);
  if (!cap) {
    ev = d->pring[slot];
    for (int k = 0; k < 3; ++k)
      if (!ev[k]) FL_HIP(hipEventCreate(&ev[k]));
    FL_HIP(hipEventRecord(ev[0], st));
  }
  // inside a capture: a cooperative kernel node (persist_capmode 0) or a plain one (1; residency was checked
  // by the uncaptured cooperative launches and persist_device_ok)
  const int lrc = pk::persist_launch(P, st, !cap || tn().persist_capmode == 0);
  if (lrc) return lrc;
  if (!cap) {
    FL_HIP(hipEventRecord(ev[1], st));
    FL_HIP(hipMemcpyAsync(d->pfail_host, d->pfail, sizeof(int), hipMemcpyDeviceToHost, st));
    // this launch's own error word (set by its first failing workgroup, zeroed by the next launch's prologue, which
    // is stream-ordered behind this copy)
    FL_HIP(hipMemcpyAsync(d->perr_host + slot, P.ctr + pk::CT_ERR, sizeof(int), hipMemcpyDeviceToHost, st));
    FL_HIP(hipEventRecord(ev[2], st));
    ++d->pring_n;
  }
  ++d->pruns;
  return kOk;
}

static int graph_chunk(int nfe) {
  const int gs = tn().graph_steps;
  for (int g = gs < nfe ? gs : nfe; g > 1; --g)
    if (nfe % g == 0) return g;
  return 1;
}

}  // namespace fl

extern "C" {

FLAMED_API int flamed_den_velocity(flamed_den_t h, const float* x, const float* mods, int mod_div, int B, int T,
                                   float* v_out, void* ws, size_t ws_bytes, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev, "flamed_den_velocity: handle not loaded");
  FL_REQUIRE(x && mods && v_out && ws && B > 0 && T > 0 && mod_div > 0, "flamed_den_velocity: bad args");
  FL_DEN_CALL(d);
  FL_REQUIRE_ON(x, d->device, "flamed_den_velocity");
  if (ws_bytes < den_ws_bytes(d, B, T)) {
    set_error("flamed_den_velocity: workspace too small (%zu < %zu)", ws_bytes, den_ws_bytes(d, B, T));
    return kNoWorkspace;
  }
  return den_step(d, const_cast<float*>(x), mods, mod_div, B, T, 0.f, v_out, ws, st);
}

FLAMED_API int flamed_den_step(flamed_den_t h, float* xt, const float* mods, int mod_div, int B, int T, float dt,
                               void* ws, size_t ws_bytes, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev, "flamed_den_step: handle not loaded");
  FL_REQUIRE(xt && mods && ws && B > 0 && T > 0 && mod_div > 0, "flamed_den_step: bad args");
  FL_DEN_CALL(d);
  FL_REQUIRE_ON(xt, d->device, "flamed_den_step");
  if (ws_bytes < den_ws_bytes(d, B, T)) {
    set_error("flamed_den_step: workspace too small");
    return kNoWorkspace;
  }
  return den_step(d, xt, mods, mod_div, B, T, dt, nullptr, ws, st);
}

FLAMED_API int flamed_den_solve_chunk(flamed_den_t h, int nfe) {
  Den* d = reinterpret_cast<Den*>(h);
  if (!d || nfe <= 0) return -1;
  FL_DEN_CALL(d);
  return graph_chunk(nfe);
}

FLAMED_API int flamed_den_persist_info(flamed_den_t h, int* runs, int* broken, float* last_ms) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && runs && broken && last_ms, "flamed_den_persist_info: bad args");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  DeviceGuard dg(d->device);
  *last_ms = 0.f;
  if (d->pring_n > 0) {  // waits for the last uncaptured launch (a diagnostic query, not the call path)
    hipEvent_t* ev = d->pring[(d->pring_n - 1) % Den::kPRing];
    FL_HIP(hipEventSynchronize(ev[1]));
    FL_HIP(hipEventElapsedTime(last_ms, ev[0], ev[1]));
  }
  persist_poll_fails(d);
  *runs = d->pruns;
  *broken = d->pbroken ? 1 : 0;
  return kOk;
}

FLAMED_API int flamed_den_persist_status(flamed_den_t h, int* runs, int* fails) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && runs && fails, "flamed_den_persist_status: bad args");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  *runs = d->pruns;
  *fails = d->pfail_host ? __atomic_load_n(d->pfail_host, __ATOMIC_RELAXED) : 0;
  persist_poll_fails(d);
  return kOk;
}

FLAMED_API int flamed_den_persist_fails(flamed_den_t h, int* fails) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && fails, "flamed_den_persist_fails: bad args");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  DeviceGuard dg(d->device);
  *fails = 0;
  if (!d->pmem) return kOk;
  pk::Params P{};
  persist_layout(d->pmem, &P);
  FL_HIP(hipDeviceSynchronize());  // captured launches leave no event: wait for everything (diagnostic)
  FL_HIP(hipMemcpy(fails, P.sticky + pk::SY_FAILS, sizeof(int), hipMemcpyDeviceToHost));
  if (d->pfail_host) __atomic_store_n(d->pfail_host, *fails, __ATOMIC_RELAXED);
  persist_poll_fails(d);
  return kOk;
}

FLAMED_API int flamed_den_persist_last(flamed_den_t h, long long* seq) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && seq, "flamed_den_persist_last: bad args");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  *seq = d->pring_n - 1;
  return kOk;
}

FLAMED_API int flamed_den_persist_query(flamed_den_t h, long long seq, int* state) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && state, "flamed_den_persist_query: bad args");
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  FL_REQUIRE(seq >= 0 && seq < d->pring_n, "flamed_den_persist_query: no such launch");
  if (seq < d->pring_n - Den::kPRing) {
    *state = 3;  // its ring slot has been reused
    return kOk;
  }
  DeviceGuard dg(d->device);
  const int slot = (int)(seq % Den::kPRing);
  const hipError_t e = hipEventQuery(d->pring[slot][2]);
  if (e == hipErrorNotReady) {
    *state = 2;
    return kOk;
  }
  FL_HIP(e);
  *state = __atomic_load_n(d->perr_host + slot, __ATOMIC_RELAXED) != 0 ? 1 : 0;
  return kOk;
}

FLAMED_API int flamed_den_persist_times(flamed_den_t h, float* ms, int n) {
  Den* d = reinterpret_cast<Den*>(h);
  if (!d || !ms || n < 0) {
    set_error("flamed_den_persist_times: bad args");
    return -1;
  }
  std::lock_guard<std::recursive_mutex> lk(d->mu);
  DeviceGuard dg(d->device);
  int k = (long long)n < d->pring_n ? n : (int)d->pring_n;
  if (k > Den::kPRing) k = Den::kPRing;
  for (int i = 0; i < k; ++i) {
    hipEvent_t* ev = d->pring[(d->pring_n - k + i) % Den::kPRing];
    if (hipEventSynchronize(ev[1]) != hipSuccess || hipEventElapsedTime(ms + i, ev[0], ev[1]) != hipSuccess) {
      set_error("flamed_den_persist_times: event query failed");
      return -1;
    }
  }
  return k;
}

FLAMED_API int flamed_den_solve(flamed_den_t h, float* xt, const float* mods, int nfe, int B, int T, void* ws,
                                size_t ws_bytes, int use_graph, hipStream_t st) {
  return flamed_den_solve_part(h, xt, mods, nfe, B, T, ws, ws_bytes, use_graph, 0, nfe, st);
}

// Hardware-queue probe for two streams: a one-lane kernel on stream a waits (bounded: 2 ms of s_memrealtime)
// for a flag that a kernel on stream b sets.  If b's launch sits on a's hardware queue it cannot start until
// a's kernel has timed out, and the pair is reported as serialising.  Both kernels stamp s_memrealtime (the wait
// kernel its start and end, the set kernel its start), so a pair that was not concurrent is told apart: the set
// kernel starting within 50 us after the wait kernel ended is the queue's back-to-back dispatch (serialising);
// any other timing means the device was busy (e.g. another handle's cooperative launch holding every CU) and the
// result is inconclusive -- ADVICE r5.
__global__ void qprobe_wait_kernel(int* w) {
  if (threadIdx.x != 0) return;
  unsigned long long* ts = reinterpret_cast<unsigned long long*>(w + 4);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int ok = 0;
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < 200000) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) { ok = 1; break; }
    __builtin_amdgcn_s_sleep(2);
  }
  ts[0] = t0;
  ts[1] = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(w + 1, ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void qprobe_set_kernel(int* w) {
  if (threadIdx.x == 0) {
    reinterpret_cast<unsigned long long*>(w + 4)[2] = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// *state: 0 concurrent, 1 serialising (back-to-back on one queue), 2 inconclusive (device busy)
static int streams_concurrent(int* w, hipStream_t a, hipStream_t b, int* state) {
  int h[10] = {};
  FL_HIP(hipMemcpy(w, h, sizeof(h), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(qprobe_wait_kernel, dim3(1), dim3(64), 0, a, w);
  FL_LAUNCH_CHECK();
  hipLaunchKernelGGL(qprobe_set_kernel, dim3(1), dim3(64), 0, b, w);
  FL_LAUNCH_CHECK();
  FL_HIP(hipStreamSynchronize(a));
  FL_HIP(hipStreamSynchronize(b));
  FL_HIP(hipMemcpy(h, w, sizeof(h), hipMemcpyDeviceToHost));
  unsigned long long ts[3];
  memcpy(ts, h + 4, sizeof(ts));
  const long long gap = (long long)(ts[2] - ts[1]);  // set start - wait end, 10 ns ticks
  *state = h[1] == 1 ? 0 : (gap >= 0 && gap < 5000) ? 1 : 2;
  return kOk;
}

// Replay streams of the split chains (tune split_prio).  HIP maps each stream to one of GPU_MAX_HW_QUEUES (4)
// hardware queues by current use, so two normal-priority streams -- or a graph's own branch streams -- can
// share the launch stream's queue and serialise the chains: the round-4 single graph with parallel branches
// (split_graph 1) measured 295-322 ms at B = 64 on some process histories and 341-348 ms on others (e.g. with
// its streams created after a cooperative launch; tools/coop_stream_probe.py shows stream pairs that
// serialise).  Priority streams come from queues of their own (probe: every high / low pair concurrent), so
// the chains replay on them.  split_prio 0: chain 0 on the caller's stream, chain 1 at the highest priority
// (chains 2 / 3 low / normal); 1: every chain on a low-priority stream of its own; 2: every chain on a
// high-priority stream.
static int den_chain_streams(Den* d, int S, hipStream_t st) {
  const int pm = tn().split_prio;
  int plo = 0, phi = 0;
  FL_HIP(hipDeviceGetStreamPriorityRange(&plo, &phi));
  const int k0 = pm == 0 && !tn().prio_all ? 1 : 0;
  for (int k = k0; k < S; ++k) {  // (S = 1: chain 0's stream only)
    if (d->run_aux[pm][k]) continue;
    const int pr = pm == 1 ? plo : pm == 2 ? phi : (k == 1 ? phi : k == 2 ? plo : 0);
    // a new stream that serialises with an earlier chain's is parked (kept alive, so its hardware queue stays
    // counted as used) and another one is created; the probe needs host syncs, so it is skipped inside a capture
    const bool probe = k > k0 && !stream_capturing(st);
    if (probe && !d->qprobe) FL_HIP(hipMalloc(&d->qprobe, 64));
    for (int tries = 0;; ++tries) {
      hipStream_t sk = nullptr;
      FL_HIP(hipStreamCreateWithPriority(&sk, hipStreamNonBlocking, pr));
      bool ok = true;
      for (int j = k0; probe && ok && j < k; ++j) {
        int c1 = 0, c2 = 0;
        const int rc1 = streams_concurrent(d->qprobe, d->run_aux[pm][j], sk, &c1);
        const int rc2 = rc1 ? rc1 : streams_concurrent(d->qprobe, sk, d->run_aux[pm][j], &c2);
        if (rc2) { (void)hipStreamDestroy(sk); return rc2; }
        if (c1 == 2 || c2 == 2) ++d->qprobe_busy;  // inconclusive: keep the stream (only a measured serialisation parks)
        ok = c1 != 1 && c2 != 1;
      }
      if (ok || tries >= Den::kMaxParked || d->n_parked >= Den::kMaxParked) {
        d->run_aux[pm][k] = sk;
        d->qprobe_retries += tries;
        break;
      }
      d->parked[d->n_parked++] = sk;
    }
  }
  return kOk;
}

FLAMED_API int flamed_den_solve_part(flamed_den_t h, float* xt, const float* mods, int nfe, int B, int T, void* ws,
                                     size_t ws_bytes, int use_graph, int s0, int s1, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev, "flamed_den_solve: handle not loaded");
  FL_REQUIRE(xt && mods && ws && B > 0 && T > 0 && nfe > 0, "flamed_den_solve: bad args");
  FL_REQUIRE(0 <= s0 && s0 < s1 && s1 <= nfe, "flamed_den_solve_part: bad step range [%d, %d) of %d", s0, s1, nfe);
  FL_DEN_CALL(d);
  FL_REQUIRE_ON(xt, d->device, "flamed_den_solve");
  if (ws_bytes < den_solve_ws(d, B, T)) {
    set_error("flamed_den_solve: workspace too small");
    return kNoWorkspace;
  }
  // delta_t = 1 / nfe as a python float, applied in fp32 (prob_generator.py:441,445)
  const float dt = (float)(1.0 / (double)nfe);
  const size_t step_stride = (size_t)B * d->MS;
  const int S = den_split(d, B, T), Bk = B / S;
  const size_t wsk = S > 1 ? den_split_ws(d, B, T, S) : 0;
  auto sub = [&](int k, float*& xk, const float*& mk, void*& wk) {  // chain k's state, table rows, workspace
    xk = xt + (size_t)k * Bk * T * d->C;
    mk = mods + (size_t)k * Bk * d->MS;
    wk = static_cast<char*>(ws) + k * wsk;
  };
  if (!(use_graph & 1)) {
    for (int s = s0; s < s1; ++s)
      for (int k = 0; k < S; ++k) {
        float* xk; const float* mk; void* wk;
        sub(k, xk, mk, wk);
        int rc = den_step(d, xk, mk + s * step_stride, T, Bk, T, dt, nullptr, wk, st, nullptr, nullptr, B, k, S);
        if (rc) return rc;
      }
    return kOk;
  }
  const int G = graph_chunk(nfe);
  FL_REQUIRE(s0 % G == 0 && (s1 % G == 0 || s1 == nfe), "flamed_den_solve_part: range [%d, %d) not on %d-step graph chunks",
             s0, s1, G);
  // the parts of one solve must run one step structure: a knob change between parts is rejected, and the
  // path (one persistent launch per part, or the graph of launches) is decided once, by the step-0 part
  if (s0 == 0) {
    d->part_epoch = d->tune_ver;
    d->ppath = !(use_graph & 2) && persist_eligible(d, B, T) ? 1 : 0;  // bit 2: the caller's retry, no persistent launch
    d->ppath_key[0] = B; d->ppath_key[1] = T; d->ppath_key[2] = nfe;
  }
  FL_REQUIRE(d->part_epoch == d->tune_ver, "flamed_den_solve_part: knobs changed since step 0 of this solve (part [%d, %d))",
             s0, s1);
  FL_REQUIRE(d->ppath >= 0 && d->ppath_key[0] == B && d->ppath_key[1] == T && d->ppath_key[2] == nfe,
             "flamed_den_solve_part: part [%d, %d) of a solve whose step-0 part did not run on this handle", s0, s1);
  if (d->ppath == 1) {  // one persistent launch for the whole range (B = 1)
    const int prc = persist_solve(d, xt, mods, nfe, B, T, s0, s1, st);
    if (prc == kOk || s0 != 0 || prc != kBadArg) return prc;
    // the runtime refused the cooperative grid (not all 256 workgroups co-resident): this device never
    // runs the persistent solve; this solve (still at step 0) takes the graph of launches
    d->pdev_ok = 0;
    d->ppath = 0;
  }
  if (!d->ctr) FL_HIP(hipMalloc(&d->ctr, 256));
  // fused Euler steps: 25 launches per step instead of 26 (the combine rides in the next proj_in); the
  // state ping-pongs between xt (even steps) and the workspace's XP (odd steps), so G must be even
  const bool fused = S == 1 && den_fused_ok(d, B, T) && G % 2 == 0;
  const bool fbig = !fused && den_fused_big(d, Bk, T);  // large M: in-place fused steps, per chain
  const bool br = S > 1 && tn().split_graph == 1;
  DenWs w;
  den_ws_layout(d, B, T, ws, &w);
  // the graph bakes in dt = 1/nfe, so nfe is part of the key
  const bool hit = d->gexec && d->g_B == B && d->g_T == T && d->g_nfe == nfe && d->g_xt == xt && d->g_mods == mods && d->g_ws == ws &&
                   d->g_epoch == d->tune_ver;
  if (!hit) {
    retire_graph(d->gexec);
    for (auto& g : d->gexec_c) retire_graph(g);
    if (!d->cap_stream) FL_HIP(hipStreamCreateWithFlags(&d->cap_stream, hipStreamNonBlocking));
    if (S > 1 && !br) {
      const int rc = den_chain_streams(d, S, st);
      if (rc) return rc;
    }
    for (int k = 0; k < Den::kMaxSplit; ++k)
      if (!d->cap_ev[k]) FL_HIP(hipEventCreateWithFlags(&d->cap_ev[k], hipEventDisableTiming));
    if (br) {  // tune split_graph 1 (round 4): one graph, the chains as parallel branches (fork / join events)
      for (int k = 1; k < S; ++k)
        if (!d->cap_aux[k]) FL_HIP(hipStreamCreateWithFlags(&d->cap_aux[k], hipStreamNonBlocking));
      FL_HIP(hipStreamBeginCapture(d->cap_stream, hipStreamCaptureModeRelaxed));
      FL_HIP(hipEventRecord(d->cap_ev[0], d->cap_stream));
      for (int k = 1; k < S; ++k) FL_HIP(hipStreamWaitEvent(d->cap_aux[k], d->cap_ev[0], 0));
      int rc = kOk;
      for (int k = 0; k < S && rc == kOk; ++k) {
        float* xk; const float* mk; void* wk;
        sub(k, xk, mk, wk);
        hipStream_t cs = k == 0 ? d->cap_stream : d->cap_aux[k];
        for (int s = 0; s < G && rc == kOk; ++s) rc = den_step(d, xk, mk, T, Bk, T, dt, nullptr, wk, cs, d->ctr + 16 * k, fbig ? xk : nullptr, B, k, S);
      }
      for (int k = 1; k < S && rc == kOk; ++k) {
        FL_HIP(hipEventRecord(d->cap_ev[k], d->cap_aux[k]));
        FL_HIP(hipStreamWaitEvent(d->cap_stream, d->cap_ev[k], 0));
      }
      hipGraph_t g = nullptr;
      hipError_t e = hipStreamEndCapture(d->cap_stream, &g);
      if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
      FL_HIP(e);
      hipError_t ie = hipGraphInstantiate(&d->gexec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      FL_HIP(ie);
    }
    // one graph per chain (G steps of its sub-batch), captured one after another on cap_stream
    for (int k = 0; k < (br ? 0 : S); ++k) {
      FL_HIP(hipStreamBeginCapture(d->cap_stream, hipStreamCaptureModeRelaxed));
      int rc = kOk;
      float* xk; const float* mk; void* wk;
      sub(k, xk, mk, wk);
      for (int s = 0; s < G && rc == kOk; ++s) {
        if (fused) rc = den_step(d, s % 2 ? w.XP : xt, mods, T, B, T, dt, nullptr, ws, d->cap_stream, d->ctr, s % 2 ? xt : w.XP);
        else rc = den_step(d, xk, mk, T, Bk, T, dt, nullptr, wk, d->cap_stream, d->ctr + 16 * k, fbig ? xk : nullptr, B, k, S);
      }
      hipGraph_t g = nullptr;
      hipError_t e = hipStreamEndCapture(d->cap_stream, &g);
      if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
      FL_HIP(e);
      hipGraphExec_t& ex = k == 0 ? d->gexec : d->gexec_c[k];
      hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      FL_HIP(ie);
    }
    d->g_B = B; d->g_T = T; d->g_nfe = nfe; d->g_epoch = d->tune_ver; d->g_xt = xt; d->g_mods = mods; d->g_ws = ws;
  }
  const size_t n = (size_t)B * T * d->C;
  if (s0 == 0) {
    if (fused) {  // counter -1: each step's proj_in advances it before the step's first modulation read
      hipLaunchKernelGGL(euler_init_kernel, dim3((n + 255) / 256), dim3(256), 0, st, xt, d->bout, w.XP, w.Y, B * T, d->C);
      FL_LAUNCH_CHECK();
      FL_HIP(hipMemsetAsync(d->ctr, 0xff, sizeof(int), st));
    } else if (fbig) {  // every chain: Y whose combine is exactly 0, counter -1 (its euler_cast advances it)
      for (int k = 0; k < S; ++k) {
        float* xk; const float* mk; void* wk;
        sub(k, xk, mk, wk);
        DenWs wc;
        den_ws_layout(d, Bk, T, wk, &wc);
        const size_t nk = (size_t)Bk * T * d->C;
        hipLaunchKernelGGL(euler_init_kernel, dim3((nk + 255) / 256), dim3(256), 0, st, xk, d->bout, (float*)nullptr, wc.Y, Bk * T, d->C);
        FL_LAUNCH_CHECK();
        FL_HIP(hipMemsetAsync(d->ctr + 16 * k, 0xff, sizeof(int), st));
      }
    } else {
      FL_HIP(hipMemsetAsync(d->ctr, 0, 256, st));  // the step counters of every chain (16 ints apart)
    }
  }
  if ((S > 1 && !br) || tn().prio_all) {  // fork: every chain replays its graph for the whole range on its stream, then join
    const int NG = br ? 1 : S;  // graphs to replay
    if (NG == 1) {
      const int rc = den_chain_streams(d, 1, st);  // (prio_all: the single graph on a chain stream too)
      if (rc) return rc;
    }
    const int pm = tn().split_prio;
    const bool own0 = pm != 0 || tn().prio_all;  // chain 0 off the caller's stream
    FL_HIP(hipEventRecord(d->cap_ev[0], st));
    for (int k = 0; k < NG; ++k) {
      hipStream_t cs = (k == 0 && !own0) ? st : d->run_aux[pm][k];
      if (cs != st) FL_HIP(hipStreamWaitEvent(cs, d->cap_ev[0], 0));
      for (int r = s0 / G; r < s1 / G; ++r) FL_HIP(hipGraphLaunch(k == 0 ? d->gexec : d->gexec_c[k], cs));
    }
    for (int k = 0; k < NG; ++k) {
      hipStream_t cs = (k == 0 && !own0) ? st : d->run_aux[pm][k];
      if (cs == st) continue;
      FL_HIP(hipEventRecord(d->cap_ev[1 + k % (Den::kMaxSplit - 1)], cs));  // (S <= kMaxSplit: k < 3 or pm == 0)
      FL_HIP(hipStreamWaitEvent(st, d->cap_ev[1 + k % (Den::kMaxSplit - 1)], 0));
    }
  } else {
    for (int r = s0 / G; r < s1 / G; ++r) FL_HIP(hipGraphLaunch(d->gexec, st));
  }
  note_graph_use(d->gexec, st);
  for (int k = 1; k < (br ? 1 : S); ++k) note_graph_use(d->gexec_c[k], st);  // st has joined chain k's replays
  if (fused && s1 == nfe) {  // the last step's combine + Euler update: x_nfe = XP + dt * v (nfe even: XP holds x_{nfe-1})
    hipLaunchKernelGGL(conv3_combine_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w.Y, d->bout, xt, nullptr, B * T, T,
                       d->C, dt, nullptr, w.XP);
    FL_LAUNCH_CHECK();
  }
  if (fbig && s1 == nfe) {  // every chain's last combine + Euler update, in place
    for (int k = 0; k < S; ++k) {
      float* xk; const float* mk; void* wk;
      sub(k, xk, mk, wk);
      DenWs wc;
      den_ws_layout(d, Bk, T, wk, &wc);
      const size_t nk = (size_t)Bk * T * d->C;
      hipLaunchKernelGGL(conv3_combine_kernel, dim3((nk + 255) / 256), dim3(256), 0, st, wc.Y, d->bout, xk, nullptr, Bk * T, T,
                         d->C, dt, nullptr, nullptr);
      FL_LAUNCH_CHECK();
    }
  }
  return kOk;
}

}  // extern "C"

extern "C" {

#ifdef FL_STAMPS  // diagnostic library only (include/flamed_diag.h)
FLAMED_API int flamed_stamp_buffer(void* buf) {
  g_stamp_dev = reinterpret_cast<unsigned long long*>(buf);
  return kOk;
}
#endif

// In-graph per-launch cost of every kernel class: a graph of `steps` Euler steps (dt = 0) is timed
// as captured and again with one class launched twice per occurrence (flamed_tune dup_class); the
// difference over the number of duplicated launches is what one launch of the class costs inside a
// replayed step (dispatch included, event overhead excluded).  ms_out[c] per launch, ms_out[kClasses]
// = one whole step.
FLAMED_API int flamed_den_time_kernels_graph(flamed_den_t h, float* xt, const float* mods, int B, int T, void* ws,
                                             size_t ws_bytes, int reps, float* ms_out, hipStream_t st) {
  Den* d = reinterpret_cast<Den*>(h);
  FL_REQUIRE(d && d->dev && xt && mods && ws && ms_out && reps > 0, "flamed_den_time_kernels_graph: bad args");
  FL_DEN_CALL(d);
  if (ws_bytes < den_ws_bytes(d, B, T)) {
    set_error("flamed_den_time_kernels_graph: workspace too small");
    return kNoWorkspace;
  }
  constexpr int kSteps = 4;
  if (!d->cap_stream) FL_HIP(hipStreamCreateWithFlags(&d->cap_stream, hipStreamNonBlocking));
  // every exit (early error returns included) restores the handle's knob snapshot and frees the events
  struct Restore {
    Den* d;
    int dup;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    ~Restore() {
      d->tune.dup_class = dup;
      if (e0) (void)hipEventDestroy(e0);
      if (e1) (void)hipEventDestroy(e1);
    }
  } guard{d, d->tune.dup_class};
  FL_HIP(hipEventCreate(&guard.e0));
  FL_HIP(hipEventCreate(&guard.e1));
  hipEvent_t e0 = guard.e0, e1 = guard.e1;
  const int saved_dup = guard.dup;  // the handle's active snapshot (this call's TuneScope)
  // the step structure the solve graph uses: fused Euler steps (no combine launches) where it fuses
  const bool fused = den_fused_ok(d, B, T);
  const bool fbig = !fused && den_fused_big(d, B, T);
  DenWs w;
  den_ws_layout(d, B, T, ws, &w);
  if (fused || fbig) {
    const size_t n = (size_t)B * T * d->C;
    hipLaunchKernelGGL(euler_init_kernel, dim3((n + 255) / 256), dim3(256), 0, st, xt, d->bout, fused ? w.XP : (float*)nullptr,
                       w.Y, B * T, d->C);
    FL_LAUNCH_CHECK();
  }
  auto timed = [&](int dup, float* ms) -> int {
    d->tune.dup_class = dup;
    FL_HIP(hipStreamBeginCapture(d->cap_stream, hipStreamCaptureModeRelaxed));
    int rc = kOk;
    for (int i = 0; i < kSteps && rc == kOk; ++i) {
      if (fused) rc = den_step(d, i % 2 ? w.XP : xt, mods, T, B, T, 0.f, nullptr, ws, d->cap_stream, nullptr, i % 2 ? xt : w.XP);
      else rc = den_step(d, xt, mods, T, B, T, 0.f, nullptr, ws, d->cap_stream, nullptr, fbig ? xt : nullptr);
    }
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(d->cap_stream, &g);
    d->tune.dup_class = saved_dup;
    if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
    FL_HIP(e);
    hipGraphExec_t ex;
    hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    FL_HIP(ie);
    FL_HIP(hipGraphLaunch(ex, st));
    FL_HIP(hipGraphLaunch(ex, st));
    FL_HIP(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) FL_HIP(hipGraphLaunch(ex, st));
    FL_HIP(hipEventRecord(e1, st));
    FL_HIP(hipEventSynchronize(e1));
    FL_HIP(hipEventElapsedTime(ms, e0, e1));
    *ms /= (float)(reps * kSteps);
    (void)hipGraphExecDestroy(ex);
    return kOk;
  };
  float base = 0.f;
  int rc = timed(-1, &base);
  const int NB = d->NB;
  const int per_step[FLAMED_DEN_KERNEL_CLASSES] = {1, NB + 1, 0, NB + 1, NB + 1, NB, NB, 1, fused ? 0 : 1};
  for (int c = 0; c < FLAMED_DEN_KERNEL_CLASSES && rc == kOk; ++c) {
    float t = base;
    if (per_step[c] > 0 && (c != 2 || d->gcnt == nullptr)) rc = timed(c, &t);
    ms_out[c] = per_step[c] > 0 ? (t - base) / (float)per_step[c] : 0.f;
  }
  ms_out[FLAMED_DEN_KERNEL_CLASSES] = base;
  return rc;
}

}  // extern "C"
