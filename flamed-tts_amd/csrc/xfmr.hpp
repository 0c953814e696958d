// Transformer building blocks shared by the prior stack (prior.hip) and the FaCodec timbre encoder
// (prompt.hip): row LayerNorm (+ key-padding mask), LDS-staged fp32 attention, residual GEMM epilogue.
#pragma once
#include "gemm.hpp"

#include <cmath>
#include <vector>

namespace fl {

// LayerNorm (eps 1e-5, affine) + masked_fill(mask, 0), one wave per row.  With `embs` the rows j >= P
// of utterance b are also written to embs[b][q][j - P] (the decoder's target slice, :181-182).
template <int D>
__global__ __launch_bounds__(256) void ln_mask_kernel(const float* __restrict__ R, const float* __restrict__ g,
                                                      const float* __restrict__ bb, const uint8_t* __restrict__ mask,
                                                      float* __restrict__ X, int M, int n, float* __restrict__ embs,
                                                      int P, int T, int nq, int q) {
  constexpr int PER = D / 64;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  const float* r = R + (size_t)m * D;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = r[lane + 64 * j];
    s += v[j];
  }
  const float mean = wave_sum64(s) / (float)D;
  float qv = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    float d = v[j] - mean;
    qv += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum64(qv) / (float)D + 1e-5f);
  const bool pad = mask && mask[m] != 0;
  float* x = X + (size_t)m * D;
  const int b = m / n, l = m - b * n;
  float* e = (embs && l >= P) ? embs + (((size_t)b * nq + q) * T + (l - P)) * D : nullptr;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    int c = lane + 64 * j;
    float y = pad ? 0.f : ((v[j] - mean) * rstd) * g[c] + bb[c];
    x[c] = y;
    if (e) e[c] = y;
  }
}

// Scaled dot-product attention with an optional key-padding mask (prior: Modules.py:14-25,
// SubLayers.py:38-52; timbre encoder: nn.MultiheadAttention without a mask, facodec/transformer.py:116).
// QKV rows (B*n, 3D): Q at column h*DK, K at D + h*DK, V at 2D + h*DK.  Out O (B*n, D), head h at h*DK.
// Block: 512 threads = 8 waves; lane = query of a 64-query tile, wave w takes keys [8w, 8w+8) of every
// 64-key chunk (all lanes read the same K/V row: LDS broadcast).  K/V chunks are double-buffered in LDS
// and the next chunk's global loads are issued before the current chunk's math (registers -> LDS after
// it), so one HBM/L2 latency per chunk is hidden.  Each wave keeps an online-softmax state (max, sum,
// acc[DK]); the eight states of a query are merged through LDS at the end.
constexpr int kAttnWaves = 8;
constexpr int kAttnKC = 64;  // keys per chunk
constexpr size_t attn_lds_bytes(int DK) {
  const size_t buf = (size_t)2 * 2 * kAttnKC * DK * 4;            // 2 buffers x (K, V)
  const size_t merge = (size_t)kAttnWaves * 64 * (DK + 2) * 4;    // per-wave (acc, max, sum) of 64 queries
  return (buf > merge ? buf : merge) + 2 * kAttnKC;               // + 2 mask chunks
}
template <int DK>
__global__ __launch_bounds__(512) void attn_kernel(const float* __restrict__ QKV, const uint8_t* __restrict__ kmask,
                                                   int n, int D, float temp, float* __restrict__ O) {
  constexpr int NW = kAttnWaves, KC = kAttnKC, KW = KC / NW;
  constexpr int V4 = KC * DK / 4;              // float4s per operand chunk
  constexpr int PT = (2 * V4 + 511) / 512;     // float4s per thread per chunk (K and V)
  constexpr int DS = DK / NW;                  // output dims per thread in the merge
  static_assert(DK % NW == 0 && DK % 4 == 0, "head width");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  uint8_t* msk = reinterpret_cast<uint8_t*>(sm) + attn_lds_bytes(DK) - 2 * KC;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const int qi = blockIdx.x * 64 + lane;
  const int ld = 3 * D;
  const float* base = QKV + (size_t)b * n * ld;

  float qv[DK];
  {
    const float* qp = base + (size_t)(qi < n ? qi : n - 1) * ld + h * DK;
#pragma unroll
    for (int d = 0; d < DK; d += 4) {
      float4 t = ld4(qp + d);
      qv[d] = t.x; qv[d + 1] = t.y; qv[d + 2] = t.z; qv[d + 3] = t.w;
    }
  }
  float4 pf[PT];
  uint8_t pm = 1;
  auto fetch = [&](int k0) {
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = tid + j * 512;
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < 2 * V4) {
        const int op = i / V4, r = i - op * V4;
        const int key = r / (DK / 4), c = (r - key * (DK / 4)) * 4;
        const int kk = k0 + key;
        if (kk < n) t = ld4(base + (size_t)kk * ld + (op + 1) * D + h * DK + c);
      }
      pf[j] = t;
    }
    if (tid < KC) {
      const int kk = k0 + tid;
      pm = kk < n ? (kmask ? kmask[(size_t)b * n + kk] : 0) : 1;
    }
  };
  auto stash = [&](int buf) {
    float* KV = sm + buf * 2 * KC * DK;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = tid + j * 512;
      if (i < 2 * V4) *reinterpret_cast<float4*>(KV + (size_t)i * 4) = pf[j];  // K rows then V rows
    }
    if (tid < KC) msk[buf * KC + tid] = pm;
  };

  float mx = -INFINITY, sum = 0.f, acc[DK];
#pragma unroll
  for (int d = 0; d < DK; ++d) acc[d] = 0.f;
  const int nch = (n + KC - 1) / KC;
  fetch(0);
  stash(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    if (c + 1 < nch) fetch((c + 1) * KC);  // in flight during this chunk's math
    const float* Ks = sm + buf * 2 * KC * DK;
    const float* Vs = Ks + KC * DK;
    const uint8_t* ms = msk + buf * KC;
    float s[KW];
    float cmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < KW; ++j) {
      const int key = w * KW + j;
      const float* kr = Ks + key * DK;
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < DK; d += 4) {
        float4 kv = *reinterpret_cast<const float4*>(kr + d);
        dot = fmaf(qv[d], kv.x, dot);
        dot = fmaf(qv[d + 1], kv.y, dot);
        dot = fmaf(qv[d + 2], kv.z, dot);
        dot = fmaf(qv[d + 3], kv.w, dot);
      }
      s[j] = ms[key] ? -INFINITY : dot / temp;
      cmax = fmaxf(cmax, s[j]);
    }
    if (cmax != -INFINITY) {  // uniform per wave: every key of this wave's slice may be padding
      const float nm = fmaxf(mx, cmax);
      const float sc = __expf(mx - nm);  // mx = -inf on the first live slice: 0
      sum *= sc;
#pragma unroll
      for (int d = 0; d < DK; ++d) acc[d] *= sc;
#pragma unroll
      for (int j = 0; j < KW; ++j) {
        const float p = __expf(s[j] - nm);  // masked keys: 0
        sum += p;
        const float* vr = Vs + (w * KW + j) * DK;
#pragma unroll
        for (int d = 0; d < DK; d += 4) {
          float4 vv = *reinterpret_cast<const float4*>(vr + d);
          acc[d] = fmaf(p, vv.x, acc[d]);
          acc[d + 1] = fmaf(p, vv.y, acc[d + 1]);
          acc[d + 2] = fmaf(p, vv.z, acc[d + 2]);
          acc[d + 3] = fmaf(p, vv.w, acc[d + 3]);
        }
      }
      mx = nm;
    }
    if (c + 1 < nch) stash(buf ^ 1);  // that buffer's last readers finished before the previous barrier
    __syncthreads();
  }
  // merge the eight waves' partial softmax states: acc as [w][d][lane] (conflict-free), then (max, sum)
  float* pa = sm;                          // NW * DK * 64
  float* pmx = sm + NW * DK * 64;          // NW * 64
  float* psm = pmx + NW * 64;              // NW * 64
#pragma unroll
  for (int d = 0; d < DK; ++d) pa[(w * DK + d) * 64 + lane] = acc[d];
  pmx[w * 64 + lane] = mx;
  psm[w * 64 + lane] = sum;
  __syncthreads();
  if (qi >= n) return;
  float M = -INFINITY;
#pragma unroll
  for (int u = 0; u < NW; ++u) M = fmaxf(M, pmx[u * 64 + lane]);
  float f[NW], L = 0.f;
#pragma unroll
  for (int u = 0; u < NW; ++u) {
    f[u] = __expf(pmx[u * 64 + lane] - M);  // all keys padded: M = -inf -> NaN, as the reference's softmax
    L += psm[u * 64 + lane] * f[u];
  }
  float* o = O + ((size_t)b * n + qi) * D + h * DK + w * DS;
#pragma unroll
  for (int d = 0; d < DS; ++d) {
    float a = 0.f;
#pragma unroll
    for (int u = 0; u < NW; ++u) a += pa[(u * DK + w * DS + d) * 64 + lane] * f[u];
    o[d] = a / L;
  }
}

// The same attention on the fp32 matrix cores (v_mfma_f32_16x16x4_f32).  Per workgroup 16 QW queries of one
// (utterance, head); 8 waves = KG key groups x QW query waves: wave (g, w) owns queries [16 w, 16 w + 16)
// and the 64-key chunks c = g (mod KG).  Transposed products keep every operand where the next MFMA wants
// it without a shuffle: S^T (keys x queries) = K . Q^T leaves lane (c, r) holding P^T[key 4 r + i][query c],
// which is exactly that lane's B operand of O^T (dims x queries) = V^T . P^T when the MFMA's four K slots
// are mapped to keys {4 r + i} (the same permutation on V^T's A operand, read from a transposed V chunk).
// Online softmax per query column (max / sum over the 4 lanes of a column by two xor shuffles), the two
// key groups merged through LDS at the end.  Chunks are staged K row-major and V transposed, rows padded
// by 16 B, the next chunk's global loads in registers while the current one is computed.
// QW query waves x KG key groups = 8 waves: 16 QW queries per workgroup; key group g takes chunks c = g
// (mod KG).  Two configs: (4, 2) and, where the LDS of four double-buffered groups fits (32-wide heads, the
// prior decoders at n = 640: 120 -> 240 workgroups), (2, 4).
template <int DK, int QW>
struct AttnM {
  static constexpr int KG = 8 / QW, GT = 64 * QW;                 // key groups, threads per group
  static constexpr int KC = 64, KS = DK + 4, VS = KC + 4;         // padded LDS row strides (floats)
  static constexpr int BUF = KC * KS + DK * VS;                   // K chunk + V^T chunk
  static constexpr int V4 = KC * DK / 4;                          // float4s per operand chunk
  static constexpr int PT = (2 * V4 + GT - 1) / GT;               // float4s per thread of a group
  static constexpr size_t lds() {
    return (size_t)2 * KG * BUF * 4 + 2 * KG * KC + (size_t)(KG - 1) * QW * 64 * (2 + 4 * (DK / 16)) * 4;
  }
};
template <int DK, int QW>
__global__ __launch_bounds__(512) void attn_mfma_kernel(const float* __restrict__ QKV, const uint8_t* __restrict__ kmask,
                                                        int n, int D, float temp, float* __restrict__ O) {
  using A = AttnM<DK, QW>;
  constexpr int KC = A::KC, NT = KC / 16, SB = DK / 16, DT = DK / 16, PT = A::PT, KG = A::KG, GT = A::GT;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  // buffers: [group][2] x (K [KC][KS], V^T [DK][VS]); masks [group][2][KC] bytes; merge area after
  uint8_t* msk = reinterpret_cast<uint8_t*>(sm + 2 * KG * A::BUF);
  float* mrg = reinterpret_cast<float*>(msk + 2 * KG * KC);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), grp = w / QW, wq = w % QW, gt = tid % GT;
  const int h = blockIdx.y, b = blockIdx.z;
  const int c = lane & 15, r = lane >> 4;
  const int ld = 3 * D;
  const float* base = QKV + (size_t)b * n * ld;
  const int qi = blockIdx.x * (16 * QW) + wq * 16 + c;  // this lane's query (column of every MFMA tile)
  float4 qr[SB];
  {
    const float* qp = base + (size_t)(qi < n ? qi : n - 1) * ld + h * DK;
#pragma unroll
    for (int sb = 0; sb < SB; ++sb) qr[sb] = ld4(qp + 16 * sb + 4 * r);
  }
  float4 pf[PT];
  uint8_t pm = 1;
  auto fetch = [&](int k0) {  // this group's next chunk into registers
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = gt + j * GT;
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < 2 * A::V4) {
        const int op = i / A::V4, rr = i - op * A::V4;
        const int key = rr / (DK / 4), cc = (rr - key * (DK / 4)) * 4;
        if (k0 + key < n) t = ld4(base + (size_t)(k0 + key) * ld + (op + 1) * D + h * DK + cc);
      }
      pf[j] = t;
    }
    if (gt < KC) {
      const int kk = k0 + gt;
      pm = kk < n ? (kmask ? kmask[(size_t)b * n + kk] : 0) : 1;
    }
  };
  auto stash = [&](int buf) {  // registers -> this group's LDS buffer (K row-major, V transposed)
    float* Kb = sm + (grp * 2 + buf) * A::BUF;
    float* Vt = Kb + KC * A::KS;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = gt + j * GT;
      if (i < 2 * A::V4) {
        const int op = i / A::V4, rr = i - op * A::V4;
        const int key = rr / (DK / 4), cc = (rr - key * (DK / 4)) * 4;
        if (op == 0) {
          *reinterpret_cast<float4*>(Kb + key * A::KS + cc) = pf[j];
        } else {
          Vt[(cc + 0) * A::VS + key] = pf[j].x;
          Vt[(cc + 1) * A::VS + key] = pf[j].y;
          Vt[(cc + 2) * A::VS + key] = pf[j].z;
          Vt[(cc + 3) * A::VS + key] = pf[j].w;
        }
      }
    }
    if (gt < KC) msk[(grp * 2 + buf) * KC + gt] = pm;
  };

  float m = -INFINITY, l = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nch = (n + KC - 1) / KC, iters = (nch + KG - 1) / KG;
  fetch(grp * KC);
  stash(0);
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    const int buf = it & 1, ch = KG * it + grp;
    if (it + 1 < iters) fetch((ch + KG) * KC);  // in flight during this chunk's math
    const float* Kb = sm + (grp * 2 + buf) * A::BUF;
    const float* Vt = Kb + KC * A::KS;
    const uint8_t* mk = msk + (grp * 2 + buf) * KC;
    if (ch < nch) {
      f32x4 s[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
          const float4 kf = *reinterpret_cast<const float4*>(Kb + (16 * t + c) * A::KS + 16 * sb + 4 * r);
          s[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.x, qr[sb].x, s[t], 0, 0, 0);
          s[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.y, qr[sb].y, s[t], 0, 0, 0);
          s[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.z, qr[sb].z, s[t], 0, 0, 0);
          s[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.w, qr[sb].w, s[t], 0, 0, 0);
        }
      }
      // S^T lane (c, r): keys 16 t + 4 r + i of query c; scale, mask, chunk max over the query's 64 keys
      float cmax = -INFINITY;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = mk[16 * t + 4 * r + i] ? -INFINITY : s[t][i] / temp;
          s[t][i] = v;
          cmax = fmaxf(cmax, v);
        }
      cmax = fmaxf(cmax, __shfl_xor(cmax, 16));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32));
      const float nm = fmaxf(m, cmax);
      float rs = 0.f;
      if (nm != -INFINITY) {  // (per query: a column whose keys so far are all padding keeps m = -inf)
        const float sc = __expf(m - nm);  // m = -inf: 0
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __expf(s[t][i] - nm);
            s[t][i] = p;
            rs += p;
          }
        l *= sc;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= sc;
        m = nm;
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      rs += __shfl_xor(rs, 16);
      rs += __shfl_xor(rs, 32);
      l += rs;
      // O^T += V^T . P^T: MFMA (t, i) maps K slot r to key 16 t + 4 r + i on both operands
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float4 vf = *reinterpret_cast<const float4*>(Vt + (16 * dt + c) * A::VS + 16 * t + 4 * r);
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf.x, s[t][0], o[dt], 0, 0, 0);
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf.y, s[t][1], o[dt], 0, 0, 0);
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf.z, s[t][2], o[dt], 0, 0, 0);
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf.w, s[t][3], o[dt], 0, 0, 0);
        }
    }
    if (it + 1 < iters) stash(buf ^ 1);  // that buffer's last readers finished before the previous barrier
    __syncthreads();
  }
  // merge the key groups: groups 1.. leave (m, l, o) per lane, group 0 combines them in group order
  constexpr int MS = 2 + 4 * DT;
  if (grp > 0) {
    float* mw = mrg + (((grp - 1) * QW + wq) * 64 + lane) * MS;
    mw[0] = m;
    mw[1] = l;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) mw[2 + 4 * dt + i] = o[dt][i];
  }
  __syncthreads();
  if (grp > 0) return;
  float M = m;
#pragma unroll
  for (int g = 1; g < KG; ++g) M = fmaxf(M, mrg[(((g - 1) * QW + wq) * 64 + lane) * MS]);
  float f[KG];
  f[0] = __expf(m - M);  // all keys padded: M = -inf -> NaN, as the reference's softmax
  float L = l * f[0];
#pragma unroll
  for (int g = 1; g < KG; ++g) {
    const float* mw = mrg + (((g - 1) * QW + wq) * 64 + lane) * MS;
    f[g] = __expf(mw[0] - M);
    L += mw[1] * f[g];
  }
  if (qi >= n) return;
  float* op = O + ((size_t)b * n + qi) * D + h * DK;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = o[dt][i] * f[0];
#pragma unroll
      for (int g = 1; g < KG; ++g) a += mrg[(((g - 1) * QW + wq) * 64 + lane) * MS + 2 + 4 * dt + i] * f[g];
      v[i] = a / L;
    }
    *reinterpret_cast<float4*>(op + 16 * dt + 4 * r) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// ------------------------------------------------------------------ epilogues

// (acc + bias) + residual  (fc(out) + residual, SubLayers.py:54-55; w_2(...) + residual, :91-93)
struct EpiBiasRes {
  const float* __restrict__ bias;
  const float* __restrict__ res;
  float* __restrict__ out;
  int ldo;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int m, int n, float acc, const float*, int) const {
    return (acc + bias[n]) + res[(size_t)m * ldo + n];
  }
  __device__ void store(int m, int n, float v) const { out[(size_t)m * ldo + n] = v; }
  __device__ void store4(int m, int n, const float* v) const { store_val4<float>(out + (size_t)m * ldo + n, v); }
  __device__ void store_stats(int, int, float, float) const {}
};

// fp32 GEMM of the transformer stacks: the shape-driven config, but 32 x 32 tiles when 32 x 64 tiles
// would not give every CU a workgroup (N = 384 outputs at a few hundred rows: long K chains on few CUs).
template <class AL, class EP>
static int xf_gemm(const AL& al, const float* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  if (M < 2048 && (size_t)(N / 64) * ((M + 31) / 32) < 256 && N % 32 == 0)
    return launch_gemm_cfg<32, 32, 3, float>(al, W, ldw, ep, M, N, K, st);
  return launch_gemm<float>(al, W, ldw, ep, M, N, K, st);
}

template <int D>
static int launch_ln(const float* R, const float* g, const float* b, const uint8_t* mask, float* X, int M, int n,
                     float* embs, int P, int T, int nq, int q, hipStream_t st) {
  hipLaunchKernelGGL(ln_mask_kernel<D>, dim3((M + 3) / 4), dim3(256), 0, st, R, g, b, mask, X, M, n, embs, P, T, nq, q);
  FL_LAUNCH_CHECK();
  return kOk;
}
static int ln_mask(int D, const float* R, const float* g, const float* b, const uint8_t* mask, float* X, int M, int n,
                   float* embs, int P, int T, int nq, int q, hipStream_t st) {
  switch (D) {
    case 192: return launch_ln<192>(R, g, b, mask, X, M, n, embs, P, T, nq, q, st);
    case 256: return launch_ln<256>(R, g, b, mask, X, M, n, embs, P, T, nq, q, st);
    case 384: return launch_ln<384>(R, g, b, mask, X, M, n, embs, P, T, nq, q, st);
    default: FL_REQUIRE(false, "layer norm: unsupported model width %d", D);
  }
}
template <int DK>
static int launch_attn(const float* QKV, const uint8_t* mask, int B, int n, int D, int H, float temp, float* O, hipStream_t st) {
  if (tn().attn_mfma) {
    constexpr int QW = AttnM<DK, 2>::lds() <= 160 * 1024 ? 2 : 4;
    const size_t lds = AttnM<DK, QW>::lds();
    auto kern = attn_mfma_kernel<DK, QW>;
    if (lds > 64 * 1024) FL_HIP(set_max_lds(reinterpret_cast<const void*>(kern)));
    hipLaunchKernelGGL(kern, dim3((n + 16 * QW - 1) / (16 * QW), H, B), dim3(512), lds, st, QKV, mask, n, D, temp, O);
    FL_LAUNCH_CHECK();
    return kOk;
  }
  const size_t lds = attn_lds_bytes(DK);
  auto kern = attn_kernel<DK>;
  if (lds > 64 * 1024) FL_HIP(set_max_lds(reinterpret_cast<const void*>(kern)));
  hipLaunchKernelGGL(kern, dim3((n + 63) / 64, H, B), dim3(512), lds, st, QKV, mask, n, D, temp, O);
  FL_LAUNCH_CHECK();
  return kOk;
}
// softmax(Q K^T / sqrt(dk)) V per head; `mask` (B x n, 1 = padded key) may be null.  temperature =
// np.power(d_k, 0.5) applied as a division (SubLayers.py:21, Modules.py:17).
static int attention(int DK, const float* QKV, const uint8_t* mask, int B, int n, int D, int H, float* O, hipStream_t st) {
  const float temp = (float)std::sqrt((double)DK);
  switch (DK) {
    case 32: return launch_attn<32>(QKV, mask, B, n, D, H, temp, O, st);
    case 48: return launch_attn<48>(QKV, mask, B, n, D, H, temp, O, st);
    case 64: return launch_attn<64>(QKV, mask, B, n, D, H, temp, O, st);
    default: FL_REQUIRE(false, "attention: unsupported head width %d", DK);
  }
}


// One cached hipGraph of a whole stack call, re-captured when the call's key (pointers, shapes) changes.
struct CapGraph {
  hipGraphExec_t exec = nullptr;
  hipStream_t cap = nullptr;
  std::vector<const void*> key;
  void release() {
    retire_graph(exec);
    if (cap) (void)hipStreamDestroy(cap);
    *this = CapGraph();
  }
};

template <class F>
static int with_graph(CapGraph& g, const std::vector<const void*>& key_in, bool use_graph, hipStream_t st, F&& body) {
  if (!use_graph) return body(st);
  // the captured launches bake in the knobs the body read: the process tune epoch is part of the key
  std::vector<const void*> key = key_in;
  key.push_back((const void*)(intptr_t)tune_epoch());
  if (!g.exec || g.key != key) {
    retire_graph(g.exec);
    if (!g.cap) FL_HIP(hipStreamCreateWithFlags(&g.cap, hipStreamNonBlocking));
    FL_HIP(hipStreamBeginCapture(g.cap, hipStreamCaptureModeRelaxed));
    int r = body(g.cap);
    hipGraph_t gr = nullptr;
    hipError_t e = hipStreamEndCapture(g.cap, &gr);
    if (r) { if (gr) (void)hipGraphDestroy(gr); return r; }
    FL_HIP(e);
    hipError_t ie = hipGraphInstantiate(&g.exec, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    FL_HIP(ie);
    g.key = key;
  }
  FL_HIP(hipGraphLaunch(g.exec, st));
  note_graph_use(g.exec, st);
  return kOk;
}

}  // namespace fl
