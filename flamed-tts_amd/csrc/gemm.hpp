// MFMA GEMM template for gfx950: C[M][N] = A[M][K] · W[N][K]^T with a pluggable A-operand loader
// (fused prologue: dtype conversion, LayerNorm+AdaLN modulation, conv tap gathers, ...) and a
// pluggable epilogue (bias, activations, gated residuals, LayerNorm row-partials, Euler update).
//
// Geometry: 256 threads = 4 waves in a 2x2 grid; wave tile (BM/2)x(BN/2) built from 16x16 MFMA
// fragments.  One K-step stages BM (and BN) rows x KCH 16-byte chunks through double-buffered LDS
// (rows padded by 16 B).  DT selects the MFMA:
//   bf16 : v_mfma_f32_16x16x32_bf16, one MFMA per 64 B of row (lane group q = lane>>4 owns 16 B);
//   f32  : v_mfma_f32_16x16x4_f32, four MFMAs per 64 B of row: lane group q owns k = 4q..4q+3 and
//          MFMA j consumes element j — a permutation of the K order applied identically to A and W,
//          so the result is an exact fp32 FMA chain (parity mode).
#pragma once
#include "common.hpp"

namespace fl {

constexpr int kGemmThreads = 256;

template <int BM, int BN, int KCH, class AL, class EP>
struct GemmSmem {
  static constexpr int ROWB = KCH * 16 + 16;
  static constexpr int tiles = 2 * (BM + BN) * ROWB;
  static constexpr int a_stats = AL::stat_rows(BM) * 2 * 4;
  static constexpr int e_stats = EP::stat_rows(BM) * 2 * 4;
  static constexpr int red = BM * 2 * 4;
  static constexpr int bytes = ((tiles > red ? tiles : red) + a_stats + e_stats + 15) / 16 * 16;
};

// LayerNorm row statistics from producer partials: S[m][NT] = (tile mean, tile M2) over `tw` columns.
__device__ __forceinline__ void row_stats_from_partials(const float* __restrict__ S, int m, int NT, int tw,
                                                        float eps, float& mean, float& rstd) {
  const float2* p = reinterpret_cast<const float2*>(S) + (size_t)m * NT;
  float s = 0.f;
  for (int i = 0; i < NT; ++i) s += p[i].x;
  mean = s / (float)NT;
  float m2 = 0.f;
  for (int i = 0; i < NT; ++i) {
    float2 q = p[i];
    float d = q.x - mean;
    m2 += q.y + (float)tw * d * d;
  }
  float var = m2 / (float)(NT * tw);
  rstd = 1.0f / sqrtf(var + eps);
}

template <int BM, int BN, int KCH, typename DT, class AL, class EP>
__global__ __launch_bounds__(kGemmThreads) void gemm_kernel(AL al, const DT* __restrict__ W, int ldw, EP ep,
                                                             int M, int N, int K) {
  using SM = GemmSmem<BM, BN, KCH, AL, EP>;
  constexpr int EPC = DTraits<DT>::EPC;
  constexpr int ROWB = SM::ROWB;
  constexpr int BKE = KCH * EPC;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int ACH = BM * KCH / kGemmThreads;
  constexpr int BCH = BN * KCH / kGemmThreads;
  static_assert(ACH >= 1 && BCH >= 1, "tile too small for 256 threads");
  static_assert(KCH % 4 == 0, "KCH must be a multiple of 4 (64 B)");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* tileA0 = smem;
  char* tileA1 = smem + BM * ROWB;
  char* tileB0 = smem + 2 * BM * ROWB;
  char* tileB1 = tileB0 + BN * ROWB;
  float* a_stats = reinterpret_cast<float*>(smem + (SM::tiles > SM::red ? SM::tiles : SM::red));
  float* e_stats = a_stats + AL::stat_rows(BM) * 2;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int bn = blockIdx.x * BN;
  const int bm = blockIdx.y * BM;

  al.prologue(bm, BM, M, a_stats);
  ep.prologue(bm, BM, M, e_stats);
  __syncthreads();

  typename AL::Raw ra[ACH];
  uint4 rb[BCH];
  const int nsteps = K / BKE;

  auto issue = [&](int s) {
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      int m = bm + r;
      m = m < M ? m : M - 1;
      ra[j] = al.issue(m, s * BKE + kc * EPC);
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      rb[j] = *reinterpret_cast<const uint4*>(W + (size_t)(bn + r) * ldw + s * BKE + kc * EPC);
    }
  };
  auto commit = [&](int s, char* tA, char* tB) {
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      int m = bm + r;
      m = m < M ? m : M - 1;
      *reinterpret_cast<uint4*>(tA + r * ROWB + kc * 16) = al.template finish<DT>(ra[j], m, s * BKE + kc * EPC, a_stats, bm);
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      *reinterpret_cast<uint4*>(tB + r * ROWB + kc * 16) = rb[j];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  commit(0, tileA0, tileB0);
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int s = 0; s < nsteps; ++s) {
    const bool cur1 = (s & 1);
    char* tA = cur1 ? tileA1 : tileA0;
    char* tB = cur1 ? tileB1 : tileB0;
    if (s + 1 < nsteps) issue(s + 1);
#pragma unroll
    for (int kk = 0; kk < KCH / 4; ++kk) {
      uint4 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[i] = *reinterpret_cast<const uint4*>(tA + (wr * WTM + i * 16 + fr) * ROWB + (kk * 4 + fq) * 16);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j] = *reinterpret_cast<const uint4*>(tB + (wc * WTN + j * 16 + fr) * ROWB + (kk * 4 + fq) * 16);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (DTraits<DT>::kCode == 1) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&a[i]),
                                                                *reinterpret_cast<bf16x8*>(&b[j]), acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].x), __uint_as_float(b[j].x), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].y), __uint_as_float(b[j].y), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].z), __uint_as_float(b[j].z), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].w), __uint_as_float(b[j].w), acc[i][j], 0, 0, 0);
          }
        }
    }
    if (s + 1 < nsteps) commit(s + 1, cur1 ? tileA0 : tileA1, cur1 ? tileB0 : tileB1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  float val[FM][FN][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = bm + wr * WTM + i * 16 + fq * 4 + r;
        int n = bn + wc * WTN + j * 16 + fr;
        int mc = m < M ? m : M - 1;
        val[i][j][r] = ep.value(mc, n, acc[i][j][r], e_stats, bm);
      }

  if constexpr (EP::kRowStats) {
    float* red = reinterpret_cast<float*>(smem);  // tiles are dead after the final barrier
    float mean[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) s += val[i][j][r];
        s = wave_sum16(s);
        if (fr == 0) red[(wr * WTM + i * 16 + fq * 4 + r) * 2 + wc] = s;
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int rl = wr * WTM + i * 16 + fq * 4 + r;
        mean[i][r] = (red[rl * 2] + red[rl * 2 + 1]) * (1.0f / BN);
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float d = val[i][j][r] - mean[i][r];
          s += d * d;
        }
        s = wave_sum16(s);
        if (fr == 0) red[(wr * WTM + i * 16 + fq * 4 + r) * 2 + wc] = s;
      }
    __syncthreads();
    if (wc == 0 && fr == 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int rl = wr * WTM + i * 16 + fq * 4 + r;
          int m = bm + rl;
          if (m < M) ep.store_stats(m, blockIdx.x, mean[i][r], red[rl * 2] + red[rl * 2 + 1]);
        }
    }
  }

#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = bm + wr * WTM + i * 16 + fq * 4 + r;
        int n = bn + wc * WTN + j * 16 + fr;
        if (m < M) ep.store(m, n, val[i][j][r]);
      }
}

// ------------------------------ generic loaders ------------------------------

// A = DT matrix, row stride ld (elements).
template <typename DT>
struct LoadPlain {
  const DT* __restrict__ p;
  int ld;
  struct Raw { uint4 v; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const { return Raw{*reinterpret_cast<const uint4*>(p + (size_t)m * ld + k)}; }
  template <typename D> __device__ uint4 finish(const Raw& r, int, int, const float*, int) const { return r.v; }
};

// A = fp32 matrix converted to DT on the fly.
template <typename DT>
struct LoadF32 {
  const float* __restrict__ p;
  int ld;
  struct Raw { float v[DTraits<DT>::EPC]; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    Raw r;
    const float* q = p + (size_t)m * ld + k;
#pragma unroll
    for (int j = 0; j < DTraits<DT>::EPC; j += 4) {
      float4 t = ld4(q + j);
      r.v[j] = t.x; r.v[j + 1] = t.y; r.v[j + 2] = t.z; r.v[j + 3] = t.w;
    }
    return r;
  }
  template <typename D> __device__ uint4 finish(const Raw& r, int, int, const float*, int) const { return pack_chunk<D>(r.v); }
};

// ------------------------------ generic epilogues ------------------------------

template <typename OT, int ACT>  // ACT: 0 none, 1 GELU(erf), 2 SiLU, 3 ReLU
struct EpiBiasAct {
  const float* __restrict__ bias;
  OT* __restrict__ out;
  int ldo;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int, int n, float acc, const float*, int) const {
    float v = acc + (bias ? bias[n] : 0.f);
    if constexpr (ACT == 1) v = gelu_erf(v);
    if constexpr (ACT == 2) v = silu(v);
    if constexpr (ACT == 3) v = fmaxf(v, 0.f);
    return v;
  }
  __device__ void store(int m, int n, float v) const { store_val<OT>(out + (size_t)m * ldo + n, v); }
  __device__ void store_stats(int, int, float, float) const {}
};

// fp32 output (+ optional ReLU) + per-(row, N-tile) LayerNorm partials (mean, M2) for the
// consumer's LayerNorm.
template <bool RELU = false>
struct EpiBiasStatsT {
  const float* __restrict__ bias;
  float* __restrict__ out;
  int ldo;
  float* __restrict__ S;
  int NT;
  static constexpr bool kRowStats = true;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int, int n, float acc, const float*, int) const {
    float v = acc + bias[n];
    return RELU ? fmaxf(v, 0.f) : v;
  }
  __device__ void store(int m, int n, float v) const { out[(size_t)m * ldo + n] = v; }
  __device__ void store_stats(int m, int nt, float mean, float m2) const {
    reinterpret_cast<float2*>(S)[(size_t)m * NT + nt] = make_float2(mean, m2);
  }
};
using EpiBiasStats = EpiBiasStatsT<false>;

// Conv1d (kernel KT, pad KT/2, zero padding at each sequence edge) as a GEMM over K = tap*Cin + c,
// source rows optionally LayerNorm'ed (affine) from producer partials.  Row m = b*L + l.
template <typename DT, bool LN>
struct LoadConvRows {
  const float* __restrict__ x;
  int Cin;
  int L;
  int KT;
  int dil;
  const float* __restrict__ S;  // LN partials of x rows (LN only)
  int NT, tw;
  float eps;
  const float* __restrict__ g;
  const float* __restrict__ bb;
  static constexpr int EPC = DTraits<DT>::EPC;
  struct Raw { float v[EPC], w[LN ? EPC : 1], b[LN ? EPC : 1]; int src; };
  static constexpr int stat_rows(int BM) { return LN ? BM + 8 : 0; }
  __device__ void prologue(int bm, int BM, int M, float* st) const {
    if constexpr (LN) {
      const int h = KT / 2;
      for (int r = threadIdx.x; r < BM + 2 * h; r += blockDim.x) {
        int m = bm - h + r;
        m = m < 0 ? 0 : (m < M ? m : M - 1);
        row_stats_from_partials(S, m, NT, tw, eps, st[2 * r], st[2 * r + 1]);
      }
    }
  }
  __device__ Raw issue(int m, int k) const {
    Raw r;
    int tap = k / Cin, c = k - tap * Cin;
    int off = (tap - KT / 2) * dil;
    int l = m % L + off;
    r.src = (l >= 0 && l < L) ? m + off : -1;
    if (r.src >= 0) {
      const float* px = x + (size_t)r.src * Cin + c;
#pragma unroll
      for (int j = 0; j < EPC; j += 4) {
        float4 a = ld4(px + j);
        r.v[j] = a.x; r.v[j + 1] = a.y; r.v[j + 2] = a.z; r.v[j + 3] = a.w;
        if constexpr (LN) {
          float4 w = ld4(g + c + j), b = ld4(bb + c + j);
          r.w[j] = w.x; r.w[j + 1] = w.y; r.w[j + 2] = w.z; r.w[j + 3] = w.w;
          r.b[j] = b.x; r.b[j + 1] = b.y; r.b[j + 2] = b.z; r.b[j + 3] = b.w;
        }
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
    } else if constexpr (LN) {
      int i = r.src - (bm - KT / 2);
      const float mean = st[2 * i], rstd = st[2 * i + 1];
#pragma unroll
      for (int j = 0; j < EPC; ++j) o[j] = ((r.v[j] - mean) * rstd) * r.w[j] + r.b[j];
    } else {
#pragma unroll
      for (int j = 0; j < EPC; ++j) o[j] = r.v[j];
    }
    return pack_chunk<D>(o);
  }
};

// Dilated conv gather over a DT activation (no transform): K index = tap*Cin + c.
template <typename DT>
struct LoadConvPlain {
  const DT* __restrict__ x;
  int Cin;
  int L;
  int KT;
  int dil;
  struct Raw { uint4 v; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    int tap = k / Cin, c = k - tap * Cin;
    int off = (tap - KT / 2) * dil;
    int l = m % L + off;
    if (l < 0 || l >= L) return Raw{make_uint4(0u, 0u, 0u, 0u)};
    return Raw{*reinterpret_cast<const uint4*>(x + (size_t)(m + off) * Cin + c)};
  }
  template <typename D> __device__ uint4 finish(const Raw& r, int, int, const float*, int) const { return r.v; }
};

// Host-side launcher.
template <int BM, int BN, int KCH, typename DT, class AL, class EP>
inline int launch_gemm(const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  constexpr int BKE = KCH * DTraits<DT>::EPC;
  FL_REQUIRE(M > 0 && N % BN == 0 && K % BKE == 0, "gemm: unsupported shape M=%d N=%d K=%d (BN=%d BK=%d)", M, N, K, BN, BKE);
  using SM = GemmSmem<BM, BN, KCH, AL, EP>;
  dim3 grid(N / BN, (M + BM - 1) / BM);
  auto kern = gemm_kernel<BM, BN, KCH, DT, AL, EP>;
  if (SM::bytes > 64 * 1024) {
    static bool attr_set = false;
    if (!attr_set) {
      FL_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, SM::bytes));
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, grid, dim3(kGemmThreads), SM::bytes, st, al, W, ldw, ep, M, N, K);
  FL_LAUNCH_CHECK();
  return kOk;
}

}  // namespace fl
