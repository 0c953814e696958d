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
#include <type_traits>

#include "common.hpp"

namespace fl {

constexpr int kGemmThreads = 256;

// Optional per-column vector caches in LDS: a loader with kVec > 0 stages kVec floats per K column
// (e.g. two modulation rows x (alpha, beta)) in its prologue; an epilogue with kEVec > 0 stages
// kEVec floats per output column of its tile.  Detected by these traits (0 when absent).
template <class T, class = void> struct kvec_of { static constexpr int value = 0; };
template <class T> struct kvec_of<T, std::void_t<decltype(T::kVec)>> { static constexpr int value = T::kVec; };
// Per-column epilogue vectors are stored field-major with this column stride (>= every N tile that
// stages them), so the lanes of a row read consecutive floats (conflict-free, vectorisable).
constexpr int kEVecStride = 128;
template <class T, class = void> struct kevec_of { static constexpr int value = 0; };
template <class T> struct kevec_of<T, std::void_t<decltype(T::kEVec)>> { static constexpr int value = T::kEVec; };
// Epilogues with kPre read one global value per output element (e.g. the residual X); the kernel
// fetches it through ep.pre(m, n) before the main loop (small tiles) so its latency is hidden, and
// passes it to value_v as the last argument.
template <class T, class = void> struct kpre_of { static constexpr bool value = false; };
template <class T> struct kpre_of<T, std::void_t<decltype(T::kPre)>> { static constexpr bool value = T::kPre; };

// Epilogues with a side output that needs the staged per-column vectors (store_v / store4_v) get them
// at the store; the others take plain store / store4.
template <class T, class = void> struct kstorev_of { static constexpr bool value = false; };
template <class T> struct kstorev_of<T, std::void_t<decltype(T::kStoreV)>> { static constexpr bool value = T::kStoreV; };
template <class EP>
__device__ __forceinline__ void ep_store(const EP& ep, int m, int n, float v, const float* vec, bool use, int bm, int bn) {
  if constexpr (kstorev_of<EP>::value) ep.store_v(m, n, v, vec, use, bm, bn);
  else ep.store(m, n, v);
}

template <int BM, int BN, int KCH, int NSTAGE, class AL, class EP>
struct GemmSmem {
  static constexpr int ROWB = KCH * 16;  // unpadded; 16-B chunks XOR-swizzled by row
  static constexpr int tiles = NSTAGE * (BM + BN) * ROWB;
  static constexpr int a_stats = AL::stat_rows(BM) * 2 * 4;
  static constexpr int e_stats = EP::stat_rows(BM) * 2 * 4;
  static constexpr int e_vec = kevec_of<EP>::value * kEVecStride * 4;
  static_assert(kevec_of<EP>::value == 0 || BN <= kEVecStride, "per-column vectors: BN <= kEVecStride");
  static constexpr int red = BM * 2 * 4;
  static constexpr int base = (tiles > red ? tiles : red) + 16;  // + 16 B: split-K "last arriver" flag
  static constexpr int flag = base - 16;
  static constexpr int bytes = (base + a_stats + e_stats + e_vec + 15) / 16 * 16;  // + kVec*K*4 (runtime)
};

// Split-K over gridDim.z (small-M GEMMs, where one block's K chain is the latency).  Every slice
// stores its fp32 partial tile as a slab in MFMA-fragment order, then takes a ticket on the tile's
// counter (agent-scope release before, acquire after — cdna_hip_programming.md §5 "Projection GEMM
// at M = 256" item 2); the last arriver sums all `n` slabs in slice order (deterministic), resets the
// counter and runs the fused epilogue.  n == 1: no split.
constexpr int kMaxSplit = 4;
struct SplitK {
  int n;  // 1..kMaxSplit
  float* slab;  // tiles x n x BM x BN floats
  int* cnt;     // tiles counters, zero between launches
  int strips = 0;  // > 0: XCD-aware placement in column strips of this many tiles (xcd_tile)
};

// XCD-aware tile placement for small grids: dispatch round-robins workgroup ids over the 8 XCDs (each
// with a private L2), so by default column tile x always lands on XCD x mod 8 and every A row panel
// is fetched by all 8 L2s.  Here the id is first made consecutive per XCD (bijective, guide §5 T1),
// then walked through column strips of `sw` tiles in row-major order inside each strip: an XCD gets a
// compact block of about (gy / (8 * sw / gx)) rows x sw columns, so A panels are shared by gx / sw
// XCDs and W panels by 8 * sw / gx.  Requires gx % sw == 0.
__device__ __forceinline__ void xcd_tile(int sw, int& tx, int& ty) {
  const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy, id = blockIdx.y * gx + blockIdx.x;
  const int xcd = id & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (id >> 3);
  const int per_strip = gy * sw;
  const int strip = wg / per_strip, w = wg - strip * per_strip;
  ty = w / sw;
  tx = strip * sw + (w - ty * sw);
}

// LayerNorm row statistics from producer partials: S[m][NT] = (tile mean, tile M2) over `tw` columns,
// NT <= 32.  All partials are loaded before reducing (independent loads in flight together).
template <int MAXNT>
__device__ __forceinline__ void row_stats_n(const float2* __restrict__ p, int NT, int tw, float eps, float& mean, float& rstd) {
  float2 q[MAXNT];
#pragma unroll
  for (int i = 0; i < MAXNT; ++i) q[i] = i < NT ? p[i] : make_float2(0.f, 0.f);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXNT; ++i) s += q[i].x;
  mean = s / (float)NT;
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXNT; ++i) {
    if (i < NT) {
      float d = q[i].x - mean;
      m2 += q[i].y + (float)tw * d * d;
    }
  }
  float var = m2 / (float)(NT * tw);
  rstd = 1.0f / sqrtf(var + eps);
}
// The 32-partial form (BN = 32 tiles) stays out of line: inlined next to the 16-partial form it cost
// ~6 us per consuming GEMM at B = 1 even when never executed (register allocation of the prologue).
__device__ __noinline__ void row_stats_32(const float2* __restrict__ p, int NT, int tw, float eps, float& mean, float& rstd) {
  row_stats_n<32>(p, NT, tw, eps, mean, rstd);
}
__device__ __forceinline__ void row_stats_from_partials(const float* __restrict__ S, int m, int NT, int tw,
                                                        float eps, float& mean, float& rstd) {
  const float2* p = reinterpret_cast<const float2*>(S) + (size_t)m * NT;
  if (NT <= 16) row_stats_n<16>(p, NT, tw, eps, mean, rstd);
  else row_stats_32(p, NT, tw, eps, mean, rstd);
}

// Byte offset of 16-B chunk `c` of LDS tile row `r` (128-B rows, two per 256-B bank line).  A 16-lane
// ds_read_b128 group reads rows r0..r0+15 at one chunk; its 16-B slot is (r & 1) * 8 + (c ^ ((r >> 1) & 7)),
// distinct for all 16 rows -> conflict-free.  (XOR with r & 7 put rows r and r + 8 in the same slot: a
// 2-way conflict on every fragment read, SQ_LDS_BANK_CONFLICT.)  The commit writes (two rows x 8 chunks
// per 16 lanes) stay conflict-free.
template <int KCH>
__device__ __forceinline__ int lds_off(int r, int c) {
  static_assert(KCH == 8, "128-B rows");
  return r * (KCH * 16) + ((c ^ ((r >> 1) & 7)) << 4);
}

// NSTAGE = 2: LDS double buffer, loads issued one K-step ahead.
// NSTAGE = 3: LDS ring of 3, two register stages, loads issued two K-steps ahead (small-M latency).
template <int BM, int BN, int KCH, int NSTAGE, typename DT, class AL, class EP>
__global__ __launch_bounds__(kGemmThreads) void gemm_kernel(AL al, const DT* __restrict__ W, int ldw, EP ep,
                                                             int M, int N, int K, SplitK sk) {
  using SM = GemmSmem<BM, BN, KCH, NSTAGE, AL, EP>;
  constexpr int EPC = DTraits<DT>::EPC;
  constexpr int BKE = KCH * EPC;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int ACH = BM * KCH / kGemmThreads;
  constexpr int BCH = BN * KCH / kGemmThreads;
  constexpr int TILE = (BM + BN) * SM::ROWB;
  static_assert(ACH >= 1 && BCH >= 1, "tile too small for 256 threads");
  static_assert(KCH == 8, "K-step is 128 B per row");
  static_assert(NSTAGE >= 2 && NSTAGE <= 7 && (NSTAGE <= 3 || (NSTAGE - 1) % 2 == 0), "2, 3, 5 or 7 stages");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* a_stats = reinterpret_cast<float*>(smem + SM::base);
  int* s_flag = reinterpret_cast<int*>(smem + SM::flag);
  float* e_stats = a_stats + AL::stat_rows(BM) * 2;
  float* e_vec = e_stats + EP::stat_rows(BM) * 2;
  float* a_vec = e_vec + kevec_of<EP>::value * kEVecStride;
  constexpr bool AV = kvec_of<AL>::value > 0;
  constexpr bool EV = kevec_of<EP>::value > 0;

  FL_STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  int tx = blockIdx.x, ty = blockIdx.y;
  if (sk.strips > 0) xcd_tile(sk.strips, tx, ty);
  const int bn = tx * BN;
  const int bm = ty * BM;

  bool a_uv = false, e_uv = false;  // set by the prologue (per-column vectors staged in LDS)
  typename AL::Raw ra0[ACH], ra1[ACH];
  u32x4 rb0[BCH], rb1[BCH];
  const int kslice = K / sk.n;
  const int k0 = blockIdx.z * kslice;
  const int nsteps = kslice / BKE;

  auto issue = [&](int s, typename AL::Raw (&ra)[ACH], u32x4 (&rb)[BCH]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      int m = bm + r;
      m = m < M ? m : M - 1;
      if constexpr (AV) ra[j] = al.issue_v(m, k0 + s * BKE + kc * EPC);
      else ra[j] = al.issue(m, k0 + s * BKE + kc * EPC);
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      rb[j] = *reinterpret_cast<const u32x4*>(W + (size_t)(bn + r) * ldw + k0 + s * BKE + kc * EPC);
    }
  };
  auto commit = [&](int s, const typename AL::Raw (&ra)[ACH], const u32x4 (&rb)[BCH], char* t) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      int m = bm + r;
      m = m < M ? m : M - 1;
      if constexpr (AV)
        *reinterpret_cast<u32x4*>(t + lds_off<KCH>(r, kc)) = al.template finish_v<DT>(ra[j], m, k0 + s * BKE + kc * EPC, a_stats, a_vec, a_uv, bm);
      else
        *reinterpret_cast<u32x4*>(t + lds_off<KCH>(r, kc)) = al.template finish<DT>(ra[j], m, k0 + s * BKE + kc * EPC, a_stats, bm);
    }
    char* tb = t + BM * SM::ROWB;
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      int c = tid + j * kGemmThreads;
      int r = c / KCH, kc = c % KCH;
      *reinterpret_cast<u32x4*>(tb + lds_off<KCH>(r, kc)) = rb[j];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](const char* t) __attribute__((always_inline)) {
    const char* tb = t + BM * SM::ROWB;
#pragma unroll
    for (int kk = 0; kk < KCH / 4; ++kk) {
      u32x4 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const u32x4*>(t + lds_off<KCH>(wr * WTM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const u32x4*>(tb + lds_off<KCH>(wc * WTN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (DTraits<DT>::kCode == 1) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[i]),
                                                                __builtin_bit_cast(bf16x8, b[j]), acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].x), __uint_as_float(b[j].x), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].y), __uint_as_float(b[j].y), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].z), __uint_as_float(b[j].z), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].w), __uint_as_float(b[j].w), acc[i][j], 0, 0, 0);
          }
        }
    }
  };

  // The first K-steps' operand loads go out before the fused prologue (LN statistics, per-column
  // vectors, epilogue prefetch), whose own loads then overlap them.
  constexpr bool PRE = kpre_of<EP>::value;
  constexpr bool PRE_EARLY = PRE && FM * FN <= 4;
  float pre[FM][FN][4];
  auto fetch_pre = [&]() __attribute__((always_inline)) {
    if constexpr (PRE) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            int m = bm + wr * WTM + i * 16 + fq * 4 + r;
            pre[i][j][r] = ep.pre(m < M ? m : M - 1, bn + wc * WTN + j * 16 + fr);
          }
    }
  };
  auto prologue = [&]() __attribute__((always_inline)) {
    if constexpr (PRE_EARLY) fetch_pre();
    if constexpr (AV) a_uv = al.prologue_v(bm, BM, M, K, a_stats, a_vec);
    else al.prologue(bm, BM, M, a_stats);
    if constexpr (EV) e_uv = ep.prologue_v(bm, bn, BM, BN, M, e_stats, e_vec);
    else ep.prologue(bm, BM, M, e_stats);
    __syncthreads();
    FL_STAMP(1);
  };

  if constexpr (NSTAGE == 2) {
    issue(0, ra0, rb0);
    prologue();
    commit(0, ra0, rb0, smem);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      char* cur = smem + (s & 1) * TILE;
      char* nxt = smem + ((s + 1) & 1) * TILE;
      issue(s + 1 < nsteps ? s + 1 : s, ra0, rb0);  // unconditional (clamped) keeps the staging in VGPRs
      compute(cur);
      if (s + 1 < nsteps) commit(s + 1, ra0, rb0, nxt);
      __syncthreads();
    }
  } else if constexpr (NSTAGE >= 4) {
    // Deep register prefetch for latency-bound (small-M) GEMMs whose weights stream from MALL/HBM:
    // R = NSTAGE-1 register sets keep R K-steps of loads in flight; LDS is double-buffered.
    // At step s: compute LDS[s&1]; commit step s+1 (register set (s+1)%R) into LDS[(s+1)&1]; reissue
    // that set with step s+1+R (clamped, so the loads stay unconditional); barrier.
    constexpr int R = NSTAGE - 1;
    typename AL::Raw ra[R][ACH];
    u32x4 rb[R][BCH];
    const int last = nsteps - 1;
#pragma unroll
    for (int u = 0; u < R; ++u) issue(u < last ? u : last, ra[u], rb[u]);
    prologue();
    commit(0, ra[0], rb[0], smem);
    issue(R < last ? R : last, ra[0], rb[0]);
    __syncthreads();
    for (int s0 = 0; s0 < nsteps; s0 += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int s = s0 + u;
        if (s < nsteps) {
          compute(smem + (u & 1) * TILE);
          if (s + 1 < nsteps) {
            commit(s + 1, ra[(u + 1) % R], rb[(u + 1) % R], smem + ((u + 1) & 1) * TILE);
            const int nx = s + 1 + R;
            issue(nx < last ? nx : last, ra[(u + 1) % R], rb[(u + 1) % R]);
          }
          __syncthreads();
        }
      }
    }
  } else {
    // invariant at iteration s: LDS holds steps s, s+1; register set (s&1) holds loads of step s+2
    const int last = nsteps - 1;
    issue(0, ra0, rb0);
    issue(last < 1 ? last : 1, ra1, rb1);
    prologue();
    commit(0, ra0, rb0, smem);
    if (nsteps > 1) commit(1, ra1, rb1, smem + TILE);
    issue(last < 2 ? last : 2, ra0, rb0);
    __syncthreads();
    int b0 = 0;  // LDS slot of step s
    for (int s = 0; s < nsteps; s += 2) {
      {  // even step: issue s+3 into set 1, commit set 0 (step s+2)
        int b2 = b0 + 2 >= 3 ? b0 - 1 : b0 + 2;
        issue(s + 3 < nsteps ? s + 3 : last, ra1, rb1);
        compute(smem + b0 * TILE);
        if (s + 2 < nsteps) commit(s + 2, ra0, rb0, smem + b2 * TILE);
        __syncthreads();
        b0 = b0 == 2 ? 0 : b0 + 1;
      }
      if (s + 1 < nsteps) {  // odd step: issue s+4 into set 0, commit set 1 (step s+3)
        int b2 = b0 + 2 >= 3 ? b0 - 1 : b0 + 2;
        issue(s + 4 < nsteps ? s + 4 : last, ra0, rb0);
        compute(smem + b0 * TILE);
        if (s + 3 < nsteps) commit(s + 3, ra1, rb1, smem + b2 * TILE);
        __syncthreads();
        b0 = b0 == 2 ? 0 : b0 + 1;
      }
    }
  }

  FL_STAMP(2);
  // ---------------- split-K: slab hand-off, the last arriver reduces ----------------
  // Write-through form (cdna_hip_programming.md §6 Guideline 16, R1 + sc1 consume): every slab store
  // is a 16-B sc1 buffer store, every storing wave drains (vmcnt 0) before the block barrier, one lane
  // takes a relaxed agent-scope ticket; the last arriver reads ALL slabs with sc1 loads.  No release
  // fence (buffer_wbl2 writes back the XCD L2's dirty lines: ~6 us after a kernel that dirtied it) and
  // no acquire (sc1 loads bypass this CU's L1).
  if (sk.n > 1) {
    const int tile = ty * gridDim.x + tx;
    float* slabs = sk.slab + (size_t)tile * sk.n * (BM * BN);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slabs, 0, sk.n * BM * BN * 4, 0x00020000);
    const int mine = blockIdx.z * (BM * BN * 4);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                               mine + ((i * FN + j) * kGemmThreads + tid) * 16, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(sk.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == sk.n - 1;
      if (last) __hip_atomic_store(sk.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      *s_flag = last;
    }
    __syncthreads();
    if (!*s_flag) return;  // block-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: keeps the sc1 loads below the ticket
    // load all kMaxSplit slab slots unconditionally (no per-element register/load select, guide §5
    // item 4(c)): slots >= n lie past the descriptor's range and read as zero; sum in slice order
    u32x4 q[FM][FN][kMaxSplit];
#pragma unroll
    for (int z = 0; z < kMaxSplit; ++z)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          q[i][j][z] = __builtin_amdgcn_raw_buffer_load_b128(rs, z * (BM * BN * 4) + ((i * FN + j) * kGemmThreads + tid) * 16, 0, 16);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        f32x4 sum = __builtin_bit_cast(f32x4, q[i][j][0]);
#pragma unroll
        for (int z = 1; z < kMaxSplit; ++z) sum += __builtin_bit_cast(f32x4, q[i][j][z]);
        acc[i][j] = sum;
      }
  }

  // ---------------- epilogue (values overwrite the accumulators in place) ----------------
  if constexpr (PRE && !PRE_EARLY) fetch_pre();
  auto& val = acc;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = bm + wr * WTM + i * 16 + fq * 4 + r;
        int n = bn + wc * WTN + j * 16 + fr;
        int mc = m < M ? m : M - 1;
        if constexpr (PRE) val[i][j][r] = ep.value_v(mc, n, acc[i][j][r], e_stats, e_vec, e_uv, bm, bn, pre[i][j][r]);
        else if constexpr (EV) val[i][j][r] = ep.value_v(mc, n, acc[i][j][r], e_stats, e_vec, e_uv, bm, bn);
        else val[i][j][r] = ep.value(mc, n, acc[i][j][r], e_stats, bm);
      }

  FL_STAMP(3);
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
          if (m < M) ep.store_stats(m, tx, mean[i][r], red[rl * 2] + red[rl * 2 + 1]);
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
        if (m < M) ep_store(ep, m, n, val[i][j][r], e_vec, e_uv, bm, bn);
      }
  FL_STAMP(4);
}

// ------------------------------ generic loaders ------------------------------

// A = DT matrix, row stride ld (elements).
template <typename DT>
struct LoadPlain {
  const DT* __restrict__ p;
  int ld;
  struct Raw { u32x4 v; };
  static constexpr int kSrcBytes = sizeof(DT);  // DMA path: raw source rows, no transform when == 2
  __device__ const char* src_row(int m) const { return reinterpret_cast<const char*>(p + (size_t)m * ld); }
  struct XRow {};  // unused: bf16 rows are consumed in place
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const { return Raw{*reinterpret_cast<const u32x4*>(p + (size_t)m * ld + k)}; }
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return r.v; }
};

// A = fp32 matrix converted to DT on the fly.
template <typename DT>
struct LoadF32 {
  const float* __restrict__ p;
  int ld;
  struct Raw { float v[DTraits<DT>::EPC]; };
  static constexpr int kSrcBytes = 4;
  __device__ const char* src_row(int m) const { return reinterpret_cast<const char*>(p + (size_t)m * ld); }
  // DMA-path transform (gemm_dma.hpp): per-thread row context hoisted out of the K loop
  struct XRow {};
  __device__ XRow xrow(int, const float*, const float*, bool, int) const { return {}; }
  template <typename D> __device__ u32x4 xform(const XRow&, const Raw& r, int, const float*, const float*, int) const { return pack_chunk<D>(r.v); }
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
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return pack_chunk<D>(r.v); }
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
    if constexpr (ACT == 1) {
      if constexpr (std::is_same<OT, bf16>::value) v = gelu_fast(v);  // bf16 output: 4.7e-7 erf error is invisible
      else v = gelu_erf(v);                                            // fp32 parity mode: ocml erff
    }
    if constexpr (ACT == 2) v = silu(v);
    if constexpr (ACT == 3) v = fmaxf(v, 0.f);
    return v;
  }
  __device__ void store(int m, int n, float v) const { store_val<OT>(out + (size_t)m * ldo + n, v); }
  __device__ void store4(int m, int n, const float* v) const { store_val4<OT>(out + (size_t)m * ldo + n, v); }
  __device__ void store_stats(int, int, float, float) const {}
};

// fp32 (or bf16: the large-M bf16 residual stream) output (+ optional ReLU) + per-(row, N-tile)
// LayerNorm partials (mean, M2, of the fp32 values) for the consumer's LayerNorm.
template <bool RELU = false, typename OT = float>
struct EpiBiasStatsT {
  const float* __restrict__ bias;
  OT* __restrict__ out;
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
  __device__ void store(int m, int n, float v) const { store_val<OT>(out + (size_t)m * ldo + n, v); }
  __device__ void store4(int m, int n, const float* v) const { store_val4<OT>(out + (size_t)m * ldo + n, v); }
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
  __device__ u32x4 finish(const Raw& r, int, int, const float* st, int bm) const {
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
  struct Raw { u32x4 v; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    int tap = k / Cin, c = k - tap * Cin;
    int off = (tap - KT / 2) * dil;
    int l = m % L + off;
    if (l < 0 || l >= L) return Raw{u32x4{0u, 0u, 0u, 0u}};
    return Raw{*reinterpret_cast<const u32x4*>(x + (size_t)(m + off) * Cin + c)};
  }
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return r.v; }
};

// Host-side launcher.  Tile configurations (BM, BN, NSTAGE) are selected by the callers:
//   small M  : 32 x 64, 3-stage ring (latency-bound at ~400 rows: more workgroups, deeper prefetch)
//   mid M    : 64 x 64, 3-stage
//   large M  : 128 x 64, 3-stage (measured with flamed_probe_gemm at M = 25600, N = 1024: 461 TF at
//              K = 1024 vs 358 TF for 128 x 128, whose 4x4 fragments per wave double the VGPRs)
// Split-K context: a caller that owns slab memory and zeroed counters installs it (SplitScope) around
// its launches; launch_gemm_cfg then splits bf16 GEMMs whose tile grid is small.
struct SplitCtx {
  float* slab = nullptr;
  size_t slab_floats = 0;
  int* cnt = nullptr;
  int cnt_n = 0;
  int target = 1;  // aim for about this many workgroups (tiles x splits); 1 = no split
  int max_split = 4;
  bool f32 = false;  // also split exact-fp32 GEMMs (PVA nets: a fixed slice order is still deterministic)
};
extern thread_local SplitCtx* g_split;
// Pipeline depth of the small-M (32 x 64) config: tn().small_stages 3 = LDS ring of 3 / 2 K-steps in
// flight, 5 / 7 = 4 / 6 K-steps of register prefetch; XCD strip width of small/mid-M tile placement:
// tn().xcd_strips (SplitK::strips, 0 = off).

struct SplitScope {
  SplitCtx* prev;
  explicit SplitScope(SplitCtx* c) : prev(g_split) { g_split = c; }
  ~SplitScope() { g_split = prev; }
};

template <int BM, int BN, typename DT>
inline SplitK choose_split(int M, int N, int K) {
  constexpr int BKE = 8 * DTraits<DT>::EPC;
  SplitK sk{1, nullptr, nullptr, 0};
  {
    const int gx = N / BN;
    const int xs = tn().xcd_strips;
    if (xs > 0 && gx % xs == 0 && M < 8192) sk.strips = xs;
  }
  SplitCtx* c = g_split;
  if (!c || (DTraits<DT>::kCode != 1 && !c->f32)) return sk;  // the denoiser's fp32 parity mode keeps one FMA chain
  const int tiles = (N / BN) * ((M + BM - 1) / BM);
  int n = 1;
  while (n * 2 <= c->max_split && tiles * n * 2 <= c->target && (K / BKE) % (n * 2) == 0 && K / (n * 2) >= 2 * BKE) n *= 2;
  if (n == 1 || tiles > c->cnt_n || (size_t)tiles * n * BM * BN > c->slab_floats) return sk;
  return SplitK{n, c->slab, c->cnt, sk.strips};
}

template <int BM, int BN, int NSTAGE, typename DT, class AL, class EP>
inline int launch_gemm_cfg(const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  constexpr int KCH = 8;
  constexpr int BKE = KCH * DTraits<DT>::EPC;
  FL_REQUIRE(M > 0 && N % BN == 0 && K % BKE == 0, "gemm: unsupported shape M=%d N=%d K=%d (BN=%d BK=%d)", M, N, K, BN, BKE);
  using SM = GemmSmem<BM, BN, KCH, NSTAGE, AL, EP>;
  const SplitK sk = choose_split<BM, BN, DT>(M, N, K);
  dim3 grid(N / BN, (M + BM - 1) / BM, sk.n);
  auto kern = gemm_kernel<BM, BN, KCH, NSTAGE, DT, AL, EP>;
  const size_t bytes = SM::bytes + (size_t)kvec_of<AL>::value * K * 4;
  FL_REQUIRE(bytes <= 160 * 1024, "gemm: LDS request %zu B too large (K=%d)", bytes, K);
  if (bytes > 64 * 1024) FL_HIP(set_max_lds(reinterpret_cast<const void*>(kern)));
  hipLaunchKernelGGL(kern, grid, dim3(kGemmThreads), bytes, st, al, W, ldw, ep, M, N, K, sk);
  FL_LAUNCH_CHECK();
  return kOk;
}

// Tile selection by shape.  `BNf` fixes the N tile when the epilogue's row partials need a known
// width (0 = free choice).
enum GemmCfg { kCfgSmall = 0, kCfgMid = 1, kCfgLarge = 2, kCfgTiny = 3 /* denoiser only: 32 x 32 tiles */ };
inline GemmCfg pick_cfg(int M) { return M < 2048 ? kCfgSmall : (M < 8192 ? kCfgMid : kCfgLarge); }
// Tiny-M tiles are 32 columns wide: half the weight panel per workgroup, twice the workgroups.
inline int cfg_bn(GemmCfg c) { return c == kCfgTiny ? 32 : 64; }

template <typename DT, class AL, class EP>
inline int launch_gemm_auto(GemmCfg c, const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  if (c == kCfgSmall) {
    if (tn().small_stages == 5) return launch_gemm_cfg<32, 64, 5, DT>(al, W, ldw, ep, M, N, K, st);
    if (tn().small_stages == 7) return launch_gemm_cfg<32, 64, 7, DT>(al, W, ldw, ep, M, N, K, st);
    return launch_gemm_cfg<32, 64, 3, DT>(al, W, ldw, ep, M, N, K, st);
  }
  if (c == kCfgMid) return launch_gemm_cfg<64, 64, 3, DT>(al, W, ldw, ep, M, N, K, st);
  return launch_gemm_cfg<128, 64, 3, DT>(al, W, ldw, ep, M, N, K, st);
}

// kWideA: the A loader transforms fp32 rows (LayerNorm / GroupNorm apply); at large M a 128 x 128 tile
// halves how often those rows are re-read (B = 64 measurement: 128 x 64 slowed these GEMMs by ~30 %).
constexpr bool kWideA = true;

template <typename DT, class AL, class EP>
inline int launch_gemm_auto(GemmCfg c, bool wide_a, const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K,
                            hipStream_t st) {
  if (c == kCfgLarge && wide_a && N % 128 == 0 && !EP::kRowStats)
    return launch_gemm_cfg<128, 128, 3, DT>(al, W, ldw, ep, M, N, K, st);
  return launch_gemm_auto<DT>(c, al, W, ldw, ep, M, N, K, st);
}

// Shape-driven convenience: choose the config from M (row partial width = cfg_bn(pick_cfg(M)) when
// N allows 128-wide tiles).
template <typename DT, class AL, class EP>
inline int launch_gemm(const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  return launch_gemm_auto<DT>(pick_cfg(M), al, W, ldw, ep, M, N, K, st);
}

}  // namespace fl
