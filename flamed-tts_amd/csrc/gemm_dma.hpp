// LDS-DMA pipelined bf16 GEMM for the latency-bound small/mid-M regime (denoiser at B*T < 8192 rows).
//
// Why a second main loop: the register-staged ring of gemm_kernel is serialised by hipcc — the
// staging VGPRs of the next K-steps are reused as ds_read destinations and control-flow joins flush
// the wait counters, so the emitted loop waits `s_waitcnt vmcnt(0)` every K-step (read in the .s of
// the 32x64 3-stage instantiation) and only one K-step of operand traffic is ever in flight.  Here
// every global operand byte travels by `global_load_lds_dwordx4` straight into an NS-deep LDS ring
// (no VGPR destinations, so nothing for the compiler to wait on), completion is tracked with an
// explicit counted `s_waitcnt vmcnt(ahead * G)` and raw `s_barrier`s (cdna_hip_programming.md §5
// "Pipelining across barriers"), and NS-1 K-steps stay in flight.
//
// Operand images (128-B bf16 rows, XOR-swizzled exactly as lds_off<8>): glds writes a wave's 64 lanes
// lane-linearly, so the swizzle is applied to each lane's SOURCE chunk (an involution) and the
// fragment reads use lds_off (guide §5.4 rule 21).  An A loader whose source is fp32 (LayerNorm /
// GroupNorm / conversion prologues, kSrcBytes == 4) has its raw 256-B rows staged linearly; one
// LDS->LDS pass per K-step applies the loader's own finish/finish_v transform into a double-buffered
// bf16 image.  The fused prologue (row statistics, per-column vectors) and epilogue policies are the
// gemm_kernel ones, unchanged.
#pragma once
#include "gemm.hpp"

#include <utility>

namespace fl {


// One wave-instruction of LDS-DMA: 64 lanes x 16 B from per-lane `g` to LDS [lds, lds + 1024).  Written
// as inline asm (M0 saved and restored inside the statement, guide §5.7): hipcc does not see the DMA,
// so it neither drains it before every ds_read (it cannot prove the reads do not alias the DMA target
// and emits vmcnt(0) — read in the .s of the builtin form) nor at barriers; completion is ours to count.
__device__ __forceinline__ void glds16(const void* g, char* lds) {
  const unsigned l = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)(lds)));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(l)
               : "memory");
}

// s_waitcnt vmcnt(n * G) for a runtime n in [0, NMAX] (the count is an instruction immediate).
template <int G, int NMAX>
__device__ __forceinline__ void wait_vm(int n) {
  static_assert(NMAX * G <= 63, "vmcnt immediate is 6 bits");
#define FL_WV(i) \
  case i:        \
    if constexpr (i <= NMAX) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(i * G) : "memory"); \
    break;
  switch (n) {
    FL_WV(0) FL_WV(1) FL_WV(2) FL_WV(3) FL_WV(4) FL_WV(5) FL_WV(6) FL_WV(7) FL_WV(8) FL_WV(9)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
#undef FL_WV
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Four consecutive columns of one row through a residual epilogue (kPre): value4_v when the epilogue has one (its
// staged per-column vectors read as float4 -- four scalar reads at a 4-word lane stride are 2-way LDS bank conflicts),
// else value_v per column.  value4_v evaluates each column with value_v's expression, so the results are the same.
template <class T, class = void> struct has_value4 { static constexpr bool value = false; };
template <class T> struct has_value4<T, std::void_t<decltype(&T::value4_v)>> { static constexpr bool value = true; };
template <class EP>
__device__ __forceinline__ void value4_pre(const EP& ep, int m, int n, const float* av, const float* st, const float* vec,
                                           bool use, int bm, int bn, const float* x, float* v) {
  if constexpr (has_value4<EP>::value) {
    ep.value4_v(m, n, av, st, vec, use, bm, bn, x, v);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = ep.value_v(m, n + e, av[e], st, vec, use, bm, bn, x[e]);
  }
}
// ... and through an epilogue with staged per-column vectors but no residual (kEVec, no kPre: the LayerNorm fold)
template <class EP>
__device__ __forceinline__ void value4_ev(const EP& ep, int m, int n, const float* av, const float* st, const float* vec,
                                          bool use, int bm, int bn, float* v) {
  if constexpr (has_value4<EP>::value) {
    ep.value4_v(m, n, av, st, vec, use, bm, bn, nullptr, v);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = ep.value_v(m, n + e, av[e], st, vec, use, bm, bn);
  }
}

// Four consecutive outputs of one row: the epilogue's own store4 when it has one, else four stores.
template <class T, class = void> struct has_store4 { static constexpr bool value = false; };
template <class T>
struct has_store4<T, std::void_t<decltype(std::declval<const T&>().store4(0, 0, (const float*)nullptr))>> {
  static constexpr bool value = true;
};
template <class EP>
__device__ __forceinline__ void store4(const EP& ep, int m, int n, const float* v, const float* vec, bool use, int bm, int bn) {
  if constexpr (kstorev_of<EP>::value) {
    ep.store4_v(m, n, v, vec, use, bm, bn);
  } else if constexpr (has_store4<EP>::value) {
    ep.store4(m, n, v);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) ep.store(m, n + e, v[e]);
  }
}

// Byte offset of 16-B chunk c of row r in a K-step image with CPR chunks per row (CPR = 8: lds_off;
// CPR = 4, 64-B rows: slot (r & 3) * 4 + (c ^ ((r >> 2) & 3)) of the 256-B bank line, distinct for the
// 16 rows a ds_read_b128 lane group reads at one chunk).
template <int CPR>
__device__ __forceinline__ int lds_offk(int r, int c) {
  if constexpr (CPR == 8) return lds_off<8>(r, c);
  else return r * 64 + ((c ^ ((r >> 2) & 3)) << 4);
}
template <int CPR>
__device__ __forceinline__ int lds_swz(int r) { return CPR == 8 ? ((r >> 1) & 7) : ((r >> 2) & 3); }

template <int BM, int BN, int NS, class AL, class EP, int KB = 64>
struct DmaSmem {
  static constexpr int AE = AL::kSrcBytes;                 // 2 (bf16 A, used in place) or 4 (fp32, transformed)
  static constexpr bool XF = AE == 4;
  static_assert(KB == 64 || (KB == 32 && !XF), "K-step: 64, or 32 for bf16 A");
  static constexpr int CPR = KB / 8;                       // 16-B chunks per bf16 row of one K-step
  static constexpr int A_RAW = BM * KB * AE;               // one K-step of A source rows
  static constexpr int W_ST = BN * KB * 2;                 // one K-step of W rows (bf16)
  static constexpr int STAGE = A_RAW + W_ST;
  static constexpr int ABF = XF ? BM * 128 : 0;            // transformed bf16 A image (x2, alternating)
  static constexpr int ring = NS * STAGE;
  static constexpr int red = BM * 2 * 4;
  // big tiles (more than 4 MFMA fragments per wave) run the row-vectorised epilogue through an fp32
  // image of the whole output tile in LDS
  static constexpr bool VEPI = (BM / 32) * (BN / 32) > 4;
  static constexpr int ctile = VEPI ? BM * BN * 4 : 0;
  static constexpr int body0 = ring + 2 * ABF > red ? ring + 2 * ABF : red;
  static constexpr int body = body0 > ctile ? body0 : ctile;
  static constexpr int a_stats = AL::stat_rows(BM) * 2 * 4;
  static constexpr int e_stats = EP::stat_rows(BM) * 2 * 4;
  static constexpr int e_vec = kevec_of<EP>::value * kEVecStride * 4;
  static_assert(kevec_of<EP>::value == 0 || BN <= kEVecStride, "per-column vectors: BN <= kEVecStride");
  static constexpr int bytes = (body + a_stats + e_stats + e_vec + 15) / 16 * 16;  // + kVec*K*4 (runtime)
  // glds instructions per thread per K-step
  static constexpr int GW = BN * CPR / 256;                // W: BN rows x CPR chunks / 64 lanes / 4 waves
  static constexpr int GA = XF ? BM / 16 : BM * CPR / 256; // A: BM rows x (16 | CPR) chunks / 64 / 4
  static constexpr int G = GW + GA;
};

// XCD = true: workgroup ids are remapped so the ~nwg/8 tiles one XCD receives (dispatch round-robins
// ids over the 8 XCDs) are consecutive in row-major tile order — a row panel of A is then fetched by
// one XCD's L2 instead of all eight (large M, where A is the big operand; guide §5 T1, bijective form).
template <int BM, int BN, int NS, class AL, class EP, int XCD = 0, int KB = 64>
__global__ __launch_bounds__(kGemmThreads) void gemm_dma_kernel(AL al, const bf16* __restrict__ W, int ldw, EP ep,
                                                                 int M, int N, int K) {
  using SM = DmaSmem<BM, BN, NS, AL, EP, KB>;
  constexpr int CPR = SM::CPR, RPI = 64 / CPR;  // rows per DMA wave-instruction
  constexpr bool XF = SM::XF;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int BKE = KB;
  static_assert(BM % 32 == 0 && BN % 32 == 0 && NS >= (SM::XF ? 3 : 2) && NS - 2 <= 9, "dma gemm tile");
  static_assert(!XF || BM * 8 % kGemmThreads == 0, "transform pass: whole chunks per thread");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* a_stats = reinterpret_cast<float*>(smem + SM::body);
  float* e_stats = a_stats + AL::stat_rows(BM) * 2;
  float* e_vec = e_stats + EP::stat_rows(BM) * 2;
  float* a_vec = e_vec + kevec_of<EP>::value * kEVecStride;
  constexpr bool AV = kvec_of<AL>::value > 0;
  constexpr bool EV = kevec_of<EP>::value > 0;

  FL_STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tx = blockIdx.x, ty = blockIdx.y;
  if constexpr (XCD == 2) {
    // column strips: XCD x (= dispatch id mod 8) owns tile columns [x*gx/8, (x+1)*gx/8), so each XCD's
    // L2 pulls 1/8 of the weight panel (the larger operand at small M) and all of A (gx % 8 == 0)
    const int gx = gridDim.x, id = blockIdx.y * gx + blockIdx.x, sw = gx >> 3;
    const int xcd = id & 7, k = id >> 3;
    ty = k / sw;
    tx = xcd * sw + (k - ty * sw);
  } else if constexpr (XCD == 1) {
    const int gx = gridDim.x, nwg = gx * gridDim.y, id = blockIdx.y * gx + blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (id >> 3);
    ty = wg / gx;
    tx = wg - ty * gx;
  }
  const int bn = tx * BN;
  const int bm = ty * BM;
  const int nsteps = K / BKE;

  // ---- per-lane DMA sources (K-step 0); a K-step advances every source by 128 (bf16) / 256 (fp32) B
  const char* wsrc[SM::GW];
#pragma unroll
  for (int j = 0; j < SM::GW; ++j) {
    const int r = (wave * SM::GW + j) * RPI + lane / CPR;
    const int c = (lane % CPR) ^ lds_swz<CPR>(r);
    wsrc[j] = reinterpret_cast<const char*>(W + (size_t)(bn + r) * ldw) + c * 16;
  }
  const char* asrc[SM::GA];
#pragma unroll
  for (int j = 0; j < SM::GA; ++j) {
    if constexpr (XF) {  // 4 rows x 16 linear chunks per instruction
      const int r = (wave * SM::GA + j) * 4 + (lane >> 4);
      const int m = bm + r < M ? bm + r : M - 1;
      asrc[j] = al.src_row(m) + (lane & 15) * 16;
    } else {             // 8 rows x 8 swizzled chunks per instruction
      const int r = (wave * SM::GA + j) * RPI + lane / CPR;
      const int m = bm + r < M ? bm + r : M - 1;
      asrc[j] = al.src_row(m) + ((lane % CPR) ^ lds_swz<CPR>(r)) * 16;
    }
  }
  auto issue = [&](int s) __attribute__((always_inline)) {
    char* st = smem + (s % NS) * SM::STAGE;
#pragma unroll
    for (int j = 0; j < SM::GA; ++j)
      glds16(asrc[j] + (size_t)s * (KB * SM::AE), st + (wave * SM::GA + j) * 1024);
#pragma unroll
    for (int j = 0; j < SM::GW; ++j) glds16(wsrc[j] + (size_t)s * (KB * 2), st + SM::A_RAW + (wave * SM::GW + j) * 1024);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- kPreIssue K-steps go out before the fused prologue (whose loads then overlap them, and whose
  // waits — in-order vmcnt — drain only those), the rest of the NS-1 deep ring right after it
  constexpr int kPreIssue = 2;
  const int ring_n = nsteps < NS - 1 ? nsteps : NS - 1;
  const int pre_n = ring_n < kPreIssue ? ring_n : kPreIssue;
  for (int s = 0; s < pre_n; ++s) issue(s);

  constexpr bool PRE = kpre_of<EP>::value;
  // Small tiles fetch the residual (X) before the K loop; at 128 x 128 that costs 64 VGPRs and drops the
  // kernel to one workgroup per CU (B = 64: conv_3 222 -> 234 us, mlp.2 183 -> 204 us), so it waits.
  constexpr bool PRE_EARLY = PRE && FM * FN <= 4;
  float pre[FM][FN][4];
  const int fr = lane & 15, fq = lane >> 4;
  bool a_uv = false, e_uv = false;
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
  if constexpr (PRE_EARLY) fetch_pre();
  if constexpr (AV) a_uv = al.prologue_v(bm, BM, M, K, a_stats, a_vec);
  else al.prologue(bm, BM, M, a_stats);
  if constexpr (EV) e_uv = ep.prologue_v(bm, bn, BM, BN, M, e_stats, e_vec);
  else ep.prologue(bm, BM, M, e_stats);
  FL_STAMP(1);
  for (int s = pre_n; s < ring_n; ++s) issue(s);

  // transform pass (fp32-source loaders): raw K-step s -> bf16 image Abf[s & 1].  A thread transforms
  // the same rows at every K-step, so its row context (statistics, vector slot) is built once here.
  constexpr int PR = XF ? BM * 8 / kGemmThreads : 1;
  typename AL::XRow xr[PR];  // filled after the first barrier (the prologue's LDS writes)
  auto transform = [&](int s) __attribute__((always_inline)) {
    if constexpr (XF) {
      const char* st = smem + (s % NS) * SM::STAGE;
      char* abf = smem + SM::ring + (s & 1) * SM::ABF;
#pragma unroll
      for (int p = 0; p < BM * 8 / kGemmThreads; ++p) {
        const int q = tid + p * kGemmThreads;
        const int r = q >> 3, c = q & 7;
        const float* row = reinterpret_cast<const float*>(st + r * 256);
        // odd rows read their two 16-B halves in the other order: the 16 lanes of a ds_read_b128
        // group (two rows) then hit 16 distinct slots of the 256-B bank line
        const int h0 = (r & 1), h1 = h0 ^ 1;
        const float4 x0 = *reinterpret_cast<const float4*>(row + c * 8 + h0 * 4);
        const float4 x1 = *reinterpret_cast<const float4*>(row + c * 8 + h1 * 4);
        const float4 lo = h0 ? x1 : x0, hi = h0 ? x0 : x1;
        typename AL::Raw raw;
        raw.v[0] = lo.x; raw.v[1] = lo.y; raw.v[2] = lo.z; raw.v[3] = lo.w;
        raw.v[4] = hi.x; raw.v[5] = hi.y; raw.v[6] = hi.z; raw.v[7] = hi.w;
        const u32x4 o = al.template xform<bf16>(xr[p], raw, s * BKE + c * 8, a_stats, a_vec, bm);
        *reinterpret_cast<u32x4*>(abf + lds_off<8>(r, c)) = o;
      }
    }
  };
  auto mfma_step = [&](const char* ta, const char* tb) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < KB / 32; ++kk) {
      u32x4 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const u32x4*>(ta + lds_offk<CPR>(wr * WTM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const u32x4*>(tb + lds_offk<CPR>(wc * WTN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[i]), __builtin_bit_cast(bf16x8, b[j]),
                                                              acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (XF) {
    // ---- main loop, transform one K-step ahead: at step s the A image of s is complete (transformed
    // during step s-1), so one barrier per step orders {transform s+1 -> Abf[(s+1)&1]} against
    // {MFMA s <- Abf[s&1]} and the DMA reissue into the slot step s-1 used.
    wait_vm<SM::G, NS - 2>(ring_n - 1);  // K-step 0 landed (ring_n - 1 younger K-steps in flight)
    lds_barrier();
#pragma unroll
    for (int p = 0; p < PR; ++p) {
      const int r = (tid + p * kGemmThreads) >> 3;
      const int m = bm + r < M ? bm + r : M - 1;
      xr[p] = al.xrow(m, a_stats, a_vec, a_uv, bm);
    }
    transform(0);
    for (int s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) {
        const int ahead = (nsteps - 2 - s) < (NS - 3) ? (nsteps - 2 - s) : (NS - 3);
        wait_vm<SM::G, NS - 2>(ahead);  // K-step s+1 landed
      }
      lds_barrier();
      if (s + NS - 1 < nsteps) issue(s + NS - 1);  // into slot (s-1) % NS: transformed at s-2, W read at s-1
      if (s + 1 < nsteps) transform(s + 1);
      mfma_step(smem + SM::ring + (s & 1) * SM::ABF, smem + (s % NS) * SM::STAGE + SM::A_RAW);
    }
  } else {
    // ---- main loop: wait for K-step s (counted), barrier, reissue the slot of s-1, MFMA in place
    for (int s = 0; s < nsteps; ++s) {
      const int ahead = (nsteps - 1 - s) < (NS - 2) ? (nsteps - 1 - s) : (NS - 2);
      wait_vm<SM::G, NS - 2>(ahead);
      lds_barrier();
      if (s + NS - 1 < nsteps) issue(s + NS - 1);  // into the slot K-step s-1 used (all waves are past it)
      const char* st = smem + (s % NS) * SM::STAGE;
      mfma_step(st, st + SM::A_RAW);
    }
  }
  lds_barrier();  // every wave's fragment reads are done before the epilogue reuses the ring
  FL_STAMP(2);
  if constexpr (PRE && !PRE_EARLY && !SM::VEPI) fetch_pre();

  if constexpr (SM::VEPI) {
    // ---- row-vectorised epilogue: accumulators -> fp32 tile image in LDS (16-float column blocks
    // XOR-swizzled by (row >> 2) & 3: the four rows of one fragment write are 4 fq + r for a fixed r, so they
    // differ in bits 2..3 -- the round-5 swizzle by row & 3 was constant within a write and left it 4-way
    // bank-conflicted), then each thread handles 16 x (one row, 4 consecutive columns): 16-B residual loads /
    // stores, row statistics over a half-wave per row.
    float* ct = reinterpret_cast<float*>(smem);
    auto cidx = [](int row, int col) __attribute__((always_inline)) { return row * BN + (col ^ (((row >> 2) & 3) << 4)); };
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ct[cidx(wr * WTM + i * 16 + fq * 4 + r, wc * WTN + j * 16 + fr)] = acc[i][j][r];
    __syncthreads();
    FL_STAMP(3);
    constexpr int C4 = BN / 4, IT = BM * C4 / kGemmThreads, RPI = kGemmThreads / C4;  // rows per iteration
    static_assert(C4 == 32, "row-vectorised epilogue: a row is one half-wave of float4 columns");
    float xr[IT][4];
    if constexpr (PRE) {
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int row = it * RPI + (tid >> 5), c = (tid & 31) * 4;
        const int m = bm + row < M ? bm + row : M - 1;
#pragma unroll
        for (int e = 0; e < 4; ++e) xr[it][e] = ep.pre(m, bn + c + e);
      }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int row = it * RPI + (tid >> 5), c = (tid & 31) * 4;
      const int m = bm + row < M ? bm + row : M - 1;
      const float4 a4 = *reinterpret_cast<const float4*>(ct + cidx(row, c));
      const float av[4] = {a4.x, a4.y, a4.z, a4.w};
      float v[4];
      if constexpr (PRE) {
        value4_pre(ep, m, bn + c, av, e_stats, e_vec, e_uv, bm, bn, xr[it], v);
      } else if constexpr (EV) {
        value4_ev(ep, m, bn + c, av, e_stats, e_vec, e_uv, bm, bn, v);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ep.value(m, bn + c + e, av[e], e_stats, bm);
      }
      if constexpr (EP::kRowStats) {
        float sum = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) sum += __shfl_xor(sum, o);
        const float mean = sum * (1.0f / BN);
        float q = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[e] - mean;
          q += d * d;
        }
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o);
        if ((tid & 31) == 0 && bm + row < M) ep.store_stats(bm + row, tx, mean, q);
      }
      if (bm + row < M) store4(ep, bm + row, bn + c, v, e_vec, e_uv, bm, bn);
    }
  } else {
    // ---- epilogue (gemm_kernel's, verbatim in effect)
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
      float* red = reinterpret_cast<float*>(smem);
      float mean[FM][4];
  #pragma unroll
      for (int i = 0; i < FM; ++i)
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sum = 0.f;
  #pragma unroll
          for (int j = 0; j < FN; ++j) sum += val[i][j][r];
          sum = wave_sum16(sum);
          if (fr == 0) red[(wr * WTM + i * 16 + fq * 4 + r) * 2 + wc] = sum;
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
          float sum = 0.f;
  #pragma unroll
          for (int j = 0; j < FN; ++j) {
            float d = val[i][j][r] - mean[i][r];
            sum += d * d;
          }
          sum = wave_sum16(sum);
          if (fr == 0) red[(wr * WTM + i * 16 + fq * 4 + r) * 2 + wc] = sum;
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
  }
  FL_STAMP(4);
}

// Deepest ring that fits 160 KB next to the prologue/epilogue LDS (at most NSMAX stages).
template <int BM, int BN, int NS, class AL, class EP>
inline int launch_gemm_dma_ns(const AL& al, const bf16* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  using SM = DmaSmem<BM, BN, NS, AL, EP>;
  const size_t bytes = SM::bytes + (size_t)kvec_of<AL>::value * K * 4;
  if constexpr (NS > 3) {
    if (bytes > 160 * 1024) return launch_gemm_dma_ns<BM, BN, NS - 1>(al, W, ldw, ep, M, N, K, st);
  }
  FL_REQUIRE(bytes <= 160 * 1024, "gemm_dma: LDS request %zu B too large (K=%d)", bytes, K);
  auto kern = gemm_dma_kernel<BM, BN, NS, AL, EP>;
  if (bytes > 64 * 1024) {
    FL_HIP(set_max_lds(reinterpret_cast<const void*>(kern)));
  }
  hipLaunchKernelGGL(kern, dim3(N / BN, (M + BM - 1) / BM), dim3(kGemmThreads), bytes, st, al, W, ldw, ep, M, N, K);
  FL_LAUNCH_CHECK();
  return kOk;
}

// Fixed ring depth, optional XCD-aware placement (large-M tiles).
template <int BM, int BN, int NS, int XCD, class AL, class EP, int KB = 64>
inline int launch_gemm_dma_fixed(const AL& al, const bf16* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  FL_REQUIRE(M > 0 && N % BN == 0 && K % KB == 0, "gemm_dma: unsupported shape M=%d N=%d K=%d (BN=%d)", M, N, K, BN);
  using SM = DmaSmem<BM, BN, NS, AL, EP, KB>;
  const size_t bytes = SM::bytes + (size_t)kvec_of<AL>::value * K * 4;
  FL_REQUIRE(bytes <= 160 * 1024, "gemm_dma: LDS request %zu B too large (K=%d)", bytes, K);
  auto kern = gemm_dma_kernel<BM, BN, NS, AL, EP, XCD, KB>;
  if (bytes > 64 * 1024) {
    FL_HIP(set_max_lds(reinterpret_cast<const void*>(kern)));
  }
  hipLaunchKernelGGL(kern, dim3(N / BN, (M + BM - 1) / BM), dim3(kGemmThreads), bytes, st, al, W, ldw, ep, M, N, K);
  FL_LAUNCH_CHECK();
  return kOk;
}

template <int BM, int BN, class AL, class EP>
inline int launch_gemm_dma(const AL& al, const bf16* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  FL_REQUIRE(M > 0 && N % BN == 0 && K % 64 == 0, "gemm_dma: unsupported shape M=%d N=%d K=%d (BN=%d)", M, N, K, BN);
  switch (tn().dma_ns) {  // ring depth (flamed_tune "dma_ns"); deeper rings fall back while LDS does not fit
    case 8: return launch_gemm_dma_ns<BM, BN, 8>(al, W, ldw, ep, M, N, K, st);
    case 6: return launch_gemm_dma_ns<BM, BN, 6>(al, W, ldw, ep, M, N, K, st);
    case 4: return launch_gemm_dma_ns<BM, BN, 4>(al, W, ldw, ep, M, N, K, st);
    default: return launch_gemm_dma_ns<BM, BN, 3>(al, W, ldw, ep, M, N, K, st);
  }
}

}  // namespace fl
