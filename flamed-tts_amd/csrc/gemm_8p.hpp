// 256 x 256-tile bf16 GEMM for the MFMA-bound large-M regime (denoiser at B*T >= big_rows):
// C[M][N] = A[M][K] . W[N][K]^T with A bf16 rows (LoadPlain) and any epilogue policy of gemm.hpp.
//
// Structure (cdna_hip_programming.md §5 "The 256^2 8-phase template"): 512 threads = 8 waves as
// 2 (M) x 4 (N), each wave a 128 x 64 output block of 8 x 4 MFMA fragments (v_mfma_f32_16x16x32_bf16).
// One K-tile = 64 deep: A 256 x 64 and W 256 x 64 bf16 (32 KB each) in a double-buffered LDS image
// (128 KB).  Every operand byte travels by global_load_lds_dwordx4 (source-side XOR swizzle, lds_off<8>
// reads), 16 KB "half-tiles" at a time: A_lo = the first 64 rows of each wave row's 128 (read by quadrant
// Q0), A_hi = the last 64 (Q2), B_lo = the first 32 columns of each wave column's 64 (Q0, kept in
// registers for Q3), B_hi = the other 32 (Q1).  A wave's 128 x 64 block is computed in four quadrant
// phases per K-tile, 16 MFMAs each (Q0: A_lo x B_lo, Q1: A_lo x B_hi, Q2: A_hi x B_hi, Q3: A_hi x B_lo),
// so each half-tile slot is read in exactly one phase:
//   phase  1    2    3    4  |  5    6    7    8      (even K-tile in buffer 0, odd in buffer 1)
//   reads  E.lo E.Bh E.Ah -  |  O.lo O.Bh O.Ah -
//   loads  O.Bh O.Ah E'.Al E'.Bl | E'.Bh E'.Ah O'.Al O'.Bl     (E' = E + 2, O' = O + 2)
//   waits               vm(4) |                vm(4)
// Each phase: ds_reads of the phase's fragments, one half-tile of LDS-DMA (2 instructions per thread),
// [counted vmcnt], s_barrier, lgkmcnt(0), 16 MFMAs at raised priority, s_barrier.  The two wave rows run
// one barrier apart (the wr == 1 waves take one extra barrier up front), so one group's ds_reads overlap
// the other's MFMAs.  Ordering rules (§5): a half-tile is read one phase after the wait that retires it
// (the stagger needs that one barrier more), and restaged at least two phases after its last read — both
// hold for every slot in the table above.  The wait counts are the DMA instructions issued after the
// tile that must have landed (2 per later half-tile; fewer in the last iteration, when nothing follows).
// Epilogue: the accumulators go through an fp32 LDS image of 256 x 128 (one column half at a time), read
// back row-vectorised (16-B residual loads/stores, LayerNorm row partials of 128 columns over a half-wave).
//
// MX-fp8 variant (F8 = true; BASELINE configs[4] "fp8 pointwise projections"): A and W are OCP e4m3 bytes
// with one e8m0 scale per 32-element K block of every row (both operands), and each quadrant runs 8
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the K of the bf16 form per MFMA, twice its cycles: 2x bf16 per
// clock).  A K-tile is 128 elements = the same 128-B rows, so the DMA ring, the swizzle and the fragment
// reads are byte-for-byte the bf16 ones.  Lane group g (lanes 16 g .. 16 g + 15) reads chunks g and 4 + g
// of its row — instruction K [16 g, +16) in VGPRs 0-3, [64 + 16 g, +16) in VGPRs 4-7 (measured,
// tools/probe_mx.py) — and passes the scale of K block g, which the hardware applies to instruction K
// [32 g, 32 g + 32) = memory bytes [32 g, 32 g + 32) of the K-tile row: an MX block is 32 contiguous
// elements.  The scales of the tile's 256 rows / columns over all of K (256 x K / 32 bytes each; K <= 1024)
// are staged in LDS before the main loop, in the order the fragment reads want (mx_a_index / mx_b_index:
// a lane reads its 8 A-row scales with one ds_read_b64 and its 4 W-column scales with one ds_read_b32 per
// K-tile, picked by the MFMA's op_sel byte).
#pragma once
#include "gemm.hpp"

#ifndef FL_8P_EPI_U
#define FL_8P_EPI_U 4  // epilogue row-iterations whose residual loads are in flight together (16 spills)
#endif
#include "gemm_dma.hpp"

namespace fl {

constexpr int k8pThreads = 512;

constexpr int kMxMaxK = 1024;  // fp8 path: largest K whose scales are staged whole (256 x K/32 B per operand)

template <class EP, bool F8 = false>
struct G8Smem {
  static constexpr int HALF = 16 * 1024;           // one half-tile: 128 rows x 128 B
  static constexpr int BUF = 4 * HALF;             // one K-tile: A (32 KB) then W (32 KB)
  static constexpr int ring = 2 * BUF;             // 128 KB
  static constexpr int ctile = 256 * 128 * 4;      // epilogue image: 256 rows x 128 fp32 columns (128 KB)
  static constexpr int body = ring > ctile ? ring : ctile;
  static constexpr int e_stats = EP::stat_rows(256) * 2 * 4;
  static constexpr int e_vec = kevec_of<EP>::value * kEVecStride * 4;  // per 128-column half (two copies)
  static constexpr int mx = F8 ? 2 * 256 * (kMxMaxK / 32) : 0;          // A then W scale bytes
  static constexpr int bytes = (body + e_stats + 2 * e_vec + mx + 15) / 16 * 16;
};

// Position of the e8m0 scale of (row m, K block kb) of an fp8 A operand with K columns: per 256-row tile
// a contiguous 256 x K/32-byte image, ordered [kb][row half][row % 16][row % 128 / 16] (a lane's 8
// fragment rows are 8 consecutive bytes).  Rows are padded to a multiple of 256.
__host__ __device__ __forceinline__ size_t mx_a_index(int m, int kb, int K) {
  const int r = m & 255;
  return (size_t)(m >> 8) * (size_t)(8 * K) + (size_t)(((kb * 2 + (r >> 7)) << 7) + ((r & 15) << 3) + ((r & 127) >> 4));
}
// ... of (column n, K block kb) of an fp8 W: per 256-column tile [kb][column quarter][n % 16][n % 64 / 16].
__host__ __device__ __forceinline__ size_t mx_b_index(int n, int kb, int K) {
  const int c = n & 255;
  return (size_t)(n >> 8) * (size_t)(8 * K) + (size_t)(((kb * 4 + (c >> 6)) << 6) + ((c & 15) << 2) + ((c & 63) >> 4));
}
// Bytes of the scale image of an fp8 operand of `rows` rows (or W columns) and K columns.
inline size_t mx_scale_bytes(size_t rows, int K) { return (rows + 255) / 256 * 256 * (size_t)(K / 32); }

// MX block exponent of the HIP recipe: the smallest e with amax * 2^-e <= 448 (no element saturates;
// e = ceil(log2(amax / 448)), tests/fp8_sim.py "mxfp8c"), clamped to the e8m0 range.
__device__ __forceinline__ int mx_exp(float amax) {
  const unsigned u = __float_as_uint(amax);
  const int be = (int)((u >> 23) & 0xff);
  if (be == 0) return -127;  // zero / denormal block: any scale represents it
  int e = be - 127 - 8;      // amax * 2^-e in [256, 512)
  if (amax * __uint_as_float((unsigned)(127 - e) << 23) > 448.f) ++e;
  return e < -126 ? -126 : (e > 127 ? 127 : e);
}
__device__ __forceinline__ float mx_inv(int e) { return __uint_as_float((unsigned)(127 - e) << 23); }  // 2^-e
// Four values (already scaled into [-448, 448]) -> four e4m3 bytes, v[0] in the low byte.
__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

// tile row (A) / tile column (W) of row q in [0, 128) of half-tile h (0: lo, 1: hi)
__device__ __forceinline__ int g8_arow(int h, int q) { return (q & 63) + ((q >> 6) << 7) + (h << 6); }
__device__ __forceinline__ int g8_bcol(int h, int q) { return (q & 31) + ((q >> 5) << 6) + (h << 5); }

// One block-scaled MX-fp8 MFMA accumulating in place (D == C, tied): the builtin's destination is not tied
// to its accumulator input, and at 2 waves / SIMD the untied form spills the 256 x 256 tile's 128
// accumulators.  A scale byte IB / JB of the scale word: op_sel bit = byte & 1, op_sel_hi bit = byte >> 1.
typedef int mx_i32x8 __attribute__((ext_vector_type(8)));
template <int IB, int JB>
__device__ __forceinline__ void mx_mfma_inplace(f32x4& acc, const mx_i32x8& a, const mx_i32x8& b, unsigned sa, unsigned sb) {
  if constexpr (IB == 0 && JB == 0)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0]" : "+v"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
  else
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[%5,%6,0] op_sel_hi:[%7,%8,0]"
                 : "+v"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb), "i"(IB & 1), "i"(JB & 1), "i"(IB >> 1), "i"(JB >> 1));
}

// Epilogues whose output is the next GEMM's MX-fp8 operand (EP::kF8Out; store_f8 hook).
template <class T, class = void> struct kf8out_of { static constexpr bool value = false; };
template <class T> struct kf8out_of<T, std::void_t<decltype(T::kF8Out)>> { static constexpr bool value = T::kF8Out; };

// Four consecutive residual values of an epilogue with kPre: one vector load when the epilogue has pre4.
template <class T, class = void> struct has_pre4 { static constexpr bool value = false; };
template <class T>
struct has_pre4<T, std::void_t<decltype(std::declval<const T&>().pre4(0, 0, (float*)nullptr))>> {
  static constexpr bool value = true;
};
template <class EP>
__device__ __forceinline__ void pre4(const EP& ep, int m, int n, float* x) {
  if constexpr (has_pre4<EP>::value) {
    ep.pre4(m, n, x);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = ep.pre(m, n + e);
  }
}

// A producer thread's 8 consecutive columns of row m (K columns) -> e4m3 + the block scale; the 4 lanes
// of one 32-column block (consecutive lanes, 32-column aligned) combine their maxima with two shuffles.
__device__ __forceinline__ void store_f8x8(const float* o, unsigned char* dst, unsigned char* sc, int m, int k, int K) {
  float am = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(o[j]));
  am = fmaxf(am, __shfl_xor(am, 1));
  am = fmaxf(am, __shfl_xor(am, 2));
  const int e = mx_exp(am);
  const float inv = mx_inv(e);
  const uint2 q = make_uint2(pack4_fp8(o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv),
                             pack4_fp8(o[4] * inv, o[5] * inv, o[6] * inv, o[7] * inv));
  *reinterpret_cast<uint2*>(dst + (size_t)m * K + k) = q;
  if ((k & 31) == 0) sc[mx_a_index(m, k >> 5, K)] = (unsigned char)(e + 127);
}

// fp32 weight W[N][K] -> e4m3 rows + the W scale image (mx_b_index): one thread per (row, 32-block).
static __global__ void quant_w_f8_kernel(const float* __restrict__ src, int N, int K, unsigned char* __restrict__ dst,
                                  unsigned char* __restrict__ sc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, KB = K / 32;
  if (i >= N * KB) return;
  const int n = i / KB, kb = i - n * KB;
  const float* p = src + (size_t)n * K + kb * 32;
  float v[32], am = 0.f;
#pragma unroll
  for (int j = 0; j < 32; j += 4) {
    const float4 f = ld4(p + j);
    v[j] = f.x; v[j + 1] = f.y; v[j + 2] = f.z; v[j + 3] = f.w;
  }
#pragma unroll
  for (int j = 0; j < 32; ++j) am = fmaxf(am, fabsf(v[j]));
  const int e = mx_exp(am);
  const float inv = mx_inv(e);
  unsigned q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = pack4_fp8(v[4 * j] * inv, v[4 * j + 1] * inv, v[4 * j + 2] * inv, v[4 * j + 3] * inv);
  u32x4* d = reinterpret_cast<u32x4*>(dst + (size_t)n * K + kb * 32);
  d[0] = u32x4{q[0], q[1], q[2], q[3]};
  d[1] = u32x4{q[4], q[5], q[6], q[7]};
  sc[mx_b_index(n, kb, K)] = (unsigned char)(e + 127);
}

// Bias + activation (EpiBiasAct<bf16, ACT>'s arithmetic) written as the next GEMM's MX-fp8 A operand:
// e4m3 rows (row stride ldo bytes) + the scale image (mx_a_index with K = ldo).  gemm8p epilogues only.
template <int ACT>
struct EpiBiasActF8 {
  static constexpr bool kF8Out = true;
  const float* __restrict__ bias;
  unsigned char* __restrict__ out;
  unsigned char* __restrict__ sc;
  int ldo;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int, int n, float acc, const float*, int) const {
    float v = acc + bias[n];
    if constexpr (ACT == 1) v = gelu_fast(v);
    if constexpr (ACT == 2) v = silu(v);
    return v;
  }
  __device__ void store(int, int, float) const {}
  __device__ void store_stats(int, int, float, float) const {}
  __device__ void store_f8(int m, int n, unsigned packed, int e, bool lead) const {
    *reinterpret_cast<unsigned*>(out + (size_t)m * ldo + n) = packed;
    if (lead) sc[mx_a_index(m, n >> 5, ldo)] = (unsigned char)(e + 127);
  }
};

// A / W: bf16 (F8 = false) or e4m3 bytes with scale images SA / SW (F8 = true); lda / ldw in elements.
template <class EP, bool F8 = false>
__global__ __launch_bounds__(k8pThreads) void gemm8p_kernel(const void* __restrict__ Av, int lda, const void* __restrict__ Wv,
                                                            int ldw, EP ep, int M, int N, int K,
                                                            const unsigned char* __restrict__ SA,
                                                            const unsigned char* __restrict__ SW) {
  using SM = G8Smem<EP, F8>;
  constexpr int ES = F8 ? 1 : 2;  // bytes per element
  const char* A = reinterpret_cast<const char*>(Av);
  const char* W = reinterpret_cast<const char*>(Wv);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* e_stats = reinterpret_cast<float*>(smem + SM::body);
  float* e_vec0 = e_stats + EP::stat_rows(256) * 2;
  float* e_vec1 = e_vec0 + kevec_of<EP>::value * kEVecStride;
  unsigned char* mxs = reinterpret_cast<unsigned char*>(e_vec1 + kevec_of<EP>::value * kEVecStride);  // F8 scales

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // XCD-aware tile order (guide §5 T1, bijective): the ~nwg/8 tiles one XCD receives are consecutive in
  // row-major tile order, so an A row panel is fetched into one XCD's L2
  int tx, ty;
  {
    const int gx = gridDim.x, nwg = gx * gridDim.y, id = blockIdx.y * gx + blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (id >> 3);
    ty = wg / gx;
    tx = wg - ty * gx;
  }
  const int bm = ty * 256, bn = tx * 256;
  const int NT = K * ES / 128;  // 128-B K-tiles

  // ---- per-lane DMA sources: wave w moves rows q = 16 w + 8 j + lane / 8 (j = 0, 1) of a half-tile;
  // lane % 8 picks the 16-B chunk, XOR-swizzled on the source (lds_off<8> on the read, rule 21).  Kept as
  // 32-bit byte offsets from the (uniform) operand bases: 8 VGPRs instead of 8 pointers.
  unsigned aoff[2][2], woff[2][2];  // [half][j]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = wave * 16 + j * 8 + (lane >> 3);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ar = g8_arow(h, q), wn = g8_bcol(h, q);
      const int m = bm + ar < M ? bm + ar : M - 1;
      aoff[h][j] = (unsigned)m * (unsigned)(lda * ES) + (unsigned)(((lane & 7) ^ ((ar >> 1) & 7)) << 4);
      woff[h][j] = (unsigned)(bn + wn) * (unsigned)(ldw * ES) + (unsigned)(((lane & 7) ^ ((wn >> 1) & 7)) << 4);
    }
  }
  // A image rows are tile rows (byte r * 128 of the K-tile's A region); half-tile h row q lands at tile
  // row g8_arow(h, q): the 8 rows of one instruction are consecutive there, so its 1 KB is contiguous.
  auto issue = [&](int t, int which) __attribute__((always_inline)) {
    // which: 0 A_lo, 1 B_lo, 2 B_hi, 3 A_hi
    char* buf = smem + (t & 1) * SM::BUF;
    const bool isA = which == 0 || which == 3;
    const int h = (which == 2 || which == 3) ? 1 : 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q0 = wave * 16 + j * 8;  // first row of this instruction in the half-tile
      if (isA) glds16(A + aoff[h][j] + (unsigned)t * 128u, buf + g8_arow(h, q0) * 128);
      else glds16(W + woff[h][j] + (unsigned)t * 128u, buf + 2 * SM::HALF + g8_bcol(h, q0) * 128);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 a[4][2], blo[2][2], bhi[2][2];  // bf16: fragment i / j, 16-B chunk kk
  // F8: the same two chunks read straight into the halves of the MFMA's 8-dword operand (no copies into
  // fresh register tuples: the fp8 loop otherwise spills at 2 waves / SIMD)
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  typedef int i32x8 __attribute__((ext_vector_type(8)));
  i32x8 a8[4], blo8[2], bhi8[2];
  // fragment read addresses: row (wr*128 + i*16 + fr) / (wc*64 + j*16 + fr) at chunk kk*4 + fq; the lds_off
  // swizzle ((row >> 1) & 7) reduces to (fr >> 1) & 7, so fragment i / j is +2048 B (an immediate offset)
  const int swz = (fr >> 1) & 7;
  const int lda0 = (wr * 128 + fr) * 128, ldb0 = 2 * SM::HALF + (wc * 64 + fr) * 128;
  const int kc0 = ((fq ^ swz) & 7) << 4, kc1 = (((4 + fq) ^ swz) & 7) << 4;
  auto read_a = [&](const char* ta, int i0) __attribute__((always_inline)) {
    const char* p0 = ta + lda0 + kc0;
    const char* p1 = ta + lda0 + kc1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (F8) {
        a8[i].lo = *reinterpret_cast<const i32x4*>(p0 + (i0 + i) * 2048);
        a8[i].hi = *reinterpret_cast<const i32x4*>(p1 + (i0 + i) * 2048);
      } else {
        a[i][0] = *reinterpret_cast<const u32x4*>(p0 + (i0 + i) * 2048);
        a[i][1] = *reinterpret_cast<const u32x4*>(p1 + (i0 + i) * 2048);
      }
    }
  };
  auto read_b = [&](int hi, const char* tb, int j0) __attribute__((always_inline)) {  // hi: into bhi (else blo)
    const char* p0 = tb + ldb0 + kc0;
    const char* p1 = tb + ldb0 + kc1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (F8) {
        i32x8(&b)[2] = hi ? bhi8 : blo8;
        b[j].lo = *reinterpret_cast<const i32x4*>(p0 + (j0 + j) * 2048);
        b[j].hi = *reinterpret_cast<const i32x4*>(p1 + (j0 + j) * 2048);
      } else {
        u32x4(&b)[2][2] = hi ? bhi : blo;
        b[j][0] = *reinterpret_cast<const u32x4*>(p0 + (j0 + j) * 2048);
        b[j][1] = *reinterpret_cast<const u32x4*>(p1 + (j0 + j) * 2048);
      }
    }
  };
  // F8: this lane's scale words of the current K-tile (A rows i = 0..7 as two words, W columns j = 0..3)
  unsigned sa_w[2] = {0u, 0u}, sw_w = 0u;
  auto read_s = [&](int t) __attribute__((always_inline)) {
    if constexpr (F8) {
      // the scale words are MFMA operands of the previous K-tile's (inline-asm, hazard-unaware) MFMAs:
      // wait out the longest MFMA read-after-issue window before overwriting them
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");
      const int kb = t * 4 + fq;
      const uint2 v = *reinterpret_cast<const uint2*>(mxs + ((kb * 2 + wr) << 7) + (fr << 3));
      sa_w[0] = v.x;
      sa_w[1] = v.y;
      sw_w = *reinterpret_cast<const unsigned*>(mxs + 256 * (kMxMaxK / 32) + ((kb * 4 + wc) << 6) + (fr << 2));
    }
  };
  auto mfma_q = [&](int i0, int j0, int hi) __attribute__((always_inline)) {  // hi: B fragments from bhi
    if constexpr (F8) {
      const i32x8(&b8)[2] = hi ? bhi8 : blo8;
      const unsigned sa = i0 ? sa_w[1] : sa_w[0];
      // op_sel picks the byte of the scale word: A row i0 + i -> byte i, W column j0 + j -> byte j0 + j
#define FL_MXQ(I, J, JB) mx_mfma_inplace<I, JB>(acc[i0 + I][j0 + J], a8[I], b8[J], sa, sw_w)
      if (j0 == 0) {
        FL_MXQ(0, 0, 0); FL_MXQ(0, 1, 1); FL_MXQ(1, 0, 0); FL_MXQ(1, 1, 1);
        FL_MXQ(2, 0, 0); FL_MXQ(2, 1, 1); FL_MXQ(3, 0, 0); FL_MXQ(3, 1, 1);
      } else {
        FL_MXQ(0, 0, 2); FL_MXQ(0, 1, 3); FL_MXQ(1, 0, 2); FL_MXQ(1, 1, 3);
        FL_MXQ(2, 0, 2); FL_MXQ(2, 1, 3); FL_MXQ(3, 0, 2); FL_MXQ(3, 1, 3);
      }
#undef FL_MXQ
    } else {
      const u32x4(&b)[2][2] = hi ? bhi : blo;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, a[i][kk]), __builtin_bit_cast(bf16x8, b[j][kk]), acc[i0 + i][j0 + j], 0, 0, 0);
    }
  };
  auto bar = []() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // one phase: reads (R), one half-tile of DMA (issued when `ld`), optional counted wait, barrier,
  // lgkmcnt(0), MFMAs, barrier
  auto mid = []() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto tail = []() __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- the epilogue's row statistics and per-column vectors (both 128-column halves) are staged first,
  // outside the operand ring: its ordinary global loads complete before any LDS-DMA is in flight, and the
  // accumulators are not yet live (staging them after the main loop spilled: 128 accumulators + staging)
  constexpr bool EV = kevec_of<EP>::value > 0;
  bool e_uv0 = false, e_uv1 = false;
  if constexpr (EV) {
    e_uv0 = ep.prologue_v(bm, bn, 256, 128, M, e_stats, e_vec0);
    e_uv1 = ep.prologue_v(bm, bn + 128, 256, 128, M, e_stats, e_vec1);
  } else {
    ep.prologue(bm, 256, M, e_stats);
  }
  if constexpr (F8) {  // the tile's A-row and W-column scale images (8 * K bytes each), before any DMA
    const int n16 = K / 2;  // 16-B pieces per image (8 K bytes)
    const u32x4* sa = reinterpret_cast<const u32x4*>(SA + (size_t)ty * (size_t)(8 * K));
    const u32x4* sw = reinterpret_cast<const u32x4*>(SW + (size_t)tx * (size_t)(8 * K));
    for (int q = tid; q < n16; q += k8pThreads) {
      reinterpret_cast<u32x4*>(mxs)[q] = sa[q];
      reinterpret_cast<u32x4*>(mxs + 256 * (kMxMaxK / 32))[q] = sw[q];
    }
    __syncthreads();
  }

  // ---- prologue: K-tile 0 whole, K-tile 1's A_lo / B_lo (the steady state's phase 7 / 8 loads)
  issue(0, 0); issue(0, 1); issue(0, 2); issue(0, 3);
  if (NT > 1) { issue(1, 0); issue(1, 1); }
  if (NT > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (wr == 1) bar();  // the second wave row runs one barrier behind

  for (int t = 0; t < NT; t += 2) {
    const char* E = smem + 0 * SM::BUF;
    const char* O = smem + 1 * SM::BUF;
    const bool e2 = t + 2 < NT, o2 = t + 3 < NT;  // NT is even: the odd K-tile t + 1 always exists
    // phase 1: E.Q0 (A_lo x B_lo)
    read_s(t);
    read_b(0, E, 0);
    read_a(E, 0);
    issue(t + 1, 2);
    mid(); mfma_q(0, 0, 0); tail();
    // phase 2: E.Q1 (A_lo x B_hi)
    read_b(1, E, 2);
    issue(t + 1, 3);
    mid(); mfma_q(0, 2, 1); tail();
    // phase 3: E.Q2 (A_hi x B_hi)
    read_a(E, 4);
    if (e2) issue(t + 2, 0);
    mid(); mfma_q(4, 2, 1); tail();
    // phase 4: E.Q3 (A_hi x B_lo); wait: the odd K-tile has landed (E'.A_lo / B_lo may fly)
    if (e2) issue(t + 2, 1);
    if (e2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mid(); mfma_q(4, 0, 0); tail();
    // phase 5: O.Q0
    read_s(t + 1);
    read_b(0, O, 0);
    read_a(O, 0);
    if (e2) issue(t + 2, 2);
    mid(); mfma_q(0, 0, 0); tail();
    // phase 6: O.Q1
    read_b(1, O, 2);
    if (e2) issue(t + 2, 3);
    mid(); mfma_q(0, 2, 1); tail();
    // phase 7: O.Q2
    read_a(O, 4);
    if (o2) issue(t + 3, 0);
    mid(); mfma_q(4, 2, 1); tail();
    // phase 8: O.Q3; wait: the next even K-tile has landed (O'.A_lo / B_lo may fly)
    if (o2) issue(t + 3, 1);
    if (o2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mid(); mfma_q(4, 0, 0); tail();
  }
  if (wr == 0) bar();  // realign the two wave rows: every LDS read of the main loop is complete after this
  bar();
  // F8: the last MFMAs were inline asm (the compiler's hazard recognizer does not see them): the XDL
  // write -> VALU / DS read window of a 16-pass MFMA (18 wait states) before the epilogue reads acc
  if constexpr (F8) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  // ---- epilogue, one 128-column half at a time through a 256 x 128 fp32 image
  float* ct = reinterpret_cast<float*>(smem);
  // 16-float column blocks XOR-swizzled by (row >> 2) & 3 = fq: a fragment write's four rows (4 fq + r) hit distinct
  // banks (swizzling by row & 3, constant within one write, left it 4-way conflicted)
  auto cidx = [](int row, int col) __attribute__((always_inline)) { return row * 128 + (col ^ (((row >> 2) & 3) << 4)); };
  constexpr bool PRE = kpre_of<EP>::value;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int bnh = bn + h * 128;
    if ((wc >> 1) == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ct[cidx(wr * 128 + i * 16 + fq * 4 + r, (wc & 1) * 64 + j * 16 + fr)] = acc[i][j][r];
    }
    const bool e_uv = h ? e_uv1 : e_uv0;
    const float* e_vec = h ? e_vec1 : e_vec0;
    __syncthreads();
    constexpr int IT = 256 * 32 / k8pThreads, RPI = k8pThreads / 32;  // 16 rows per iteration
    constexpr int U = FL_8P_EPI_U;  // iterations whose residual loads are in flight together (16-B vector loads)
#pragma unroll 1
    for (int it0 = 0; it0 < IT; it0 += U) {
      float xr[U][4];
      if constexpr (PRE) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int row = (it0 + u) * RPI + (tid >> 5), c = (tid & 31) * 4;
          pre4(ep, bm + row < M ? bm + row : M - 1, bnh + c, xr[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = (it0 + u) * RPI + (tid >> 5), c = (tid & 31) * 4;
        const int m = bm + row < M ? bm + row : M - 1;
        const float4 a4 = *reinterpret_cast<const float4*>(ct + cidx(row, c));
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
        float v[4];
        if constexpr (PRE) {
          value4_pre(ep, m, bnh + c, av, e_stats, e_vec, e_uv, bm, bnh, xr[u], v);
        } else if constexpr (EV) {
          value4_ev(ep, m, bnh + c, av, e_stats, e_vec, e_uv, bm, bnh, v);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = ep.value(m, bnh + c + e, av[e], e_stats, bm);
        }
        if constexpr (kf8out_of<EP>::value) {  // MX-fp8 output: 8 lanes = one 32-column block of the row
          float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
#pragma unroll
          for (int o = 1; o < 8; o <<= 1) am = fmaxf(am, __shfl_xor(am, o));
          const int e = mx_exp(am);
          const float inv = mx_inv(e);
          if (bm + row < M) ep.store_f8(bm + row, bnh + c, pack4_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv), e, (tid & 7) == 0);
          continue;
        }
        if constexpr (EP::kRowStats) {
          float sum = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) sum += __shfl_xor(sum, o);
          const float mean = sum * (1.0f / 128);
          float q = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = v[e] - mean;
            q += d * d;
          }
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o);
          if ((tid & 31) == 0 && bm + row < M) ep.store_stats(bm + row, bnh / 128, mean, q);
        }
        if (bm + row < M) store4(ep, bm + row, bnh + c, v, e_vec, e_uv, bm, bnh);
      }
    }
    __syncthreads();  // the image is rewritten by the next half
  }
}

// Shapes: N % 256 == 0, K % 128 == 0 (an even number of 64-deep K-tiles), any M (rows clamped / masked).
template <class EP>
inline int launch_gemm8p(const bf16* A, int lda, const bf16* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  FL_REQUIRE(M > 0 && N % 256 == 0 && K % 128 == 0, "gemm8p: unsupported shape M=%d N=%d K=%d", M, N, K);
  using SM = G8Smem<EP>;
  static_assert(SM::bytes <= 160 * 1024, "gemm8p: LDS");
  auto kern = gemm8p_kernel<EP, false>;
  FL_HIP(set_max_lds(reinterpret_cast<const void*>(kern)));
  hipLaunchKernelGGL(kern, dim3(N / 256, (M + 255) / 256), dim3(k8pThreads), SM::bytes, st, (const void*)A, lda, (const void*)W, ldw,
                     ep, M, N, K, (const unsigned char*)nullptr, (const unsigned char*)nullptr);
  FL_LAUNCH_CHECK();
  return kOk;
}

// MX-fp8: A (M x K e4m3, row stride lda bytes) with scale image SA (mx_a_index, rows padded to 256), W
// (N x K e4m3) with SW (mx_b_index).  Shapes: N % 256 == 0, K % 256 == 0 (an even number of 128-deep
// K-tiles), K <= kMxMaxK.
template <class EP>
inline int launch_gemm8p_f8(const unsigned char* A, const unsigned char* SA, int lda, const unsigned char* W,
                            const unsigned char* SW, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  FL_REQUIRE(M > 0 && N % 256 == 0 && K % 256 == 0 && K <= kMxMaxK && A && SA && W && SW,
             "gemm8p_f8: unsupported shape M=%d N=%d K=%d", M, N, K);
  using SM = G8Smem<EP, true>;
  static_assert(SM::bytes <= 160 * 1024, "gemm8p_f8: LDS");
  auto kern = gemm8p_kernel<EP, true>;
  FL_HIP(set_max_lds(reinterpret_cast<const void*>(kern)));
  hipLaunchKernelGGL(kern, dim3(N / 256, (M + 255) / 256), dim3(k8pThreads), SM::bytes, st, (const void*)A, lda, (const void*)W, ldw,
                     ep, M, N, K, SA, SW);
  FL_LAUNCH_CHECK();
  return kOk;
}

}  // namespace fl
