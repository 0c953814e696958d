// Persistent PVA flow kernel (design notes: pvaflow.hpp).
#include "flamed_hip.h"
#include "pvaflow.hpp"

#include <type_traits>

namespace fl {
namespace pv {

// Diagnostic build only (FL_STAMPS, libflamed_hip_stamps.so; tools/pva_timeline.py): thread 0 of every
// workgroup records s_memrealtime at fixed points of step pst_step.
#ifdef FL_STAMPS
#define PVST()                                                                                   \
  do {                                                                                           \
    if (s == P.pst_step && P.pst && threadIdx.x == 0 && pst_k < kStampSlots)                     \
      P.pst[blockIdx.x * kStampSlots + pst_k] = __builtin_amdgcn_s_memrealtime();                 \
    ++pst_k;                                                                                     \
  } while (0)
static unsigned long long* g_pva_pst = nullptr;
static int g_pva_pst_step = -1;
#else
#define PVST() ((void)0)
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
// sc1 (write-through) stores and sc1 loads of hand-off data (aux 16 = sc1)
__device__ __forceinline__ void st4_wt(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 16);
}
__device__ __forceinline__ void st8_wt(__amdgpu_buffer_rsrc_t r, unsigned off, float a, float b) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(a), __float_as_uint(b)}, r, off, 0, 16);
}
__device__ __forceinline__ void st16_wt(__amdgpu_buffer_rsrc_t r, unsigned off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);
}
__device__ __forceinline__ float4 ld16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// Every storing wave drains its write-through stores, the workgroup meets, one lane takes the ticket.
__device__ __forceinline__ void signal(int* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Abandon the flow: the first workgroup to set the error word also counts the failed launch in the sticky word.
__device__ __forceinline__ void raise_err(int* err, int* fails) {
  int expected = 0;
  if (__hip_atomic_compare_exchange_strong(err, &expected, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    __hip_atomic_fetch_add(fails, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 polls the counters of row groups rg - 1, rg, rg + 1 (those that exist) until each reaches
// `target`; bounded by tmo, and an error word set by any workgroup ends every wait.  false: abandon.
__device__ __forceinline__ bool wait3(int* err, int* fails, long long tmo, int* base, int rg, int RG, int target, int* flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x, g = rg - 1 + lane;
    const bool need = lane < 3 && g >= 0 && g < RG;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    for (unsigned it = 0;; ++it) {
      bool mine = true;
      if (need) mine = __hip_atomic_load(base + g * kLine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
      if (__all(mine)) break;
      if ((it & 31) == 31) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) { ok = false; break; }
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > tmo) {
          if (lane == 0) raise_err(err, fails);
          ok = false;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) *flag = ok ? 1 : 0;
  }
  __syncthreads();
  const bool ok = *flag != 0;
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: hand-off loads stay below the poll
  return ok;
}

// K blocks [kb0, kb1) of 16 (a multiple of kBatch blocks) of one 16 x 16 fp32 tile: lane (c, q) supplies A
// elements k = 16 kb + 4 q .. + 3 of its row (af) and reads the same four K of weight column c from the
// resident LDS panel (row stride K floats, 16-B chunks XOR-swizzled by the column); MFMA j of a block
// consumes element j of every lane's chunk, so both operands see one K permutation.  A batch's A loads
// all go out before its MFMAs, so a wave pays one hand-off read latency per batch: the batch is the whole
// K range of the wave up to 18 blocks (72 VGPRs; 36 spilled at 512 VGPRs).  (Batches of 9 blocks
// made conv2 six serial sc1 latencies: 6.9 us of a 19.6 us step at L = 60.)
template <int kBatch, class AF>
__device__ __forceinline__ void kloop(f32x4& acc, const float* W, int K, int kb0, int kb1, int c, int q, const AF& af) {
  for (int kb = kb0; kb < kb1; kb += kBatch) {
    float4 a[kBatch];
#pragma unroll
    for (int i = 0; i < kBatch; ++i) a[i] = af.raw(kb + i);  // global loads only: one latency per batch
#pragma unroll
    for (int i = 0; i < kBatch; ++i) {
      a[i] = af.fin(kb + i, a[i]);  // the transform's LDS vectors are read block by block
      const float4 b = *reinterpret_cast<const float4*>(W + c * K + 4 * ((4 * (kb + i) + q) ^ c));
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b.w, acc, 0, 0, 0);
    }
  }
}

// conv1's A element of this lane's row m (tap gather over proj + time embedding, pva.py:227-230):
// P[src] + w0 * x_t[src] + temb, zero outside the utterance.
template <int D>
struct AConv1 {
  const float* P;
  const float *w0, *te, *xs;
  int m, lm, L, xa, q;
  bool live;
  __device__ bool valid(int kb, int& src, int& ch) const {
    const int k0 = 16 * kb + 4 * q, tap = k0 / D, l = lm + tap - 1;
    ch = k0 - tap * D;
    src = m + tap - 1;
    return live && l >= 0 && l < L;
  }
  __device__ float4 raw(int kb) const {
    int src, ch;
    return valid(kb, src, ch) ? ld4(P + (size_t)src * D + ch) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __device__ float4 fin(int kb, float4 p) const {
    int src, ch;
    if (!valid(kb, src, ch)) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 w = *reinterpret_cast<const float4*>(w0 + ch);
    const float4 e = *reinterpret_cast<const float4*>(te + ch);
    const float x = xs[src - xa];
    return make_float4((p.x + w.x * x) + e.x, (p.y + w.y * x) + e.y, (p.z + w.z * x) + e.z, (p.w + w.w * x) + e.w);
  }
};
// conv2's A element: LayerNorm_1(R1[src]) (statistics of the window rows in LDS), zero outside.
template <int F>
struct AConv2 {
  __amdgpu_buffer_rsrc_t r1;
  const float *st, *g, *b;
  int m, lm, L, xa, q;
  bool live;
  __device__ bool valid(int kb, int& src, int& ch) const {
    const int k0 = 16 * kb + 4 * q, tap = k0 / F, l = lm + tap - 1;
    ch = k0 - tap * F;
    src = m + tap - 1;
    return live && l >= 0 && l < L;
  }
  __device__ float4 raw(int kb) const {
    int src, ch;
    return valid(kb, src, ch) ? ld16_sc1(r1, (unsigned)((src * F + ch) * 4)) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __device__ float4 fin(int kb, float4 v) const {
    int src, ch;
    if (!valid(kb, src, ch)) return make_float4(0.f, 0.f, 0.f, 0.f);
    const int i = src - xa;
    const float mean = st[2 * i], rstd = st[2 * i + 1];
    const float4 gg = *reinterpret_cast<const float4*>(g + ch);
    const float4 bb = *reinterpret_cast<const float4*>(b + ch);
    return make_float4(((v.x - mean) * rstd) * gg.x + bb.x, ((v.y - mean) * rstd) * gg.y + bb.y,
                       ((v.z - mean) * rstd) * gg.z + bb.z, ((v.w - mean) * rstd) * gg.w + bb.w);
  }
};

// One-tile row groups (B * L <= 80): the window's A rows are staged in LDS by coalesced 16-B loads (a wave
// instruction = 1 KB of consecutive rows) instead of each lane gathering 16 rows x 64 B per instruction
// straight from the hand-off buffer, and read back per block (rows padded by 16 B: conflict-free).
// conv1: P rows (w0 x + temb added per block); conv2: LayerNorm_1(R1) rows (applied while staging).
template <int D, int F>
struct AConv1S {
  const float *sa, *w0, *te, *xs;
  int m, lm, L, xa, q;
  bool live;
  __device__ bool valid(int kb, int& src, int& ch) const {
    const int k0 = 16 * kb + 4 * q, tap = k0 / D, l = lm + tap - 1;
    ch = k0 - tap * D;
    src = m + tap - 1;
    return live && l >= 0 && l < L;
  }
  __device__ float4 raw(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ float4 fin(int kb, float4) const {
    int src, ch;
    if (!valid(kb, src, ch)) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 p = *reinterpret_cast<const float4*>(sa + (src - xa) * (F + 4) + ch);
    const float4 w = *reinterpret_cast<const float4*>(w0 + ch);
    const float4 e = *reinterpret_cast<const float4*>(te + ch);
    const float x = xs[src - xa];
    return make_float4((p.x + w.x * x) + e.x, (p.y + w.y * x) + e.y, (p.z + w.z * x) + e.z, (p.w + w.w * x) + e.w);
  }
};
template <int F>
struct AConv2S {
  const float* sa;
  int m, lm, L, xa, q;
  bool live;
  __device__ float4 raw(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ float4 fin(int kb, float4) const {
    const int k0 = 16 * kb + 4 * q, tap = k0 / F, l = lm + tap - 1, ch = k0 - tap * F;
    if (!(live && l >= 0 && l < L)) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *reinterpret_cast<const float4*>(sa + (m + tap - 1 - xa) * (F + 4) + ch);
  }
};

// ST (Params::stage): row groups of >= 2 tiles take conv_st (the per-lane gather loops of those groups are not
// compiled in, so the staged kernel does not carry their registers)
template <int D, int F, bool ST>
__global__ __launch_bounds__(kThreads, 1) void pva_persist_kernel(Params P) {
  using LY = Lds<D, F>;
  constexpr int K1 = LY::K1, K2 = LY::K2, CS = LY::CS, NB1 = K1 / 16, NB2 = K2 / 16;
  static_assert(NB1 % 36 == 0 && NB2 % 36 == 0, "K blocks split 1 / 2 / 4 ways");
  static_assert(CS < 32 && CS % 2 == 0, "head constants, paired LN1 partial loads");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* W1 = reinterpret_cast<float*>(smem + LY::W1);
  float* W2 = reinterpret_cast<float*>(smem + LY::W2);
  float* vw0 = reinterpret_cast<float*>(smem + LY::W0);
  float* vg1 = reinterpret_cast<float*>(smem + LY::G1);
  float* vb1 = reinterpret_cast<float*>(smem + LY::B1);
  float* vte = reinterpret_cast<float*>(smem + LY::TE);
  float* xs = reinterpret_cast<float*>(smem + LY::XS);   // x_t of window rows r0 - 1 .. r0 + nr
  float* st = reinterpret_cast<float*>(smem + LY::ST);   // LN1 (mean, rstd) of the same rows
  float* gs = reinterpret_cast<float*>(smem + LY::GS);   // G_s of the CS slices, [CS] = sum b2 lw
  float4* red = reinterpret_cast<float4*>(smem + LY::RED);
  float* sa = reinterpret_cast<float*>(smem + LY::SA);  // staged A window (one-tile groups)
  float* uv = reinterpret_cast<float*>(smem + LY::UV);  // staged conv1: U[tap][c] = W1_tap,c . w0, V[tap][c] = W1_tap,c . temb_s
  int* flag = reinterpret_cast<int*>(smem + LY::FLAG);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int per = CS * P.RG;
  const int net = blockIdx.x / per, rem = blockIdx.x - net * per, rg = rem / CS, cs = rem - rg * CS;
  const NetP& N = P.net[net];
  const int M = P.M, L = P.L;
  const int tb = rg * P.MT / P.RG, te = (rg + 1) * P.MT / P.RG;
  const int r0 = 16 * tb, nr = min(16 * te, M) - r0, nt = te - tb;
  const int col0 = cs * kCols, xa = r0 - 1, nw = nr + 2;
  int* h1 = P.ctr + CT_H1 + net * kMaxRG * kLine;
  int* h2 = P.ctr + CT_H2 + net * kMaxRG * kLine;
  int* errw = P.ctr + CT_ERR;
  int* fails = P.sticky;
  const long long tmo = P.tmo;
  // Every workgroup leaves through here, after its last counter access: a failed flow writes NaN into its rows
  // of x_t (slice-0 workgroups own the write-back); the last workgroup to count its exit zeroes the counters
  // this launch used, for the next launch.
  auto leave = [&](bool ok) {
    if (!ok && cs == 0)
      for (int i = tid; i < nr; i += kThreads) N.xt[r0 + i] = __builtin_nanf("");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      flag[1] = __hip_atomic_fetch_add(P.ctr + CT_EXIT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == P.grid - 1;
    __syncthreads();
    if (flag[1]) {
      const int n = 2 * P.RG;  // per net and row group: an H1 and an H2 counter
      if (tid < 2 * n) {
        const int which = tid / n, k = tid - which * n, nn = k / P.RG, g = k - nn * P.RG;
        __hip_atomic_store(P.ctr + (which ? CT_H2 : CT_H1) + (nn * kMaxRG + g) * kLine, 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      } else if (tid == 2 * n) {
        __hip_atomic_store(P.ctr + CT_ERR, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (tid == 2 * n + 1) {
        __hip_atomic_store(P.ctr + CT_EXIT, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };

  // ---- resident state: this workgroup's weight columns of both convs, shared vectors, x_t window
  for (int i = tid; i < kCols * K1 / 4; i += kThreads) {
    const int n = i / (K1 / 4), j = i - n * (K1 / 4);
    *reinterpret_cast<float4*>(W1 + n * K1 + 4 * (j ^ (n & 15))) = ld4(N.c1w + (size_t)(col0 + n) * K1 + 4 * j);
  }
  for (int i = tid; i < kCols * K2 / 4; i += kThreads) {
    const int n = i / (K2 / 4), j = i - n * (K2 / 4);
    *reinterpret_cast<float4*>(W2 + n * K2 + 4 * (j ^ (n & 15))) = ld4(N.c2w + (size_t)(col0 + n) * K2 + 4 * j);
  }
  for (int i = tid; i < D; i += kThreads) vw0[i] = N.w0[i];
  for (int i = tid; i < F; i += kThreads) {
    vg1[i] = N.g1[i];
    vb1[i] = N.b1[i];
  }
  if (tid < CS) {
    float g = 0.f;
    for (int k = 0; k < kCols; ++k) g = fmaf(N.g2[kCols * tid + k], N.lw[kCols * tid + k], g);
    gs[tid] = g;
  } else if (tid == 32) {
    float bl = 0.f;
    for (int k = 0; k < F; ++k) bl = fmaf(N.b2[k], N.lw[k], bl);
    gs[CS] = bl;
  }
  for (int i = tid; i < nw; i += kThreads) {
    const int r = xa + i;
    xs[i] = (r >= 0 && r < M) ? N.xt[r] : 0.f;
  }
  const float bias1 = N.c1b[col0 + c], bias2 = N.c2b[col0 + c];
  const float gl = N.g2[col0 + c] * N.lw[col0 + c];
  const float lb = N.lb[0];
  const __amdgpu_buffer_rsrc_t rR1 = rsrc(N.R1, (unsigned)M * F * 4);
  const __amdgpu_buffer_rsrc_t rP = rsrc(N.P, (unsigned)M * D * 4);  // conv1's P rows (constant during the flow)
  const __amdgpu_buffer_rsrc_t rS1 = rsrc(N.S1, (unsigned)M * CS * 8);
  const __amdgpu_buffer_rsrc_t rS2 = rsrc(N.S2, (unsigned)M * CS * 16);
  __syncthreads();

  // waves -> (tile, K part): one tile split over 4 / 2 waves, or tiles w, w + 4 whole
  const int KS = nt == 1 ? 4 : (nt == 2 ? 2 : 1);
  const int part = wave % KS;

  // one conv: every wave's K part of its tile(s), the K parts summed through LDS in part order, then the
  // epilogue by the part-0 waves
  auto conv = [&](const float* W, int K, auto nbtag, auto af, auto afs, auto epi) {
    constexpr int NB = decltype(nbtag)::value;
    constexpr int B4 = NB / 4 < 18 ? NB / 4 : 18, B2 = NB / 2 < 18 ? NB / 2 : 18, B1 = NB < 18 ? NB : 18;
    static_assert((NB / 4) % B4 == 0 && (NB / 2) % B2 == 0 && NB % B1 == 0, "K blocks per wave");
    if (KS > 1) {
      const int t = wave / KS;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (KS == 4) kloop<B4>(acc, W, K, part * NB / 4, (part + 1) * NB / 4, c, q, afs(t));
      else if constexpr (!ST) kloop<B2>(acc, W, K, part * NB / 2, (part + 1) * NB / 2, c, q, af(t));
      red[wave * 64 + lane] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      __syncthreads();
      if (part == 0) {
        for (int p = 1; p < KS; ++p) {
          const float4 o = red[(wave + p) * 64 + lane];
          acc[0] += o.x; acc[1] += o.y; acc[2] += o.z; acc[3] += o.w;
        }
        epi(t, acc);
      }
    } else if constexpr (!ST) {
      for (int t = wave; t < nt; t += 4) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        kloop<B1>(acc, W, K, 0, NB, c, q, af(t));
        epi(t, acc);
      }
    }
  };

  // Row groups of >= 2 tiles (Params::stage): the conv's A window (rows xa .. xa + nw - 1, C channels) goes
  // through LDS in 64-channel chunks.  Each chunk is one coalesced pass of 16-B row loads (a wave instruction =
  // 4 rows x 256 B, instead of 16 lanes gathering 16 rows each), transformed by xf (conv1: P + w0 x + temb;
  // conv2: LayerNorm_1) while written to one of two LDS buffers, further chunks' loads in flight in registers;
  // then every wave runs the chunk's 3 taps x 2 K-blocks of its tiles (w, w + 4).  K is summed chunk-major
  // (the launch path sums it tap-major: the same terms, fp32 rounding apart, inside the parity bar).
  // One barrier per chunk: a buffer is rewritten two chunks later, after the next chunk's barrier, which
  // every wave reaches only when done with this chunk.
  // IPT 16-B items per thread per chunk cover a 66-row window (4 tiles + halo); RD - 1 chunks' loads in flight
  // ahead of the one being staged.  Groups of 5..8 tiles run two passes (tiles w and w + 4, window rows
  // from 0 and from 64), so every wave holds one tile's accumulator at a time.
  constexpr int FC = LY::FC, CBS = LY::CBS, PROWS = LY::PROWS, RD = 3;
  constexpr int IPT = (PROWS * (FC / 4) + kThreads - 1) / kThreads;
  static_assert(2 * 64 + 2 >= LY::WMAX, "two passes cover a group");
  auto conv_st = [&](const float* W, int K, auto ctag, auto ld, auto xf, auto epi, auto tick) {  // tick: FL_STAMPS
    constexpr int C = decltype(ctag)::value, NCH = C / FC;
    constexpr int NBT = FC / 16;  // K-blocks per tap in a chunk
    static_assert(C % FC == 0 && NBT % 2 == 0, "chunks of an even number of K-blocks per tap");
    // two-tile groups: waves (tile w & 1, part w >> 1) split each chunk by K-block (part kp takes blocks kp, kp + 2,
    // ... of every tap), the two parts summed through LDS at the end (part 0 + part 1: deterministic)
    const bool kh = nt == 2;
    const int tw = kh ? (wave & 1) : wave, kp = kh ? (wave >> 1) : 0;
    const int npass = nt > 4 ? 2 : 1;
    for (int pass = 0; pass < npass; ++pass) {
      const int w0 = 64 * pass, nwp = min(nw - w0, PROWS);  // this pass's window rows (window index w0 + row)
      float4 ring[RD][IPT];
      // every load is issued unconditionally (rows outside the pass window or the batch read past the buffer's
      // range, which returns zeros): with no branch around them the compiler's vmcnt waits stay counted, so chunk
      // k waits only for its own loads, not for the chunks in flight behind it
      auto issue = [&](float4 (&dst)[IPT], int k) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
          const int i = tid + kThreads * j, row = i / (FC / 4), c4 = i - row * (FC / 4);
          const int r = xa + w0 + row;
          dst[j] = ld(row < nwp && r >= 0 && r < M ? r : -1, FC * k + 4 * c4);
        }
      };
      // two accumulators (even / odd units), so consecutive MFMA groups do not wait on each other's result;
      // summed once at the end (acc0 + acc1: deterministic)
      f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const int t = tw + 4 * pass;
      const int m = r0 + 16 * t + c;
      const bool live = t < nt && m < r0 + nr;
      const int lm = live ? m % L : 0;
      auto stage = [&](int k) __attribute__((always_inline)) {
        float* buf = sa + (k & 1) * (PROWS + 1) * CBS;
        // branch-free: items past the pass window go to the buffer's spare row PROWS (a load consumed only inside
        // a branch was sunk into it by the compiler, and its wait became vmcnt(0) behind the chunks in flight)
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
          const int i = tid + kThreads * j, row = i / (FC / 4), c4 = i - row * (FC / 4);
          const int r = xa + w0 + row;
          const bool inw = row < nwp;
          const float4 v = P.stage == 3 ? ring[k % RD][j] : xf(w0 + (inw ? row : 0), FC * k + 4 * c4, ring[k % RD][j]);  // (3: no transform)
          // rows outside the batch are zero: a bit mask, not a select (a select became a branch again)
          const unsigned msk = (r >= 0 && r < M) ? ~0u : 0u;
          const float4 o = make_float4(__uint_as_float(__float_as_uint(v.x) & msk), __uint_as_float(__float_as_uint(v.y) & msk),
                                       __uint_as_float(__float_as_uint(v.z) & msk), __uint_as_float(__float_as_uint(v.w) & msk));
          *reinterpret_cast<float4*>(buf + (inw ? row : PROWS) * CBS + 4 * c4) = o;
        }
      };
      auto compute = [&](int k, auto khtag) __attribute__((always_inline)) {
        const float* buf = sa + (k & 1) * (PROWS + 1) * CBS;
        constexpr bool KH = decltype(khtag)::value;  // compile-time: no branch around the MFMAs
        constexpr int NU = 3 * (KH ? NBT / 2 : NBT);  // (tap, K-block) units of this wave in the chunk
        if (t >= nt) return;
        // unit u = (tap u / NB, block): its A fragment (the window row of tap, zeroed outside the utterance by a
        // bit mask on an always-issued read -- the row is inside the pass window for every t < nt) and its B
        // fragment (weight columns c, the block's 4 K per lane)
        auto frag = [&](int u, float4& a, float4& b) __attribute__((always_inline)) {
          constexpr int NB = KH ? NBT / 2 : NBT;
          const int tap = u / NB, bi = u - tap * NB, blk = KH ? 2 * bi + kp : bi;
          a = *reinterpret_cast<const float4*>(buf + (m + tap - 1 - xa - w0) * CBS + 4 * q + 16 * blk);
          const int kb = (tap * C + FC * k) / 16 + blk;
          b = *reinterpret_cast<const float4*>(W + c * K + 4 * ((4 * kb + q) ^ c));
        };
        // units in groups of UG: the group's 2 UG LDS reads are issued together, then its 4 UG MFMAs
        constexpr int UG = NU % 4 == 0 ? 4 : 3;
#pragma unroll
        for (int u0 = 0; u0 < NU; u0 += UG) {
          float4 ar[UG], br[UG];
#pragma unroll
          for (int v = 0; v < UG; ++v) frag(u0 + v, ar[v], br[v]);
          __builtin_amdgcn_sched_barrier(0);  // the scheduler would sink each read to its MFMAs (one LDS latency each)
#pragma unroll
          for (int v = 0; v < UG; ++v) {
            const int u = u0 + v, tap = u / (NU / 3), l = lm + tap - 1;
            const unsigned vm = (live && l >= 0 && l < L) ? ~0u : 0u;
            const float4 a = make_float4(__uint_as_float(__float_as_uint(ar[v].x) & vm), __uint_as_float(__float_as_uint(ar[v].y) & vm),
                                         __uint_as_float(__float_as_uint(ar[v].z) & vm), __uint_as_float(__float_as_uint(ar[v].w) & vm));
            const float4 b = br[v];
            f32x4& ac = (u & 1) ? acc1 : acc;
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, ac, 0, 0, 0);
          }
        }
      };
      // software pipeline, one barrier per chunk: iteration k stages chunk k + 1 (into the other buffer, last read by
      // chunk k - 1's MFMAs, which every wave finished before the previous barrier) and runs chunk k's MFMAs, so a
      // wave's staging VALU / LDS work can issue in the MFMA gaps
#pragma unroll
      for (int k = 0; k < RD - 1; ++k)
        if (k < NCH) issue(ring[k], k);
      stage(0);
      __syncthreads();
      if (pass == 0) tick();
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        if (k + RD - 1 < NCH) issue(ring[(k + RD - 1) % RD], k + RD - 1);
        if (k + 1 < NCH) stage(k + 1);
        if (P.stage != 2) {  // (diagnostic 2: no MFMAs)
          if (kh) compute(k, std::true_type{});
          else compute(k, std::false_type{});
        }
        __syncthreads();
        if (pass == 0 && (k & 1)) tick();
      }
      acc[0] += acc1[0]; acc[1] += acc1[1]; acc[2] += acc1[2]; acc[3] += acc1[3];
      if (kh) {
        red[wave * 64 + lane] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        __syncthreads();
        if (kp == 0) {
          const float4 o = red[(wave + 2) * 64 + lane];
          acc[0] += o.x; acc[1] += o.y; acc[2] += o.z; acc[3] += o.w;
          epi(tw, acc);
        }
      } else if (t < nt) {
        epi(t, acc);
      }
      __syncthreads();  // the chunk buffers (sa) and red are reused by the next pass / conv / step
    }
  };
  const bool staged = ST && nt >= 2;

  // conv1 is linear in its input A[src] = P[src] + w0 x_t[src] + temb_s (pva.py:227-230; the conv taps cut at
  // the utterance edges), so for the staged groups it is split once per flow:
  //   conv1[m, n] = CP[m, n] + sum_tap valid(m, tap) (x_t[m + tap - 1] U[tap][n] + V_s[tap][n])
  // with CP = conv1 of the constant P rows (one MFMA pass here, kept in registers in the accumulator layout),
  // U[tap][n] = W1[n, tap, :] . w0 (once) and V_s[tap][n] = W1[n, tap, :] . temb_s (per step, 48 dots of D).  A
  // step's conv1 is then elementwise; the sums are regrouped (fp32 rounding apart, inside the parity bar).
  f32x4 cp[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  // dot of weight column c, tap `tap` with an LDS vector v over D (the W1 panel is 16-B-chunk swizzled by column)
  auto w1dot = [&](int tap, int cc, const float* v, int d0, int d1) {
    float acc = 0.f;
    for (int d = d0; d < d1; d += 4) {
      const int k = tap * D + d;
      const float4 w = *reinterpret_cast<const float4*>(W1 + cc * K1 + 4 * ((k >> 2) ^ (cc & 15)));
      const float4 x = *reinterpret_cast<const float4*>(v + d);
      acc = fmaf(w.x, x.x, acc);
      acc = fmaf(w.y, x.y, acc);
      acc = fmaf(w.z, x.z, acc);
      acc = fmaf(w.w, x.w, acc);
    }
    return acc;
  };
  if (staged) {
    conv_st(W1, K1, std::integral_constant<int, D>{},
            [&](int r, int ch) {  // r < 0: past the range (zeros)
              return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rP, r < 0 ? 0xfffffff0u : (unsigned)((r * D + ch) * 4), 0, 0));
            },
            [&](int, int, float4 p) { return p; },
            [&](int t, const f32x4& acc) { cp[t >= 4 ? 1 : 0] = acc; }, [] {});
    if (tid < 3 * kCols) uv[tid] = w1dot(tid / kCols, tid % kCols, vw0, 0, D);
    __syncthreads();
  }

  for (int s = 0; s < P.nfe; ++s) {
#ifdef FL_STAMPS
    int pst_k = 0;
#endif
    if (s == P.inject_step) {  // diagnostic failure injection
      if (tid == 0) raise_err(errw, fails);
      leave(false);
      return;
    }
    for (int i = tid; i < D; i += kThreads) vte[i] = N.temb[(size_t)s * D + i];
    if (nt == 1)  // conv1's P window rows (constant, but the staging area is shared with conv2's rows)
      for (int i = tid; i < nw * (D / 4); i += kThreads) {
        const int row = i / (D / 4), c4 = i - row * (D / 4), rr = xa + row;
        *reinterpret_cast<float4*>(sa + row * (F + 4) + 4 * c4) =
            (rr >= 0 && rr < M) ? ld4(N.P + (size_t)rr * D + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    __syncthreads();
    PVST();

    // ---- conv1 (pva.py:221-230: proj(cat(x_t, enc)) + temb -> Conv k3 -> ReLU) + LN1 partials
    auto epi1 = [&](int t, const f32x4& acc) {
#pragma unroll
           for (int i = 0; i < 4; ++i) {
             const int row = 16 * t + 4 * q + i;
             const float v = fmaxf(acc[i] + bias1, 0.f);
             if (row < nr) st4_wt(rR1, (unsigned)(((r0 + row) * F + col0 + c) * 4), v);
             const float mean = wave_sum16(v) * (1.0f / kCols);
             const float d = v - mean;
             const float m2 = wave_sum16(d * d);
             if (c == 0 && row < nr) st8_wt(rS1, (unsigned)(((r0 + row) * CS + cs) * 8), mean, m2);
           }
         };
    if (staged) {
      // V_s: 48 dots of D = 192, four threads per dot (quarters of D, combined in order by shuffles)
      if (tid < 4 * 3 * kCols) {
        const int o = tid >> 2, part = tid & 3;
        float v = w1dot(o / kCols, o % kCols, vte, part * (D / 4), (part + 1) * (D / 4));
        const float v1 = __shfl_xor(v, 1);
        v = (part & 1) ? v1 + v : v + v1;  // (p0 + p1), (p2 + p3) in every lane of the pair
        const float v2 = __shfl_xor(v, 2);
        v = (part & 2) ? v2 + v : v + v2;  // (p0 + p1) + (p2 + p3)
        if (part == 0) uv[3 * kCols + o] = v;
      }
      __syncthreads();
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        const int t = wave + 4 * ti;
        if (t >= nt) break;
        f32x4 acc = cp[ti];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 16 * t + 4 * q + i, m = r0 + row;
          const int lm = m < M ? m % L : 0;
          float sum = 0.f;
#pragma unroll
          for (int tap = 0; tap < 3; ++tap) {
            const int l = lm + tap - 1;
            const float x = xs[row + tap];  // window index of frame m + tap - 1 (xa = r0 - 1)
            const float term = fmaf(x, uv[tap * kCols + c], uv[3 * kCols + tap * kCols + c]);
            sum += (m < r0 + nr && l >= 0 && l < L) ? term : 0.f;
          }
          acc[i] += sum;
        }
        epi1(t, acc);
      }
    } else {
    conv(W1, K1, std::integral_constant<int, NB1>{},
         [&](int t) {
           const int m = r0 + 16 * t + c;
           const bool live = m < r0 + nr;
           return AConv1<D>{N.P, vw0, vte, xs, m, live ? m % L : 0, L, xa, q, live};
         },
         [&](int t) {
           const int m = r0 + 16 * t + c;
           const bool live = m < r0 + nr;
           return AConv1S<D, F>{sa, vw0, vte, xs, m, live ? m % L : 0, L, xa, q, live};
         },
         epi1);
    }
    PVST();
    signal(h1 + rg * kLine);
    PVST();
    if (!wait3(errw, fails, tmo, h1, rg, P.RG, CS * (s + 1), flag)) { leave(false); return; }
    PVST();

    // LN1 statistics of the window rows from the CS partials (equal-count combine, as the launch path)
    if (tid < nw) {
      const int r = xa + tid;
      float mean = 0.f, rstd = 0.f;
      if (r >= 0 && r < M) {
        float2 pp[CS];  // two partials per 16-B load (CS even)
#pragma unroll
        for (int k = 0; k < CS; k += 2) {
          const float4 v = ld16_sc1(rS1, (unsigned)((r * CS + k) * 8));
          pp[k] = make_float2(v.x, v.y);
          pp[k + 1] = make_float2(v.z, v.w);
        }
        float sm = 0.f;
#pragma unroll
        for (int k = 0; k < CS; ++k) sm += pp[k].x;
        mean = sm / (float)CS;
        float m2 = 0.f;
#pragma unroll
        for (int k = 0; k < CS; ++k) {
          const float d = pp[k].x - mean;
          m2 += pp[k].y + (float)kCols * d * d;
        }
        rstd = 1.0f / sqrtf(m2 / (float)(CS * kCols) + 1e-5f);
      }
      st[2 * tid] = mean;
      st[2 * tid + 1] = rstd;
    }
    __syncthreads();
    if (nt == 1) {  // conv2's window rows, LayerNorm_1 applied (Layers: Conv -> ReLU -> LN -> Conv)
      for (int i = tid; i < nw * (F / 4); i += kThreads) {
        const int row = i / (F / 4), c4 = i - row * (F / 4), rr = xa + row;
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rr >= 0 && rr < M) {
          const float4 v = ld16_sc1(rR1, (unsigned)((rr * F + 4 * c4) * 4));
          const float mean = st[2 * row], rstd = st[2 * row + 1];
          const float4 g = *reinterpret_cast<const float4*>(vg1 + 4 * c4);
          const float4 b = *reinterpret_cast<const float4*>(vb1 + 4 * c4);
          o = make_float4(((v.x - mean) * rstd) * g.x + b.x, ((v.y - mean) * rstd) * g.y + b.y,
                          ((v.z - mean) * rstd) * g.z + b.z, ((v.w - mean) * rstd) * g.w + b.w);
        }
        *reinterpret_cast<float4*>(sa + row * (F + 4) + 4 * c4) = o;
      }
      __syncthreads();
    }
    PVST();

    // ---- conv2 (Conv k3 over LN1 -> ReLU) + head partials over the slice
    auto epi2 = [&](int t, const f32x4& acc) {
#pragma unroll
           for (int i = 0; i < 4; ++i) {
             const int row = 16 * t + 4 * q + i;
             const float v = fmaxf(acc[i] + bias2, 0.f);
             const float mean = wave_sum16(v) * (1.0f / kCols);
             const float d = v - mean;
             const float m2 = wave_sum16(d * d);
             const float sg = wave_sum16(d * gl);
             if (c == 0 && row < nr) st16_wt(rS2, (unsigned)(((r0 + row) * CS + cs) * 16), make_float4(mean, m2, sg, 0.f));
           }
         };
    if (staged) {
      conv_st(W2, K2, std::integral_constant<int, F>{},
              [&](int r, int ch) { return ld16_sc1(rR1, r < 0 ? 0xfffffff0u : (unsigned)((r * F + ch) * 4)); },
              [&](int row, int ch, float4 v) {
                const float mean = st[2 * row], rstd = st[2 * row + 1];
                const float4 g = *reinterpret_cast<const float4*>(vg1 + ch);
                const float4 b = *reinterpret_cast<const float4*>(vb1 + ch);
                return make_float4(((v.x - mean) * rstd) * g.x + b.x, ((v.y - mean) * rstd) * g.y + b.y,
                                   ((v.z - mean) * rstd) * g.z + b.z, ((v.w - mean) * rstd) * g.w + b.w);
              },
              epi2, [&] { PVST(); });
    } else {
    conv(W2, K2, std::integral_constant<int, NB2>{},
         [&](int t) {
           const int m = r0 + 16 * t + c;
           const bool live = m < r0 + nr;
           return AConv2<F>{rR1, st, vg1, vb1, m, live ? m % L : 0, L, xa, q, live};
         },
         [&](int t) {
           const int m = r0 + 16 * t + c;
           const bool live = m < r0 + nr;
           return AConv2S<F>{sa, m, live ? m % L : 0, L, xa, q, live};
         },
         epi2);
    }
    PVST();
    signal(h2 + rg * kLine);
    PVST();
    if (!wait3(errw, fails, tmo, h2, rg, P.RG, CS * (s + 1), flag)) { leave(false); return; }
    PVST();

    // ---- head (LN2 . lw + lb, masked_fill) + Euler update of the window rows (pva.py:104-109, 234-238)
    if (tid < nw) {
      const int r = xa + tid;
      if (r >= 0 && r < M) {
        float4 pp[CS];
#pragma unroll
        for (int k = 0; k < CS; ++k) pp[k] = ld16_sc1(rS2, (unsigned)((r * CS + k) * 16));
        float sm = 0.f;
#pragma unroll
        for (int k = 0; k < CS; ++k) sm += pp[k].x;
        const float mean = sm / (float)CS;
        float m2 = 0.f;
#pragma unroll
        for (int k = 0; k < CS; ++k) {
          const float d = pp[k].x - mean;
          m2 += pp[k].y + (float)kCols * d * d;
        }
        const float rstd = 1.0f / sqrtf(m2 / (float)F + 1e-5f);
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < CS; ++k) dot += pp[k].z + (pp[k].x - mean) * gs[k];
        const float vel = P.mask[r] ? 0.f : (rstd * dot + gs[CS]) + lb;
        xs[tid] = __fadd_rn(xs[tid], __fmul_rn(P.dt, vel));
      }
    }
    __syncthreads();
    PVST();
  }
  if (cs == 0)
    for (int i = tid; i < nr; i += kThreads) N.xt[r0 + i] = xs[i + 1];
  leave(true);
}

size_t pva_persist_lds() { return (size_t)Lds<192, 384>::BYTES; }

bool pva_persist_device_ok(int device, int grid) {
  int cus = 0, nb = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < grid) return false;
  for (const void* k : {reinterpret_cast<const void*>(pva_persist_kernel<192, 384, true>),
                        reinterpret_cast<const void*>(pva_persist_kernel<192, 384, false>)}) {
    if (set_max_lds(k) != hipSuccess) return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kThreads, Lds<192, 384>::BYTES) != hipSuccess || nb < 1)
      return false;
  }
  return true;
}

int pva_persist_launch(const Params& Pin, hipStream_t st) {
  Params P = Pin;
#ifdef FL_STAMPS
  P.pst = g_pva_pst;
  P.pst_step = g_pva_pst_step;
#endif
  P.grid = 2 * Lds<192, 384>::CS * P.RG;
  // cooperative: the runtime checks the grid against the occupancy and refuses it up front; a captured
  // cooperative launch replays cooperatively
  void* args[] = {&P};
  const void* kern = P.stage ? reinterpret_cast<const void*>(pva_persist_kernel<192, 384, true>)
                             : reinterpret_cast<const void*>(pva_persist_kernel<192, 384, false>);
  // tune coop 0: plain launch (profiling, README "Known issues"); residency checked by pva_persist_eligible
  const hipError_t e = tn().coop ? hipLaunchCooperativeKernel(kern, dim3(P.grid), dim3(kThreads), args, Lds<192, 384>::BYTES, st)
                                 : hipLaunchKernel(kern, dim3(P.grid), dim3(kThreads), args, Lds<192, 384>::BYTES, st);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error("persistent PVA flow: hipLaunchCooperativeKernel -> %s", hipGetErrorString(e));
    return e == hipErrorCooperativeLaunchTooLarge ? kBadArg : kHip;
  }
  return kOk;
}

}  // namespace pv
}  // namespace fl

#ifdef FL_STAMPS
extern "C" FLAMED_API int flamed_pva_stamps(void* buf, int step) {
  fl::pv::g_pva_pst = reinterpret_cast<unsigned long long*>(buf);
  fl::pv::g_pva_pst_step = step;
  return fl::kOk;
}
#endif
