// Persistent B = 1 Euler solve kernel (design notes: persist.hpp).
#include <cstdio>
#include <cstdlib>

#include "flamed_hip.h"
#include "flamed_diag.h"
#include "persist.hpp"
#include "gemm_dma.hpp"

namespace fl {
namespace pk {

// Diagnostic build only (FL_STAMPS, libflamed_hip_stamps.so): thread 0 of every workgroup records
// s_memrealtime (100 MHz, chip-wide) at each wait / compute / signal point of one chosen step into
// g_pst[workgroup][k] (flamed_persist_stamps; tools/persist_timeline.py).
#ifdef FL_STAMPS
constexpr int kStampSlots = 160;
#define PST(step)                                                                                       \
  do {                                                                                                  \
    if ((step) == P.pst_step && P.pst && threadIdx.x == 0 && pst_k < kStampSlots)                       \
      P.pst[blockIdx.x * kStampSlots + pst_k] = __builtin_amdgcn_s_memrealtime();                      \
    ++pst_k;                                                                                            \
  } while (0)
// the address of the next stamp slot (or null), for a stamp taken inside a helper
#define PSTP(step) \
  (((step) == P.pst_step && P.pst && pst_k < kStampSlots) ? P.pst + blockIdx.x * kStampSlots + pst_k++ : (++pst_k, nullptr))
// GroupNorm exchange dump (flamed_persist_gndump): lane tid < 32 of workgroup (g, s), hand-off blk of step gnd_step
#define GND(k, v)                                                                                       \
  do {                                                                                                  \
    if (cur_step == P.gnd_step && P.gnd)                                                                \
      P.gnd[(((size_t)blk * kWGs + g * kSlots + s) * 32 + (tid & 31)) * 32 + (k)] = (v);                \
  } while (0)
#else
#define GND(k, v) ((void)0)
#define PST(step) ((void)0)
#define PSTP(step) nullptr
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
// write-through (sc1) 16-B store / sc1 16-B load (aux 16 = sc1)
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
// plain 16-B store: the line stays in this XCD's L2 (group-local hand-offs when groups are XCDs)
__device__ __forceinline__ void st16p(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ float4 as_f4(u32x4 v) { return __builtin_bit_cast(float4, v); }
// An opaque copy of a lane index: address arithmetic derived from it is computed where it is used, inside
// the step loop, instead of being hoisted into hundreds of loop-invariant registers (LDS fragment
// offsets, DMA source addresses of every phase).
__device__ __forceinline__ int opq(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Row range of group g.  Default: ceil(T / 8) consecutive frames per group (T = 400: 50 rows each, the last
// groups short or empty).  persist_opt bit 2: whole 16-row tiles, group gi of an utterance taking tiles
// [gi MT / gpu, (gi + 1) MT / gpu) (T = 400: seven 48-row groups and one 64-row group); measured faster (r05bm:
// 20.7 vs 21.1 ms at B = 1 T = 400) but not default yet (csrc/common.hpp Tune::persist_opt).  Rows
// past nr in a wave's last 16-row fragment read as zero through the buffer range and are never stored.
// Several utterances (B = 2, 4 or 8, each of T frames; rows u T .. u T + T - 1): utterance u owns the 8 / B
// groups u 8/B .. + 8/B - 1 and splits its frames among them the same way, so a group never spans two
// utterances (its modulation row, GroupNorm statistics and zero padding are its utterance's).
__device__ __forceinline__ void group_rows(int g, int T, int B, int& r0, int& nr, int opt) {
  const int gpu = kGroups / B, u = g / gpu, gi = g - u * gpu;
  if (opt & 2) {  // whole 16-row tiles [gi MT / gpu, (gi + 1) MT / gpu) of the utterance
    const int MT = (T + 15) >> 4;
    const int tb = gi * MT / gpu, te = (gi + 1) * MT / gpu;
    r0 = u * T + 16 * tb;
    nr = max(min(16 * te, T) - 16 * tb, 0);
    return;
  }
  const int R = (T + gpu - 1) / gpu;
  r0 = u * T + gi * R;
  nr = max(min(R, T - gi * R), 0);
}

// ---- hand-off primitives ----
// Every storing wave drains its (sc1) stores, the workgroup meets, one lane adds to the counter.
__device__ __forceinline__ void signal(int* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The same signal issued AFTER the next phase's weight DMA (persist_opt 4096): vmcnt counts loads, stores and
// LDS-DMA together in issue order, so waiting until only this wave's kDma youngest operations (its DMA pieces)
// are outstanding drains exactly the older hand-off stores -- the drain's round trip overlaps the DMA issue
// instead of preceding it, and the DMA stays in flight across the barrier.
template <int kDma>
__device__ __forceinline__ void signal_dma(int* ctr) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kDma) : "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Abandon the solve: the first workgroup to set the error word also counts the failed launch in the sticky
// word the host reads later (the per-launch counter block is zeroed before every launch, `fails` is not).
__device__ __forceinline__ void raise_err(int* err, int* fails, int code) {
  int expected = 0;
  if (__hip_atomic_compare_exchange_strong(err, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    __hip_atomic_fetch_add(fails, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 polls n counters (base + k * stride, k < n) with sc1 loads until all reach `target` (s_sleep
// between polls); bounded by P.tmo, and an error word set by any workgroup ends every wait.  The
// other waves meet it at a barrier.  Returns false when the solve is being abandoned.
__device__ __forceinline__ bool wait_ge(int* err, int* fails, long long tmo, int* base, int stride, int n, int target, int* flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    for (unsigned it = 0;; ++it) {
      bool mine = true;
      if (lane < n) mine = __hip_atomic_load(base + lane * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
      // the last lane watches the error word in the same poll: a wait whose counters are already complete still
      // stops once any workgroup has given the launch up (a deferred seal check, persist_opt 65536, fails
      // without stalling anyone)
      else if (lane == 63) mine = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
      if (__all(mine)) break;
      if ((it & 31) == 31) {  // the error word and the clock only every 32 polls: one round trip per poll
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) { ok = false; break; }
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > tmo) {
          if (lane == 0) raise_err(err, fails, 1);
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
  __syncthreads();  // the flag word is rewritten by the next wait
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: hand-off loads stay below the poll
  return ok;
}

// The reset prologue's grid-wide arrival: wave 0 polls a monotonic (wrapping) ticket counter until it has
// reached `target` (no error word yet: the counter block is being reset); a timeout leaves the launch.
__device__ __forceinline__ bool arrive_wait(unsigned* ctr, unsigned target, long long tmo, int* flag) {
  if (threadIdx.x < 64) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    for (unsigned it = 0;; ++it) {
      if (arrive_reached(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), target)) break;
      if ((it & 31) == 31 && (long long)(__builtin_amdgcn_s_memrealtime() - t0) > tmo) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0) *flag = ok ? 1 : 0;
  }
  __syncthreads();
  const bool ok = *flag != 0;
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: later hand-off loads stay below
  return ok;
}

// Seal check (persist_opt 16384, a verification mode): every producer stores, write-through and ahead of the
// drain that precedes its counter add, the number of the group hand-off it is completing into its seal; a
// consumer that has seen a counter reach hand-off `target` then requires every seal it depends on to show
// >= target.  A seal behind its counter would mean the ordering that the hand-off protocol relies on
// (MI355X_MICROARCH.md, Valid forms row 1) did not hold: the consumer spins on it, and gives the launch up
// (error 4, NaN-poisoned x) if it never arrives.  Wave 0 checks n seals from sp; the others meet it.
__device__ __forceinline__ bool seals_ok(const int* sp, int n, int target, int* err, int* fails, long long tmo, int* flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    for (;;) {
      bool mine = true;
      for (int i = lane; i < n; i += 64)
        mine = mine && __hip_atomic_load(sp + 4 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
      if (__all(mine)) break;
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > tmo) {
        if (lane == 0) raise_err(err, fails, 4);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) *flag = ok ? 1 : 0;
  }
  __syncthreads();
  const bool ok = *flag != 0;
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok;
}

// ---- weight panels: 32 rows (output columns) x K bf16, 16-B chunks XOR-swizzled by row & 15 (the 16
// lanes of a ds_read_b128 group hit 16 distinct 16-B slots); the swizzle is applied to each lane's DMA
// SOURCE chunk (an involution), since LDS-DMA writes a wave's 64 lanes linearly.
template <int K>
__device__ __forceinline__ int woff(int n, int j) { return n * (2 * K) + ((j ^ (n & 15)) << 4); }

template <int K, class RowF>
// Issued by waves 1..3 only: wave 0 goes straight to polling the next hand-off (issuing 64 LDS-DMA
// wave-instructions takes ~1 us of a wave's time), and its vmcnt never waits for weight traffic.
__device__ __forceinline__ void dma_panel(char* dst, RowF rowp, int wave, int lane_in, int opt) {
  constexpr int kRowB = 2 * K, kNI = 32 * kRowB / 1024;
  const int lane = opq(lane_in);
  const bool w4 = opt & 1;  // all four waves issue
  if (wave == 0 && !w4) return;
  for (int i = w4 ? wave : wave - 1; i < kNI; i += w4 ? 4 : 3) {
    const int pos = i * 1024 + lane * 16;
    const int n = pos / kRowB, jl = (pos % kRowB) >> 4;
    glds16(reinterpret_cast<const char*>(rowp(n)) + ((jl ^ (n & 15)) << 4), dst + i * 1024);
  }
}

// The same panel issued by all four waves (persist_opt 1) with the per-piece work cut to the bone: the j loop
// unrolled, the row base a scalar pointer (global_load_lds with saddr) and the lane's 32-bit byte offset
// row n * 2K + swizzled chunk; rowb(n) gives row n's byte offset from `base`.  (The generic loop above
// spent ~1.3 us of every wave per 64 KB panel: 64-bit address math and a rolled loop per piece.)
// w4 = false: waves 1..3 issue (wave 0 goes straight to polling the next hand-off, its vmcnt free of weights).
template <int K, class RowB>
__device__ __forceinline__ void dma_panel4(char* dst, const void* base, RowB rowb, int wave, int lane_in, bool w4 = true) {
  constexpr int kRowB = 2 * K, kNI = 32 * kRowB / 1024;
  static_assert(kNI % 4 == 0, "pieces per wave");
  if (!w4 && wave == 0) return;
  const int w0 = w4 ? wave : wave - 1, ws = w4 ? 4 : 3;
  const int lane = opq(lane_in);
  const unsigned long long b = (unsigned long long)(uintptr_t)base;
  // (readfirstlane returns int: widen through unsigned, or a low word >= 2^31 sign-extends into the high one)
  const unsigned blo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned bhi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const unsigned long long bs = ((unsigned long long)bhi << 32) | (unsigned long long)blo;
  const unsigned l0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)(dst)));
#pragma unroll
  for (int j = 0; j < (kNI + 2) / 3; ++j) {
    const int i = w0 + ws * j;
    if (i >= kNI) break;
    const unsigned pos = (unsigned)i * 1024u + (unsigned)lane * 16u;
    const int n = (int)(pos / kRowB);
    const unsigned jl = (pos % kRowB) >> 4;
    const unsigned off = rowb(n) + ((jl ^ (unsigned)(n & 15)) << 4);
    const unsigned l = l0 + (unsigned)i * 1024u;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(off), "s"(bs), "s"(l)
                 : "memory");
  }
}

// ---- one GEMM phase: wave w < ntile computes rows [16 w, 16 w + 16) of the group's tile x the slot's 32
// columns: A (bf16 rows, K) straight to registers with sc1 loads (rows >= nr read as 0: buffer range),
// B fragments from the LDS weight panel.  The MFMA takes the weight fragment as its A operand and the activation
// fragment as its B operand (D = W . A^T), so lane (c, q) ends up holding TRANSPOSED output: acc[nt][r] = row c of
// the tile, column 16 nt + 4 q + r -- one row and 4 consecutive columns per 16-column half, the consumer's fragment
// order in 8-byte pieces (store_op_t), so no epilogue stages through LDS.  Same products, same K order: swapping
// the operands changes only where the results land.
// Fragment-major A image (persist_opt 64): group g's rows as [tile t < 4][K-step ks][lane][8 bf16], lane =
// (row c, K-quarter q) exactly as a v_mfma_f32_16x16x32_bf16 A operand takes it, so a wave's 16-B/lane load
// of one K-step is ONE contiguous 1 KB (8 full lines) instead of 16 half-lines of 16 rows; rows past the
// group's last row are stored as zeros.
__device__ __forceinline__ unsigned frag_group_bytes(int KST) { return (unsigned)(4 * kMaxNTW * KST * 1024); }

template <int K>
// tile: the group's 16-row tile this wave multiplies (wave + 4 i for chunk i); first: the phase's first tile,
// which waits for the weight panel's DMA and meets the other waves (the panel is then in LDS for the rest).
__device__ __forceinline__ void gemm(const bf16* A, int r0, int nr, const char* wl, f32x4 (&acc)[2], int wave, int lane_in,
                                     unsigned long long* stamp = nullptr, int g = 0, bool frag = false, int tile = -1,
                                     bool first = true) {
  constexpr int KST = K / 32;
  const int lane = opq(lane_in);
  if (tile < 0) tile = wave;
  acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntile = (nr + 15) >> 4;
  const int c = lane & 15, q = lane >> 4;
  u32x4 a[KST];
  if (tile < ntile) {
    if (frag) {
      const __amdgpu_buffer_rsrc_t rs =
          rsrc(reinterpret_cast<const char*>(A) + (size_t)g * frag_group_bytes(KST), frag_group_bytes(KST));
      const unsigned base = (unsigned)(((tile * KST) * 64 + lane) * 16);
#pragma unroll
      for (int ks = 0; ks < KST; ++ks) a[ks] = ld16(rs, base + ks * 1024);
    } else {
      const __amdgpu_buffer_rsrc_t rs = rsrc(A + (size_t)r0 * K, (unsigned)nr * K * 2);
      const unsigned base = (unsigned)(((16 * tile + c) * K + q * 8) * 2);
#pragma unroll
      for (int ks = 0; ks < KST; ++ks) a[ks] = ld16(rs, base + ks * 64);
    }
    if (first) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(KST) : "memory");  // this wave's (older) weight DMA landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (first) __syncthreads();  // every wave's DMA: the whole panel is in LDS
  if (first && stamp && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();  // FL_STAMPS timeline only
  if (tile < ntile) {
    // B fragments read kBP K-steps ahead of the MFMAs that consume them (a ring of registers), so the
    // LDS latency overlaps the matrix pipe instead of one lgkmcnt(0) per MFMA
    constexpr int kBP = 4;
    u32x4 b0[kBP], b1[kBP];
#pragma unroll
    for (int p = 0; p < kBP; ++p) {
      b0[p] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * p + q));
      b1[p] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * p + q));
    }
#pragma unroll
    for (int ks = 0; ks < KST; ++ks) {
      const u32x4 x0 = b0[ks % kBP], x1 = b1[ks % kBP];
      if (ks + kBP < KST) {
        b0[ks % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * (ks + kBP) + q));
        b1[ks % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * (ks + kBP) + q));
      }
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x0), __builtin_bit_cast(bf16x8, a[ks]), acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x1), __builtin_bit_cast(bf16x8, a[ks]), acc[1], 0, 0, 0);
    }
  }
}

// Several chunks (NTW > 1): every tile of the wave (wave + 4 i) in one pass, the A fragments streamed in half-tile
// units (K / 2 deep) through a two-unit register ring, so the next unit's loads are in flight during this unit's
// MFMAs (and no epilogue stores sit in the wave's vmcnt queue between them: the epilogues run after the pass).
// Per tile the K-steps accumulate in the same order as gemm(): bitwise the same products.
template <int K, int NTW>
__device__ __forceinline__ void gemm_multi(const bf16* A, int r0, int nr, const char* wl, f32x4 (&acc)[NTW][2], int wave,
                                           int lane_in, unsigned long long* stamp, int g, bool frag) {
  constexpr int KST = K / 32, KU = KST / 2, U = 2 * NTW;
  static_assert(KST % 2 == 0, "half-tile units");
  const int lane = opq(lane_in);
  const int ntile = (nr + 15) >> 4;
  const int c = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rs = frag ? rsrc(reinterpret_cast<const char*>(A) + (size_t)g * frag_group_bytes(KST), frag_group_bytes(KST))
                                         : rsrc(A + (size_t)r0 * K, (unsigned)nr * K * 2);
  u32x4 a[2][KU];
  auto load = [&](u32x4 (&dst)[KU], int u) __attribute__((always_inline)) {
    const int tile = wave + 4 * (u >> 1), k0 = (u & 1) * KU;
    if (tile >= ntile) return;
    if (frag) {
      const unsigned base = (unsigned)(((tile * KST + k0) * 64 + lane) * 16);
#pragma unroll
      for (int ks = 0; ks < KU; ++ks) dst[ks] = ld16(rs, base + ks * 1024);
    } else {
      const unsigned base = (unsigned)(((16 * tile + c) * K + k0 * 32 + q * 8) * 2);
#pragma unroll
      for (int ks = 0; ks < KU; ++ks) dst[ks] = ld16(rs, base + ks * 64);
    }
  };
  load(a[0], 0);
  if (wave < ntile) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(KU) : "memory");  // this wave's (older) weight DMA landed
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's DMA: the whole panel is in LDS
  if (stamp && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();  // FL_STAMPS timeline only
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int tile = wave + 4 * (u >> 1), k0 = (u & 1) * KU;
    const bool next = u + 1 < U && wave + 4 * ((u + 1) >> 1) < ntile;
    if (u + 1 < U) load(a[(u + 1) & 1], u + 1);
    if (next) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(KU) : "memory");  // this unit's loads (older) have landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f32x4(&ac)[2] = acc[u >> 1];
    if (k0 == 0) {
      ac[0] = f32x4{0.f, 0.f, 0.f, 0.f};
      ac[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (tile < ntile) {
      constexpr int kBP = 4;
      u32x4 b0[kBP], b1[kBP];
#pragma unroll
      for (int p = 0; p < kBP; ++p) {
        b0[p] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * (k0 + p) + q));
        b1[p] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * (k0 + p) + q));
      }
#pragma unroll
      for (int ks = 0; ks < KU; ++ks) {
        const u32x4 x0 = b0[ks % kBP], x1 = b1[ks % kBP];
        if (ks + kBP < KU) {
          b0[ks % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * (k0 + ks + kBP) + q));
          b1[ks % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * (k0 + ks + kBP) + q));
        }
        const u32x4 av = a[u & 1][ks];
        ac[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x0), __builtin_bit_cast(bf16x8, av), ac[0], 0, 0, 0);
        ac[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x1), __builtin_bit_cast(bf16x8, av), ac[1], 0, 0, 0);
      }
    }
  }
}

// Several chunks, one gemm() per chunk (persist_opt 262144, A/B against gemm_multi): each chunk's whole A tile is in
// flight at once (32 loads per wave) before its MFMAs, the panel already in LDS after the first chunk.
template <int K, int NTW>
__device__ __forceinline__ void gemm_seq(const bf16* A, int r0, int nr, const char* wl, f32x4 (&acc)[NTW][2], int wave,
                                         int lane_in, unsigned long long* stamp, int g, bool frag) {
#pragma unroll
  for (int ci = 0; ci < NTW; ++ci) gemm<K>(A, r0, nr, wl, acc[ci], wave, lane_in, ci == 0 ? stamp : nullptr, g, frag, wave + 4 * ci, ci == 0);
}

// Several chunks, K-outer (persist_opt 524288): K-step by K-step over every tile of the wave, so each pair of B
// fragments read from LDS feeds all NTW tiles (the panel is read once per wave per phase, not NTW times) and the
// A fragments stream through a ring D K-steps deep (D NTW 16-B loads in flight, <= 128 VGPRs), the loads of every
// chunk overlapping the MFMAs of every other.  Tiles past the group's last one load from outside the buffer range
// (zeros, no memory traffic) so every K-step issues the same NTW loads.  Per tile the K-steps accumulate in the
// same order as gemm(): bitwise the same products.
// Ring depth (K-steps in flight) per chunk count, measured (r06y/r06z, same box, ms per solve): NTW = 5 depth 3
// (T = 2400: 109.4-110.2 vs 110.8 at 4, 111.5 at 2, 126.9 at 6), NTW = 4 depth 5 (B = 4 T = 400: 42.9 vs 44.6 at
// 4, 47.1 at 8, 44.9 at 6), NTW = 3 depth 7 (r06an: T = 1500 35.05-35.09 ms vs 35.6-36.0 at 8, 37.7-37.9 at 10; r06aa: 8 vs 35.9 at 6,
// 36.7-37.0 at 4), NTW = 2
// depth 8 (r06ag / r06ah: B = 2 T = 400 25.3-25.7 ms vs 26.2 at 10 and 7, 25.7-25.9 at 9, 26.6-26.7 at 6),
// NTW = 6..8 depth 2 (r06ad: 3 is 4-5 % slower); deeper rings spill.  Overridable per chunk count for A/B builds.
#ifndef FL_KO_D2
#define FL_KO_D2 8
#endif
#ifndef FL_KO_D3
#define FL_KO_D3 7
#endif
#ifndef FL_KO_D4
#define FL_KO_D4 5
#endif
#ifndef FL_KO_D5
#define FL_KO_D5 3
#endif
#ifndef FL_KO_D6
#define FL_KO_D6 2  // NTW = 6..8 (B x T up to 4096)
#endif
template <int K, int NTW>
__device__ __forceinline__ void gemm_ko(const bf16* A, int r0, int nr, const char* wl, f32x4 (&acc)[NTW][2], int wave,
                                        int lane_in, unsigned long long* stamp, int g, bool frag) {
  constexpr int KST = K / 32, D0 = NTW == 2 ? FL_KO_D2 : NTW == 3 ? FL_KO_D3 : NTW == 4 ? FL_KO_D4 : NTW == 5 ? FL_KO_D5 : FL_KO_D6;
  constexpr int D = D0 > KST ? KST : D0;
  const int lane = opq(lane_in);
  const int ntile = (nr + 15) >> 4;
  const int c = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rs = frag ? rsrc(reinterpret_cast<const char*>(A) + (size_t)g * frag_group_bytes(KST), frag_group_bytes(KST))
                                         : rsrc(A + (size_t)r0 * K, (unsigned)nr * K * 2);
  const unsigned oob = 0x7ff00000u;
  unsigned base[NTW];
#pragma unroll
  for (int ci = 0; ci < NTW; ++ci) {
    const int tile = wave + 4 * ci;
    base[ci] = tile >= ntile ? oob
               : frag        ? (unsigned)(((tile * KST) * 64 + lane) * 16)
                             : (unsigned)(((16 * tile + c) * K + q * 8) * 2);
  }
  const unsigned kstride = frag ? 1024u : 64u;
  u32x4 a[D][NTW];
#pragma unroll
  for (int p = 0; p < D - 1; ++p)
#pragma unroll
    for (int ci = 0; ci < NTW; ++ci) a[p][ci] = ld16(rs, base[ci] + p * kstride);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"((D - 1) * NTW) : "memory");  // this wave's (older) weight DMA landed
  __syncthreads();  // every wave's DMA: the whole panel is in LDS
  if (stamp && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();  // FL_STAMPS timeline only
#pragma unroll
  for (int ci = 0; ci < NTW; ++ci) acc[ci][0] = acc[ci][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int kBP = 4;
  u32x4 b0[kBP], b1[kBP];
#pragma unroll
  for (int p = 0; p < kBP; ++p) {
    b0[p] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * p + q));
    b1[p] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * p + q));
  }
#pragma unroll
  for (int ks = 0; ks < KST; ++ks) {
    if (ks + D - 1 < KST)
#pragma unroll
      for (int ci = 0; ci < NTW; ++ci) a[(ks + D - 1) % D][ci] = ld16(rs, base[ci] + (ks + D - 1) * kstride);
    const u32x4 x0 = b0[ks % kBP], x1 = b1[ks % kBP];
    if (ks + kBP < KST) {
      b0[ks % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * (ks + kBP) + q));
      b1[ks % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * (ks + kBP) + q));
    }
#pragma unroll
    for (int ci = 0; ci < NTW; ++ci) {
      if (wave + 4 * ci < ntile) {
        const u32x4 av = a[ks % D][ci];
        acc[ci][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x0), __builtin_bit_cast(bf16x8, av), acc[ci][0], 0, 0, 0);
        acc[ci][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x1), __builtin_bit_cast(bf16x8, av), acc[ci][1], 0, 0, 0);
      }
    }
  }
}

// A multi-chunk GEMM phase (NTW > 1): the K-outer gemm_ko (persist_opt 524288, default), else the per-chunk sequence
// (262144) or the streamed gemm_multi -- A/B variants for up to five chunks only (6..8 always take gemm_ko).  Compiling
// the alternatives out of the 2..5-chunk kernels (-DFL_KO_ONLY) changes their register allocation, not for the better:
// T = 2400 115.0 vs 106.6 ms, B = 4 T = 400 43.6 vs 42.8, B = 2 T = 400 25.9 vs 26.0-26.5 (r06ae, same box).
template <int K, int NTW>
__device__ __forceinline__ void gemm_chunks(const bf16* A, int r0, int nr, const char* wl, f32x4 (&acc)[NTW][2], int wave,
                                            int lane_in, unsigned long long* stamp, int g, bool frag, int opt) {
#ifdef FL_KO_ONLY
  constexpr bool only = true;
#else
  constexpr bool only = NTW > 5;
#endif
  if constexpr (only) {
    gemm_ko<K, NTW>(A, r0, nr, wl, acc, wave, lane_in, stamp, g, frag);
  } else {
    if (opt & 524288) gemm_ko<K, NTW>(A, r0, nr, wl, acc, wave, lane_in, stamp, g, frag);
    else if (opt & 262144) gemm_seq<K, NTW>(A, r0, nr, wl, acc, wave, lane_in, stamp, g, frag);
    else gemm_multi<K, NTW>(A, r0, nr, wl, acc, wave, lane_in, stamp, g, frag);
  }
}

// The same product with the work split 2 x 2 (persist_opt 1024): wave w = (pair p, half h) multiplies row tiles
// 2p and 2p + 1 by K-steps [h KST/2, (h + 1) KST/2), so each B fragment read from LDS feeds two row tiles and
// the panel is read twice per workgroup instead of four times; the two halves of tile w are then summed
// through LDS (K-half 0 + K-half 1, the same order in every wave: deterministic) and wave w holds row tile w
// exactly where gemm() leaves it.
template <int K>
__device__ __forceinline__ void gemm_kh(const bf16* A, int r0, int nr, char* wl, f32x4 (&acc)[2], int wave, int lane_in,
                                        unsigned long long* stamp = nullptr, int g = 0, bool frag = false) {
  constexpr int KST = K / 32, KH = KST / 2;
  const int lane = opq(lane_in);
  const int ntile = (nr + 15) >> 4;
  const int c = lane & 15, q = lane >> 4;
  const int tp = wave >> 1, kh = wave & 1, t0 = 2 * tp;
  const int k0 = __builtin_amdgcn_readfirstlane(kh * KH);
  u32x4 a[2][KH];
  if (frag) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(reinterpret_cast<const char*>(A) + (size_t)g * frag_group_bytes(KST), frag_group_bytes(KST));
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int kk = 0; kk < KH; ++kk) a[t][kk] = ld16(rs, (unsigned)((((t0 + t) * KST + k0 + kk) * 64 + lane) * 16));
  } else {
    const __amdgpu_buffer_rsrc_t rs = rsrc(A + (size_t)r0 * K, (unsigned)nr * K * 2);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int kk = 0; kk < KH; ++kk) a[t][kk] = ld16(rs, (unsigned)(((16 * (t0 + t) + c) * K + (k0 + kk) * 32 + q * 8) * 2));
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * KH) : "memory");  // this wave's (older) weight DMA landed
  __syncthreads();  // every wave's DMA: the whole panel is in LDS
  if (stamp && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();  // FL_STAMPS timeline only
  f32x4 p[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) p[t][0] = p[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool use0 = t0 < ntile, use1 = t0 + 1 < ntile;
  constexpr int kBP = 4;
  u32x4 b0[kBP], b1[kBP];
#pragma unroll
  for (int pp = 0; pp < kBP; ++pp) {
    b0[pp] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * (k0 + pp) + q));
    b1[pp] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * (k0 + pp) + q));
  }
#pragma unroll
  for (int kk = 0; kk < KH; ++kk) {
    const u32x4 x0 = b0[kk % kBP], x1 = b1[kk % kBP];
    if (kk + kBP < KH) {
      b0[kk % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(c, 4 * (k0 + kk + kBP) + q));
      b1[kk % kBP] = *reinterpret_cast<const u32x4*>(wl + woff<K>(16 + c, 4 * (k0 + kk + kBP) + q));
    }
    if (use0) {
      p[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x0), __builtin_bit_cast(bf16x8, a[0][kk]), p[0][0], 0, 0, 0);
      p[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x1), __builtin_bit_cast(bf16x8, a[0][kk]), p[0][1], 0, 0, 0);
    }
    if (use1) {
      p[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x0), __builtin_bit_cast(bf16x8, a[1][kk]), p[1][0], 0, 0, 0);
      p[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x1), __builtin_bit_cast(bf16x8, a[1][kk]), p[1][1], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave has read the panel: its buffer now carries the partials
  f32x4* red = reinterpret_cast<f32x4*>(wl);  // [tile][K-half][nt][lane]
  const int other = t0 + (1 - kh);             // the tile whose other half this wave computed
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) red[((other * 2 + kh) * 2 + nt) * 64 + lane] = p[1 - kh][nt];
  __syncthreads();
  acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (wave < ntile) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const f32x4 mine = p[kh][nt], theirs = red[((wave * 2 + (1 - kh)) * 2 + nt) * 64 + lane];
      acc[nt] = kh == 0 ? mine + theirs : theirs + mine;  // K-half 0 + K-half 1
    }
  }
}

// LayerNorm partials (mean, M2 over the slot's 32 columns) of row 16 tile + c, from the transposed accumulator
// layout (lane (c, q): columns 16 nt + 4 q + r): 8 values per lane, summed over the row's four q lanes (c, c + 16,
// c + 32, c + 48; ((s0 + s1) + (s2 + s3)) in every lane, by commutativity), two passes; write-through 8-B store.
__device__ __forceinline__ void store_partials_t(float2* xpart, const float (&x)[2][4], int r0, int nr, int s, int tile, int lane_in) {
  const int lane = opq(lane_in);
  const int c = lane & 15, q = lane >> 4;
  float sm = ((x[0][0] + x[0][1]) + (x[0][2] + x[0][3])) + ((x[1][0] + x[1][1]) + (x[1][2] + x[1][3]));
  sm += __shfl_xor(sm, 16);
  sm += __shfl_xor(sm, 32);
  const float mean = sm * (1.0f / kCols);
  float m2 = 0.f;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = x[nt][r] - mean;
      m2 = fmaf(d, d, m2);
    }
  m2 += __shfl_xor(m2, 16);
  m2 += __shfl_xor(m2, 32);
  const int row = 16 * tile + c;
  if (q == 0 && row < nr)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(xpart + (size_t)(r0 + row) * kSlots + s),
                       __builtin_bit_cast(unsigned long long, make_float2(mean, m2)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
// The lane's two 4-column pieces of row 16 tile + c (transposed layout), bf16, written through straight from the
// registers: fragment-major (frag: group g's [tile][K-step s][lane' = row + 16 (2 nt + q / 2)][8 bf16], byte 8 (q & 1)
// of the 16-B piece; rows >= nr as zeros) or row-major (T x H, rows >= nr not stored).
__device__ __forceinline__ void store_op_t(bf16* dst, int g, int s, int tile, const float (&v)[2][4], int r0, int nr,
                                           int col0, int TT, int lane_in, bool frag) {
  constexpr int KST = kH / 32;
  const int lane = opq(lane_in);
  const int c = lane & 15, q = lane >> 4;
  const int row = 16 * tile + c;
  const bool live = row < nr;
  u32x2 piece[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const bf16x4 b = {(bf16)v[nt][0], (bf16)v[nt][1], (bf16)v[nt][2], (bf16)v[nt][3]};
    piece[nt] = live ? __builtin_bit_cast(u32x2, b) : u32x2{0u, 0u};
  }
  if (frag) {
    const __amdgpu_buffer_rsrc_t rs =
        rsrc(reinterpret_cast<char*>(dst) + (size_t)g * frag_group_bytes(KST), frag_group_bytes(KST));
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const unsigned off = (unsigned)(((tile * KST + s) * 64 + c + 16 * (2 * nt + (q >> 1))) * 16 + (q & 1) * 8);
      __builtin_amdgcn_raw_buffer_store_b64(piece[nt], rs, off, 0, 16);
    }
    // (r06aj: swapping halves between lanes q and q ^ 1 for one 16-B store per lane measured no faster at B = 1 and
    // 4 % slower at T = 2400, profiles/r06aj_op16_ab.txt)
  } else if (live) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(dst, (unsigned)TT * kH * 2);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      __builtin_amdgcn_raw_buffer_store_b64(piece[nt], rs, (unsigned)(((size_t)(r0 + row) * kH + col0 + 16 * nt + 4 * q) * 2), 0, 16);
  }
}

// The fp32 residual rows other groups read: only the kHalo rows at each end of the group (the depthwise halo of its
// neighbours), two 16-B write-through stores per lane straight from the transposed registers; the middle rows never
// leave the workgroup.
__device__ __forceinline__ void store_halo_t(float* ximg, const float (&x)[2][4], int r0, int nr, int col0, int tile, int TT,
                                             int lane_in) {
  const int lane = opq(lane_in);
  const int c = lane & 15, q = lane >> 4;
  const int row = 16 * tile + c;
  if (row < nr && (row < kHalo || row >= nr - kHalo)) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(ximg, (unsigned)TT * kH * 4);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      st16(rs, (unsigned)(((size_t)(r0 + row) * kH + col0 + 16 * nt + 4 * q) * 4),
           __builtin_bit_cast(u32x4, make_float4(x[nt][0], x[nt][1], x[nt][2], x[nt][3])));
  }
}

// Column vector p[16 nt + 4 q + r] of the lane's columns (transposed layout): two 16-B loads (p 16-B aligned: the
// weight arena, and modulation rows of MS floats, MS % 4 == 0 -- persist_solve checks it)
__device__ __forceinline__ void ld_cols(float (&v)[2][4], const float* p, int q) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const float4 a = *reinterpret_cast<const float4*>(p + 16 * nt + 4 * q);
    v[nt][0] = a.x; v[nt][1] = a.y; v[nt][2] = a.z; v[nt][3] = a.w;
  }
}
__device__ __forceinline__ void fill_cols(float (&v)[2][4], float x) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[nt][r] = x;
}

// (mean, rstd) of rows [ra, rb) from the 32 slots' partials (sc1 loads), into st[2 (r - rbase)]; two
// lanes per row (16 partials each), combined as row_stats_from_partials does (tile width 32, eps 1e-6).
__device__ __forceinline__ void row_stats(const float2* xpart, int T, int ra, int rb, int rbase, float* st) {
  const int n2 = 2 * (rb - ra);
  const __amdgpu_buffer_rsrc_t rs = rsrc(xpart, (unsigned)T * kSlots * 8);
  for (int idx = opq(threadIdx.x); idx < ((n2 + 63) & ~63); idx += kThreads) {
    const bool act = idx < n2;
    const int row = ra + (act ? idx >> 1 : 0), half = idx & 1;
    float mv[16], qv[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float4 v = as_f4(ld16(rs, (unsigned)((row * kSlots + half * 16 + 2 * k) * 8)));
      mv[2 * k] = v.x; qv[2 * k] = v.y; mv[2 * k + 1] = v.z; qv[2 * k + 1] = v.w;
    }
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) sm += mv[k];
    sm = dpp_add<kDppXor1>(sm);
    const float mean = sm * (1.0f / kSlots);
    float m2 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float d = mv[k] - mean;
      m2 += qv[k] + (float)kCols * d * d;
    }
    m2 = dpp_add<kDppXor1>(m2);
    if (act && half == 0) {
      st[2 * (row - rbase)] = mean;
      st[2 * (row - rbase) + 1] = 1.0f / sqrtf(m2 * (1.0f / kH) + 1e-6f);
    }
  }
}

// A staged tile (the GroupNorm apply's bf16 rows: thread -> channel, not an MFMA layout) written through with 16-B sc1
// stores (rows [ra, rb) of the tile) into dst (row stride ld).
// Each wave writes the rows it staged itself ([16 w, 16 w + 16) of the chunk), so a stage -> flush pair needs no
// workgroup barrier (persist_opt 32768: the wave's own LDS writes are ordered before its reads).
template <typename OT>
__device__ __forceinline__ void flush_tile(const char* stg, OT* dst, int ld, int r0, int ra, int rb, int col0, int T,
                                           bool local = false) {
  constexpr int CPR = kCols * (int)sizeof(OT) / 16;  // 16-B chunks per staged row
  const __amdgpu_buffer_rsrc_t rs = rsrc(dst, (unsigned)T * ld * (unsigned)sizeof(OT));
  const int w16 = 16 * (threadIdx.x >> 6);
  for (int it = opq(threadIdx.x & 63); it < 16 * CPR; it += 64) {
    const int row = w16 + it / CPR, ch = it % CPR;
    if (row < ra || row >= rb) continue;
    const u32x4 v = *reinterpret_cast<const u32x4*>(stg + (row * kCols * sizeof(OT)) + ch * 16);
    const unsigned off = (unsigned)(((size_t)(r0 + row) * ld + col0) * sizeof(OT) + ch * 16);
    if (local) st16p(rs, off, v);
    else st16(rs, off, v);
  }
}

// ... or, fragment-major (persist_opt 64): the staged bf16 chunk (rows x this slot's 32 columns = K-step s of
// the consumer) as group g's fragments (t0 + t, s): one contiguous 1 KB per 16-row tile, rows >= nr (the
// chunk's rows) as zeros; t0 = the chunk's first tile.
__device__ __forceinline__ void flush_frag(const char* stg, bf16* dst, int g, int s, int nr, int KST, bool local, int t0 = 0) {
  const int ntile = (nr + 15) >> 4;
  const __amdgpu_buffer_rsrc_t rs = rsrc(reinterpret_cast<char*>(dst) + (size_t)g * frag_group_bytes(KST), frag_group_bytes(KST));
  for (int idx = opq(threadIdx.x); idx < ntile * 64; idx += kThreads) {
    const int t = idx >> 6, ln = idx & 63, row = 16 * t + (ln & 15), q = ln >> 4;
    const u32x4 v = row < nr ? *reinterpret_cast<const u32x4*>(stg + row * (kCols * 2) + q * 16) : u32x4{0u, 0u, 0u, 0u};
    const unsigned off = (unsigned)((((t0 + t) * KST + s) * 64 + ln) * 16);
    if (local) st16p(rs, off, v);
    else st16(rs, off, v);
  }
}

__device__ __forceinline__ void acc_to(float (&v)[2][4], const f32x4 (&acc)[2]) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) v[nt][i] = acc[nt][i];
}

// GroupNorm statistics of one channel from the 8 groups' (count, mean, M2), Chan-combined in group order over this
// utterance's groups only (another utterance's entries are masked whole: a zero count alone would still add its M2),
// and the (mean, scale) the apply uses.  One code path for both exchange forms, every operation rounded on its own
// (chan_combine_rn), so the granule and counter forms give the same bits for any row partition.
__device__ __forceinline__ float2 gn_finalize(const float (&nv)[kGroups], const float (&mv)[kGroups], const float (&qv)[kGroups],
                                              int utt, int gpu, int T, float gw) {
#pragma clang fp contract(off)
  float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    const bool mine = k / gpu == utt;
    chan_combine_rn(n, mean, m2, mine ? nv[k] : 0.f, mine ? mv[k] : 0.f, mine ? qv[k] : 0.f);
  }
  return make_float2(mean, (1.0f / sqrtf(m2 * (1.0f / (float)T) + 1e-5f)) * gw);
}

// KH: GEMM phases split 2 x 2 over the waves (gemm_kh, persist_opt 1024): a template parameter, so each variant
// gets its own register allocation
// NTW: chunks of 64 rows per group (template: registers are indexed by it), 1..kMaxNTW; KH only with NTW == 1.
template <bool KH, int NTW>
__global__ __launch_bounds__(kThreads, 1) void den_persist_kernel(Params P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = P.T;            // frames per utterance
  const int TT = P.B * P.T;     // rows of the batch (buffer ranges)
  const int H = kH;
  // Group / slot: group = blockIdx % 8 (the round-robin dispatch puts it on one XCD: speed only).
  int g = blockIdx.x % kGroups, s = blockIdx.x / kGroups;
  // opt & 8: the XCDs as a 2 x 4 grid of (row half, column quarter): XCD x holds row groups
  // 4 (x / 4) .. + 3 and column slots 8 (x % 4) .. + 7, so per GEMM phase an XCD's L2 pulls 4 row
  // panels of A (each read by 8 of its CUs) and 8 weight panels (each read by 4) -- ~0.9 MB per XCD
  // instead of 1 row panel + all 32 weight panels (2.1 MB): 2.3x less Infinity-Cache traffic per phase.
  // A row group's 32 producers then span 4 XCDs, so every hand-off stays write-through.
  if (P.opt & 8) {
    const int x = g, j = s;
    g = 4 * (x / 4) + (j % 4);
    s = 8 * (x % 4) + j / 4;
  }
  constexpr bool xloc = false;  // (plain stores kept for an XCD-local group layout; every hand-off is write-through)
  const bool frag = (P.opt & 64) != 0;        // fragment-major GEMM A images (a2, u, xa, xs)
  const bool gran = (P.opt & 512) != 0;       // GroupNorm partials as tagged granules (gnp zeroed per launch)
  int r0, nr;
  group_rows(g, T, P.B, r0, nr, P.opt);
  const int gpu = kGroups / P.B, utt = g / gpu;  // this group's utterance and its frames [ub, ue)
  const int ub = utt * T, ue = ub + T;
  // padded batch (P.Bx): an idle utterance runs the same phases on zeros (every group still takes part in every
  // hand-off), without touching xt; its modulation row is the last real utterance's
  const bool idle = P.Bx > 0 && utt >= P.Bx;
  const int MB = P.Bx > 0 ? P.Bx : P.B, mutt = idle ? P.Bx - 1 : utt;
  const int c = lane & 15, q = lane >> 4;
  const int col0 = kCols * s;
  char* stg = smem + L_HS;  // epilogue staging (aliases the dwconv window)
  float* hs = reinterpret_cast<float*>(smem + L_HS);
  float* st = reinterpret_cast<float*>(smem + L_ST);  // window frame r0 - 15 + p -> (mean, rstd) at st[2 p]
  float* red = reinterpret_cast<float*>(smem + L_RED);
  float4* gnv = reinterpret_cast<float4*>(smem + L_GNV);
  int* flag = reinterpret_cast<int*>(smem + L_FLAG);
  int* grp = P.ctr + CT_GRP;
  int* mygrp = grp + 16 * g;
  int* gnc = P.ctr + CT_GN + 16 * s;
  int* errw = P.ctr + CT_ERR;
  int* fails = P.sticky + SY_FAILS;
  const long long tmo = P.tmo;
  int L = 0;    // group signals so far (the same sequence in every workgroup)
  int ndg = 0;  // GroupNorm hand-offs so far
  int wb = 0;   // LDS buffer holding (or receiving) the weights of the next GEMM phase
#ifdef FL_STAMPS
  int pst_k = 0;
#endif
  // after a GEMM phase: the next GEMM's panel goes into the buffer the finished one did not use
  [[maybe_unused]] int cur_step = P.s0;  // (FL_STAMPS builds: the step a helper lambda stamps)
  const bool fastdma = !(P.opt & 256);  // persist_opt 256: the generic issue loop (A/B)
  const bool w4 = (P.opt & 1) != 0;
  // drain behind the next panel's DMA (signal_dma): needs the four-wave fast issue, whose per-wave piece count
  // is fixed (16 for a 32 x 1024 panel, 4 for proj_in's 32 x 256)
  const bool dmafirst = (P.opt & 4096) != 0 && w4 && !(P.opt & 256);
  auto next_w = [&](const bf16* W) {
    wb ^= 1;
    if (fastdma)
      dma_panel4<kH>((smem + wb * kWPanel), W + (size_t)col0 * kH, [](int n) { return (unsigned)(n * 2 * kH); }, wave, lane, w4);
    else
      dma_panel<kH>((smem + wb * kWPanel), [&](int n) { return W + (size_t)(col0 + n) * kH; }, wave, lane, P.opt);
#ifdef FL_STAMPS
    if (P.opt & 32) {  // diagnostic: when this wave's weight DMA has landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      PST(cur_step);
    }
#endif
  };
  auto next_win = [&]() {
    wb ^= 1;
    if (fastdma)
      dma_panel4<kC>((smem + wb * kWPanel), P.win + (size_t)col0 * kC, [](int n) { return (unsigned)(n * 2 * kC); }, wave, lane, w4);
    else
      dma_panel<kC>((smem + wb * kWPanel), [&](int n) { return P.win + (size_t)(col0 + n) * kC; }, wave, lane, P.opt);
  };
  auto issue_out = [&]() {  // the conv_out panel (taps stacked): panel row n < 24 is tap n / 8 of channel 8 s + n % 8
    if (fastdma) {
      const int s8 = kCh * s;
      dma_panel4<kH>((smem + (wb ^ 1) * kWPanel), P.wout, [s8](int n) {
        const int m = n < 24 ? n : n - 24;
        return (unsigned)(((m >> 3) * kC + s8 + (m & 7)) * 2 * kH);
      }, wave, lane, w4);
    } else {
      dma_panel<kH>((smem + (wb ^ 1) * kWPanel), [&](int n) {
        const int m = n < 24 ? n : n - 24;
        return P.wout + (size_t)((m >> 3) * kC + kCh * s + (m & 7)) * kH;
      }, wave, lane, P.opt);
    }
  };

  // rows of chunk i: [kChunk i, kChunk i + crows(i)) of the group
  auto crows = [&](int i) { return max(min(kChunk, nr - kChunk * i), 0); };
  // Euler state: thread -> row kChunk i + xr_row of chunk i, channels 8 s + 2 (tid & 3) + {0, 1}
  const int xr_row = tid >> 2, xch = kCh * s + 2 * (tid & 3);
  float xs0[NTW], xs1[NTW];
#pragma unroll
  for (int i = 0; i < NTW; ++i) {
    xs0[i] = 0.f;
    xs1[i] = 0.f;
    const int row = kChunk * i + xr_row;
    if (row < nr && !idle) {
      xs0[i] = P.xt[(size_t)(r0 + row) * kC + xch];
      xs1[i] = P.xt[(size_t)(r0 + row) * kC + xch + 1];
    }
  }
  // An abandoned solve leaves NaN in this workgroup's part of x (every workgroup leaves through here or
  // finishes normally), so a failure can never pass for a result.
  // seal mode: this workgroup's seal, written before each group signal; the check after each group wait
  const bool seal = (P.opt & 16384) != 0;
  // deferred seals (persist_opt 65536): the same seals, but wave 0 only ISSUES the seal loads after the counter
  // wait (they travel with the phase's A fetch) and checks them at the next seal_put, a phase later; a seal
  // behind its counter then fails the launch (error 4, NaN at every workgroup's next wait) instead of being
  // waited for -- detection without a round trip on the hand-off chain
  const bool dseal = (P.opt & 65536) != 0;
  int dseal_v = 0x7fffffff, dseal_tgt = 0;  // wave 0: min of the seals loaded at the last wait, and its target
  auto dseal_check = [&]() {
    if (dseal && wave == 0) {
      const bool ok = __all(dseal_v >= dseal_tgt);
      if (!ok && lane == 0) raise_err(errw, fails, 4);
      return ok;
    }
    return true;
  };
  auto seal_put = [&]() {
    dseal_check();
    if ((seal || dseal) && tid == 0 && !(cur_step == P.seal_skip && blockIdx.x == 5))
      __hip_atomic_store(P.seal + 4 * (g * kSlots + s), L + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto seal_wait = [&](int g0, int ng) -> bool {
    if (dseal) {
      if (wave == 0) {
        // one load per lane: the group's 32 seals (twice), or for the all-group waits (depthwise halo, Euler
        // boundary rows) the seals of the two neighbouring groups whose rows this workgroup reads
        const int gi = ng == 1 ? g0 : (lane < 32 ? (g + kGroups - 1) % kGroups : (g + 1) % kGroups);
        dseal_v = __hip_atomic_load(P.seal + 4 * (gi * kSlots + (lane & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dseal_tgt = L;
      }
      return true;
    }
    return !seal || seals_ok(P.seal + 4 * g0 * kSlots, ng * kSlots, L, P.ctr + CT_ERR, P.sticky + SY_FAILS, P.tmo,
                             reinterpret_cast<int*>(smem + L_FLAG));
  };
  auto fail_exit = [&]() {
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
      const int row = kChunk * i + xr_row;
      if (row < nr && !idle) {
        P.xt[(size_t)(r0 + row) * kC + xch] = __builtin_nanf("");
        P.xt[(size_t)(r0 + row) * kC + xch + 1] = __builtin_nanf("");
      }
    }
  };
  // Staged hand-off rows are written and flushed by the same wave (stage_tile / GroupNorm apply rows 16 w .. 16 w + 15,
  // flush_frag / flush_tile / publish_xs by wave): persist_opt 32768 orders them with the wave's own LDS wait instead
  // of a workgroup barrier.
  const bool wlocal = (P.opt & 32768) != 0;
  auto stage_sync = [&]() {
    if (wlocal) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else __syncthreads();
  };
  // weights of the first GEMM (proj_in) while the state is published
  dma_panel<kC>(smem, [&](int n) { return P.win + (size_t)(col0 + n) * kC; }, wave, lane, P.opt);
  // bf16 rows of x (proj_in's operand): 16 B per tile row, staged in LDS
  auto publish_xs = [&]() {
    bf16* t = reinterpret_cast<bf16*>(stg);
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
      const int nrc = crows(i);
      if (i > 0) stage_sync();  // the previous chunk's rows have left the staging tile
      t[xr_row * kCh + 2 * (tid & 3)] = (bf16)xs0[i];
      t[xr_row * kCh + 2 * (tid & 3) + 1] = (bf16)xs1[i];
      stage_sync();
      // each wave writes the 16 rows it staged (lanes 0..15: one row of 16 B each)
      const int prow = 16 * wave + lane;
      if (frag) {  // channels 8 s .. 8 s + 7 = K-step s / 4, quarter s % 4 of proj_in's fragments
        if (lane < 16 && 16 * wave < nrc) {
          const __amdgpu_buffer_rsrc_t rs =
              rsrc(reinterpret_cast<char*>(P.xs) + (size_t)g * frag_group_bytes(kC / 32), frag_group_bytes(kC / 32));
          const int tt = 4 * i + wave, ln = lane + 16 * (s & 3);
          const u32x4 v = prow < nrc ? *reinterpret_cast<const u32x4*>(stg + prow * 16) : u32x4{0u, 0u, 0u, 0u};
          const unsigned off = (unsigned)(((tt * (kC / 32) + (s >> 2)) * 64 + ln) * 16);
          if (xloc) st16p(rs, off, v);
          else st16(rs, off, v);
        }
      } else if (lane < 16 && prow < nrc) {
        const __amdgpu_buffer_rsrc_t rs = rsrc(P.xs, (unsigned)TT * kC * 2);
        const unsigned off = (unsigned)(((size_t)(r0 + kChunk * i + prow) * kC + kCh * s) * 2);
        if (xloc) st16p(rs, off, *reinterpret_cast<const u32x4*>(stg + prow * 16));
        else st16(rs, off, *reinterpret_cast<const u32x4*>(stg + prow * 16));
      }
    }
    seal_put();
    signal(mygrp);
    ++L;
  };
  // ---- reset prologue: this launch zeroes its own counter block (and the GroupNorm granule tags), so no
  // host memset node has to be ordered before the kernel (a memset node replayed in a captured graph did not
  // reset the counters of later replays).  Two grid-wide arrivals on monotonic counters that are never
  // reset: the first says every workgroup of this launch has started (so the previous launch, stream-
  // ordered before it, is done with the block), the second that every share has been zeroed.
  {
    unsigned* const a0 = reinterpret_cast<unsigned*>(P.sticky + SY_ARRIVE0);
    unsigned* const a1 = reinterpret_cast<unsigned*>(P.sticky + SY_ARRIVE1);
    unsigned* tk = reinterpret_cast<unsigned*>(smem + L_FLAG);
    if (tid == 0) tk[1] = __hip_atomic_fetch_add(a0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned target = arrive_target(tk[1]);
    __syncthreads();
    const bool ok0 = arrive_wait(a0, target, tmo, flag);
    if (ok0) {
      if (tid < 4 && kCtrInts > 4 * (int)blockIdx.x + tid)
        __hip_atomic_store(P.ctr + 4 * blockIdx.x + tid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid < 4) __hip_atomic_store(P.seal + 4 * blockIdx.x + tid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (gran && tid < 32) {  // 512 B of the 128 KB granule block per workgroup
        const __amdgpu_buffer_rsrc_t rq = rsrc(P.gnp, kGroups * kH * 16);
        st16(rq, (unsigned)((blockIdx.x * 32 + tid) * 16), u32x4{0u, 0u, 0u, 0u});
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // every workgroup adds to the second counter exactly once, also after a failed first wait, so both counters
    // stay kWGs per launch and in phase for every later launch
    if (tid == 0) __hip_atomic_fetch_add(a1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool ok1 = arrive_wait(a1, target, tmo, flag);
    if (!ok0 || !ok1) {
      // counted once per launch in the sticky failure word (the error word sits in the block being reset):
      // the first workgroup to record this launch's target in SY_PFAIL adds the failure
      if (tid == 0) {
        unsigned* pf = reinterpret_cast<unsigned*>(P.sticky + SY_PFAIL);
        if (__hip_atomic_exchange(pf, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != target)
          __hip_atomic_fetch_add(fails, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // and in this launch's error word (zeroed before the second arrival), which the host copies per launch
        // (flamed_den_persist_query); the workgroups that did get through stop at their first wait
        __hip_atomic_store(errw, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      fail_exit();
      return;
    }
  }
  publish_xs();

  float X[NTW][2][4];  // residual stream tiles (this wave's tiles wave + 4 i: 16 rows x 32 columns each), MFMA layout

  for (int step = P.s0; step < P.s1; ++step) {
    const float* md = P.mods + (size_t)(step * MB + mutt) * P.MS;  // this utterance's modulation row
    cur_step = step;
    if (step == P.inject_step) {  // diagnostic failure injection: every workgroup abandons here
      if (tid == 0) raise_err(errw, fails, 3);
      fail_exit();
      return;
    }
#ifdef FL_STAMPS
    pst_k = 0;
#endif
    // ------------------------------ proj_in (:361) ------------------------------
    float binv[2][4];  // epilogue vectors of the lane's columns (transposed layout), before the wait
    ld_cols(binv, P.bin + col0, q);
    PST(step);
    if (!wait_ge(errw, fails, tmo, mygrp, 0, 1, 32 * L, flag) || !seal_wait(g, 1)) { fail_exit(); return; }
    PST(step);
    f32x4 accm[NTW][2];  // every tile's products (several chunks: one streamed pass, epilogues after it)
    if constexpr (KH) gemm_kh<kC>(P.xs, r0, nr, (smem + wb * kWPanel), accm[0], wave, lane, PSTP(step), g, frag);
    else if constexpr (NTW == 1) gemm<kC>(P.xs, r0, nr, (smem + wb * kWPanel), accm[0], wave, lane, PSTP(step), g, frag);
    else gemm_chunks<kC, NTW>(P.xs, r0, nr, (smem + wb * kWPanel), accm, wave, lane, PSTP(step), g, frag, P.opt);
    PST(step);
#pragma unroll
    for (int ci = 0; ci < NTW; ++ci) {
      const int tl = wave + 4 * ci;
      const f32x4(&acc)[2] = accm[ci];
      acc_to(X[ci], acc);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) X[ci][nt][i] += binv[nt][i];
      if (16 * tl < nr) {
        store_partials_t(P.xpart[0], X[ci], r0, nr, s, tl, lane);
        store_halo_t(P.ximg, X[ci], r0, nr, col0, tl, TT, lane);
      }
    }
    seal_put();
    if (dmafirst) {
      next_w(P.blk[0].w2);
      signal_dma<16>(mygrp);
    } else {
      signal(mygrp);
      next_w(P.blk[0].w2);
    }
    PST(step);
    ++L;

    for (int blk = 0; blk <= P.NB; ++blk) {
      const bool fin = blk == P.NB;
      const BlockW& bw = P.blk[blk];
      const float* mb = md + (size_t)blk * 6 * H;  // [sh, sc, gate] of the ConvNeXt LN (+ [sh, sc, gate] of the next)

      // -------- LN + modulate + depthwise k31 + GroupNorm(H, H) over T (prob_generator.py:81-89, 153-156)
      // what this phase reads that no other workgroup writes goes out before the wait (its latency hides in
      // the poll): the modulation vectors of the thread's columns, the depthwise taps and bias of channel cc,
      // the GroupNorm affine of the GN-combining lanes
      const int cc = tid & 31, rg = tid >> 5;
      // raw loads only before the wait (the arithmetic that consumes them after it: computed here, the compiler
      // put the loads' wait ahead of the poll instead of behind it)
      float hsc[4], hsh[4], hlw[4], hlb[4], osc[2][4], osh[2][4], olw[2][4], olb[2][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = col0 + 4 * (tid & 7) + e;
        hsc[e] = mb[H + col];
        hsh[e] = mb[col];
        hlw[e] = fin ? 1.0f : bw.lnw[col];
        hlb[e] = fin ? 0.0f : bw.lnb[col];
      }
      ld_cols(osc, mb + H + col0, q);  // the lane's own columns (transposed layout)
      ld_cols(osh, mb + col0, q);
      if (fin) {
        fill_cols(olw, 1.0f);
        fill_cols(olb, 0.0f);
      } else {
        ld_cols(olw, bw.lnw + col0, q);
        ld_cols(olb, bw.lnb + col0, q);
      }
      float w[kTaps];
#pragma unroll
      for (int j = 0; j < kTaps; ++j) w[j] = bw.dww[(size_t)j * H + col0 + cc];
      const float dbias = bw.dwb[col0 + cc];
      float gwv = 0.f, gbv = 0.f;
      if (tid < kCols) {
        gwv = bw.gnw[col0 + tid];
        gbv = bw.gnb[col0 + tid];
      }
      PST(step);
      if (!wait_ge(errw, fails, tmo, grp, 16, kGroups, 32 * L, flag) || !seal_wait(0, kGroups)) { fail_exit(); return; }  // every group: the halo rows of the neighbours
      PST(step);
      // va = w (1 + sc), vb = b (1 + sc) + sh (vab's arithmetic; w = 1, b = 0 without the affine)
      float hva[4], hvb[4], ova[2][4], ovb[2][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float sc1 = 1.0f + hsc[e];
        hva[e] = fin ? sc1 : hlw[e] * sc1;
        hvb[e] = fin ? hsh[e] : hlb[e] * sc1 + hsh[e];
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sc1 = 1.0f + osc[nt][r];
          ova[nt][r] = fin ? sc1 : olw[nt][r] * sc1;
          ovb[nt][r] = fin ? osh[nt][r] : olb[nt][r] * sc1 + osh[nt][r];
        }
      const int wa = max(r0 - kHalo, ub), wz = min(r0 + nr + kHalo, ue);  // the utterance's frames only
      // Everything this phase reads that does not wait on another phase goes out first, so the loads'
      // latencies overlap: the thread's halo item (its 4 columns col0 + 4 (tid & 7)), their modulation vectors,
      // the depthwise taps of channel cc, the row statistics.  Halo items: the group's kHalo rows above and
      // below it (window index hp, frame r0 - kHalo + hp; 30 rows x 8 column quads, threads < 240).
      const int hid = tid >> 3, hp = hid < kHalo ? hid : nr + hid;
      float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
      {
        const __amdgpu_buffer_rsrc_t rx = rsrc(P.ximg, (unsigned)TT * H * 4);
        const int r = r0 - kHalo + hp;
        if (hid < 2 * kHalo && r >= ub && r < ue) hv = as_f4(ld16(rx, (unsigned)(((size_t)r * H + col0 + 4 * (tid & 7)) * 4)));
      }
      row_stats(P.xpart[0], TT, wa, wz, r0 - kHalo, st);
      __syncthreads();
      PST(step);  // halo rows + row statistics in
      // per chunk: window hs[pw] = frame r0 + c0 - kHalo + pw (pw < kWin): own rows from X (registers), halo rows
      // from ximg, 0 outside the utterance; then the depthwise conv of the chunk's rows (zero padding at the
      // utterance edges): thread -> channel cc, chunk rows 8 rg .. 8 rg + 7
      float d[NTW][8];
#pragma unroll
      for (int ci = 0; ci < NTW; ++ci) {
        const int c0 = kChunk * ci;
        if (ci > 0) __syncthreads();  // the previous chunk's window has been read
        if (hid < 2 * kHalo) {
          const int pw = hp - c0, r = r0 - kHalo + hp;
          if (pw >= 0 && pw < kWin) {
            float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r >= ub && r < ue) {
              const float mean = st[2 * hp], rstd = st[2 * hp + 1];
              o.x = ((hv.x - mean) * rstd) * hva[0] + hvb[0];
              o.y = ((hv.y - mean) * rstd) * hva[1] + hvb[1];
              o.z = ((hv.z - mean) * rstd) * hva[2] + hvb[2];
              o.w = ((hv.w - mean) * rstd) * hva[3] + hvb[3];
            }
            *reinterpret_cast<float4*>(hs + pw * kHsLd + 4 * (tid & 7)) = o;
          }
        }
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int tb = 16 * (wave + 4 * j);  // first row of this wave's tile j
          if (tb < nr && tb + 16 > c0 - kHalo && tb < c0 + kChunk + kHalo) {
            const int row = tb + c, pw = row - c0 + kHalo;  // the lane's row, 4 consecutive columns per half
            if (row < nr && pw >= 0 && pw < kWin) {
              const int p = row + kHalo;
              const float mean = st[2 * p], rstd = st[2 * p + 1];
#pragma unroll
              for (int nt = 0; nt < 2; ++nt) {
                float o[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = ((X[j][nt][r] - mean) * rstd) * ova[nt][r] + ovb[nt][r];
                *reinterpret_cast<float4*>(hs + pw * kHsLd + 16 * nt + 4 * q) = make_float4(o[0], o[1], o[2], o[3]);
              }
            }
          }
        }
        __syncthreads();
        if (ci == 0) PST(step);  // normalised window in LDS
        {
          float win[8 + kTaps - 1];
#pragma unroll
          for (int j = 0; j < 8 + kTaps - 1; ++j) win[j] = hs[(8 * rg + j) * kHsLd + cc];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float a = dbias;
#pragma unroll
            for (int j = 0; j < kTaps; ++j) a = fmaf(w[j], win[k + j], a);
            d[ci][k] = a;
          }
        }
      }
      PST(step);  // depthwise conv done
      // GroupNorm partials of this group's frames: exact two passes (sum, squared deviations)
      {
        float sm = 0.f;
#pragma unroll
        for (int ci = 0; ci < NTW; ++ci) {
          const int nv = min(max(crows(ci) - 8 * rg, 0), 8);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (k < nv) sm += d[ci][k];
        }
        red[rg * kCols + cc] = sm;
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) tot += red[k * kCols + cc];
        const float mg = nr > 0 ? tot / (float)nr : 0.f;
        __syncthreads();
        float m2 = 0.f;
#pragma unroll
        for (int ci = 0; ci < NTW; ++ci) {
          const int nv = min(max(crows(ci) - 8 * rg, 0), 8);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (k < nv) {
              const float e = d[ci][k] - mg;
              m2 = fmaf(e, e, m2);
            }
        }
        red[rg * kCols + cc] = m2;
        __syncthreads();
        if (tid < kCols) {
          float m2t = 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) m2t += red[k * kCols + cc];
          GND(26, mg);
          GND(27, m2t);
          GND(28, (float)nr);
          if (gran) {  // (mean, M2) as two tagged granules: the data is the flag (no drain, no counter)
            unsigned long long* gq = reinterpret_cast<unsigned long long*>(P.gnp) + ((size_t)g * H + col0 + cc) * 2;
            const unsigned long long tag = (unsigned long long)(ndg + 1) << 32;
            __hip_atomic_store(gq, tag | __float_as_uint(mg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gq + 1, tag | __float_as_uint(m2t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            const __amdgpu_buffer_rsrc_t rq = rsrc(P.gnp, kGroups * kH * 16);
            st16(rq, (unsigned)((g * H + col0 + cc) * 16), __builtin_bit_cast(u32x4, make_float4((float)nr, mg, m2t, 0.f)));
          }
        }
      }
      if (!gran) signal(gnc);
      PST(step);
      ++ndg;
      PST(step);
      if (gran) {
        // wave 0: lane cc < 32 re-reads the 8 groups' granules of channel col0 + cc until every tag is this
        // hand-off's, then Chan-combines them in group order (group k's row count from group_rows)
        bool ok = true;
        if (tid < 64) {
          const unsigned long long* gq = reinterpret_cast<const unsigned long long*>(P.gnp) + (size_t)(col0 + (tid & 31)) * 2;
          float mv[kGroups], qv[kGroups];
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          for (unsigned it = 0;; ++it) {
            bool mine = true;
            if (tid < kCols) {
#pragma unroll
              for (int k = 0; k < kGroups; ++k) {
                const unsigned long long a = __hip_atomic_load(gq + (size_t)k * H * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long b = __hip_atomic_load(gq + (size_t)k * H * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                mine = mine && (unsigned)(a >> 32) == (unsigned)ndg && (unsigned)(b >> 32) == (unsigned)ndg;
                mv[k] = __uint_as_float((unsigned)a);
                qv[k] = __uint_as_float((unsigned)b);
              }
            }
            if (__all(mine)) break;
            if ((it & 31) == 31) {
              if (__hip_atomic_load(errw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) { ok = false; break; }
              if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > tmo) {
                if (tid == 0) raise_err(errw, fails, 1);
                ok = false;
                break;
              }
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (tid == 0) *flag = ok ? 1 : 0;
          if (ok && tid < kCols) {
            float nv[kGroups];  // group k's row count from group_rows
#pragma unroll
            for (int k = 0; k < kGroups; ++k) {
              int ka, kn;
              group_rows(k, T, P.B, ka, kn, P.opt);
              nv[k] = (float)kn;
              GND(3 * k, nv[k]);
              GND(3 * k + 1, mv[k]);
              GND(3 * k + 2, qv[k]);
            }
            const float2 ms = gn_finalize(nv, mv, qv, utt, gpu, T, gwv);
            GND(24, ms.x);
            GND(25, ms.y);
            gnv[tid] = make_float4(ms.x, ms.y, gbv, 0.f);
          }
        }
        __syncthreads();
        const bool okw = *flag != 0;
        __syncthreads();
        if (!okw) { fail_exit(); return; }
        PST(step);
      } else {
      if (!wait_ge(errw, fails, tmo, gnc, 0, 1, kGroups * ndg, flag)) { fail_exit(); return; }
      PST(step);
      if (tid < kCols) {  // the 8 groups' partials of this channel, Chan-combined in group order
        const __amdgpu_buffer_rsrc_t rq = rsrc(P.gnp, kGroups * kH * 16);
        float nv[kGroups], mv[kGroups], qv[kGroups];  // the producers' (count, mean, M2)
#pragma unroll
        for (int k = 0; k < kGroups; ++k) {
          const float4 v = as_f4(ld16(rq, (unsigned)((k * H + col0 + tid) * 16)));
          nv[k] = v.x;
          mv[k] = v.y;
          qv[k] = v.z;
          GND(3 * k, v.x);
          GND(3 * k + 1, v.y);
          GND(3 * k + 2, v.z);
        }
        const float2 ms = gn_finalize(nv, mv, qv, utt, gpu, T, gwv);
        GND(24, ms.x);
        GND(25, ms.y);
        gnv[tid] = make_float4(ms.x, ms.y, gbv, 0.f);
      }
      }
      __syncthreads();
      {
        const float4 gv = gnv[cc];
        bf16* t = reinterpret_cast<bf16*>(stg);
#pragma unroll
        for (int ci = 0; ci < NTW; ++ci) {
          if (ci > 0) stage_sync();  // the previous chunk's rows have left the staging tile
#pragma unroll
          for (int k = 0; k < 8; ++k) t[(8 * rg + k) * kCols + cc] = (bf16)((d[ci][k] - gv.x) * gv.y + gv.z);
          stage_sync();
          if (frag) flush_frag(stg, P.a2, g, s, crows(ci), kH / 32, xloc, 4 * ci);
          else flush_tile<bf16>(stg, P.a2, H, r0 + kChunk * ci, 0, crows(ci), col0, TT, xloc);
        }
      }
      seal_put();
      signal(mygrp);
      PST(step);
      ++L;

      // -------- conv_2 (1x1) + GELU (:90-91)
      float b2v[2][4];  // epilogue vectors before the wait
      ld_cols(b2v, bw.b2 + col0, q);
      PST(step);
      if (!wait_ge(errw, fails, tmo, mygrp, 0, 1, 32 * L, flag) || !seal_wait(g, 1)) { fail_exit(); return; }
      PST(step);
      f32x4 accm_c2[NTW][2];  // every tile's products (several chunks: one streamed pass, epilogues after it)
      if constexpr (KH) gemm_kh<kH>(P.a2, r0, nr, (smem + wb * kWPanel), accm_c2[0], wave, lane, PSTP(step), g, frag);
      else if constexpr (NTW == 1) gemm<kH>(P.a2, r0, nr, (smem + wb * kWPanel), accm_c2[0], wave, lane, PSTP(step), g, frag);
      else gemm_chunks<kH, NTW>(P.a2, r0, nr, (smem + wb * kWPanel), accm_c2, wave, lane, PSTP(step), g, frag, P.opt);
      PST(step);
#pragma unroll
      for (int ci = 0; ci < NTW; ++ci) {
        const int tl = wave + 4 * ci;
        const f32x4(&acc)[2] = accm_c2[ci];
        float v[2][4];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[nt][i] = gelu_fast(acc[nt][i] + b2v[nt][i]);
        }
        if (16 * tl < nr) store_op_t(P.u, g, s, tl, v, r0, nr, col0, TT, lane, frag);
        if (ci == 0) PST(step);  // (FL_STAMPS: the conv_2 epilogue broken down -- hand-off stores issued)
      }
      seal_put();
      if (dmafirst) {
        next_w(bw.w3);
        signal_dma<16>(mygrp);
      } else {
#ifdef FL_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PST(step);  // wave 0's hand-off stores acknowledged
        __syncthreads();
        PST(step);  // every wave's
#endif
        signal(mygrp);
        next_w(bw.w3);
      }
      PST(step);
      ++L;

      // -------- conv_3 (1x1) + ConvNeXt residual + gated residual (:92-93, 109, 156); x * alpha for the fold
      // (ova / ovb of the dwconv phase are this epilogue's LN vectors); raw loads only before the wait: alpha =
      // w (1 + scale) of the LayerNorm the next GEMM consumes (mlp / FinalLayer's second) is formed after it, or the
      // compiler waits for these loads ahead of the poll
      float g3[2][4], b3v[2][4], alv[2][4], alw[2][4];
      ld_cols(g3, mb + 2 * H + col0, q);
      ld_cols(b3v, bw.b3 + col0, q);
      ld_cols(alv, mb + 4 * H + col0, q);
      if (fin) fill_cols(alw, 1.0f);
      else ld_cols(alw, bw.lnmw + col0, q);
      PST(step);
      if (!wait_ge(errw, fails, tmo, mygrp, 0, 1, 32 * L, flag) || !seal_wait(g, 1)) { fail_exit(); return; }
      PST(step);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) alv[nt][r] = fin ? 1.0f + alv[nt][r] : alw[nt][r] * (1.0f + alv[nt][r]);
      f32x4 accm_c3[NTW][2];  // every tile's products (several chunks: one streamed pass, epilogues after it)
      if constexpr (KH) gemm_kh<kH>(P.u, r0, nr, (smem + wb * kWPanel), accm_c3[0], wave, lane, PSTP(step), g, frag);
      else if constexpr (NTW == 1) gemm<kH>(P.u, r0, nr, (smem + wb * kWPanel), accm_c3[0], wave, lane, PSTP(step), g, frag);
      else gemm_chunks<kH, NTW>(P.u, r0, nr, (smem + wb * kWPanel), accm_c3, wave, lane, PSTP(step), g, frag, P.opt);
      PST(step);
#pragma unroll
      for (int ci = 0; ci < NTW; ++ci) {
        const int tl = wave + 4 * ci;
        const f32x4(&acc)[2] = accm_c3[ci];
        float v[2][4];
        const int p = 16 * tl + c + kHalo;  // the lane's row (transposed layout)
        const float mean = st[2 * p], rstd = st[2 * p + 1];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float xh = (X[ci][nt][i] - mean) * rstd;
            const float h = xh * ova[nt][i] + ovb[nt][i];
            X[ci][nt][i] = X[ci][nt][i] + g3[nt][i] * (h + (acc[nt][i] + b3v[nt][i]));
            v[nt][i] = X[ci][nt][i] * alv[nt][i];
          }
        }
        if (16 * tl < nr) {
          store_partials_t(P.xpart[1], X[ci], r0, nr, s, tl, lane);
          store_op_t(P.xa, g, s, tl, v, r0, nr, col0, TT, lane, frag);
        }
      }
      seal_put();
      if (dmafirst) {
        if (fin) issue_out();  // conv_out's panel (into the other buffer; the flip follows the loop)
        else next_w(bw.m0);
        signal_dma<16>(mygrp);
      } else {
        signal(mygrp);
        if (fin) issue_out();
        else next_w(bw.m0);
      }
      PST(step);
      ++L;
      if (fin) break;  // conv_out follows the FinalLayer's conv_3

      // -------- mlp.0 + SiLU, the LayerNorm folded into the epilogue (:157-158)
      const float* fo0 = md + P.MS0 + (size_t)blk * 2 * H;  // [W alpha, W beta + b] of this modulation row
      float fa0[2][4], fb0[2][4];
      ld_cols(fa0, fo0 + col0, q);
      ld_cols(fb0, fo0 + H + col0, q);
      PST(step);
      if (!wait_ge(errw, fails, tmo, mygrp, 0, 1, 32 * L, flag) || !seal_wait(g, 1)) { fail_exit(); return; }
      PST(step);
      // the epilogue's row statistics of x (conv_3's partials) before the GEMM (issued between the GEMM's A loads and
      // their wait instead, r06j measured 20.84 vs 20.63 ms per B = 1 solve: slower)
      row_stats(P.xpart[1], TT, r0, r0 + nr, r0 - kHalo, st);
      f32x4 accm_m0[NTW][2];  // every tile's products (several chunks: one streamed pass, epilogues after it)
      if constexpr (KH) gemm_kh<kH>(P.xa, r0, nr, (smem + wb * kWPanel), accm_m0[0], wave, lane, PSTP(step), g, frag);
      else if constexpr (NTW == 1) gemm<kH>(P.xa, r0, nr, (smem + wb * kWPanel), accm_m0[0], wave, lane, PSTP(step), g, frag);
      else gemm_chunks<kH, NTW>(P.xa, r0, nr, (smem + wb * kWPanel), accm_m0, wave, lane, PSTP(step), g, frag, P.opt);  // (the first tile's barrier orders the statistics)
      PST(step);
#pragma unroll
      for (int ci = 0; ci < NTW; ++ci) {
        const int tl = wave + 4 * ci;
        const f32x4(&acc)[2] = accm_m0[ci];
        float v[2][4];
        const int p = 16 * tl + c + kHalo;  // the lane's row (transposed layout)
        const float mean = st[2 * p], rstd = st[2 * p + 1];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[nt][i] = silu(rstd * (acc[nt][i] - mean * fa0[nt][i]) + fb0[nt][i]);
        }
        if (16 * tl < nr) store_op_t(P.u, g, s, tl, v, r0, nr, col0, TT, lane, frag);
      }
      seal_put();
      if (dmafirst) {
        next_w(bw.m2);
        signal_dma<16>(mygrp);
      } else {
        signal(mygrp);
        next_w(bw.m2);
      }
      PST(step);
      ++L;

      // -------- mlp.2 + gated residual (:159-160)
      float g2v[2][4], bm2[2][4];
      ld_cols(g2v, mb + 5 * H + col0, q);
      ld_cols(bm2, bw.mb2 + col0, q);
      PST(step);
      if (!wait_ge(errw, fails, tmo, mygrp, 0, 1, 32 * L, flag) || !seal_wait(g, 1)) { fail_exit(); return; }
      PST(step);
      f32x4 accm_m2[NTW][2];  // every tile's products (several chunks: one streamed pass, epilogues after it)
      if constexpr (KH) gemm_kh<kH>(P.u, r0, nr, (smem + wb * kWPanel), accm_m2[0], wave, lane, PSTP(step), g, frag);
      else if constexpr (NTW == 1) gemm<kH>(P.u, r0, nr, (smem + wb * kWPanel), accm_m2[0], wave, lane, PSTP(step), g, frag);
      else gemm_chunks<kH, NTW>(P.u, r0, nr, (smem + wb * kWPanel), accm_m2, wave, lane, PSTP(step), g, frag, P.opt);
      PST(step);
#pragma unroll
      for (int ci = 0; ci < NTW; ++ci) {
        const int tl = wave + 4 * ci;
        const f32x4(&acc)[2] = accm_m2[ci];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) X[ci][nt][i] = X[ci][nt][i] + g2v[nt][i] * (acc[nt][i] + bm2[nt][i]);
        if (16 * tl < nr) {
          store_partials_t(P.xpart[0], X[ci], r0, nr, s, tl, lane);
          store_halo_t(P.ximg, X[ci], r0, nr, col0, tl, TT, lane);
        }
      }
      seal_put();
      if (dmafirst) {
        next_w(P.blk[blk + 1].w2);
        signal_dma<16>(mygrp);
      } else {
        signal(mygrp);
        next_w(P.blk[blk + 1].w2);
      }
      PST(step);
      ++L;
    }

    // -------- conv_out k3 (taps stacked; LayerNorm + modulate folded; :238-245, 264).  Panel row n < 24 is
    // tap n / 8 of latent channel 8 s + n % 8; rows 24..31 repeat rows 0..7 (ignored)
    wb ^= 1;  // conv_out's panel was issued behind the FinalLayer's conv_3
    float fac[2][4], fbc[2][4];  // fold vectors of the lane's stacked columns (transposed layout), before the wait
    {
      const float* fo = md + P.MS0 + (size_t)P.NB * 2 * H;  // [wa (3 C), wb (3 C)]
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = 16 * nt + 4 * q, m = n < 24 ? n : n - 24;  // 4 consecutive stacked columns from ns
        const int ns = (m >> 3) * kC + kCh * s + (m & 7);
        const float4 a = *reinterpret_cast<const float4*>(fo + ns), b = *reinterpret_cast<const float4*>(fo + 3 * kC + ns);
        fac[nt][0] = a.x; fac[nt][1] = a.y; fac[nt][2] = a.z; fac[nt][3] = a.w;
        fbc[nt][0] = b.x; fbc[nt][1] = b.y; fbc[nt][2] = b.z; fbc[nt][3] = b.w;
      }
    }
    PST(step);
    if (!wait_ge(errw, fails, tmo, mygrp, 0, 1, 32 * L, flag) || !seal_wait(g, 1)) { fail_exit(); return; }
    PST(step);
    row_stats(P.xpart[1], TT, r0, r0 + nr, r0 - kHalo, st);
    f32x4 acco[NTW][2];  // every tile's products first: with several chunks Y goes into this phase's panel buffer
    if constexpr (KH) gemm_kh<kH>(P.xa, r0, nr, (smem + wb * kWPanel), acco[0], wave, lane, PSTP(step), g, frag);
    else if constexpr (NTW == 1) gemm<kH>(P.xa, r0, nr, (smem + wb * kWPanel), acco[0], wave, lane, PSTP(step), g, frag);
    else gemm_chunks<kH, NTW>(P.xa, r0, nr, (smem + wb * kWPanel), acco, wave, lane, PSTP(step), g, frag, P.opt);
    PST(step);
    // Y of the group: [row][24] fp32 (tap-major x 8 channels) -- in the staging tile (one chunk), or in the
    // panel conv_out has just finished reading (several chunks: <= 512 x 24 x 4 B; the next panel DMA goes to the
    // other buffer, and this one is not rewritten before the next step's proj_in)
    float* yl = reinterpret_cast<float*>(NTW == 1 ? stg : smem + wb * kWPanel);
    if (NTW > 1) __syncthreads();  // every wave is done with the panel
#pragma unroll
    for (int ci = 0; ci < NTW; ++ci) {
      const int row = 16 * (wave + 4 * ci) + c, p = row + kHalo;  // the lane's row (transposed layout)
      if (NTW == 1 || row < nr) {
        const float mean = st[2 * p], rstd = st[2 * p + 1];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int n0 = 16 * nt + 4 * q;  // the lane's 4 stacked columns (n >= 24 repeat 0..7: not stored)
          if (n0 < 24) {
            float y[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) y[i] = rstd * (acco[ci][nt][i] - mean * fac[nt][i]) + fbc[nt][i];
            *reinterpret_cast<float4*>(yl + row * 24 + n0) = make_float4(y[0], y[1], y[2], y[3]);
          }
        }
      }
    }
    __syncthreads();
    // publish what the neighbouring groups' Euler updates need: Y0 of the last frame, Y2 of the first
    if (tid < 4 && nr > 0) {
      const __amdgpu_buffer_rsrc_t ry = rsrc(P.yb, kWGs * 16 * 4);
      const int half = tid >> 1, k = tid & 1;
      const float* src = half == 0 ? yl + (nr - 1) * 24 + 4 * k : yl + 16 + 4 * k;
      st16(ry, (unsigned)(((g + kGroups * s) * 16 + half * 8 + 4 * k) * 4), __builtin_bit_cast(u32x4, *reinterpret_cast<const float4*>(src)));
    }
    seal_put();
    if (dmafirst && step + 1 < P.s1) {
      next_win();
      signal_dma<4>(mygrp);
    } else {
      signal(mygrp);
      if (step + 1 < P.s1) next_win();
    }
    PST(step);
    ++L;

    // -------- Euler update x += dt * v, v[t] = b + Y1[t] + Y0[t-1] + Y2[t+1] (:445; conv3_combine order)
    PST(step);
    if (!wait_ge(errw, fails, tmo, grp, 16, kGroups, 32 * L, flag) || !seal_wait(0, kGroups)) { fail_exit(); return; }
    PST(step);
    int gp = 0, gn_ = 0;  // the groups owning frames r0 - 1 and r0 + nr (nearest non-empty neighbours)
    for (int k = 0; k < kGroups; ++k) {
      int a, b;
      group_rows(k, T, P.B, a, b, P.opt);
      if (b > 0 && a + b == r0) gp = k;
      if (b > 0 && a == r0 + nr) gn_ = k;
    }
#pragma unroll
    for (int ci = 0; ci < NTW; ++ci) {
      const int row = kChunk * ci + xr_row;
      if (row < nr) {
        const int t = r0 + row;
        const __amdgpu_buffer_rsrc_t ry = rsrc(P.yb, kWGs * 16 * 4);
        float vv[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int chl = 2 * (tid & 3) + e, ch = kCh * s + chl;
          float v = P.bout[ch] + yl[row * 24 + 8 + chl];
          if (t > ub) {  // zero padding at the utterance's edges (conv_out k3)
            const float y0 = row > 0 ? yl[(row - 1) * 24 + chl]
                                     : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           ry, (unsigned)(((gp + kGroups * s) * 16 + chl) * 4), 0, 16));
            v += y0;
          }
          if (t < ue - 1) {
            const float y2 = row < nr - 1 ? yl[(row + 1) * 24 + 16 + chl]
                                          : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                ry, (unsigned)(((gn_ + kGroups * s) * 16 + 8 + chl) * 4), 0, 16));
            v += y2;
          }
          vv[e] = v;
        }
        xs0[ci] = __fadd_rn(xs0[ci], __fmul_rn(P.dt, vv[0]));
        xs1[ci] = __fadd_rn(xs1[ci], __fmul_rn(P.dt, vv[1]));
      }
    }
    __syncthreads();  // yl (staging) is rewritten by publish_xs
    if (step + 1 < P.s1) publish_xs();
  }
  if (dseal) {  // the last wait's seals (no later seal_put checks them)
    int* okf = reinterpret_cast<int*>(smem + L_FLAG);
    if (tid == 0) *okf = 1;
    __syncthreads();
    if (!dseal_check() && lane == 0) *okf = 0;
    __syncthreads();
    if (*okf == 0) { fail_exit(); return; }
  }
#pragma unroll
  for (int ci = 0; ci < NTW; ++ci) {
    const int row = kChunk * ci + xr_row;
    if (row < nr && !idle) {
      P.xt[(size_t)(r0 + row) * kC + xch] = xs0[ci];
      P.xt[(size_t)(r0 + row) * kC + xch + 1] = xs1[ci];
    }
  }
}

#ifdef FL_STAMPS
static unsigned long long* g_pst_buf = nullptr;
static int g_pst_step = -1;
static float* g_gnd_buf = nullptr;
static int g_gnd_step = -1;
int persist_gndump(void* buf, int step) {
  g_gnd_buf = reinterpret_cast<float*>(buf);
  g_gnd_step = step;
  return kOk;
}
int persist_stamps(void* buf, int step) {
  g_pst_buf = reinterpret_cast<unsigned long long*>(buf);
  g_pst_step = step;
  return kOk;
}
#endif

// Every kernel variant: [0] the 2 x 2 wave-split GEMM (persist_opt 1024, one chunk), [ntw] ntw chunks per group.
static const void* const* persist_kernels() {
  static const void* const k[kMaxNTW + 1] = {
      reinterpret_cast<const void*>(den_persist_kernel<true, 1>), reinterpret_cast<const void*>(den_persist_kernel<false, 1>),
      reinterpret_cast<const void*>(den_persist_kernel<false, 2>), reinterpret_cast<const void*>(den_persist_kernel<false, 3>),
      reinterpret_cast<const void*>(den_persist_kernel<false, 4>), reinterpret_cast<const void*>(den_persist_kernel<false, 5>),
      reinterpret_cast<const void*>(den_persist_kernel<false, 6>), reinterpret_cast<const void*>(den_persist_kernel<false, 7>),
      reinterpret_cast<const void*>(den_persist_kernel<false, 8>)};
  static_assert(kMaxNTW == 8, "kernel table");
  return k;
}

bool persist_device_ok(int device) {
  int cus = 0, nb = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus != kWGs) return false;
  for (int i = 0; i <= kMaxNTW; ++i) {
    const void* k = persist_kernels()[i];
    if (set_max_lds(k) != hipSuccess) return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kThreads, kLds) != hipSuccess || nb < 1) return false;
  }
  return true;
}

int persist_launch(const Params& Pin, hipStream_t st, bool cooperative) {
  Params P = Pin;
#ifdef FL_STAMPS
  P.pst = g_pst_buf;
  P.pst_step = g_pst_step;
  P.gnd = g_gnd_buf;
  P.gnd_step = g_gnd_step;
#endif
  // Cooperative: the runtime checks the grid against the kernel's occupancy and rejects it up front
  // (hipErrorCooperativeLaunchTooLarge) instead of queueing workgroups behind resident ones that wait for
  // them.  Capturable: a captured cooperative launch replays cooperatively (MI355X_MICROARCH.md, Residency).
  void* args[] = {&P};
  if (P.ntw < 1 || P.ntw > kMaxNTW || ((P.opt & 1024) && P.ntw != 1)) {
    set_error("persistent solve: %d row chunks per group (1..%d; the wave-split GEMM variant takes one)", P.ntw, kMaxNTW);
    return kBadArg;
  }
  const void* kern = persist_kernels()[(P.opt & 1024) ? 0 : P.ntw];
  // tune coop 0: plain launch (profiling: rocprofv3's teardown faults after cooperative launches, README);
  // residency was checked by persist_eligible either way
  const hipError_t e = cooperative && tn().coop ? hipLaunchCooperativeKernel(kern, dim3(kWGs), dim3(kThreads), args, kLds, st)
                                   : hipLaunchKernel(kern, dim3(kWGs), dim3(kThreads), args, kLds, st);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error("persistent solve: hipLaunchCooperativeKernel -> %s", hipGetErrorString(e));
    return e == hipErrorCooperativeLaunchTooLarge ? kBadArg : kHip;
  }
  return kOk;
}

}  // namespace pk
}  // namespace fl

#ifdef FL_STAMPS
extern "C" FLAMED_API int flamed_persist_stamps(void* buf, int step) { return fl::pk::persist_stamps(buf, step); }
extern "C" FLAMED_API int flamed_persist_gndump(void* buf, int step) { return fl::pk::persist_gndump(buf, step); }
#endif

// Host-side check of the reset prologue's ticket arithmetic (include/flamed_diag.h; CPU unit test).
extern "C" FLAMED_API int flamed_persist_ticket(unsigned ticket, unsigned cur, unsigned* target, int* reached) {
  if (!target || !reached) return fl::kBadArg;
  *target = fl::pk::arrive_target(ticket);
  *reached = fl::pk::arrive_reached(cur, *target) ? 1 : 0;
  return fl::kOk;
}
