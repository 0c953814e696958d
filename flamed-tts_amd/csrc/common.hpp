// Common types, error plumbing and small device helpers for the Flamed MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <set>
#include <utility>
#include <vector>

namespace fl {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // SROA-friendly (HIP uint4 is a union struct)

// ---- error reporting (thread-local last error, C-ABI flamed_last_error) ----
void set_error(const char* fmt, ...);
const char* last_error();

enum Status : int {
  kOk = 0,
  kBadArg = 1001,      // invalid dims / null pointers / unsupported config
  kNoWorkspace = 1002, // workspace too small
  kHip = 1003,         // HIP runtime failure (message has details)
};

#define FL_HIP(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      ::fl::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return ::fl::kHip;                                                                 \
    }                                                                                    \
  } while (0)

// Completion events of cached graph execs: note_graph_use records one after a call's last replay of an exec
// (outside stream capture), retire_graph waits for it before destroying the exec.  The exec owns the
// replay's kernel-argument and node storage; freeing it under a queued replay is a use-after-free in the
// runtime.  Waiting on that exec's own event (not hipDeviceSynchronize) leaves other streams and any
// concurrent global-mode capture alone.
struct GraphEvents {
  std::mutex mu;
  std::map<hipGraphExec_t, hipEvent_t> ev;
};
inline GraphEvents& graph_events() {
  static GraphEvents g;
  return g;
}
inline void note_graph_use(hipGraphExec_t ex, hipStream_t st) {
  if (!ex) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;  // nested in a capture
  GraphEvents& g = graph_events();
  std::lock_guard<std::mutex> lk(g.mu);
  hipEvent_t& e = g.ev[ex];
  if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    e = nullptr;
    (void)hipStreamSynchronize(st);  // no event: fall back to draining this stream
    return;
  }
  (void)hipEventRecord(e, st);
}
inline void retire_graph(hipGraphExec_t& ex) {
  if (!ex) return;
  hipEvent_t e = nullptr;
  {
    GraphEvents& g = graph_events();
    std::lock_guard<std::mutex> lk(g.mu);
    auto it = g.ev.find(ex);
    if (it != g.ev.end()) {
      e = it->second;
      g.ev.erase(it);
    }
  }
  if (e) {
    (void)hipEventSynchronize(e);
    (void)hipEventDestroy(e);
  }
  (void)hipGraphExecDestroy(ex);
  ex = nullptr;
}

#define FL_REQUIRE(cond, ...)        \
  do {                               \
    if (!(cond)) {                   \
      ::fl::set_error(__VA_ARGS__);  \
      return ::fl::kBadArg;          \
    }                                \
  } while (0)

#define FL_LAUNCH_CHECK()                                                                  \
  do {                                                                                     \
    hipError_t e_ = hipGetLastError();                                                     \
    if (e_ != hipSuccess) {                                                                \
      ::fl::set_error("%s:%d kernel launch -> %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return ::fl::kHip;                                                                   \
    }                                                                                      \
  } while (0)

// ---- device pinning ----
// A handle lives on the device of the weights it was loaded from (hipPointerGetAttributes); every entry
// point makes that device current for its duration and restores the caller's, so a call from a thread
// whose current device differs (e.g. `--device cuda:1` in one process) allocates and launches on the
// handle's device instead of dereferencing its memory from another GPU.
int device_of(const void* p, int* dev);  // kOk, or kBadArg for a pointer HIP does not know
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if (dev < 0) return;
    int cur = -1;
    err = hipGetDevice(&cur);
    if (err == hipSuccess && cur != dev) {
      err = hipSetDevice(dev);
      if (err == hipSuccess) prev = cur;
    }
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
#define FL_ON_DEVICE(dev)                                                          \
  ::fl::DeviceGuard dg_(dev);                                                      \
  do {                                                                             \
    if (dg_.err != hipSuccess) {                                                   \
      ::fl::set_error("%s:%d hipSetDevice(%d) -> %s", __FILE__, __LINE__, (dev),  \
                      hipGetErrorString(dg_.err));                                 \
      return ::fl::kHip;                                                           \
    }                                                                              \
  } while (0)
// `p` (a caller tensor) must live on the handle's device `dev`.
#define FL_REQUIRE_ON(p, dev, what)                                                                   \
  do {                                                                                                \
    int pd_ = -1;                                                                                     \
    if (::fl::device_of((p), &pd_) == ::fl::kOk && (dev) >= 0 && pd_ != (dev)) {                      \
      ::fl::set_error("%s: tensor on device %d but the handle lives on device %d", (what), pd_, (dev)); \
      return ::fl::kBadArg;                                                                           \
    }                                                                                                 \
  } while (0)

// ---- tuning knobs (flamed_tune / flamed_den_tune) ----
// Process defaults are set by flamed_tune under a mutex and bump an epoch; a handle snapshots them
// (or keeps its own, after flamed_den_tune) and every launch of a handle call reads the calling
// thread's active snapshot (TuneScope), so concurrent calls on different handles / threads never see a
// knob change halfway through a step.
struct Tune {
  int split_target = 1;    // split-K off by default: slower at B = 1 (profiles/r01_splitk_sweep.txt)
  int split_max = 4;
  int small_stages = 3;    // small-M register pipeline (3 | 5 | 7)
  int xcd_strips = 0;      // small/mid-M tile placement strips (0 = off)
  int bn32 = 1;            // 32 x 32 tiles below kTinyRows rows
  int use_dma = 1;         // 1: LDS-DMA main loop for bf16-A small-M GEMMs; 2: also fp32-A; 0: off
  int dma_ns = 3;          // small-M DMA ring depth
  int noctr = 0;           // diagnostic: ignore the device step counter
  int dup_class = -1;      // ablation: launch this kernel class twice per step
  int stamp_class = -1;    // diagnostic (FL_STAMPS builds)
  int dw_cg32_rows = 1536; // below: narrow depthwise workgroups
  int dw_cg_small = 32;    // their channel width (16 | 32)
  int dw_tc_big = 64;      // large-M depthwise T-chunk (64 | 128)
  int big = 1;             // large-M bf16 path
  int big_min_rows = 1536;
  int big_ns = 2;          // its LDS ring depth
  int lnfold = 1;          // LayerNorm fold into mlp.0 / conv_out epilogues (bf16)
  int fold_big_rows = 6144;
  int graph_steps = 16;    // Euler steps per captured solve graph
  int x16 = 0;             // large-M path: bf16 residual stream X and depthwise output D
  int g8p_rows = 12800;    // large-M GEMMs from this many rows on 256 x 256 8-phase tiles (0 = off); 12800: the B = 64
                           // split chains (2 x 12800 rows) take them too (311 -> 278 ms, r05bi)
  int dwgn = 1;            // large-M path: whole-utterance depthwise conv + GroupNorm kernel (T <= 512)
  int dwgn_small = 1;      // small-M bf16 path: one-workgroup-per-8-channels depthwise conv + GroupNorm (T <= 576)
  int fuse_euler = 1;      // small-M solve graphs: conv_out combine + Euler update inside the next proj_in
  int persist = 1;         // B = 1 bf16 solves: one persistent launch for all steps (persist.hpp)
  int split_batch = 2;     // large-M bf16 solves: sub-batch chains as parallel graph branches (den_split)
  int split_graph = 0;     // split chains: 0 one graph per chain on its own (priority) stream, 1 one graph with branches
  int prio_all = 0;       // experiment: every graph-path solve replays on the handle's chain-0 stream of split_prio
  int split_prio = 2;      // split chains' replay streams (den_chain_streams): 0 caller + highest, 1 all low, 2 all high
  int split_min_rows = 6144;  // ... when every chain still has this many rows
  int persist_seal_skip = -1;  // diagnostic: one workgroup skips its hand-off seals in this step (seal modes must fail)
  int persist_inject = -1; // diagnostic: every persistent launch fails at this step (-1 = never)
  int persist_pad = 1;     // persistent solve for B = 3 / 5..7 as B = 4 / 8 with idle utterances (persist_batch)
  int persist_pad_ntw = 4; // ... and a batch padded to >= 1.5x its size (B = 5 as 8) only up to this many chunks per row
                           // group: the idle utterances cost whole chunks (r06au / r06av: B = 5 T = 500, eight chunks,
                           // 84.5 ms vs 80.8 on the graph of launches, B = 5 T = 300, five chunks, 53.5 vs 50.0; B = 6 T = 300 52.7 vs 74.3, B = 3 T = 400 42.4 vs 46.6, B = 7
                           // T = 256 44.9 vs 72.6, B = 3 T = 800 (seven chunks) 73.2 vs 78.6 stay persistent)
  int persist_multi = 1;   // persistent solve also for B = 2 / 4 / 8 utterances (each group inside one utterance)
  int persist_ntw = 8;     // persistent solve up to this many 64-frame chunks per row group (1: T <= 512 per utterance)
  int persist_multi_ntw = 8;  // ... and for B > 1 up to this many (A/B knob).  r06c, with the round-5 epilogues, had the
                           // graph of launches ahead beyond 2 chunks (B = 4 T = 400: 60.4 ms persistent); with the
                           // transposed register epilogues (r06i) the persistent launch wins at every multi-chunk shape
                           // measured: B = 4 T = 400 47.4 vs 76.1 ms, B = 4 T = 300 38.6 vs 45.5, B = 8 T = 320 61.9 vs
                           // 77.3, B = 2 T = 1000 51.7 vs 76.0; B = 3 T = 400 (padded to 4) 47.5 vs 46.6.  Six to eight
                           // chunks (r06ac, K-outer GEMM; B x T <= 4096): B = 4 T = 800 73.3 vs 86.0 ms, B = 3 T = 800
                           // 73.2 vs 78.6, B = 4 T = 1024 85.7 vs 90.5, B = 8 T = 500 85.0 vs 86.1, B = 1 T = 3000 (nfe 256)
                           // 128.0 vs 174.0
  int persist_capmode = 0; // persistent launch inside a stream capture: 0 cooperative node, 1 plain kernel node
  int persist_opt = 885322;  // persistent kernel variant bits (pk::Params::opt): 8 = XCD-grouped grid,
                           // 64 = fragment-major GEMM A images, 512 = tagged-granule GroupNorm exchange
                           // (measured per B = 1 T = 400 solve: 26.4 -> 22.8 -> 21.7 ms), 65536 = deferred hand-off
                           // seals (default-on verification, +2.5 %), 262144 = one gemm() per 64-frame chunk
                           // (multi-chunk solves 8 % faster than gemm_multi), 32768 = wave-local staging order (default since
                           // r05bn: B = 2 T = 400 32.1 -> 31.7 ms, long-form 156 -> 152.6 ms, B = 1 neutral);
                           // 2 = row groups of whole 16-row tiles (default since r06c: B = 1 T = 400 20.93 -> 20.55 ms,
                           // B = 2 31.97 -> 31.43 ms; the r05 counter- vs granule-form GroupNorm divergence under it was
                           // FMA contraction in one of two inlined combines, fixed by gn_finalize);
                           // 524288 = K-outer multi-chunk GEMM gemm_ko (default since r06x, same box: T = 2400
                           // 130.7 -> 126.9 ms, B = 2 T = 400 28.0 -> 26.0, B = 4 T = 400 51.7 -> 46.9, T = 800
                           // 28.2 -> 26.2, B = 8 T = 300 32.9 -> 32.0; B = 1 T <= 512 has one chunk: unaffected);
                           // A/B bits: 1 = four-wave weight DMA (round 3
                           // default; since round 5 waves 1..3 issue, so wave 0's poll never waits behind weight loads:
                           // 21.50 -> 21.18 ms), 16384 blocking seals (+12 %),
                           // 1024 2 x 2 wave split, 4096 drain behind the DMA.  Removed after measuring: the GEMM
                           // phases' deferred seal loads issued after the GEMM (r06ap neutral as a bit, but its code
                           // slowed the default kernel 2-5 %, r06ar)
  int pva_split = 0;       // PVA nets: split-K of their small-M fp32 GEMMs (fixed slice order); measured
                           // neutral (L = 60 / 247, 64 steps: 2.70 / 2.94 vs 2.61 / 2.92 ms), so off
  int pva_persist = 1;     // PVA flow: both nets, every step, one persistent launch (pvaflow.hpp; B*L <= 640)
  int attn_mfma = 1;       // transformer attention (prior stack, timbre encoder) on fp32 MFMA (xfmr.hpp)
  int prior_split = 1;     // bf16 prior decoders: split-K of the GEMMs with small tile grids
  int pva_stage = 1;       // PVA persistent flow: conv A windows of >= 2-tile row groups staged through LDS in chunks
  int pva_inject = -1;     // diagnostic: every persistent PVA flow fails at this step (-1 = never)
  int dwgn_var = 1;        // dwgn kernel variant: 1 scalar fp32 pair math (default), diagnostics for T in (384, 448]: 0 packed, 2 scalar LDS accesses
  int coop = 1;            // persistent kernels as cooperative launches (0: plain launches, for profiling runs)
  int stop_after = -1;     // diagnostic: a denoiser evaluation returns after this many kernel-class launches (-1 = never)
};
int tune_apply(Tune& t, const char* key, int value);  // kOk or kBadArg (message set)
Tune tune_snapshot(int* epoch);                       // process defaults + their epoch
int tune_epoch();
extern thread_local const Tune* tl_tune;
const Tune& tune_defaults_unlocked();
inline const Tune& tn() { return tl_tune ? *tl_tune : tune_defaults_unlocked(); }
struct TuneScope {
  const Tune* prev;
  explicit TuneScope(const Tune* t) : prev(tl_tune) { tl_tune = t; }
  ~TuneScope() { tl_tune = prev; }
};

// Opt a kernel into 160 KB of dynamic LDS once per (kernel, device): the attribute is per device, so a
// process driving several GPUs sets it on each.
template <typename Tag = void>
inline hipError_t set_max_lds(const void* kern) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({kern, dev})) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e == hipSuccess) done.insert({kern, dev});
  return e;
}

// Copies of the caller's small vectors (biases, norm gains, activation parameters, filters) into a
// handle's own arena, so a handle never points at caller memory: collected while the arena is laid out
// (add), copied once it is allocated (commit, stream-ordered device-to-device).
struct VecCopies {
  struct Item { const float* src; size_t n; const float** dst; size_t off; };
  std::vector<Item> items;
  size_t bytes = 0;
  void add(const float* src, size_t n, const float** dst) {
    items.push_back(Item{src, n, dst, bytes});
    bytes += (4 * n + 15) & ~(size_t)15;
  }
  int commit(char* base, hipStream_t st) {
    for (const Item& it : items) {
      FL_HIP(hipMemcpyAsync(base + it.off, it.src, 4 * it.n, hipMemcpyDeviceToDevice, st));
      *it.dst = reinterpret_cast<const float*>(base + it.off);
    }
    return kOk;
  }
};

// ---- device helpers ----
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// erf by Abramowitz & Stegun 7.1.26 (|err| <= 4.7e-7 in fp32 with v_rcp_f32 / v_exp_f32, measured over
// [-6, 6]); ~15 VALU ops against ocml erff's branchy ~40 (the GELU epilogue of the B = 64 conv_2 GEMM
// spent 13.7 us per workgroup in erff).  Used only where the result is rounded to bf16 next.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  const float p = ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t + 0.254829592f) * t;
  return copysignf(1.0f - p * __expf(-ax * ax), x);
}
__device__ __forceinline__ float gelu_fast(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

// v + the value of another lane, picked by a DPP control (a VALU operand modifier: no LDS round trip, unlike
// __shfl_xor's ds_bpermute): quad_perm [1,0,3,2] = lane ^ 1, [2,3,0,1] = lane ^ 2 (within a quad),
// row_half_mirror (lane i <-> 7 - i of each 8), row_mirror (lane i <-> 15 - i of each 16).
template <int kCtrl>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), kCtrl, 0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

// Sum over the 16 lanes sharing lane >> 4.  Bitwise the same as the xor-1/2/4/8 butterfly: after the two quad
// steps every lane of a quad holds the quad sum, so the half-row and row mirrors add exactly the partner sums
// the xor-4 and xor-8 steps add (fp32 addition is commutative).
__device__ __forceinline__ float wave_sum16(float v) {
  v = dpp_add<kDppXor1>(v);
  v = dpp_add<kDppXor2>(v);
  v = dpp_add<kDppHalfMirror>(v);
  v = dpp_add<kDppMirror>(v);
  return v;
}

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Chan et al. parallel combine of (count, mean, M2) partials.
// An empty partial (nb <= 0) contributes nothing, whatever its mean / M2 words hold.
// chan_combine with every operation rounded on its own (no FMA contraction): the persistent solve's two GroupNorm
// exchange forms each inline their own copy of the combine, and -ffp-contract=fast let the compiler fuse
// `mean + d * (nb / nn)` in one copy and not in the other, so the forms parted by an ulp whenever the groups' counts
// were unequal (persist_opt bit 2 at B = 4 T = 100: groups of 48 and 52 frames; tools/rowpart_probe.py --dump).
__device__ __forceinline__ void chan_combine_rn(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
#pragma clang fp contract(off)
  if (nb <= 0.f) return;
  const float nn = n + nb;
  if (nn <= 0.f) return;
  const float d = meanb - mean;
  mean = mean + d * (nb / nn);
  m2 = m2 + (m2b + (d * d) * ((n * nb) / nn));
  n = nn;
}

__device__ __forceinline__ void chan_combine(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  if (nb <= 0.f) return;
  float nn = n + nb;
  if (nn <= 0.f) return;
  float d = meanb - mean;
  mean += d * (nb / nn);
  m2 += m2b + d * d * (n * nb / nn);
  n = nn;
}

template <typename DT> struct DTraits;
template <> struct DTraits<bf16> {
  static constexpr int EPC = 8;  // elements per 16-byte chunk
  static constexpr int kCode = 1;
};
template <> struct DTraits<float> {
  static constexpr int EPC = 4;
  static constexpr int kCode = 0;
};

// 16-byte chunk of DT built from EPC floats.
template <typename DT> __device__ __forceinline__ u32x4 pack_chunk(const float* v);
template <> __device__ __forceinline__ u32x4 pack_chunk<float>(const float* v) {
  return u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
}
template <> __device__ __forceinline__ u32x4 pack_chunk<bf16>(const float* v) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (bf16)v[j];
  return __builtin_bit_cast(u32x4, b);
}

template <typename DT> __device__ __forceinline__ void store_val(DT* p, float v) { *p = (DT)v; }
// four consecutive values (16-B fp32 / 8-B bf16 store; p aligned accordingly)
template <typename DT> __device__ __forceinline__ void store_val4(DT* p, const float* v);
template <> __device__ __forceinline__ void store_val4<float>(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void store_val4<bf16>(bf16* p, const float* v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 b;
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = (bf16)v[j];
  *reinterpret_cast<uint2*>(p) = __builtin_bit_cast(uint2, b);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Four / eight consecutive activations of type T (fp32 or bf16) as fp32 (16-B / 8-B / 16-B loads).
template <typename T> __device__ __forceinline__ float4 ldx4(const T* p);
template <> __device__ __forceinline__ float4 ldx4<float>(const float* p) { return ld4(p); }
template <> __device__ __forceinline__ float4 ldx4<bf16>(const bf16* p) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const bf16x4 b = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(p));
  return make_float4((float)b[0], (float)b[1], (float)b[2], (float)b[3]);
}
template <typename T> __device__ __forceinline__ void ldx8(const T* p, float* o);
template <> __device__ __forceinline__ void ldx8<float>(const float* p, float* o) {
  const float4 a = ld4(p), b = ld4(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <> __device__ __forceinline__ void ldx8<bf16>(const bf16* p, float* o) {
  const bf16x8 b = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p));
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (float)b[j];
}

// ---- phase stamps (diagnostic build only: -DFL_STAMPS, libflamed_hip_stamps.so) ----
// Thread 0 of every block writes s_memtime at numbered checkpoints into fl_stamp_buf[block][8]
// when the host has pointed fl_stamp_buf at a buffer (one chosen kernel class per step).
#ifdef FL_STAMPS
static __device__ unsigned long long* fl_stamp_buf = nullptr;  // per translation unit (no -fgpu-rdc)
__device__ __forceinline__ void fl_stamp(int i) {
  if (threadIdx.x == 0 && fl_stamp_buf) {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    const size_t blk = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
    fl_stamp_buf[blk * 8 + i] = t;
  }
}
#define FL_STAMP(i) ::fl::fl_stamp(i)
#else
#define FL_STAMP(i) ((void)0)
#endif

}  // namespace fl
