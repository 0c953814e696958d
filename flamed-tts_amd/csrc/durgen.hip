// PVA duration / silence flow-matching generators + integer length regulator on gfx950.
// Reference: flamed/models/synthesizer/pva.py:9-41 (SinusoidalPosEmb, TimeEmbedding), :88-116
// (PVA.sample Euler loop), :125-166 (LengthRegulator.LR), :173-238 (ProbabilisticModule),
// :241-284 (Conv); flamed/utils/tools.py:91-99 (get_mask_from_lengths), :299-317 (pad).
//
// Per Euler step and per net (dur, sil), M = B*L phoneme rows, all exact fp32 (f32 MFMA = fp32 FMA
// chains) so the rounded integer durations match the reference:
//   conv1 GEMM  A[m][tap*192+c] = P[src][c] + w0[c]*xt[src] + temb_s[c]  (proj + time embedding
//               folded in the loader; P = enc.W[:,1:]^T + b precomputed once)  -> +b, ReLU, LN partials
//   conv2 GEMM  A[m][tap*384+c] = LN1(R1[src])[c]                           -> +b, ReLU
//   head        LN2 + Linear(384->1) + masked_fill + Euler update, one wave per row
// The length regulator turns the final log-durations into frame counts (clamp(round(exp(d)-1),0),
// pva.py:111-112), builds the interleaved phone/silence repeat prefix sums, and gathers the frames.
#include "flamed_hip.h"
#include "gemm.hpp"
#include "pvaflow.hpp"

#include <mutex>
#include <vector>

namespace fl {

// SinusoidalPosEmb (pva.py:9-22), scale 1000, [sin, cos], frequency denominator (half-1).
__global__ void pos_emb_kernel(const float* __restrict__ t, int R, int dim, float* __restrict__ F) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= R * dim) return;
  int half = dim / 2;
  int r = idx / dim, j = idx - r * dim;
  int jj = j < half ? j : j - half;
  const float negemb = (float)(-9.210340371976184 / (double)(half - 1));
  float f = expf((float)jj * negemb);
  float a = (1000.0f * t[r]) * f;
  F[idx] = j < half ? sinf(a) : cosf(a);
}

// conv weight (N, Cin, KT) -> (N, KT, Cin) fp32 (K index = tap*Cin + c)
__global__ void taps_major_kernel(const float* __restrict__ src, float* __restrict__ dst, int N, int Cin, int KT) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)N * Cin * KT;
  if (i >= total) return;
  int k = i % KT;
  size_t t = i / KT;
  int c = t % Cin;
  int n = t / Cin;
  dst[((size_t)n * KT + k) * Cin + c] = src[i];
}

// proj weight (D, D+1): column 0 -> w0[D], columns 1.. -> We[D][D]
__global__ void split_proj_kernel(const float* __restrict__ src, float* __restrict__ w0, float* __restrict__ we, int D) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= D * (D + 1)) return;
  int r = i / (D + 1), c = i - r * (D + 1);
  if (c == 0) w0[r] = src[i];
  else we[(size_t)r * D + c - 1] = src[i];
}

// conv1 A operand: out0[src] = P[src] + w0 * xt[src] + temb (zero outside the utterance).  With a
// device step counter `ctr` the time-embedding row is temb + (*ctr) * Cin (graph replay).
struct LoadDurIn {
  const float* __restrict__ P;
  const float* __restrict__ w0;
  const float* __restrict__ xt;
  const float* __restrict__ temb;
  int Cin;
  int L;
  const int* __restrict__ ctr;
  struct Raw { float v[4]; };
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ Raw issue(int m, int k) const {
    Raw r;
    int tap = k / Cin, c = k - tap * Cin;
    int l = m % L + tap - 1;
    if (l < 0 || l >= L) {
      r.v[0] = r.v[1] = r.v[2] = r.v[3] = 0.f;
      return r;
    }
    int src = m + tap - 1;
    const float* tr = temb + (ctr ? (size_t)(*ctr) * Cin : 0);
    float4 p = ld4(P + (size_t)src * Cin + c), w = ld4(w0 + c), te = ld4(tr + c);
    float x = xt[src];
    r.v[0] = (p.x + w.x * x) + te.x;
    r.v[1] = (p.y + w.y * x) + te.y;
    r.v[2] = (p.z + w.z * x) + te.z;
    r.v[3] = (p.w + w.w * x) + te.w;
    return r;
  }
  template <typename D> __device__ u32x4 finish(const Raw& r, int, int, const float*, int) const { return pack_chunk<D>(r.v); }
};

// LN2 + Linear(F->1) + masked_fill(mask, 0) + Euler update; one wave per row.
template <int F>
__global__ __launch_bounds__(256) void dur_head_kernel(const float* __restrict__ R2, const float* __restrict__ g,
                                                       const float* __restrict__ b, const float* __restrict__ wl,
                                                       const float* __restrict__ bl, const uint8_t* __restrict__ mask,
                                                       float* xt, int M, float dt, int* ctr) {
  constexpr int PER = F / 64;
  if (ctr && blockIdx.x == 0 && threadIdx.x == 0) *ctr += 1;  // end of an Euler step (sil net head)
  int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (m >= M) return;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = R2[(size_t)m * F + lane + 64 * j];
    s += v[j];
  }
  float mean = wave_sum64(s) / (float)F;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    float d = v[j] - mean;
    q += d * d;
  }
  float rstd = 1.0f / sqrtf(wave_sum64(q) / (float)F + 1e-5f);
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    int c = lane + 64 * j;
    float y = ((v[j] - mean) * rstd) * g[c] + b[c];
    dot += y * wl[c];
  }
  dot = wave_sum64(dot);
  if (lane == 0) {
    float vel = mask[m] ? 0.f : dot + bl[0];
    xt[m] = __fadd_rn(xt[m], __fmul_rn(dt, vel));
  }
}

struct PvaGraph {
  hipGraphExec_t exec = nullptr;
  hipStream_t cap = nullptr, cap2 = nullptr;  // the two nets' chains are captured as parallel branches
  hipEvent_t fork = nullptr, join = nullptr;
  std::vector<const void*> key;
  int* ctr = nullptr;  // device Euler step counters: [0] duration chain, [1] silence chain
  void release() {
    retire_graph(exec);
    if (cap) (void)hipStreamDestroy(cap);
    if (cap2) (void)hipStreamDestroy(cap2);
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    if (ctr) (void)hipFree(ctr);
    *this = PvaGraph();
  }
};

struct DurNet {
  int D, F, KT;
  int device = -1;  // device of the packed weights
  std::mutex mu;    // one call at a time per handle
  char* dev = nullptr;
  float *w0, *we, *c1w, *c2w;  // packed
  const float *pb, *t1w, *t1b, *t2w, *t2b, *c1b, *g1, *b1, *c2b, *g2, *b2, *lw, *lb;  // copies in the arena
  PvaGraph graph;   // the (duration, silence) pair's cached flow graph, kept on the duration net's handle
  // split-K of the net's small-M GEMMs (their K chains, 18 / 36 fp32 K-steps, are the step's latency):
  // per-handle slab + self-resetting tile counters, so the two nets' concurrent graph branches never share
  SplitCtx split;
  char* split_mem = nullptr;
  static constexpr int kSplitTarget = 256, kSplitCounters = 1024;
  // persistent flow of the (duration, silence) pair (pvaflow.hpp), kept on the duration net's handle:
  // scratch (self-resetting counters, the sticky failure count, hand-off buffers of both nets; zeroed once at
  // allocation), a pinned copy of the failure count (refreshed asynchronously behind every uncaptured launch),
  // HIP events around the last uncaptured launch
  static constexpr int kPersistRetry = 3;  // failed launches before the pair stays on the graph path
  char* pmem = nullptr;
  int* pfail_host = nullptr;
  int pfails_seen = 0;
  hipEvent_t pev[2] = {nullptr, nullptr};
  bool pev_set = false;
  int pdev_ok[pv::kMaxRG + 1] = {-1, -1, -1, -1, -1, -1};  // per row-group count: the grid is all resident
  bool pbroken = false;
  int pruns = 0;
  void release_persist() {
    if (pev_set) (void)hipEventSynchronize(pev[1]);  // the last uncaptured launch still owns pmem
    if (pmem) (void)hipFree(pmem);
    if (pfail_host) (void)hipHostFree(pfail_host);
    for (hipEvent_t& e : pev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    pmem = nullptr;
    pfail_host = nullptr;
    pfails_seen = 0;
    pev_set = false;
  }
};

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }
static bool tune_snapshot_pva_split() { return tn().pva_split != 0; }

struct PvaWs {
  float *Fd, *TH, *TEMBd, *TEMBs, *Pd, *Ps, *R1, *S1, *R2, *R1s, *S1s, *R2s;  // R*/S* per net (chains run concurrently)
};
static size_t pva_ws_layout(const DurNet* n, int B, int L, int nfe, void* base, PvaWs* w) {
  size_t M = (size_t)B * L;
  size_t sizes[12] = {4ull * nfe * n->D, 4ull * nfe * 4 * n->D, 4ull * nfe * n->D, 4ull * nfe * n->D, 4 * M * n->D,
                      4 * M * n->D, 4 * M * n->F, 8 * M * (n->F / 64), 4 * M * n->F, 4 * M * n->F, 8 * M * (n->F / 64),
                      4 * M * n->F};
  size_t off = 0;
  float* p[12];
  for (int i = 0; i < 12; ++i) {
    p[i] = base ? (float*)((char*)base + off) : nullptr;
    off += a256(sizes[i]);
  }
  if (w) *w = PvaWs{p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9], p[10], p[11]};
  return off;
}

static int net_prepare(DurNet* n, const float* enc, int M, const float* ts, int nfe, float* F, float* TH, float* TEMB,
                       float* P, hipStream_t st) {
  const int D = n->D;
  hipLaunchKernelGGL(pos_emb_kernel, dim3((nfe * D + 255) / 256), dim3(256), 0, st, ts, nfe, D, F);
  FL_LAUNCH_CHECK();
  int rc;
  if ((rc = launch_gemm<float>(LoadF32<float>{F, D}, n->t1w, D, EpiBiasAct<float, 2>{n->t1b, TH, 4 * D}, nfe, 4 * D, D, st))) return rc;
  if ((rc = launch_gemm<float>(LoadF32<float>{TH, 4 * D}, n->t2w, 4 * D, EpiBiasAct<float, 0>{n->t2b, TEMB, D}, nfe, D, 4 * D, st))) return rc;
  if ((rc = launch_gemm<float>(LoadF32<float>{enc, D}, n->we, D, EpiBiasAct<float, 0>{n->pb, P, D}, M, D, D, st))) return rc;
  return kOk;
}

struct NetBufs {
  float *R1, *S1, *R2;
};
static int net_step(DurNet* n, const float* P, const float* temb, float* xt, const uint8_t* mask, int B, int L, float dt,
                    const NetBufs& w, hipStream_t st, const int* ctr = nullptr, int* ctr_inc = nullptr,
                    bool split = true) {
  const int M = B * L, D = n->D, F = n->F;
  const int NT = F / 64;
  SplitScope split_scope(split && n->split_mem && tune_snapshot_pva_split() ? &n->split : nullptr);
  int rc;
  if ((rc = launch_gemm_auto<float>(pick_cfg(M) == kCfgSmall ? kCfgSmall : kCfgMid, LoadDurIn{P, n->w0, xt, temb, D, L, ctr}, n->c1w, 3 * D,
                                          EpiBiasStatsT<true>{n->c1b, w.R1, F, w.S1, NT}, M, F, 3 * D, st)))
    return rc;
  if ((rc = launch_gemm<float>(LoadConvRows<float, true>{w.R1, F, L, 3, 1, w.S1, NT, 64, 1e-5f, n->g1, n->b1}, n->c2w,
                                          3 * F, EpiBiasAct<float, 3>{n->c2b, w.R2, F}, M, F, 3 * F, st)))
    return rc;
  hipLaunchKernelGGL(dur_head_kernel<384>, dim3((M + 3) / 4), dim3(256), 0, st, w.R2, n->g2, n->b2, n->lw, n->lb, mask, xt, M, dt, ctr_inc);
  FL_LAUNCH_CHECK();
  return kOk;
}

// -------- persistent flow (pvaflow.hpp) --------
static size_t pva_persist_layout(char* base, int F, pv::Params* P) {
  size_t off = 0;
  auto take = [&](size_t bytes) { char* p = base ? base + off : nullptr; off = a256(off + bytes); return p; };
  const size_t M = pv::kMaxM, CS = (size_t)F / pv::kCols;
  char* ctr = take(4 * (size_t)pv::kCtrInts);
  char* sticky = take(256);
  char* buf[2][3];
  for (int n = 0; n < 2; ++n) {
    buf[n][0] = take(M * F * 4);
    buf[n][1] = take(M * CS * 8);
    buf[n][2] = take(M * CS * 16);
  }
  if (P) {
    P->ctr = reinterpret_cast<int*>(ctr);
    P->sticky = reinterpret_cast<int*>(sticky);
    for (int n = 0; n < 2; ++n) {
      P->net[n].R1 = reinterpret_cast<float*>(buf[n][0]);
      P->net[n].S1 = reinterpret_cast<float2*>(buf[n][1]);
      P->net[n].S2 = reinterpret_cast<float4*>(buf[n][2]);
    }
  }
  return off;
}

// Row groups of the persistent flow for M rows: as many as the grid allows (48 workgroups each), at most
// kMaxTiles 16-row tiles per group; 0 = does not fit.
static int pva_persist_groups(int M, int F) {
  const int MT = (M + 15) / 16, per = 2 * F / pv::kCols;
  const int RG = std::min(std::min(MT, pv::kMaxRG), 256 / per);
  return (RG > 0 && MT <= RG * pv::kMaxTiles) ? RG : 0;
}

// Failed launches the kernel has counted since the pair's last look (the pinned copy lags at most one launch;
// exact once the stream of the last launch has been synchronised).  Never waits.
static void pva_poll_fails(DurNet* nd) {
  if (!nd->pfail_host) return;
  const int f = __atomic_load_n(nd->pfail_host, __ATOMIC_RELAXED);
  if (f <= nd->pfails_seen) return;
  nd->pfails_seen = f;
  if (f >= DurNet::kPersistRetry && !nd->pbroken) {
    nd->pbroken = true;
    fprintf(stderr, "flamed: %d persistent PVA flows failed (states NaN-poisoned); this pair uses the graph path from now on\n", f);
  } else {
    fprintf(stderr, "flamed: a persistent PVA flow failed (%d of %d allowed); its states were NaN-poisoned\n", f,
            DurNet::kPersistRetry);
  }
}

// Whether a use_graph flow of M rows runs as the persistent launch.  Allowed inside a stream capture (nothing
// on that path waits on the device).
static bool pva_persist_eligible(DurNet* nd, DurNet* ns, int M) {
  pva_poll_fails(nd);
  if (!tn().pva_persist || nd->pbroken || nd->D != 192 || nd->F != 384 || ns->D != 192 || ns->F != 384) return false;
  const int RG = pva_persist_groups(M, nd->F);
  if (RG == 0) return false;
  if (nd->pdev_ok[RG] < 0) nd->pdev_ok[RG] = pv::pva_persist_device_ok(nd->device, 2 * (nd->F / pv::kCols) * RG) ? 1 : 0;
  return nd->pdev_ok[RG] == 1;
}

static bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}

// Every step of both flows as ONE cooperative launch, only enqueued (no host synchronisation): the kernel
// resets its own counters; outside a capture HIP events around it and an async copy of the failure count follow
// it.  A failed launch leaves NaN in both states and is reported by the next call / flamed_pva_persist_status.
// *done = false: the runtime refused the cooperative grid (this row-group count never runs persistently on this
// device); the caller runs the graph path.
static int pva_persist_run(DurNet* nd, DurNet* ns, const PvaWs& w, const uint8_t* mask, float* dur_t, float* sil_t, int nfe,
                           int B, int L, float dt, hipStream_t st, bool* done) {
  *done = false;
  const int M = B * L;
  const bool cap = stream_capturing(st);
  if (!nd->pmem) {
    FL_REQUIRE(!cap, "persistent PVA flow: first use inside a stream capture (run it once uncaptured first)");
    const size_t bytes = pva_persist_layout(nullptr, nd->F, nullptr);
    FL_HIP(hipMalloc(&nd->pmem, bytes));
    FL_HIP(hipMemsetAsync(nd->pmem, 0, bytes, st));
  }
  if (!nd->pfail_host) {
    FL_REQUIRE(!cap, "persistent PVA flow: first use inside a stream capture (run it once uncaptured first)");
    FL_HIP(hipHostMalloc(reinterpret_cast<void**>(&nd->pfail_host), 16, hipHostMallocDefault));
    *nd->pfail_host = 0;
    nd->pfails_seen = 0;
  }
  pv::Params P{};
  pva_persist_layout(nd->pmem, nd->F, &P);
  P.M = M; P.L = L; P.MT = (M + 15) / 16; P.RG = pva_persist_groups(M, nd->F); P.nfe = nfe; P.dt = dt;
  P.mask = mask;
  const DurNet* nets[2] = {nd, ns};
  const float* Pn[2] = {w.Pd, w.Ps};
  const float* Tn[2] = {w.TEMBd, w.TEMBs};
  float* xn[2] = {dur_t, sil_t};
  for (int i = 0; i < 2; ++i) {
    const DurNet* n = nets[i];
    pv::NetP& o = P.net[i];
    o.P = Pn[i]; o.w0 = n->w0; o.temb = Tn[i]; o.c1w = n->c1w; o.c1b = n->c1b; o.g1 = n->g1; o.b1 = n->b1;
    o.c2w = n->c2w; o.c2b = n->c2b; o.g2 = n->g2; o.b2 = n->b2; o.lw = n->lw; o.lb = n->lb; o.xt = xn[i];
  }
  P.tmo = 50000000;  // 0.5 s of s_memrealtime (100 MHz) per wait
  P.inject_step = tn().pva_inject;
  P.stage = tn().pva_stage;
  if (!cap) {
    if (!nd->pev[0]) FL_HIP(hipEventCreate(&nd->pev[0]));
    if (!nd->pev[1]) FL_HIP(hipEventCreate(&nd->pev[1]));
    FL_HIP(hipEventRecord(nd->pev[0], st));
  }
  const int lrc = pv::pva_persist_launch(P, st);
  if (lrc == kBadArg) {  // cooperative grid refused: never again on this device for this row-group count
    nd->pdev_ok[P.RG] = 0;
    return kOk;
  }
  if (lrc) return lrc;
  if (!cap) {
    FL_HIP(hipEventRecord(nd->pev[1], st));
    nd->pev_set = true;
    FL_HIP(hipMemcpyAsync(nd->pfail_host, P.sticky, sizeof(int), hipMemcpyDeviceToHost, st));
  }
  *done = true;
  ++nd->pruns;
  return kOk;
}

// -------- length regulator --------
// One workgroup per utterance: repeats (interleaved phone/silence), exclusive prefix sum, total.
__global__ __launch_bounds__(256) void lr_lengths_kernel(const float* __restrict__ pd, const float* __restrict__ sd,
                                                         const int64_t* __restrict__ src_lens, int L, int log_domain,
                                                         int64_t* __restrict__ cum, int64_t* __restrict__ tgt_len) {
  __shared__ int64_t part[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n2 = 2 * L;
  const int per = (n2 + 255) / 256;
  const int64_t sl = src_lens[b];
  auto rep = [&](int j) -> int64_t {
    int l = j >> 1;
    float v = (j & 1) ? sd[(size_t)b * L + l] : pd[(size_t)b * L + l];
    if (log_domain) v = fmaxf(rintf(expf(v) - 1.0f), 0.0f);   // pva.py:111-112
    bool valid = l < sl;
    if (!(j & 1)) {
      int64_t r = valid ? (int64_t)rintf(v) : 0;              // pva.py:136-137 (round, clamp >= 1)
      return r < 1 ? 1 : r;
    }
    int64_t r = valid ? (int64_t)rintf(v) : 0;                // pva.py:139-140 (round, clamp >= 0)
    return r < 0 ? 0 : r;
  };
  int64_t s = 0;
  for (int q = 0; q < per; ++q) {
    int j = tid * per + q;
    if (j < n2) s += rep(j);
  }
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan of the thread totals
    int64_t v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int64_t run = tid ? part[tid - 1] : 0;
  int64_t* c = cum + (size_t)b * (n2 + 1);
  for (int q = 0; q < per; ++q) {
    int j = tid * per + q;
    if (j < n2) {
      c[j] = run;
      run += rep(j);
    }
  }
  if (tid == 255) {
    c[n2] = part[255];
    tgt_len[b] = part[255];
  }
}

// out[b][f] = x[b][src(f)] for f < tgt_len[b] (src = segment j's phoneme, silence -> phoneme 0), else 0.
__global__ __launch_bounds__(256) void lr_expand_kernel(const float* __restrict__ x, const int64_t* __restrict__ cum,
                                                        int L, int H, int T_out, float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.y;
  if (row >= T_out) return;
  const int n2 = 2 * L;
  const int64_t* c = cum + (size_t)b * (n2 + 1);
  float* o = out + ((size_t)b * T_out + row) * H;
  if ((int64_t)row >= c[n2]) {
    for (int h = lane; h < H; h += 64) o[h] = 0.f;
    return;
  }
  int lo = 0, hi = n2 - 1;  // last j with c[j] <= row and a non-empty segment
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (c[mid] <= (int64_t)row) lo = mid;
    else hi = mid - 1;
  }
  int src = (lo & 1) ? 0 : (lo >> 1);
  const float* xs = x + ((size_t)b * L + src) * H;
  for (int h = lane; h < H; h += 64) o[h] = xs[h];
}

}  // namespace fl

using namespace fl;

extern "C" {

FLAMED_API int flamed_dur_create(int input_size, int filter_size, int kernel, flamed_dur_t* out) {
  FL_REQUIRE(out, "flamed_dur_create: null out");
  FL_REQUIRE(kernel == 3, "flamed_dur_create: only kernel_size=3 is specialised (got %d)", kernel);
  FL_REQUIRE(input_size % 64 == 0 && filter_size == 384, "flamed_dur_create: unsupported dims input=%d filter=%d", input_size, filter_size);
  DurNet* n = new DurNet();
  n->D = input_size; n->F = filter_size; n->KT = kernel;
  *out = reinterpret_cast<flamed_dur_t>(n);
  return kOk;
}

FLAMED_API int flamed_dur_destroy(flamed_dur_t h) {
  DurNet* n = reinterpret_cast<DurNet*>(h);
  if (!n) return kOk;
  {
    std::lock_guard<std::mutex> lk(n->mu);
    DeviceGuard dg(n->device);
    n->graph.release();
    n->release_persist();
    if (n->dev) (void)hipFree(n->dev);
    if (n->split_mem) (void)hipFree(n->split_mem);
  }
  delete n;
  return kOk;
}

FLAMED_API int flamed_dur_load(flamed_dur_t h, const float* const* w, int nw, hipStream_t st) {
  DurNet* n = reinterpret_cast<DurNet*>(h);
  FL_REQUIRE(n && w && nw == FLAMED_DUR_W, "flamed_dur_load: expected %d weights", FLAMED_DUR_W);
  for (int i = 0; i < nw; ++i) FL_REQUIRE(w[i], "flamed_dur_load: weight %d is null", i);
  int wdev = -1;
  FL_REQUIRE(device_of(w[0], &wdev) == kOk, "flamed_dur_load: weights must be device memory");
  for (int i = 1; i < nw; ++i) FL_REQUIRE_ON(w[i], wdev, "flamed_dur_load");
  std::lock_guard<std::mutex> lk(n->mu);
  if (n->device >= 0 && n->device != wdev) {
    DeviceGuard og(n->device);
    n->graph.release();
    n->release_persist();
    for (int& v : n->pdev_ok) v = -1;
    if (n->dev) { (void)hipFree(n->dev); n->dev = nullptr; }
    if (n->split_mem) { (void)hipFree(n->split_mem); n->split_mem = nullptr; }
  }
  n->device = wdev;
  FL_ON_DEVICE(wdev);
  const int D = n->D, F = n->F;
  size_t o_w0 = 0, o_we = a256(4ull * D), o_c1 = o_we + a256(4ull * D * D), o_c2 = o_c1 + a256(4ull * F * 3 * D);
  size_t o_vec = o_c2 + a256(4ull * F * 3 * F);
  // vectors copied (the caller may free its tensors): pb D, t1w 4D x D, t1b 4D, t2w D x 4D, t2b D,
  // c1b g1 b1 c2b g2 b2 lw (F each), lb 1
  const size_t vec_floats = (size_t)D + 4ull * D * D + 4ull * D + 4ull * D * D + D + 7ull * F + 1;
  size_t total = o_vec + a256(4 * vec_floats + 64 * 4);
  if (n->dev) { FL_HIP(hipFree(n->dev)); n->dev = nullptr; }
  n->graph.release();
  FL_HIP(hipMalloc(&n->dev, total));
  if (!n->split_mem) {  // slab: up to kSplitTarget workgroups of 32 x 64 fp32 tiles; zeroed tile counters
    const size_t slab_floats = (size_t)DurNet::kSplitTarget * 32 * 64;
    FL_HIP(hipMalloc(&n->split_mem, 4 * slab_floats + 4 * DurNet::kSplitCounters));
    FL_HIP(hipMemsetAsync(n->split_mem + 4 * slab_floats, 0, 4 * DurNet::kSplitCounters, st));
    n->split.slab = reinterpret_cast<float*>(n->split_mem);
    n->split.slab_floats = slab_floats;
    n->split.cnt = reinterpret_cast<int*>(n->split_mem + 4 * slab_floats);
    n->split.cnt_n = DurNet::kSplitCounters;
    n->split.target = DurNet::kSplitTarget;
    n->split.max_split = 4;
    n->split.f32 = true;
  }
  n->w0 = (float*)(n->dev + o_w0); n->we = (float*)(n->dev + o_we);
  n->c1w = (float*)(n->dev + o_c1); n->c2w = (float*)(n->dev + o_c2);
  hipLaunchKernelGGL(split_proj_kernel, dim3((D * (D + 1) + 255) / 256), dim3(256), 0, st, w[0], n->w0, n->we, D);
  FL_LAUNCH_CHECK();
  size_t t1 = (size_t)F * D * 3, t2 = (size_t)F * F * 3;
  hipLaunchKernelGGL(taps_major_kernel, dim3((t1 + 255) / 256), dim3(256), 0, st, w[6], n->c1w, F, D, 3);
  FL_LAUNCH_CHECK();
  hipLaunchKernelGGL(taps_major_kernel, dim3((t2 + 255) / 256), dim3(256), 0, st, w[10], n->c2w, F, F, 3);
  FL_LAUNCH_CHECK();
  size_t vcur = o_vec;
  auto vec = [&](const float* src, size_t cnt, const float** dst) -> int {
    FL_HIP(hipMemcpyAsync(n->dev + vcur, src, 4 * cnt, hipMemcpyDeviceToDevice, st));
    *dst = reinterpret_cast<const float*>(n->dev + vcur);
    vcur += (4 * cnt + 15) & ~(size_t)15;  // 16-B aligned slots
    return kOk;
  };
  int rc;
#define TRY(x) do { if ((rc = (x)) != kOk) return rc; } while (0)
  TRY(vec(w[1], D, &n->pb)); TRY(vec(w[2], 4ull * D * D, &n->t1w)); TRY(vec(w[3], 4ull * D, &n->t1b));
  TRY(vec(w[4], 4ull * D * D, &n->t2w)); TRY(vec(w[5], D, &n->t2b)); TRY(vec(w[7], F, &n->c1b)); TRY(vec(w[8], F, &n->g1));
  TRY(vec(w[9], F, &n->b1)); TRY(vec(w[11], F, &n->c2b)); TRY(vec(w[12], F, &n->g2)); TRY(vec(w[13], F, &n->b2));
  TRY(vec(w[14], F, &n->lw)); TRY(vec(w[15], 1, &n->lb));
#undef TRY
  return kOk;
}

FLAMED_API size_t flamed_pva_workspace_size(flamed_dur_t h, int B, int L, int nfe) {
  DurNet* n = reinterpret_cast<DurNet*>(h);
  return n ? pva_ws_layout(n, B, L, nfe, nullptr, nullptr) : 0;
}

FLAMED_API int flamed_pva_flow(flamed_dur_t dur, flamed_dur_t sil, const float* enc, const uint8_t* mask, float* dur_t,
                               float* sil_t, const float* ts, int nfe, int B, int L, void* ws, size_t ws_bytes,
                               int use_graph, hipStream_t st) {
  DurNet* nd = reinterpret_cast<DurNet*>(dur);
  DurNet* ns = reinterpret_cast<DurNet*>(sil);
  FL_REQUIRE(nd && ns && nd->dev && ns->dev, "flamed_pva_flow: handles not loaded");
  FL_REQUIRE(nd->D == ns->D && nd->F == ns->F, "flamed_pva_flow: dur/sil nets differ in dims");
  FL_REQUIRE(enc && mask && dur_t && sil_t && ts && ws && nfe > 0 && B > 0 && L > 0, "flamed_pva_flow: bad args");
  FL_REQUIRE(nd->device == ns->device, "flamed_pva_flow: dur/sil handles live on different devices");
  std::unique_lock<std::mutex> lk_d(nd->mu, std::defer_lock), lk_s(ns->mu, std::defer_lock);
  if (nd == ns) lk_d.lock();
  else std::lock(lk_d, lk_s);
  FL_ON_DEVICE(nd->device);
  FL_REQUIRE_ON(enc, nd->device, "flamed_pva_flow");
  int tune_ep = 0;
  const Tune tsnap = tune_snapshot(&tune_ep);  // process defaults, read once for this call's GEMM launches
  TuneScope ts_(&tsnap);
  if (ws_bytes < pva_ws_layout(nd, B, L, nfe, nullptr, nullptr)) {
    set_error("flamed_pva_flow: workspace too small");
    return kNoWorkspace;
  }
  PvaWs w;
  pva_ws_layout(nd, B, L, nfe, ws, &w);
  const int M = B * L, D = nd->D;
  // delta_t = 1 / nfe as a python float, applied in fp32 (pva.py:99,106,109)
  const float dt = (float)(1.0 / (double)nfe);
  const NetBufs bd{w.R1, w.S1, w.R2}, bs{w.R1s, w.S1s, w.R2s};
  int rc;
  if ((rc = net_prepare(nd, enc, M, ts, nfe, w.Fd, w.TH, w.TEMBd, w.Pd, st))) return rc;
  if ((rc = net_prepare(ns, enc, M, ts, nfe, w.Fd, w.TH, w.TEMBs, w.Ps, st))) return rc;
  if ((use_graph & 1) && !(use_graph & 2) && pva_persist_eligible(nd, ns, M)) {
    bool done = false;
    if ((rc = pva_persist_run(nd, ns, w, mask, dur_t, sil_t, nfe, B, L, dt, st, &done))) return rc;
    if (done) return kOk;
  }
  if (!(use_graph & 1)) {
    for (int i = 0; i < nfe; ++i) {  // dur then sil on every step (pva.py:104-109)
      if ((rc = net_step(nd, w.Pd, w.TEMBd + (size_t)i * D, dur_t, mask, B, L, dt, bd, st))) return rc;
      if ((rc = net_step(ns, w.Ps, w.TEMBs + (size_t)i * D, sil_t, mask, B, L, dt, bs, st))) return rc;
    }
    return kOk;
  }
  // graph of G steps replayed nfe/G times; the step's time-embedding row comes from a device counter.
  // The duration and silence flows are independent chains (each net reads only its own x_t and the
  // encoder output, pva.py:104-109): they are captured as two parallel branches (fork/join events),
  // each with its own counter and scratch, and run concurrently.
  int G = 1;
  for (int g = 16; g > 1; --g)
    if (nfe % g == 0) { G = g; break; }
  PvaGraph& gp = nd->graph;
  if (!gp.ctr) FL_HIP(hipMalloc(&gp.ctr, 256));
  std::vector<const void*> key = {nd, ns, enc, mask, dur_t, sil_t, ts, ws, (const void*)(intptr_t)nfe,
                                  (const void*)(intptr_t)B, (const void*)(intptr_t)L, nd->dev, ns->dev,
                                  (const void*)(intptr_t)tune_ep};  // knobs (pva_split) are baked into the graph
  if (!gp.exec || gp.key != key) {
    retire_graph(gp.exec);
    if (!gp.cap) FL_HIP(hipStreamCreateWithFlags(&gp.cap, hipStreamNonBlocking));
    if (!gp.cap2) FL_HIP(hipStreamCreateWithFlags(&gp.cap2, hipStreamNonBlocking));
    if (!gp.fork) FL_HIP(hipEventCreateWithFlags(&gp.fork, hipEventDisableTiming));
    if (!gp.join) FL_HIP(hipEventCreateWithFlags(&gp.join, hipEventDisableTiming));
    FL_HIP(hipStreamBeginCapture(gp.cap, hipStreamCaptureModeRelaxed));
    int r = kOk;
    hipError_t fe = hipEventRecord(gp.fork, gp.cap);
    if (fe == hipSuccess) fe = hipStreamWaitEvent(gp.cap2, gp.fork, 0);
    if (fe != hipSuccess) r = kHip;
    // one handle for both nets: its split-K counters would be shared by the concurrent branches
    const bool split = nd != ns;
    for (int i = 0; i < G && r == kOk; ++i) r = net_step(nd, w.Pd, w.TEMBd, dur_t, mask, B, L, dt, bd, gp.cap, gp.ctr, gp.ctr, split);
    for (int i = 0; i < G && r == kOk; ++i)
      r = net_step(ns, w.Ps, w.TEMBs, sil_t, mask, B, L, dt, bs, gp.cap2, gp.ctr + 1, gp.ctr + 1, split);
    if (r == kOk) {
      fe = hipEventRecord(gp.join, gp.cap2);
      if (fe == hipSuccess) fe = hipStreamWaitEvent(gp.cap, gp.join, 0);
      if (fe != hipSuccess) r = kHip;
    }
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(gp.cap, &g);
    if (r) { if (g) (void)hipGraphDestroy(g); return r; }
    FL_HIP(e);
    hipError_t ie = hipGraphInstantiate(&gp.exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    FL_HIP(ie);
    gp.key = key;
  }
  FL_HIP(hipMemsetAsync(gp.ctr, 0, 2 * sizeof(int), st));
  for (int r = 0; r < nfe / G; ++r) FL_HIP(hipGraphLaunch(gp.exec, st));
  note_graph_use(gp.exec, st);
  return kOk;
}

FLAMED_API int flamed_pva_persist_ready(flamed_dur_t dur, flamed_dur_t sil, int B, int L, hipStream_t st) {
  DurNet* nd = reinterpret_cast<DurNet*>(dur);
  DurNet* ns = reinterpret_cast<DurNet*>(sil);
  FL_REQUIRE(nd && ns && nd->dev && ns->dev && B > 0 && L > 0, "flamed_pva_persist_ready: bad args");
  std::lock_guard<std::mutex> lk(nd->mu);
  FL_ON_DEVICE(nd->device);
  (void)st;  // the capture state no longer matters: the persistent launch is capturable
  return pva_persist_eligible(nd, ns, B * L) ? 1 : 0;
}

FLAMED_API int flamed_pva_persist_info(flamed_dur_t dur, int* runs, int* broken, float* last_ms) {
  DurNet* n = reinterpret_cast<DurNet*>(dur);
  FL_REQUIRE(n && runs && broken && last_ms, "flamed_pva_persist_info: bad args");
  std::lock_guard<std::mutex> lk(n->mu);
  DeviceGuard dg(n->device);
  *last_ms = 0.f;
  if (n->pev_set) {  // waits for the last uncaptured launch (a diagnostic query, not the call path)
    FL_HIP(hipEventSynchronize(n->pev[1]));
    FL_HIP(hipEventElapsedTime(last_ms, n->pev[0], n->pev[1]));
  }
  pva_poll_fails(n);
  *runs = n->pruns;
  *broken = n->pbroken ? 1 : 0;
  return kOk;
}

FLAMED_API int flamed_pva_persist_status(flamed_dur_t dur, int* runs, int* fails) {
  DurNet* n = reinterpret_cast<DurNet*>(dur);
  FL_REQUIRE(n && runs && fails, "flamed_pva_persist_status: bad args");
  std::lock_guard<std::mutex> lk(n->mu);
  *runs = n->pruns;
  *fails = n->pfail_host ? __atomic_load_n(n->pfail_host, __ATOMIC_RELAXED) : 0;
  pva_poll_fails(n);
  return kOk;
}

FLAMED_API int flamed_lr_lengths(const float* phone, const float* sil, const int64_t* src_lens, int B, int L,
                                 int log_domain, int64_t* cum, int64_t* tgt_len, hipStream_t st) {
  FL_REQUIRE(phone && sil && src_lens && cum && tgt_len && B > 0 && L > 0, "flamed_lr_lengths: bad args");
  int dv = -1;
  (void)device_of(cum, &dv);
  FL_ON_DEVICE(dv);
  hipLaunchKernelGGL(lr_lengths_kernel, dim3(B), dim3(256), 0, st, phone, sil, src_lens, L, log_domain, cum, tgt_len);
  FL_LAUNCH_CHECK();
  return kOk;
}

FLAMED_API int flamed_lr_expand(const float* x, const int64_t* cum, int B, int L, int H, int T_out, float* out,
                                hipStream_t st) {
  FL_REQUIRE(x && cum && out && B > 0 && L > 0 && H > 0 && T_out >= 0, "flamed_lr_expand: bad args");
  int dv = -1;
  (void)device_of(out, &dv);
  FL_ON_DEVICE(dv);
  if (T_out == 0) return kOk;
  hipLaunchKernelGGL(lr_expand_kernel, dim3((T_out + 3) / 4, B), dim3(256), 0, st, x, cum, L, H, T_out, out);
  FL_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
