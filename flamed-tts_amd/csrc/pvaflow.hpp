// Persistent PVA flow: every Euler step of BOTH flow-matching generators (duration and silence) in ONE
// launch.  Reference: flamed/models/synthesizer/pva.py:97-112 (PVA.sample loop: dur then sil each step),
// :173-238 (ProbabilisticModule: proj + time embedding -> Conv(k3) + ReLU -> LN -> Conv(k3) + ReLU -> LN ->
// Linear -> masked_fill), :241-284 (Conv).
//
// The launch-path flow (durgen.hip net_step) is three launches per net and step whose K chains are
// latency, not work (L = 60: 34 us per net evaluation for 0.18 MFLOP per row).  Here each net's two conv
// GEMMs are split over 24 workgroups of 16 output columns (F = 384) x up to 5 row groups of 16-row tiles,
// and each workgroup keeps its weight columns of BOTH convs resident in LDS for the whole solve (16 x
// (3 D + 3 F) fp32 = 110.6 KB), so a step moves only activations:
//   conv1  A = P[src] + w0 * x_t[src] + temb_s (tap gather, zero outside the utterance; P = proj's encoder
//          half + bias, hoisted) -> + b, ReLU -> R1 slice + LayerNorm partials (mean, M2 over 16 columns)
//          -> hand-off H1 (the row group and its two neighbours: conv2's taps reach one row across)
//   conv2  A = LN1(R1[src]) (statistics Chan-combined from the 24 partials, fixed order) -> + b, ReLU ->
//          per-row head partials over the slice: (mean, M2, sum (v - mean) g2 lw) -> hand-off H2
//   head   every workgroup combines the 24 partials of its rows and the halo rows (fixed order:
//          identical in every workgroup that computes a row), LN2 . lw + b2 . lw + lb, masked_fill, and
//          x_t += dt * v in LDS: no third hand-off, x_t never leaves the workgroups until the end.
// The head's dot is the centred partial form  rstd * sum_s [S_s + (mean_s - mean) G_s] + sum b2 lw + lb
// (G_s = sum over slice s of g2 lw): the same value as LN2(v) . lw to fp32 rounding.
// All arithmetic is fp32 (v_mfma_f32_16x16x4_f32, the K order permuted identically on both operands),
// as the launch path: the rounded integer durations must match the reference.
// Hand-offs follow cdna_hip_programming.md §6 Guideline 16 (write-through sc1 stores, vmcnt drain,
// barrier, relaxed agent-scope ticket; consumers poll and read with sc1 loads).  WAR safety without double
// buffers: a row group rewrites R1 / S1 only after H2 of the previous step, i.e. after every reader of
// those rows (itself and its two neighbours) has finished conv2; S2 only after H1 of the next step, i.e.
// after every reader has finished its head.  The launch is cooperative (every workgroup co-resident, or the
// runtime refuses it up front) and only enqueued: no host synchronisation, so it can be captured.  Every spin is
// bounded: a timeout sets the error word (the first to set it adds one to a sticky failure count the host reads
// asynchronously), every workgroup leaves, and x_t is written as NaN -- a failed flow is loud, never silently
// wrong (the Python wrapper waits for the flow, re-runs a failed one on the graph path, and after 3 failures the
// pair stays there).  The counter block resets itself: each workgroup counts its exit, the last one zeroes the
// block, so no memset node has to precede the kernel in a captured graph.
#pragma once
#include "common.hpp"

namespace fl {
namespace pv {

constexpr int kThreads = 256, kCols = 16, kMaxRG = 5, kMaxTiles = 8, kMaxRowsWG = 16 * kMaxTiles;
constexpr int kMaxM = kMaxRG * kMaxRowsWG;  // 640 phoneme rows (B * L)
constexpr int kLine = 16;                   // ints per counter (one 64-B line each)
constexpr int CT_H1 = 0, CT_H2 = 2 * kMaxRG * kLine, CT_ERR = 4 * kMaxRG * kLine, CT_EXIT = CT_ERR + kLine,
              kCtrInts = CT_EXIT + kLine;

struct NetP {
  const float *P, *w0, *temb, *c1w, *c1b, *g1, *b1, *c2w, *c2b, *g2, *b2, *lw, *lb;
  float* xt;    // flow state (M), read at launch start, written at the end by column slice 0
  float* R1;    // conv1 output, M x F
  float2* S1;   // LN1 partials, M x CS
  float4* S2;   // head partials, M x CS
};
struct Params {
  int M, L, RG, MT, nfe;
  float dt;
  const uint8_t* mask;
  NetP net[2];
  int* ctr;       // hand-off counters, error word, exit count: zero at launch start; the last workgroup to leave
                  // zeroes them again for the next launch (stream-ordered after this one)
  int* sticky;    // [0] failed launches so far (never reset; the host reads it asynchronously)
  int grid;       // workgroups of this launch (2 nets x CS slices x RG row groups)
  long long tmo;  // poll timeout, s_memrealtime ticks (100 MHz)
  int inject_step = -1;  // diagnostic (flamed_tune pva_inject): every workgroup abandons the flow at this step
  int stage = 1;         // row groups of >= 2 tiles: conv A windows staged through LDS in 32-channel chunks (tune pva_stage)
  unsigned long long* pst = nullptr;  // FL_STAMPS builds: per-workgroup timeline of step pst_step
  int pst_step = -1;
};
constexpr int kStampSlots = 16;

// LDS carve (bytes) for input size D, filter size F
template <int D, int F>
struct Lds {
  static constexpr int K1 = 3 * D, K2 = 3 * F, CS = F / kCols, XR = kMaxRowsWG + 4;
  static constexpr int W1 = 0, W2 = W1 + kCols * K1 * 4, W0 = W2 + kCols * K2 * 4, G1 = W0 + D * 4, B1 = G1 + F * 4,
                       TE = B1 + F * 4, XS = TE + D * 4, ST = XS + XR * 4, GS = ST + 2 * XR * 4, RED = GS + 32 * 4,
                       FLAG = RED + 4 * 64 * 16, UV = FLAG + 16, SA = UV + 2 * 3 * kCols * 4,
                       SAS = F + 4 /* staged row stride (floats) */;
  // one-tile groups: the conv A window (18 rows) staged in LDS; larger groups (Params::stage): two buffers of a
  // 64-channel chunk of a 4-tile pass window (66 rows, padded by 16 B), in the same bytes
  static constexpr int FC = 64, CBS = FC + 4, WMAX = kMaxRowsWG + 2, PROWS = 4 * 16 + 2, SA1 = 18 * SAS * 4,
                       SA2 = 2 * (PROWS + 1) * CBS * 4, BYTES = SA + (SA1 > SA2 ? SA1 : SA2);  // (+ a spare row)
  static_assert(K1 % 64 == 0 && K2 % 64 == 0 && D % 16 == 0 && F % kCols == 0, "pva persist dims");
  static_assert(RED % 16 == 0 && BYTES <= 160 * 1024, "pva persist LDS");
};

bool pva_persist_device_ok(int device, int grid);
int pva_persist_launch(const Params& P, hipStream_t st);
size_t pva_persist_lds();

}  // namespace pv
}  // namespace fl
