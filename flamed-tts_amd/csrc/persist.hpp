// Persistent B = 1 Euler solve: every step of ProbGenerator.sample's ODE loop (reference
// flamed/models/synthesizer/prob_generator.py:434-447; one SimpleMLPAdaLN.forward :349-365 per step)
// in ONE launch of 256 workgroups (one per CU), the phases of a step chained by in-launch hand-offs
// instead of 25 kernel boundaries.
//
// Work split (speed only; correctness never depends on placement).  Workgroup b is (group g, slot s); with the
// default persist_opt bit 8 the XCDs form a 2 x 4 grid: the round-robin dispatch puts b on XCD x = b % 8, which
// holds row groups 4 (x / 4) .. + 3 and slots 8 (x % 4) .. + 7 (so each weight panel is read by 2 XCDs and each
// group's hand-off rows by 4; without bit 8, g = b % 8 and s = b / 8: one group per XCD, every panel on all 8).
// Group g owns a contiguous range of <= 512 frames (equal shares of the utterance), processed as chunks of 64
// (four 16-row MFMA tiles, one per wave; NTW chunks: a kernel variant per chunk count); slot s owns hidden
// columns [32 s, 32 s + 32) and latent channels [8 s, 8 s + 8).  What stays on chip across phases:
//   * the residual stream X of the workgroup's (frames x 32 columns) tile, in registers;
//   * the Euler state x of its (frames x 8 channels), in registers across ALL steps (fp32);
//   * each GEMM phase's weight panel (32 output columns x K, bf16), LDS-DMA'd into one of two LDS
//     buffers by the previous GEMM phase, so a phase only waits for its activations.
// GEMM A operands (bf16 x_t, GroupNorm output, conv_2 / mlp.0 outputs, x * alpha) are handed over
// fragment-major (persist_opt 64, default): group g's rows as [16-row tile][32-wide K-step][lane][8 bf16],
// the exact register image of a v_mfma_f32_16x16x32_bf16 A operand, so each consumer wave's load of one
// K-step is one contiguous 1 KB (8 full lines) instead of 16 rows x 64 B (16 half-lines): the per-XCD L2
// request rate, not bytes, was what the A fetch waited on (2.4 -> 1.2 us per GEMM phase, 26.4 -> 22.8 ms).
// Every activation handed to another workgroup (bf16 GEMM operands, LayerNorm row partials, halo rows,
// GroupNorm partials, conv_out boundary rows) is stored write-through (sc1), drained by every storing
// wave, then one lane adds to a counter; consumers poll with sc1 loads and read the data with sc1
// loads only (cdna_hip_programming.md §6 Guideline 16, table row 1: no release / acquire fences).
//   group counters  grp[g]: the 32 slots of g add 1 after each group phase (GEMM operands, partials)
//   GroupNorm       gn[s]:  the 8 groups' slot-s workgroups add 1 after publishing their partials
// Per step: proj_in, 4 x (dwconv+GroupNorm, conv_2, conv_3, mlp.0, mlp.2), FinalLayer (dwconv+
// GroupNorm, conv_2, conv_3, conv_out), Euler update.  Numerics follow the bf16 launch path (bf16
// operands, fp32 accumulation / residual / statistics / state, the LayerNorm fold of mlp.0 and
// conv_out); GroupNorm statistics are exact per group (two passes) and Chan-combined across the 8
// groups in a fixed order (deterministic).  The grid is launched cooperatively (hipLaunchCooperativeKernel:
// all 256 workgroups co-resident, or the launch fails up front), so no wait depends on a workgroup that
// is not running.  Every spin is still bounded: a timeout sets the error word, every workgroup leaves and
// writes NaN into its part of x (a failed solve is loud, never silently wrong), and the first to set the
// word adds one to a sticky failure count the host reads after the fact (no host sync on the call path).
#pragma once
#include "common.hpp"

namespace fl {
namespace pk {

constexpr int kGroups = 8, kSlots = 32, kWGs = kGroups * kSlots, kThreads = 256;
constexpr int kH = 1024, kC = 256, kCols = kH / kSlots, kCh = kC / kSlots;
// A row group holds up to kMaxNTW chunks of kChunk = 64 frames (chunk i = 16-row tiles 4 i .. 4 i + 3, wave w owning
// tile 4 i + w): B x T <= 8 x 512 = 4096 frames (one 30 s utterance at 80 Hz is 2400; the reference's metadata
// batch of 4 at T = 1024).
constexpr int kChunk = 64, kMaxNTW = 8, kMaxRows = kChunk * kMaxNTW, kHalo = 15, kTaps = 31, kWin = kChunk + 2 * kHalo;
constexpr int kMaxNB = 8, kMaxT = kGroups * kMaxRows;
// LDS carve (bytes): two weight panels, the dwconv window (aliased by the epilogue staging tile), row
// statistics of the window, GroupNorm reduction scratch, poll flag
constexpr int kWPanel = kCols * kH * 2;
// dwconv window rows are padded to 36 floats: the transposed epilogue layout writes a lane's row as float4 pieces, and
// with a 32-float stride the 16 rows of one write would share 2 bank groups; at 36 they hit 16 distinct ones (and the
// depthwise conv's two rows per wave, 8 apart, fall in opposite bank halves)
constexpr int kHsLd = kCols + 4;
constexpr int L_HS = 2 * kWPanel;
constexpr int L_ST = L_HS + kWin * kHsLd * 4;
constexpr int L_RED = L_ST + (kMaxRows + 2 * kHalo) * 8;  // row statistics of the whole group window
constexpr int L_GNV = L_RED + 8 * kCols * 4;
constexpr int L_FLAG = L_GNV + kCols * 16;
constexpr int kLds = (L_FLAG + 16 + 15) / 16 * 16;
static_assert(kLds <= 160 * 1024, "persistent solve LDS");
// counters (ints, one 64-B line each); zeroed by the launch itself (its reset prologue)
constexpr int CT_GRP = 0, CT_GN = 16 * kGroups, CT_ERR = CT_GN + 16 * kSlots, kCtrInts = CT_ERR + 16;
// sticky words (never reset; zeroed once at allocation): failed launches, and the two monotonic arrival
// counters of the reset prologue, each on a 128-B line of its own
constexpr int SY_FAILS = 0, SY_ARRIVE0 = 32, SY_ARRIVE1 = 64, SY_PFAIL = 96, kStickyInts = 128;

// Reset-prologue arrival tickets, wrap-safe: every launch adds exactly kWGs to each arrival counter (unsigned),
// and 2^32 is a multiple of kWGs, so the launch a ticket belongs to starts at ticket - ticket % kWGs on either
// side of the 32-bit wrap; its arrivals are complete once the counter has moved kWGs past that base, compared
// by signed difference.  (Host-callable for the CPU unit test: flamed_persist_ticket.)
__host__ __device__ inline unsigned arrive_target(unsigned ticket) {
  return ticket - ticket % (unsigned)kWGs + (unsigned)kWGs;
}
__host__ __device__ inline bool arrive_reached(unsigned cur, unsigned target) { return (int)(cur - target) >= 0; }

struct BlockW {
  const bf16 *w2, *w3, *m0, *m2;
  const float *b2, *b3, *mb0, *mb2, *lnw, *lnb, *lnmw, *lnmb, *dww, *dwb, *gnw, *gnb;
};

struct Params {
  int T, NB, s0, s1;
  int B = 1;               // utterances (1, 2, 4 or 8), each T frames: utterance u owns row groups u 8/B .. + 8/B - 1
  int Bx = 0;              // > 0: only utterances < Bx carry data (a batch of 3 or 5..7 run as B = 4 / 8): the others
                           // compute on zeros, never read or write xt, and take modulation row Bx - 1 (mods hold
                           // nfe x Bx rows)
  float dt;
  const float* mods;
  int MS, MS0;
  const bf16* win;
  const float* bin;
  BlockW blk[kMaxNB + 1];  // [NB] = FinalLayer (w2, w3, b2, b3, dww, dwb, gnw, gnb)
  const bf16* wout;        // conv_out taps stacked (3 C) x H
  const float* bout;
  float* xt;               // Euler state (T x C), read at launch start, written at the end
  float2* xpart[2];        // LayerNorm row partials (mean, M2) over each slot's 32 columns: T x 32; [0]
                           // from proj_in / mlp.2 (read by the next dwconv phase of EVERY group: halo
                           // rows), [1] from conv_3 (read by mlp.0 / conv_out of the same group) -- two
                           // buffers, so a group's conv_3 never overwrites what a slower neighbour's
                           // dwconv phase is still reading
  float* ximg;             // X rows (fp32) near the group edges: dwconv halo of the neighbouring groups
  bf16* a2;                // GroupNorm output = conv_2 operand, T x H
  bf16* u;                 // conv_2 / mlp.0 output = conv_3 / mlp.2 operand, T x H
  bf16* xa;                // x * alpha (LayerNorm fold) = mlp.0 / conv_out operand, T x H
  bf16* xs;                // bf16(x) = proj_in operand, T x C
  float4* gnp;             // GroupNorm partials (n, mean, M2) per (group, channel): 8 x H
  float* yb;               // conv_out boundary rows per workgroup: Y0 of its last row, Y2 of its first
  int* ctr;
  int* seal;               // persist_opt 16384: per (group, slot) the number of its last group hand-off (16 B each)
  int* sticky;             // kStickyInts words never reset between launches: [SY_FAILS] failed launches so far
                           // (the host reads it after the fact), [SY_ARRIVE0/1] the reset prologue's arrivals
                           // (unsigned tickets), [SY_PFAIL] the last launch whose prologue failed (counted once)
  int inject_step = -1;    // diagnostic (flamed_tune persist_inject): every workgroup fails at this step
  int seal_skip = -1;      // diagnostic (flamed_tune persist_seal_skip): workgroup 5 does not store its seals in this step
  long long tmo;           // poll timeout, s_memrealtime ticks (100 MHz)
  int ntw = 1;             // row chunks (64 frames each) per group: the kernel variant (rows per group <= 64 ntw)
  int opt = 0;                        // experiment bits (flamed_tune persist_opt)
  unsigned long long* pst = nullptr;  // FL_STAMPS builds: timeline of step pst_step (persist_timeline.py)
  int pst_step = -1;
  float* gnd = nullptr;               // FL_STAMPS builds: GroupNorm exchange dump of step gnd_step (rowpart_probe.py)
  int gnd_step = -1;
};

// Host side (persist.hip): whether this device runs the 256-workgroup grid fully resident, and the launch.
bool persist_device_ok(int device);
// Row chunks per group for B utterances of T frames (group_rows' largest share; opt bit 2: whole 16-row tiles).
inline int persist_ntw(int B, int T, int opt) {
  const int gpu = kGroups / B;
  int R = (T + gpu - 1) / gpu;
  if (opt & 2) R = ((T + 15) / 16 + gpu - 1) / gpu * 16;
  return (R + kChunk - 1) / kChunk;
}
int persist_launch(const Params& P, hipStream_t st, bool cooperative = true);

}  // namespace pk
}  // namespace fl
