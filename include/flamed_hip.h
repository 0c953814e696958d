/* flamed_hip.h — C-ABI of the MI355X (gfx950) Flamed-TTS flow-matching hot path.
 *
 * The reference (nghiahuynh-ai/Flamed-TTS) is pure Python/PyTorch with no FFI layer; its drop-in
 * boundary is the Python module API.  This library is what the build's Python
 * modules (flamed-tts_amd/flamed/...) bind through ctypes; each entry point below names the
 * reference function whose work it replaces.
 *
 * Conventions: every tensor argument is a DEVICE pointer owned by the caller, row-major, fp32
 * unless stated; work is enqueued on `stream` and is stream-ordered (no host synchronisation
 * inside, so every call is hipGraph-capturable except the *_load / *_create calls and the documented
 * diagnostic queries).  Scratch memory
 * comes from a caller-provided workspace sized by the matching *_workspace_size query.
 * Handles: *_load copies or packs every weight and vector into the handle's own device arena (the
 * caller's tensors may be freed afterwards) on the device those tensors live on; each call on a
 * handle runs on that device and is serialised per handle (one stream at a time: the handle's step
 * counters and cached graphs are per handle).  Diagnostic probes live in include/flamed_diag.h
 * (libflamed_diag.so), not in this library.
 * Return value: 0 on success, otherwise a status code (1001 bad argument, 1002 workspace too small,
 * 1003 HIP runtime error); flamed_last_error() describes the last failure of the calling thread.
 */
#ifndef FLAMED_HIP_H
#define FLAMED_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLAMED_API __attribute__((visibility("default")))

/* Compute dtypes.  FLAMED_FP8 (denoiser handles only): FLAMED_BF16 everywhere, plus MX-fp8 (OCP e4m3 with
 * one e8m0 scale per 32 input channels, weights and activations) for the four H x H pointwise GEMMs of
 * every block (conv_2, conv_3, mlp.0, mlp.2; BASELINE configs[4]) on the large-M path (B*T >= the
 * g8p_rows knob, default 12800); below it the handle computes exactly as FLAMED_BF16. */
enum { FLAMED_F32 = 0, FLAMED_BF16 = 1, FLAMED_FP8 = 2 };

FLAMED_API const char* flamed_last_error(void);
FLAMED_API int flamed_version(void);

/* ============================ denoiser: SimpleMLPAdaLN + Euler loop ============================
 * Replaces prob_generator.py:349-365 (SimpleMLPAdaLN.forward) and the Euler loop of
 * ProbGenerator.sample, prob_generator.py:439-447.
 *
 * Weight pointer order for flamed_den_load (fp32 device tensors exactly as in the state dict,
 * prefix prob_generator.denoiser.):
 *   head  (8):  time_embed.mlp.0.{weight,bias}, time_embed.mlp.2.{weight,bias}, cond_embed.{weight,bias},
 *               proj_in.{weight,bias}
 *   block (18 per res_blocks.i): adaLN_modulation.1.{weight,bias}, ln_conv.{weight,bias},
 *               conv_in.conv_1.{weight,bias}, conv_in.ln_1.{weight,bias}, conv_in.conv_2.{weight,bias},
 *               conv_in.conv_3.{weight,bias}, ln_mlp.{weight,bias}, mlp.0.{weight,bias}, mlp.2.{weight,bias}
 *   final (12): final_layer.adaLN_modulation.1.{weight,bias}, final_layer.conv_in.conv_1.{weight,bias},
 *               final_layer.conv_in.ln_1.{weight,bias}, final_layer.conv_in.conv_2.{weight,bias},
 *               final_layer.conv_in.conv_3.{weight,bias}, final_layer.conv_out.{weight,bias}
 * GEMM weights are packed (cast / tap-reordered) and every other vector (biases, norm gains, depthwise
 * taps) copied into the handle's own device arena.
 */
enum { FLAMED_DEN_HEAD_W = 8, FLAMED_DEN_BLOCK_W = 18, FLAMED_DEN_FINAL_W = 12 };
typedef struct flamed_den_s* flamed_den_t;

FLAMED_API int flamed_den_create(int latent_dim, int hidden, int n_blocks, int kernel, int spk_dim, int dtype,
                                 flamed_den_t* out);
FLAMED_API int flamed_den_destroy(flamed_den_t h);
FLAMED_API int flamed_den_num_weights(flamed_den_t h);
FLAMED_API int flamed_den_load(flamed_den_t h, const float* const* weights, int n_weights, hipStream_t stream);

/* AdaLN precompute for R modulation rows (TimestepEmbedder :35-72, cond_embed :358, y = t + c :359,
 * every adaLN_modulation Linear :131-134/:224-227 at once).  Row r uses t_vals[tidx[r]] and
 * spk[sidx[r]] (tidx/sidx: device int32[R]).  mods: R x flamed_den_mods_stride(h) fp32; per row
 * first the (6*n_blocks+5)*hidden modulation floats — chunks [shift_c, scale_c, gate_c, shift_m,
 * scale_m, gate_m] per block then the final layer's [shift_c, scale_c, gate_c, shift_o, scale_o] —
 * and, for bf16 handles, the LayerNorm-fold tables of the LN-consuming GEMMs: per block
 * [W_mlp0 alpha_m, W_mlp0 beta_m + b_mlp0] (2 x hidden), then [W_out alpha_o, W_out beta_o]
 * (2 x 3 latent_dim; alpha = w (1 + scale), beta = b (1 + scale) + shift of that LayerNorm). */
FLAMED_API int flamed_den_mods_stride(flamed_den_t h);
FLAMED_API size_t flamed_den_adaln_workspace_size(flamed_den_t h, int n_t, int n_spk);
FLAMED_API int flamed_den_adaln(flamed_den_t h, const float* t_vals, int n_t, const float* spk, int n_spk,
                                const int* tidx, const int* sidx, int R, float* mods, void* ws, size_t ws_bytes,
                                hipStream_t stream);

/* Workspace for B utterances of T frames (all velocity/step/solve calls). */
FLAMED_API size_t flamed_den_workspace_size(flamed_den_t h, int B, int T);

/* One velocity evaluation v = denoiser(x, t, c) (forward() parity).  x, v_out: (B*T) x latent_dim.
 * Frame row m uses modulation row m / mod_div (mod_div = T: per-utterance t, the sampling path;
 * mod_div = 1: per-frame t, the training path of prob_generator.py:423). */
FLAMED_API int flamed_den_velocity(flamed_den_t h, const float* x, const float* mods, int mod_div, int B, int T,
                                   float* v_out, void* ws, size_t ws_bytes, hipStream_t stream);

/* One Euler step in place: xt += dt * denoiser(xt, t, c)  (prob_generator.py:444-445). */
FLAMED_API int flamed_den_step(flamed_den_t h, float* xt, const float* mods, int mod_div, int B, int T, float dt,
                               void* ws, size_t ws_bytes, hipStream_t stream);

/* The whole nfe-step Euler solve in place on xt ((B*T) x latent_dim).  mods holds nfe*B rows in
 * step-major order (row s*B + b = step s, utterance b; produced by flamed_den_adaln).
 * use_graph bit 1 captures the nfe steps once into a hipGraph (cached per shape/pointers) and
 * replays it (0: plain launches); bit 2 never takes the persistent solve below (a caller's re-run of a
 * solve whose persistent launch reported a failure). */
FLAMED_API int flamed_den_solve(flamed_den_t h, float* xt, const float* mods, int nfe, int B, int T, void* ws,
                                size_t ws_bytes, int use_graph, hipStream_t stream);
/* Steps per captured solve graph for nfe steps (the granularity of flamed_den_solve_part); -1 on error. */
FLAMED_API int flamed_den_solve_chunk(flamed_den_t h, int nfe);
/* Steps [s0, s1) of the same solve (s0, s1 on flamed_den_solve_chunk boundaries, or s1 = nfe), so a
 * caller can start the solve while later AdaLN rows are still being computed on another stream:
 * s0 = 0 initialises the step counter, s1 = nfe finishes the solve.  Calls for one solve must be
 * stream-ordered and use the same arguments apart from s0 / s1. */
FLAMED_API int flamed_den_solve_part(flamed_den_t h, float* xt, const float* mods, int nfe, int B, int T, void* ws,
                                     size_t ws_bytes, int use_graph, int s0, int s1, hipStream_t stream);
/* The persistent solve (one launch of 256 workgroups for every step, flamed_tune "persist"; taken by
 * flamed_den_solve / _solve_part with use_graph != 0 on a bf16 handle for one utterance of 16..4096 frames,
 * or -- "persist_multi", default on -- for B = 2 / 4 / 8 equal-length utterances with B x T <= 4096 (and, knob
 * "persist_pad", B = 3 / 5..7 as B = 4 / 8 with idle utterances);
 * decided once per solve by its step-0 part, and later parts follow it).  The launch is
 * cooperative (all workgroups co-resident or refused up front, then this device uses the graph of launches)
 * and is only ENQUEUED: no host synchronisation, so it may be captured into a hipGraph (the captured node
 * replays cooperatively).  A launch whose in-kernel wait times out leaves NaN in xt and adds one to a sticky
 * device failure count that later calls read asynchronously; after 3 failures the handle uses the graph of
 * launches.  Lifetime: a solve captured into a caller's graph (persistent or not) points at this handle's
 * scratch, counters and graph execs, which flamed_den_destroy / _load free after waiting only for the handle's
 * own uncaptured work -- keep the handle alive while a captured graph can still replay.
 * flamed_den_persist_info: *runs = persistent launches enqueued on this handle, *broken = 1 once
 * it has given up the persistent path, *last_ms = device time of the last uncaptured launch (HIP events
 * around the kernel on the launch stream; waits for it). */
FLAMED_API int flamed_den_persist_info(flamed_den_t h, int* runs, int* broken, float* last_ms);
/* Never waits: *runs = persistent launches enqueued on this handle, *fails = its failed launches as of the
 * last completed asynchronous copy of the device's failure count (exact once the stream of the last launch has
 * been synchronised: the copy is ordered behind the launch).  Retry-budget bookkeeping; a caller that must
 * know whether one particular solve failed uses flamed_den_persist_last / _query. */
FLAMED_API int flamed_den_persist_status(flamed_den_t h, int* runs, int* fails);
/* Per-launch outcome, never waiting.  flamed_den_persist_last: *seq = sequence number of this handle's most recent
 * uncaptured persistent launch (-1 if none; call it right after a flamed_den_solve that took the persistent path).
 * flamed_den_persist_query: *state = 0 the launch finished and succeeded, 1 it finished and failed (its xt is
 * NaN-poisoned: re-run the solve with use_graph | 2), 2 not finished yet (query again later, or synchronise the
 * launch stream first), 3 unknown (more than 64 uncaptured persistent launches ago).  Each launch's own error word
 * is copied behind it into pinned memory, so the answer concerns that launch only, not earlier captured replays.
 * The Python wrapper (DenoiserHIP.settle) checks pending solves this way at its next call or at the caller's sync
 * point and re-runs a failed one in place. */
FLAMED_API int flamed_den_persist_last(flamed_den_t h, long long* seq);
FLAMED_API int flamed_den_persist_query(flamed_den_t h, long long seq, int* state);
/* Device times (ms, oldest first) of the up to n most recent uncaptured persistent launches (a ring of 64
 * HIP event pairs; waits for them); returns how many were written, -1 on error. */
FLAMED_API int flamed_den_persist_times(flamed_den_t h, float* ms, int n);

/* Kernel classes of an Euler step (flamed_den_time_kernels_graph): 0 proj_in GEMM, 1 LN/mod +
 * depthwise conv (+ GroupNorm partials, + finalize by the last-arriving T-chunk), 2 standalone GroupNorm
 * finalize (only when B x H/64 exceeds the handle's counters; otherwise ~0), 3 GN-apply + conv_2 GEMM +
 * GELU, 4 conv_3 GEMM + gated residual, 5 LN/mod + mlp.0 GEMM + SiLU, 6 mlp.2 GEMM + gated residual,
 * 7 LN/mod + conv_out tap-stacked GEMM, 8 conv_out tap combine + Euler update. */
enum { FLAMED_DEN_KERNEL_CLASSES = 9 };

/* Measurement API (bench.py's live per-kernel timing): in-graph device time per launch (ms) of each
 * kernel class: a captured graph of 4
 * dt = 0 Euler steps is replayed `reps` times as is and once per class with that class's launches
 * doubled (flamed_tune "dup_class"); ms_out[c] = (t_dup - t_base) / launches of c, and
 * ms_out[FLAMED_DEN_KERNEL_CLASSES] = t_base per step.  ms_out holds FLAMED_DEN_KERNEL_CLASSES + 1
 * floats.  Class 2 reads 0 when the GroupNorm finalize is fused into class 1. */
FLAMED_API int flamed_den_time_kernels_graph(flamed_den_t h, float* xt, const float* mods, int B, int T, void* ws,
                                             size_t ws_bytes, int reps, float* ms_out, hipStream_t stream);

/* Tuning knobs.  flamed_tune sets the process defaults (thread-safe; every handle re-snapshots them at
 * its next call); flamed_den_tune gives one denoiser handle its own values (the defaults no longer
 * apply to it).  A handle call reads one snapshot for its whole duration.  Keys:
 *   "splitk_target" — bf16 small-M GEMMs (M < 2048 rows) split K over workgroups until about this
 *                     many workgroups are launched (default 1 = off: slower at B = 1 on gfx950);
 *   "splitk_max"    — maximum number of K slices (1, 2 or 4; default 4).
 *   "small_stages"  — pipeline of the small-M GEMM tile (M < 2048 rows): 3 (LDS ring, 2 K-steps in
 *                     flight), 5 or 7 (4 or 6 K-steps of register prefetch);
 *   "dma"           — 1 (default): small-M bf16 GEMMs whose A operand is bf16 run on the LDS-DMA
 *                     pipeline (gemm_dma.hpp); 2: also those with fp32 (LayerNorm/GroupNorm) A
 *                     operands; 0: the register-staged main loop only;
 *   "dma_ns"        — LDS ring depth of those tiles: 3 (default), 4, 6 or 8;
 *   "lnfold"        — 1 (default, bf16 handles): mlp.0 and conv_out run as plain bf16 GEMMs on
 *                     x * alpha (written by the preceding conv_3 epilogue) with the LayerNorm and
 *                     modulation folded into their epilogues; 0: applied in the A-operand loader;
 *   "fold_rows"     — on the large-M path the fold is used from this many rows (default 6144);
 *   "graph_steps"   — Euler steps per captured solve graph (largest divisor of nfe up to this; 16);
 *   "bn32"          — 1 (default): denoiser GEMMs over fewer than 320 rows use 32 x 32 tiles (LN row
 *                     partials 32 columns wide); 0: 32 x 64 as above 320 rows;
 *   "big"           — 1 (default): bf16 denoiser steps over >= big_rows rows write each transforming A
 *                     operand once as bf16 rows and run 128 x 128 LDS-DMA GEMM tiles with XCD-aware
 *                     placement; 0: fused register-staged GEMMs;
 *   "big_rows"      — smallest B*T on that path (default 1536, >= 1024);
 *   "big_ns"        — LDS ring depth of those tiles: 2 (default, two workgroups per CU) or 3;
 *   "dw_tc"         — frames per depthwise-conv workgroup at >= 8192 rows: 64 (default) or 128;
 *   "dw_cg32"       — below this many rows (default 1536) the depthwise conv uses narrow channel
 *                     groups of "dw_cg" channels (16 or 32; default 32);
 *   "xcd_strips"    — XCD strip width of small/mid-M register-staged tile placement (0 = off);
 *   "x16"           — 1: bf16 residual stream / depthwise output on the large-M path (0 default);
 *   "g8p_rows"      — large-M GEMMs from this many rows on 256 x 256 8-phase tiles (12800; 0 off);
 *   "dwgn"          — 1 (default): large-M whole-utterance depthwise conv + GroupNorm kernel;
 *   "dwgn_small"    — 1 (default): small-M one-workgroup-per-8-channels depthwise conv + GroupNorm;
 *   "fuse_euler"    — 1 (default): small-M solve graphs compute the conv_out tap combine + Euler
 *                     update inside the next step's proj_in A loader (25 launches per step, state
 *                     ping-ponged through the workspace); 0: separate combine kernel (26);
 *   "persist"       — 1 (default): B = 1 bf16 solves run as one persistent cooperative launch;
 *   "persist_opt"   — persistent kernel variant bits (default 885322 = 584 + whole-16-row-tile row groups 2 +
 *                     deferred hand-off seals 65536 + per-chunk GEMMs 262144 + wave-local staging order 32768 +
 *                     K-outer multi-chunk GEMMs 524288 (over 262144 when both are set); the
 *                     others are A/B variants, csrc/common.hpp);
 *   "persist_seal_skip" — diagnostic: one workgroup skips its hand-off seals in this step (-1 default =
 *                     never): a seal mode (persist_opt 16384 / 65536) must then fail the launch;
 *   "persist_inject"— diagnostic: every persistent launch fails at this step (-1 default = never), to
 *                     exercise the NaN poisoning / failure count / retry budget;
 *   "persist_multi" — 1 (default): B = 2 / 4 / 8 equal-length utterances also run as one persistent
 *                     launch (rows per group <= 64 x persist_multi_ntw: B x T <= 4096 by default); 0: B = 1 only;
 *   "persist_pad"   — 1 (default): B = 3 / 5..7 run as the B = 4 / 8 persistent launch with idle zero utterances
 *                     in the spare row groups (4 x T / 8 x T <= 4096); 0: those B take the graph of launches;
 *   "persist_pad_ntw" — ... and a batch padded to >= 1.5x its size (B = 5 as 8) only while it needs at most this
 *                     many 64-frame chunks per row group, 1..8 (default 4: B = 5 up to T = 256);
 *   "persist_ntw"   — 64-frame chunks per persistent row group, 1..8 (default 8: T <= 4096 at B = 1);
 *   "persist_multi_ntw" — ... and for B > 1, 1..8 (default 8; an A/B knob against the graph of launches);
 *   "persist_capmode" — persistent launch inside a stream capture: 0 (default) cooperative node, 1 plain;
 *   "coop"          — 1 (default): the persistent denoiser solve and PVA flow are cooperative launches;
 *                     0: plain launches after the same residency check (profiling runs: rocprofv3's
 *                     teardown faults after a cooperative launch, README "Known issues");
 *   "split_batch"   — large-M bf16 solves as this many concurrent sub-batch chains (parallel graph
 *                     branches; default 2, bitwise equal to 1 = one chain);
 *   "split_min_rows"— ... only when every chain keeps at least this many rows (default 6144);
 *   "split_graph"   — 0 (default): one graph per chain, chains 1.. replayed on priority streams of their
 *                     own; 1: one graph with the chains as parallel branches (round 4);
 *   "split_prio"    — split chains' replay streams: 0 (default) chain 0 on the caller's stream, chain 1
 *                     on a highest-priority stream; 1 every chain on a low-priority stream; 2 all high;
 *   "pva_split"     — 1: the PVA nets' small-M exact-fp32 GEMMs split K over workgroups
 *                     (per-handle slabs, fixed slice order: deterministic); 0 (default: measured
 *                     no faster): one K chain;
 *   "pva_persist"   — 1 (default): the PVA flow of both nets runs as one persistent launch when it
 *                     fits (see flamed_pva_flow); 0: hipGraph of launches;
 *   "pva_stage"     — 1 (default): in that launch, row groups of >= 2 tiles stage their conv A windows
 *                     through LDS in 64-channel chunks (coalesced rows); 0: per-lane gathers (round 4);
 *   "pva_inject"    — diagnostic: every persistent PVA flow fails at this step (-1 default = never);
 *   "attn_mfma"     — 1 (default): transformer attention (prior stack, timbre encoder) on fp32 MFMA;
 *                     0: the LDS-broadcast FMA kernel;
 *   "prior_split"   — 1 (default): bf16 prior decoders split K of the GEMMs whose tile grid leaves CUs
 *                     idle (per-handle slabs, fixed slice order); 0: one K chain;
 *   "noctr"         — diagnostic: kernels ignore the device step counter (wrong modulation rows);
 *   "dup_class"     — ablation: launch every denoiser kernel of this class (see
 *                     FLAMED_DEN_KERNEL_CLASSES) twice per Euler step; -1 (default) = off.
 * Split-K sums the slices in a fixed order (deterministic).  Returns 1001 for an unknown key. */
FLAMED_API int flamed_tune(const char* key, int value);
FLAMED_API int flamed_den_tune(flamed_den_t h, const char* key, int value);
/* Device index the handle's weights live on (-1 before flamed_den_load).  Every call on a handle runs
 * on that device (made current for the call, the caller's restored after) and rejects tensors that
 * live on another device. */
FLAMED_API int flamed_den_device(flamed_den_t h);

/* ============================ condition fold (once per utterance) ============================
 * Replaces QuantizerEncoding (prob_generator.py:368-381) + ConditionDownSampler (:167-205, n_stages 1)
 * of ProbGenerator.sample (:435-436), SURVEY.md §8(f) f1.  Weight order for flamed_cond_load (fp32 device
 * tensors, prefix prob_generator.):
 *   quantizer_encoding.quantizer_emb.weight,
 *   cond_downsampling.resblocks.0.block.block.0.{weight,bias}, ...block.block.1.{weight,bias} (GroupNorm),
 *   cond_downsampling.downblocks.0.0.{weight,bias}, cond_downsampling.downblocks.0.1.{weight,bias} (GroupNorm),
 *   cond_downsampling.proj_out.0.{weight,bias}
 * cond: (B, n_quantizers, T, cond_dim) as the reference receives it; mask: (B, T) fp32 (1 = valid frame);
 * out: (B*T) x out_dim.  dtype FLAMED_F32 (exact fp32 MFMA) or FLAMED_BF16 GEMM operands. */
enum { FLAMED_COND_W = 11 };
typedef struct flamed_cond_s* flamed_cond_t;
FLAMED_API int flamed_cond_create(int n_quantizers, int cond_dim, int out_dim, int n_stages, int dtype, flamed_cond_t* out);
FLAMED_API int flamed_cond_destroy(flamed_cond_t h);
FLAMED_API int flamed_cond_load(flamed_cond_t h, const float* const* weights, int n_weights, hipStream_t stream);
FLAMED_API size_t flamed_cond_workspace_size(flamed_cond_t h, int B, int T);
FLAMED_API int flamed_cond_fold(flamed_cond_t h, const float* cond, const float* mask, int B, int T, float* out, void* ws,
                                size_t ws_bytes, hipStream_t stream);

/* ==================== PVA duration / silence generators + length regulator ====================
 * Replaces ProbabilisticModule.forward (pva.py:221-238) inside the Euler loop of PVA.sample
 * (pva.py:97-109) and LengthRegulator.LR (pva.py:125-166, with tools.pad :299-317).
 * Weight order for flamed_dur_load (fp32 device tensors, prefix prior_generator.pva.{duration,sil}_generator.):
 *   proj.{weight,bias}, time_emb.time_emb.1.{weight,bias}, time_emb.time_emb.3.{weight,bias},
 *   conv_layer.conv1d_1.conv.{weight,bias}, conv_layer.layer_norm_1.{weight,bias},
 *   conv_layer.conv1d_2.conv.{weight,bias}, conv_layer.layer_norm_2.{weight,bias}, linear_layer.{weight,bias}
 * Vectors are copied into the handle's arena; the proj split and conv taps are packed.  The
 * (duration, silence) pair's flow graph is cached on the duration handle. */
enum { FLAMED_DUR_W = 16 };
typedef struct flamed_dur_s* flamed_dur_t;
FLAMED_API int flamed_dur_create(int input_size, int filter_size, int kernel, flamed_dur_t* out);
FLAMED_API int flamed_dur_destroy(flamed_dur_t h);
FLAMED_API int flamed_dur_load(flamed_dur_t h, const float* const* weights, int n_weights, hipStream_t stream);
FLAMED_API size_t flamed_pva_workspace_size(flamed_dur_t h, int B, int L, int nfe);
/* Whole nfe-step flow of both generators, in place on dur_t / sil_t (B*L, the initial noise *
 * temperature).  enc: (B*L) x input_size encoder output; mask: uint8 B*L, 1 = padding (src_mask);
 * ts: nfe+1 fp32 time grid (torch.linspace(0, 1, nfe+1)).  use_graph bit 1: the fast path -- one
 * persistent launch for every step of both nets (pvaflow.hpp; input 192, filter 384, B*L <= 640, knob
 * "pva_persist"): cooperative (all workgroups co-resident, or refused up front and this row-group count then
 * takes the graph path), only enqueued (no host synchronisation; capturable once the pair has run one
 * uncaptured flow), self-resetting; a launch whose in-kernel wait times out leaves NaN in dur_t / sil_t and adds
 * one to a sticky failure count read asynchronously by later calls (flamed_pva_persist_status), and after 3
 * failures the pair takes the graph path -- else a cached hipGraph replay; bit 2: never the persistent launch
 * (a caller's re-run of a failed flow); use_graph == 0: plain launches. */
FLAMED_API int flamed_pva_flow(flamed_dur_t dur, flamed_dur_t sil, const float* enc, const uint8_t* mask, float* dur_t,
                               float* sil_t, const float* ts, int nfe, int B, int L, void* ws, size_t ws_bytes,
                               int use_graph, hipStream_t stream);
/* 1 when a flamed_pva_flow(use_graph != 0) of B x L rows on this pair, on `stream` (its capture state
 * counts), would run as the persistent launch (the caller may then pass its own buffers: no graph keyed on
 * their addresses), 0 otherwise. */
FLAMED_API int flamed_pva_persist_ready(flamed_dur_t dur, flamed_dur_t sil, int B, int L, hipStream_t stream);
/* (diagnostic) persistent PVA flows enqueued on the duration handle, whether the pair has given up the
 * persistent path (3 failed launches), device ms of the last uncaptured one (waits for it). */
FLAMED_API int flamed_pva_persist_info(flamed_dur_t dur, int* runs, int* broken, float* last_ms);
/* Never waits: persistent flows enqueued on this pair, and its failed launches as of the last completed
 * asynchronous copy of the device's failure count (exact once the flow's stream has been synchronised). */
FLAMED_API int flamed_pva_persist_status(flamed_dur_t dur, int* runs, int* fails);
/* Length regulator, phase 1: per-utterance interleaved [phone_l, silence_l] repeat counts
 * (padding phonemes -> 1 frame, 0 silence), exclusive prefix sums cum (int64 B x (2L+1)) and
 * tgt_len (int64 B).  phone/sil are frame counts, or final log-durations when log_domain != 0
 * (then clamp(round(exp(d) - 1), 0) is applied first, pva.py:111-112).  src_lens: int64 B. */
FLAMED_API int flamed_lr_lengths(const float* phone, const float* sil, const int64_t* src_lens, int B, int L,
                                 int log_domain, int64_t* cum, int64_t* tgt_len, hipStream_t stream);
/* Phase 2 (after the host has read max(tgt_len), as the reference's .tolist() does): gather frames
 * out[b][f] = x[b][src] (silence frames copy phoneme 0), zero beyond tgt_len[b], truncated at T_out. */
FLAMED_API int flamed_lr_expand(const float* x, const int64_t* cum, int B, int L, int H, int T_out, float* out,
                                hipStream_t stream);

/* ================================ FaCodec decoder (inference) ================================
 * Replaces FACodecDecoder.inference (facodec.py:630-638) and its model stack (:398-415).
 * Weight order for flamed_fac_load (fp32 device tensors as in the decoder state dict):
 *   timbre_linear.{weight,bias}, model.0.{weight_g,weight_v,bias},
 *   per DecoderBlock model.{1..n_up}.block (FLAMED_FAC_BLOCK_W = 49 each):
 *     0.act.{alpha,beta}, 0.upsample.filter, 0.downsample.lowpass.filter, 1.{weight_g,weight_v,bias},
 *     then for each ResidualUnit j in 2,3,4: j.block.0.act.{alpha,beta}, j.block.0.upsample.filter,
 *     j.block.0.downsample.lowpass.filter, j.block.1.{weight_g,weight_v,bias}, j.block.2.act.{alpha,beta},
 *     j.block.2.upsample.filter, j.block.2.downsample.lowpass.filter, j.block.3.{weight_g,weight_v,bias}
 *   final: model.{n_up+1}.act.{alpha,beta}, .upsample.filter, .downsample.lowpass.filter,
 *          model.{n_up+2}.{weight_g,weight_v,bias}
 * Weight norm is folded and conv weights packed at load; vectors are copied into the arena. */
enum { FLAMED_FAC_BLOCK_W = 49 };
typedef struct flamed_fac_s* flamed_fac_t;
FLAMED_API int flamed_fac_create(int in_channels, int upsample_initial_channel, int n_up, const int* up_ratios, int dtype,
                                 flamed_fac_t* out);
FLAMED_API int flamed_fac_destroy(flamed_fac_t h);
FLAMED_API int flamed_fac_num_weights(flamed_fac_t h);
FLAMED_API int flamed_fac_load(flamed_fac_t h, const float* const* weights, int n_weights, hipStream_t stream);
FLAMED_API size_t flamed_fac_workspace_size(flamed_fac_t h, int B, int T);
/* latents: (B, in_channels, T) channels-first as the reference passes them; spk: (B, in_channels);
 * wav: (B, hop*T) with hop = prod(up_ratios).  use_graph != 0 replays a cached hipGraph. */
FLAMED_API int flamed_fac_decode(flamed_fac_t h, const float* latents, const float* spk, int B, int T, float* wav,
                                 void* ws, size_t ws_bytes, int use_graph, hipStream_t stream);

/* ============================ FaCodec encoder (prompt encoding) ============================
 * Replaces FACodecEncoder.forward (facodec.py:183-216; EncoderBlock :136-155), SURVEY.md §8(f) f3.
 * Weight order for flamed_enc_load (fp32 device tensors as in the encoder state dict):
 *   block.0.{weight_g,weight_v,bias},
 *   per EncoderBlock block.{1..n_down}.block (FLAMED_ENC_BLOCK_W = 49 each):
 *     for each ResidualUnit j in 0,1,2: j.block.0.act.{alpha,beta}, j.block.0.upsample.filter,
 *     j.block.0.downsample.lowpass.filter, j.block.1.{weight_g,weight_v,bias}, j.block.2.act.{alpha,beta},
 *     j.block.2.upsample.filter, j.block.2.downsample.lowpass.filter, j.block.3.{weight_g,weight_v,bias};
 *     then 3.act.{alpha,beta}, 3.upsample.filter, 3.downsample.lowpass.filter, 4.{weight_g,weight_v,bias}
 *   final: block.{n_down+1}.act.{alpha,beta}, .upsample.filter, .downsample.lowpass.filter,
 *          block.{n_down+2}.{weight_g,weight_v,bias}
 * Channels: ngf at the input, doubled by every block (ngf * 2^n_down before the output conv). */
enum { FLAMED_ENC_BLOCK_W = 49 };
typedef struct flamed_enc_s* flamed_enc_t;
FLAMED_API int flamed_enc_create(int ngf, int n_down, const int* ratios, int out_channels, int dtype, flamed_enc_t* out);
FLAMED_API int flamed_enc_destroy(flamed_enc_t h);
FLAMED_API int flamed_enc_num_weights(flamed_enc_t h);
FLAMED_API int flamed_enc_load(flamed_enc_t h, const float* const* weights, int n_weights, hipStream_t stream);
/* Output frames for an n-sample input (Conv1d length arithmetic at every stride); -1 for a bad handle. */
FLAMED_API int flamed_enc_out_len(flamed_enc_t h, int n);
FLAMED_API size_t flamed_enc_workspace_size(flamed_enc_t h, int B, int n);
/* wav: (B, n) fp32 (the reference's (B, 1, n)); out: (B, out_channels, flamed_enc_out_len(n)) fp32. */
FLAMED_API int flamed_enc_encode(flamed_enc_t h, const float* wav, int B, int n, float* out, void* ws, size_t ws_bytes,
                                 int use_graph, hipStream_t stream);

/* ======================= prior transformer stack (once per utterance) =======================
 * Replaces the transformer parts of PriorGenerator.sample (prior_generator.py:141-196, SURVEY.md §8(f)
 * f2): Encoder (module/transformer/Models.py:33-100) before the PVA, and bridge + shared Decoder +
 * six prompt-prefixed Decoders (Models.py:103-171, PreEncoding prior_generator.py:12-26) + head after
 * it.  FFTBlock = post-norm MultiHeadAttention (SubLayers.py:8-57) + conv FFN (:60-95).  Exact fp32.
 * dims (17 + n_q ints): n_symbols, enc {hidden, heads, conv_filter, k0, k1, layers, max_seq_len},
 *   dec {hidden, heads, conv_filter, k0, k1, shared_layers, max_seq_len}, vocab_size, n_q,
 *   decoder_layers[n_q].  Head widths 32 or 48; hidden 192 / 256 / 384.
 * Weight order for flamed_prior_load (fp32 device tensors, prefix prior_generator.; one FFT layer =
 *   slf_attn.{w_qs,w_ks,w_vs}.{weight,bias}, slf_attn.fc.{weight,bias}, slf_attn.layer_norm.{weight,bias},
 *   pos_ffn.w_1.{weight,bias}, pos_ffn.w_2.{weight,bias}, pos_ffn.layer_norm.{weight,bias}):
 *   encoder.src_word_emb.weight, encoder.position_enc, encoder.layer_stack.* layers,
 *   bridge.{weight,bias}, code_embedding.weight, shared_decoder.position_enc, shared_decoder layers,
 *   pre_encode.{prompt_emb,target_emb,quantizer_emb.weight},
 *   for each q: prior_decoder.q.position_enc, prior_decoder.q layers; head.{weight,bias}.
 * Everything is copied / packed into the handle's arena (q/k/v concatenated, conv taps tap-major,
 * head zero-padded to a multiple of 64 rows). */
typedef struct flamed_prior_s* flamed_prior_t;
FLAMED_API int flamed_prior_create(const int* dims, int n_dims, flamed_prior_t* out);
FLAMED_API int flamed_prior_destroy(flamed_prior_t h);
FLAMED_API int flamed_prior_num_weights(flamed_prior_t h);
FLAMED_API int flamed_prior_load(flamed_prior_t h, const float* const* weights, int n_weights, hipStream_t stream);
/* Workspace for an encode of (B, L) and a decode of (B, T) targets behind P prompt frames. */
FLAMED_API size_t flamed_prior_workspace_size(flamed_prior_t h, int B, int L, int T, int P);
/* texts (B, L) int64, src_mask (B, L) uint8 (1 = padding), out (B, L, enc hidden) fp32.  pos: NULL for
 * the loaded encoder.position_enc (L <= max_seq_len), else an (L, hidden) table (Models.py:83-86). */
FLAMED_API int flamed_prior_encode(flamed_prior_t h, const int64_t* texts, const uint8_t* src_mask, int B, int L,
                                   const float* pos, float* out, void* ws, size_t ws_bytes, int use_graph,
                                   hipStream_t stream);
/* x (B, T, enc hidden) length-regulated encoder output, tgt_mask (B, T) uint8 (1 = padding), prompts
 * (B, n_q, P) int64 codes; embs (B, n_q, T, dec hidden) = prior embeddings, logits (B, vocab+1, n_q, T)
 * masked as the reference.  pos: NULL for the loaded decoder tables (P + T <= max_seq_len), else a
 * (P + T, hidden) table used by every decoder. */
FLAMED_API int flamed_prior_decode(flamed_prior_t h, const float* x, const uint8_t* tgt_mask, const int64_t* prompts,
                                   int B, int T, int P, const float* pos, float* embs, float* logits, void* ws,
                                   size_t ws_bytes, int use_graph, hipStream_t stream);
/* Operand type of the decoder-side GEMMs (bridge, shared decoder, per-quantizer decoders, head):
 * FLAMED_F32 (the C default: exact fp32 MFMA) or FLAMED_BF16 (bf16 operands, fp32 accumulation; the weights
 * are converted once on the first bf16 decode).  The encoder always runs fp32 (it feeds the durations).
 * The Python package (flamed/models/synthesizer/prior_generator.py, PriorGenerator.hip_dec_dtype) calls this
 * with FLAMED_BF16 by default; its end-to-end output is checked against the reference Flamed.sample_batch
 * fixture (tests/test_flamed_gpu.py, bf16: prior embeddings and latents rel-L2 <= 2e-2, tgt_mask exact). */
FLAMED_API int flamed_prior_set_dtype(flamed_prior_t h, int dtype);

/* ============== prompt-side quantizers + timbre encoder (once per prompt) ==============
 * Replaces FACodecDecoder.forward(vq=True) (facodec.py:470-533) after the encoder
 * conv stack: the prosody / content / residual ResidualVQs of FactorizedVectorQuantize layers
 * (quantize/rvq.py:27-73, quantize/fvq.py:35-116) and the timbre TransformerEncoder (pre-LN,
 * facodec/transformer.py:154-234) averaged over time.  Exact fp32; codes = argmax like the reference.
 * dims (3 + 2G + 6 ints): C (vq_dim, 256), codebook_dim (8), G (groups), layers[G], codebook sizes[G],
 *   timbre {hidden (= C), heads, conv_filter, kernel, layers, position-table rows}.
 * Weight order for flamed_vq_load (fp32 device tensors, prefix of the FACodecDecoder):
 *   for each group g, layer l: quantizer.g.layers.l.{in_proj.weight_g, in_proj.weight_v, in_proj.bias,
 *     out_proj.weight_g, out_proj.weight_v, out_proj.bias, _codebook.weight};
 *   timbre_encoder.position_emb.pe; per layer: ln_1.{weight,bias}, self_attn.{in_proj_weight,
 *     in_proj_bias}, self_attn.out_proj.{weight,bias}, ln_2.{weight,bias}, ffn.ffn_1.{weight,bias},
 *     ffn.ffn_2.{weight,bias}; timbre_encoder.last_ln.{weight,bias}.
 * Weight norm is folded and the codebooks normalised at load, into the handle's arena. */
typedef struct flamed_vq_s* flamed_vq_t;
FLAMED_API int flamed_vq_create(const int* dims, int n_dims, flamed_vq_t* out);
FLAMED_API int flamed_vq_destroy(flamed_vq_t h);
FLAMED_API int flamed_vq_num_weights(flamed_vq_t h);
FLAMED_API int flamed_vq_load(flamed_vq_t h, const float* const* weights, int n_weights, hipStream_t stream);
FLAMED_API size_t flamed_vq_workspace_size(flamed_vq_t h, int B, int T);
/* x (B, C, T) encoder output -> outs (B, C, T) summed quantized, codes (n_layers, B, T) int64,
 * qbuf (G, B, C, T) per-group quantized sums, spk (B, C) speaker embedding. */
FLAMED_API int flamed_vq_encode(flamed_vq_t h, const float* x, int B, int T, float* outs, int64_t* codes, float* qbuf,
                                float* spk, void* ws, size_t ws_bytes, int use_graph, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FLAMED_HIP_H */
