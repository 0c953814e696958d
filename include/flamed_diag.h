/* flamed_diag.h — diagnostic probes of the MI355X Flamed-TTS kernels (NOT the product library).
 *
 * flamed_probe_* live in libflamed_diag.so (csrc/probe.hip, `make -C flamed-tts_amd/csrc diag`);
 * flamed_stamp_buffer lives only in libflamed_hip_stamps.so (`make stamps`: the product sources built
 * with -DFL_STAMPS).  Nothing on the product path loads either library (scripts under tools/ only).
 */
#ifndef FLAMED_DIAG_H
#define FLAMED_DIAG_H

#include "flamed_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Average device time (us) per launch inside a graph of `reps` back-to-back launches.
 * flamed_probe_gemm: C[M][N] (bf16) = A[M][K] (bf16) . W[N][K]^T with tile variant
 * 0: 32x64 3-stage, 1: 64x64 3-stage, 2: 32x64 2-stage, 3: 128x128, 4: 64x128, 5: 128x64,
 * 6: 32x64 with 4 K-steps of register prefetch, 7: 32x64 with 6, 8: 64x64 with 4.  Launch i reads
 * weight matrix i % wbufs of W (wbufs x N x K), so a large wbufs streams weights from MALL/HBM as
 * in a real Euler step.
 * flamed_probe_empty: an empty kernel of `blocks` x 256 threads (the per-node floor). */
FLAMED_API int flamed_probe_gemm(int variant, int M, int N, int K, int reps, int wbufs, const void* A, const void* W,
                                 void* C, float* us_out, hipStream_t stream);
/* flamed_probe_stream: per-CU ingest — `blocks` workgroups each stream their own `kb` KB slice of src
 * (mode 1: LDS-DMA ring, mode 0: register loads).  src must hold blocks x kb KB. */
FLAMED_API int flamed_probe_stream(int blocks, int kb, int mode, int reps, const void* src, float* us_out, hipStream_t stream);
FLAMED_API int flamed_probe_empty(int blocks, int reps, float* us_out, hipStream_t stream);
/* flamed_probe_copy: STREAM-style copy of `bytes` (a multiple of 16) from src to dst by `blocks` x 256 threads, 4 float4
 * per thread per grid-stride step; mode 1 non-temporal loads / stores, 0 plain.  Average us per launch in a graph of
 * `reps` launches (bench.py's measured HBM peak: 2 x bytes / time). */
FLAMED_API int flamed_probe_copy(const void* src, void* dst, size_t bytes, int blocks, int mode, int reps, float* us_out,
                                 hipStream_t stream);
/* flamed_probe_gemm_pf: flamed_probe_gemm's chain with a concurrent L2 warm-up of the next launch's
 * weights on a second captured stream (pf_blocks workgroups, a multiple of 8; 0 = none). */
FLAMED_API int flamed_probe_gemm_pf(int variant, int M, int N, int K, int reps, int wbufs, int pf_blocks, const void* A,
                                    const void* W, void* C, float* us_out, hipStream_t stream);

/* flamed_probe_mx: one block-scaled MX-fp8 MFMA (16x16x128, e4m3, e8m0 scales) in lane layout `mode`
 * (0: a lane's 32 bytes are K [32g, 32g+32) of its row, 1: K [16g, 16g+16) and [64+16g, 64+16g+16));
 * A, B 16 x 128 bytes, sa, sb 16 x 4, C 16 x 16 fp32 = sum_k A[m][k] sa B[n][k] sb. */
FLAMED_API int flamed_probe_mx(const void* A, const void* B, const void* sa, const void* sb, float* C, int mode,
                               hipStream_t stream);

/* flamed_probe_mx_gemm: C[M][N] fp32 = MX-fp8(A[M][K]) . MX-fp8(W[N][K])^T through the product's fp8 pieces
 * (store_f8x8 producer, quant_w_f8_kernel, the 256x256 block-scaled GEMM); N % 256 == 0, K % 512 == 0,
 * K <= 1024.  Synchronous (allocates and frees its own scratch). */
FLAMED_API int flamed_probe_mx_gemm(const float* A, const float* W, int M, int N, int K, float* C, hipStream_t stream);

/* libflamed_hip_stamps.so only: device buffer of blocks x 8 u64 into which the denoiser kernels of
 * class `flamed_tune("stamp_class", c)` write s_memtime at their phase boundaries (eager steps). */
FLAMED_API int flamed_stamp_buffer(void* buf);
/* Persistent solve timeline (libflamed_hip_stamps.so only): thread 0 of each of the 256 workgroups writes
 * s_memrealtime at every wait / compute / signal point of Euler step `step` into buf[wg * 160 + k]
 * (device memory, 256 x 160 uint64); buf = NULL turns it off.  tools/persist_timeline.py. */
FLAMED_API int flamed_persist_stamps(void* buf, int step);
/* Persistent solve GroupNorm exchange dump (libflamed_hip_stamps.so only): at Euler step `step`, for every
 * GroupNorm hand-off j (0..NB), workgroup wg and channel lane c < 32, the 8 groups' (count, mean, M2) exactly as the
 * combining lane read them, then the combined (mean, scale): buf[((j * 256 + wg) * 32 + c) * 32 + k], k < 26 (device
 * memory, (NB + 1) x 256 x 32 x 32 floats); buf = NULL turns it off.  tools/rowpart_probe.py --dump. */
FLAMED_API int flamed_persist_gndump(void* buf, int step);
/* Persistent PVA flow timeline (libflamed_hip_stamps.so only): thread 0 of every workgroup writes
 * s_memrealtime at fixed points of Euler step `step` into buf[wg * 16 + k]; tools/pva_timeline.py. */
FLAMED_API int flamed_pva_stamps(void* buf, int step);

/* ---- libflamed_hip.so diagnostics ----
 * Exported by the product library for tools and tests; not part of the product contract (flamed_hip.h), and
 * nothing on the product call path uses them. */
/* Failed persistent launches so far on this handle (waits for the whole device to be idle). */
FLAMED_API int flamed_den_persist_fails(flamed_den_t h, int* fails);
/* Byte offsets inside the flamed_den_velocity / flamed_den_step workspace of its buffers X, S0, S1, D, U, GP, GNS,
 * Y, SL, A16, XA, XP (off[12]; SIZE_MAX = absent at this B, T) under the handle's current knobs. */
FLAMED_API int flamed_den_ws_offsets(flamed_den_t h, int B, int T, size_t* off);
/* The persistent solve's reset-prologue ticket arithmetic, host-side (no GPU): the arrival count `*target` that
 * completes the launch of `ticket` (a fetch_add result), and whether counter value `cur` has reached it
 * (wrap-safe across 2^32). */
FLAMED_API int flamed_persist_ticket(unsigned ticket, unsigned cur, unsigned* target, int* reached);
/* Split-chain replay streams of this handle: how many the hardware-queue probe parked (they serialised with an
 * earlier chain's stream) and how many re-creations it took in total. */
FLAMED_API int flamed_den_chain_info(flamed_den_t h, int* parked, int* retries);
/* ... and how many probe pairs were inconclusive (neither concurrent nor dispatched back-to-back: the device was busy);
 * those never park a stream. */
FLAMED_API int flamed_den_chain_busy(flamed_den_t h, int* busy);

#ifdef __cplusplus
}
#endif
#endif /* FLAMED_DIAG_H */
