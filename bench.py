#!/usr/bin/env python3
"""bench.py — Flamed-TTS flow-matching hot path on MI355X.

Metric (BASELINE.json): RTF + latent frames/sec at nsteps-denoiser=128.
One bench "step" = one full pass of the denoiser hot path over one batch: AdaLN precompute for all
nfe steps + the nfe-step Euler solve (hipGraph replay) of ProbGenerator.sample (reference
prob_generator.py:434-447), from the folded condition to the latents.  value = latent frames/s
= (all ranks' B*T) / (max-over-ranks seconds per step).  Default workload = BASELINE configs[1]:
1 utterance x 400 frames (5 s of audio), nfe=128, bf16 GEMM operands.

Also reported: per-kernel-class device times (HIP events, live) with the dominant kernel's roofline
fraction, and the oracle CPU restatement timed on the host cores (rank 0, N=1, bounded sample).
Data: synthetic — seeded random-init weights (tests' filler), N(0,1) condition/speaker.

  python bench.py [--gpus N --steps K --warmup W --batch B --frames T --nfe S --dtype bf16|f32]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import yaml  # noqa: E402

KERNEL_NAMES = ["proj_in_gemm", "lnmod_dwconv_gnpartials", "gn_finalize", "gnapply_conv2_gemm_gelu",
                "conv3_gemm_gated_resid", "lnmod_mlp0_gemm_silu", "mlp2_gemm_gated_resid", "lnmod_conv_out_gemm",
                "conv_out_combine_euler"]
N_CLASSES = len(KERNEL_NAMES)
HBM_PEAK_GBS = 8000.0                     # MI355X_MICROARCH.md chip table (spec)
MFMA_PEAK_TFS = {"bf16": 2500.0, "fp8": 5000.0, "f32": 157.3}   # dense peaks
FOLD = None  # LayerNorm fold active (set in main: bf16 and flamed_tune lnfold != 0)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=None, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i] per-GPU workload (default: 1 = B=1 T=400 nfe=128 bf16); "
                         "--batch/--frames/--nfe/--dtype override its fields")
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=None, help="latent frames per utterance (80 Hz)")
    ap.add_argument("--nfe", type=int, default=None)
    ap.add_argument("--dtype", default=None, choices=["bf16", "f32", "fp8"], help="denoiser handle dtype (fp8: MX-fp8 pointwise GEMMs at large M)")
    ap.add_argument("--no-configs3", action="store_true",
                    help="N > 1: skip the extra configs[3] leg (64 utterances per GPU on every rank)")
    ap.add_argument("--dist-single", action="store_true",
                    help="one rank: still run the multi-rank branch (an NCCL/RCCL process group of one, device-tensor "
                         "max-over-ranks timing, efficiency fields, the configs[3] leg); implied by --config 3")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel-iters", type=int, default=20, help="graph replays per kernel-class timing")
    ap.add_argument("--splitk-target", type=int, default=None, help="flamed_tune splitk_target (1 disables split-K)")
    ap.add_argument("--splitk-max", type=int, default=None, help="flamed_tune splitk_max")
    ap.add_argument("--dup-class", type=int, default=None, help="ablation: flamed_tune dup_class")
    ap.add_argument("--small-stages", type=int, default=None, help="flamed_tune small_stages (3, 5, 7)")
    ap.add_argument("--big", type=int, default=None, help="flamed_tune big (large-M bf16 path)")
    ap.add_argument("--big-rows", type=int, default=None, help="flamed_tune big_rows")
    ap.add_argument("--big-ns", type=int, default=None, help="flamed_tune big_ns (2 or 3)")
    ap.add_argument("--xcd-strips", type=int, default=None, help="flamed_tune xcd_strips (small-M tile placement)")
    ap.add_argument("--dw-cg", type=int, default=None, help="flamed_tune dw_cg (16 or 32)")
    ap.add_argument("--dma-ns", type=int, default=None, help="flamed_tune dma_ns (small-M DMA ring depth)")
    ap.add_argument("--lnfold", type=int, default=None, help="flamed_tune lnfold (LayerNorm folded into mlp.0/conv_out epilogues)")
    ap.add_argument("--graph-steps", type=int, default=None, help="flamed_tune graph_steps (Euler steps per captured graph)")
    ap.add_argument("--dw-cg32", type=int, default=None, help="flamed_tune dw_cg32 (rows below which 32-channel dwconv)")
    ap.add_argument("--dw-tc", type=int, default=None, help="flamed_tune dw_tc (large-M depthwise T-chunk)")
    ap.add_argument("--bn32", type=int, default=None, help="flamed_tune bn32 (32-wide small-M GEMM tiles)")
    ap.add_argument("--x16", type=int, default=None, help="flamed_tune x16 (large-M bf16 residual stream)")
    ap.add_argument("--g8p-rows", type=int, default=None, help="flamed_tune g8p_rows (256x256 8-phase GEMM tiles from this many rows; 0 off)")
    ap.add_argument("--dwgn", type=int, default=None, help="flamed_tune dwgn (large-M whole-utterance depthwise conv + GroupNorm kernel)")
    ap.add_argument("--dwgn-small", type=int, default=None, help="flamed_tune dwgn_small (small-M one-workgroup depthwise conv + GroupNorm)")
    ap.add_argument("--fuse-euler", type=int, default=None, help="flamed_tune fuse_euler (combine + Euler update in the next proj_in)")
    ap.add_argument("--noctr", type=int, default=None, help="diagnostic: ignore the device step counter")
    ap.add_argument("--dma", type=int, default=None, help="flamed_tune dma (0: register-staged GEMM main loop)")
    ap.add_argument("--persist", type=int, default=None, help="flamed_tune persist (B = 1: one persistent launch per solve)")
    ap.add_argument("--persist-opt", type=int, default=None, help="flamed_tune persist_opt (persistent kernel experiment bits)")
    ap.add_argument("--split-batch", type=int, default=None, help="flamed_tune split_batch (large-M sub-batch chains, 1 = off)")
    ap.add_argument("--persist-capmode", type=int, default=None, help="flamed_tune persist_capmode")
    ap.add_argument("--coop", type=int, default=None, help="flamed_tune coop (0: plain launches of the persistent kernels, for rocprofv3 runs)")
    ap.add_argument("--persist-multi", type=int, default=None, help="flamed_tune persist_multi (persistent solve for B = 2 / 4 / 8)")
    ap.add_argument("--no-peaks", action="store_true", help="skip the measured STREAM-copy / library-GEMM peaks")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU rehearsal of the launcher/timing harness over gloo (no GPU; tests/test_bench_cpu.py)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary rows (PVA flow + LR, FaCodec decode / prompt encode, end-to-end RTF)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config or 1]
    for k in ("batch", "frames", "nfe", "dtype"):
        if getattr(args, k) is None:
            setattr(args, k, cfg[k])
    return args


# BASELINE.json configs[i] as per-GPU workloads (configs[0] is the CPU plumbing case: --plumbing)
CONFIGS = {
    1: {"batch": 1, "frames": 400, "nfe": 128, "dtype": "bf16"},
    2: {"batch": 64, "frames": 400, "nfe": 128, "dtype": "bf16"},
    3: {"batch": 64, "frames": 400, "nfe": 128, "dtype": "bf16"},   # per GPU; global batch 64 x N (512 at N = 8)
    4: {"batch": 16, "frames": 2400, "nfe": 256, "dtype": "fp8"},
}


def workload_label(args, world: int) -> tuple:
    """(configs index, label) of what this run measures: --config when given, else inferred from the per-GPU
    shape and the rank count (one rank: B = 1 -> configs[1], T = 2400 -> configs[4], else configs[2]; several
    ranks: the configs[3] utterance-sharded layout).  The label states the shape that actually ran."""
    B, T, nfe, dt = args.batch, args.frames, args.nfe, args.dtype
    if args.config is not None:
        i = args.config
    elif world > 1:
        i = 3
    elif B == 1 and T <= 800:
        i = 1
    elif T >= 2400:
        i = 4
    else:
        i = 2
    ref = CONFIGS[i]
    exact = (B, T, nfe) == (ref["batch"], ref["frames"], ref["nfe"])
    audio = T * 200 / 16000.0
    shape = f"{B} utterance(s) x {T} frames ({audio:.1f} s audio) per GPU, nsteps-denoiser={nfe}, {dt}"
    if i == 3:
        text = (f"BASELINE configs[3]: {shape}, utterance-sharded over {world} GPU(s) (global batch {B * world}; "
                f"configs[3] is 64 per GPU = 512 on 8)")
    else:
        text = f"BASELINE configs[{i}]: {shape}"
    if not exact:
        text += f" [configs[{i}] layout at a non-reference size: reference is B={ref['batch']} T={ref['frames']} nfe={ref['nfe']}]"
    return i, text


def kernel_costs(cls: int, B: int, T: int, H: int, C: int, NB: int, es: int, fold: bool | None = None,
                 fused: bool = False):
    """Algorithmic (bytes, flops) per launch of each kernel class, and launches per Euler step.
    Bytes = every operand read once + every output written once.  With the
    LayerNorm fold (bf16 default) conv_3 also writes x*alpha in bf16 and mlp.0 / conv_out read it
    instead of the fp32 residual stream."""
    M = B * T
    if fold is None:  # the denoiser's default policy: folded below the large-M path and from 6144 rows on it
        fold = es == 2 and FOLD is not False and (M < 1536 or M >= 6144)
    # bf16 handles run the depthwise conv + exact two-pass GroupNorm in ONE kernel per (utterance, channel
    # group) (dwgn_small below 1536 rows with T <= 576, dwgn on the large-M path with T <= 512): it reads
    # the fp32 residual + LN partials and writes the normalised bf16 conv_2 operand; conv_2 then reads
    # that bf16 operand (no fp32 depthwise output round trip, no GroupNorm partials)
    dwgn = es == 2 and ((M < 1536 and T <= 576) or (M >= 1536 and T <= 512))
    ea = 2 if fold else 4  # bytes per A element of the LayerNorm-consuming GEMMs
    NT = H // 64
    TS = (T + 63) // 64
    stats = M * NT * 8
    if cls == 0:
        if fused:  # + the previous step's tap combine + Euler update in the loader: Y read, x_s written
            return M * C * 4 + M * 3 * C * 4 + M * C * 4 + H * C * es + M * H * 4 + stats, 2 * M * H * C + 4 * M * C, 1
        return M * C * 4 + H * C * es + M * H * 4 + stats, 2 * M * H * C, 1
    if cls == 1:
        if dwgn:
            return M * H * 4 + stats + M * H * 2, 2 * 31 * M * H, NB + 1
        return M * H * 4 + stats + M * H * 4 + B * TS * H * 12, 2 * 31 * M * H, NB + 1
    if cls == 2:
        return B * TS * H * 12 + B * H * 8, 10 * B * TS * H, NB + 1
    if cls == 3:
        if dwgn:
            return M * H * 2 + H * H * es + M * H * es, 2 * M * H * H, NB + 1
        return M * H * 4 + B * H * 8 + H * H * es + M * H * es, 2 * M * H * H, NB + 1
    if cls == 4:
        return M * H * es + H * H * es + 2 * M * H * 4 + 2 * stats + (M * H * 2 if fold else 0), 2 * M * H * H, NB + 1
    if cls == 5:
        return M * H * ea + stats + H * H * es + M * H * es, 2 * M * H * H, NB
    if cls == 6:
        return M * H * es + H * H * es + 2 * M * H * 4 + stats, 2 * M * H * H, NB
    if cls == 7:
        return M * H * ea + stats + 3 * C * H * es + M * 3 * C * 4, 2 * M * 3 * C * H, 1
    return M * 3 * C * 4 + 2 * M * C * 4, 4 * M * C, 1


def step_bytes_canonical(pg, B, T):
    """SURVEY.md §8(d) canonical HBM bytes of one fused Euler step: W (every per-frame bf16 GEMM weight
    + fp32 vectors and depthwise taps, streamed once per step; the AdaLN projections are hoisted out of
    the loop) + 54,272 B per frame (bf16 activation rows of the fused design)."""
    den = pg.denoiser
    gemm = [den.proj_in.weight]
    for blk in den.res_blocks:
        gemm += [blk.conv_in.conv_2.weight, blk.conv_in.conv_3.weight, blk.mlp[0].weight, blk.mlp[2].weight]
    fl = den.final_layer
    gemm += [fl.conv_in.conv_2.weight, fl.conv_in.conv_3.weight, fl.conv_out.weight]
    w_gemm = 2 * sum(w.numel() for w in gemm)
    hoisted = {id(p) for m in [den.time_embed, den.cond_embed] + [b.adaLN_modulation for b in den.res_blocks]
               + [fl.adaLN_modulation] for p in m.parameters()}
    gemm_ids = {id(w) for w in gemm}
    w_vec = 4 * sum(p.numel() for p in den.parameters() if id(p) not in hoisted and id(p) not in gemm_ids)
    return w_gemm + w_vec + 54272 * B * T


def measured_peaks(dev):
    """Achievable peaks on this box: a STREAM-style copy of 2 x 1 GiB (read + write bytes) --
    the best of our float4 copy probe (flamed_probe_copy: 4 float4 in flight per thread, plain or non-temporal, a
    few grid sizes; the guide measures 6.29 TB/s for a float4 copy) and torch's copy kernel, both reported -- and a
    large bf16 library GEMM (8192^3, hipBLASLt via torch.matmul)."""
    out = {}
    n = 1 << 28  # 2^28 fp32 = 1 GiB
    a = torch.empty(n, dtype=torch.float32, device=dev).uniform_()
    b = torch.empty_like(a)
    ms = _time_ms(lambda: b.copy_(a), dev, reps=10, warm=3)
    out["hbm_torch_copy_GBps"] = round(2 * 4 * n / ms / 1e6, 1)
    best = (0.0, None)
    try:
        from flamed import _native as nat
        D = nat.diag_lib()
        us = ctypes.c_float(0.0)
        for mode in (1, 0):
            for blocks in (2048, 4096, 8192):
                nat.check(D.flamed_probe_copy(nat.ptr(a), nat.ptr(b), 4 * n, blocks, mode, 10, ctypes.byref(us),
                                              nat.stream_ptr(dev)), "flamed_probe_copy")
                gbs = 2 * 4 * n / (us.value * 1e3)
                if gbs > best[0]:
                    best = (gbs, f"{'non-temporal' if mode else 'plain'} float4 copy, {blocks} x 256 threads")
    except Exception as e:  # the diagnostic library is optional for the bench
        best = (0.0, f"probe unavailable: {e}")
    out["hbm_probe_copy_GBps"] = round(best[0], 1)
    out["hbm_probe_copy_kind"] = best[1]
    out["hbm_stream_copy_GBps"] = max(out["hbm_torch_copy_GBps"], out["hbm_probe_copy_GBps"])
    del a, b
    m = 8192
    x = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
    y = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
    ms = _time_ms(lambda: torch.matmul(x, y), dev, reps=10, warm=3)
    out["bf16_gemm_TFs"] = round(2 * m ** 3 / ms / 1e9, 1)
    del x, y
    torch.cuda.empty_cache()
    return out


def host_cpu():
    """(model name, logical CPUs of the host, CPUs this process may run on)."""
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return model, os.cpu_count() or usable, usable


def _time_ms(fn, dev, reps=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / reps * 1e3


def secondary_measurements(dev, nfe):
    """The other §8 hot-path rows on the GPU, B = 1 (seeded random weights, synthetic inputs):
    PVA duration/silence flow + length regulator (a8-a10), FaCodec decode (a11-a13) and prompt encode
    (f3), and the end-to-end Flamed.sample_batch RTF in both reference definitions (a14/a15)."""
    from flamed.models.synthesizer.pva import PVA
    from flamed.utils.random_ckpt import codec_models, load_yaml
    from flamed.utils.seeded_init import fill_state_dict, randomize_module
    out = {}
    g = torch.Generator().manual_seed(7)
    prior_cfg = load_yaml("prior.yaml")
    pva = PVA(prior_cfg["variance_adaptor"]).eval()
    randomize_module(pva, 20251205)
    pva = pva.to(dev)
    enc_m, dec = codec_models(load_yaml("codec.yaml"))
    dec.load_state_dict(fill_state_dict(dec.state_dict(), 20251205))
    enc_m.load_state_dict(fill_state_dict(enc_m.state_dict(), 20251205))
    dec, enc_m = dec.eval().to(dev), enc_m.eval().to(dev)
    from flamed import Flamed
    m = Flamed({"prior_generator": prior_cfg, "prob_generator": load_yaml("prob.yaml")}).eval()
    m.load_state_dict(fill_state_dict(m.state_dict(), 20251205))
    m = m.to(dev)
    with torch.inference_mode():
        L, nfe_d = 60, 64
        enc = torch.randn(1, L, 192, generator=g).to(dev)
        src_len = torch.tensor([L], device=dev)
        mask = torch.zeros(1, L, dtype=torch.bool, device=dev)
        ms = _time_ms(lambda: pva.sample(enc, src_len, mask, nfe=nfe_d, temperature=0.3), dev)
        pruns, pbroken, pms = pva.hip().persist_info()
        out["pva_flow_lr"] = {"ms": round(ms, 3), "phonemes": L, "nsteps_durgen": nfe_d,
                              "us_per_net_eval": round(ms * 1e3 / (2 * nfe_d), 2), "dtype": "f32 (exact MFMA)",
                              "persistent_flow": {"runs": pruns, "broken": pbroken, "last_flow_ms": round(pms, 3)}}
        # the 5 s utterance's phoneme count (end_to_end_5s below)
        L5 = 285
        enc5 = torch.randn(1, L5, 192, generator=g).to(dev)
        ms5 = _time_ms(lambda: pva.sample(enc5, torch.tensor([L5], device=dev),
                                          torch.zeros(1, L5, dtype=torch.bool, device=dev), nfe=nfe_d, temperature=0.3), dev)
        out["pva_flow_lr"]["L285_ms"] = round(ms5, 3)
        T = 400
        lat = torch.randn(1, 256, T, generator=g).to(dev)
        spk = torch.randn(1, 256, generator=g).to(dev)
        ms = _time_ms(lambda: dec.inference(lat, spk), dev)
        out["facodec_decode"] = {"ms": round(ms, 3), "frames": T, "samples": T * 200,
                                 "samples_per_s": round(T * 200 / ms * 1e3, 1), "rtf": round(ms / 1e3 / (T / 80), 6),
                                 "dtype": dec.hip_dtype}
        wav = (0.1 * torch.randn(1, 1, 48000, generator=g)).to(dev)
        ms = _time_ms(lambda: enc_m(wav), dev)
        out["facodec_prompt_encode"] = {"ms": round(ms, 3), "samples": 48000, "dtype": enc_m.hip_dtype}
        z = enc_m(wav)
        ms = _time_ms(lambda: dec(z, eval_vq=False, vq=True), dev)
        out["facodec_prompt_vq_timbre"] = {"ms": round(ms, 3), "frames": int(z.shape[-1]), "dtype": "f32 (exact MFMA)",
                                           "note": "6 RVQ layers + 4-layer timbre transformer + mean (HIP)"}
        # condition fold (once per utterance, HIP) at the headline shape
        pg = m.prob_generator
        for Bc in (1, 64):
            cond = torch.randn(Bc, 6, 400, 384, generator=g).to(dev)
            cmask = torch.ones(Bc, 400, 1, dtype=torch.bool, device=dev)
            ms = _time_ms(lambda: pg.fold_condition(cond, cmask), dev)
            out[f"cond_fold_B{Bc}"] = {"ms": round(ms, 3), "frames": Bc * 400, "dtype": pg.cond_hip_dtype}
        # prior transformer stack (HIP, exact fp32, graph-captured) vs the same modules on torch-ROCm ops,
        # at the headline utterance: ~247 phonemes -> 400 target frames behind a 240-frame (3 s) prompt
        pr = m.prior_generator
        Lp, Tp, Pp = 247, 400, 240
        ids = torch.randint(1, 300, (1, Lp), generator=g).to(dev)
        smask = torch.zeros(1, Lp, dtype=torch.bool, device=dev)
        xlr = torch.randn(1, Tp, 192, generator=g).to(dev)
        tmask = torch.zeros(1, Tp, dtype=torch.bool, device=dev)
        tl = torch.tensor([Tp], device=dev)
        pcodes = torch.randint(0, 1024, (1, 6, Pp), generator=g).to(dev)
        row = {"phonemes": Lp, "frames": Tp, "prompt_frames": Pp,
               "dtype": f"encoder f32 (exact MFMA), decoders {pr.hip_dec_dtype} GEMMs (fp32 accumulation), fp32-MFMA attention"}
        row["encode_ms"] = round(_time_ms(lambda: pr.hip().encode(ids, smask), dev), 3)
        row["decode_ms"] = round(_time_ms(lambda: pr.hip().decode(xlr, tmask, pcodes, Pp), dev), 3)
        row["torch_encode_ms"] = round(_time_ms(lambda: pr.encoder(ids, smask), dev), 3)
        row["torch_decode_ms"] = round(_time_ms(lambda: pr._decode(pr.bridge(xlr), tl, tmask, pcodes, Pp), dev), 3)
        out["prior_transformer"] = row
        # end to end: Flamed.sample_batch (prior transformer + PVA + cond fold + denoiser) + decode, with
        # both reference RTF definitions (synthesize.py:209-217 prompt mode incl. decode; :293-303
        # metadata mode, decode excluded)
        z = enc_m(wav)
        _, codes, _, _, timbre = dec(z, eval_vq=False, vq=True)
        prompts = codes.permute(1, 0, 2).contiguous()

        base_phon = torch.randint(1, 300, (1, 1024), generator=torch.Generator().manual_seed(1234))

        def e2e(L, phon=None):
            phon = (phon if phon is not None else
                    torch.randint(1, 300, (1, L), generator=torch.Generator().manual_seed(L))).to(dev)
            res = {}

            def run():
                torch.manual_seed(0)
                res["o"] = m.sample_batch(phonemes=phon, src_lens=torch.tensor([L], device=dev), prompts=prompts,
                                          timbres=timbre, codec_decoder=dec, nsteps_durgen=nfe_d, nsteps_denoiser=nfe)
            total_ms = _time_ms(run, dev, reps=3, warm=1)
            o = res["o"]
            frames = int((~o["tgt_mask"]).sum().item())
            audio_s = o["wav"].shape[-1] / 16000.0
            t_sb = float(o["time"])
            return {"frames": frames, "audio_s": round(audio_s, 3), "phonemes": L, "prompt_frames": int(prompts.shape[-1]),
                    "nsteps_durgen": nfe_d, "nsteps_denoiser": nfe,
                    "sample_batch_ms": round(t_sb * 1e3, 3), "with_decode_ms": round(total_ms, 3),
                    "rtf_metadata_mode": round(t_sb / audio_s, 5),
                    "rtf_with_decode": round(total_ms / 1e3 / audio_s, 5)}
        r60 = e2e(L)
        r60["note"] = "random-init weights: the utterance length T comes from the seeded duration flow"
        out["end_to_end"] = r60
        # the headline 5 s utterance: a prefix of one fixed phoneme sequence, its length bisected until the
        # seeded duration flow yields ~400 frames (frames grow with the prefix; closest kept)
        best, lo, hi = r60, 8, 1024
        for _ in range(9):
            Lc = (lo + hi) // 2
            r = e2e(Lc, base_phon[:, :Lc])
            if abs(r["frames"] - 400) < abs(best["frames"] - 400):
                best = r
            if abs(r["frames"] - 400) <= 8 or hi - lo <= 1:
                break
            if r["frames"] < 400:
                lo = Lc
            else:
                hi = Lc
        r5 = dict(best)
        r5["note"] = ("BASELINE metric at the configs[1] length: the phoneme prefix length bisected so the seeded "
                      "duration flow gives ~400 frames (5 s); B = 1, nsteps-denoiser = 128")
        r5["duration_flips"] = duration_flips(pr, base_phon[:, :r5["phonemes"]].to(dev), nfe_d, dev)
        out["end_to_end_5s"] = r5
    return out


def duration_flips(pr, phon, nfe_d, dev, temperature=0.3):
    """Integer duration flip rate of an end-to-end run (SURVEY.md §7 hard part 2), a checker beside the
    timed run: the same encoder output and the same CPU-RNG noise (seed 0, as the timed e2e run draws it)
    through the HIP PVA flow (exact-fp32 MFMA) and through the oracle's fp32 restatement of PVA.sample's
    Euler loop (oracle.pva_flow, reference pva.py:97-109); frames = clamp(round(exp(d) - 1), 0)
    (pva.py:111-112) compared per phoneme."""
    from oracle import flamed_oracle as orc  # checker only
    L = phon.shape[1]
    smask = torch.zeros(1, L, dtype=torch.bool, device=dev)
    with torch.inference_mode():
        enc = pr.hip().encode(phon, smask)
        torch.manual_seed(0)
        d_g, s_g = pr.pva.flow(enc, smask, nfe_d, temperature)
        sd = {"prior_generator.pva." + k: v.detach().float().cpu() for k, v in pr.pva.state_dict().items()}
        torch.manual_seed(0)
        d_c, s_c = orc.pva_flow(sd, enc.float().cpu(), smask.cpu(), nfe_d, temperature)
    f = orc.log_to_frames
    flips = int((f(d_g.float().cpu()) != f(d_c)).sum()) + int((f(s_g.float().cpu()) != f(s_c)).sum())
    return {"phonemes": L, "durations_compared": 2 * L, "flips": flips, "flip_rate": flips / (2.0 * L),
            "max_abs_log_dur_diff": float(max((d_g.cpu() - d_c).abs().max(), (s_g.cpu() - s_c).abs().max())),
            "vs": "oracle.pva_flow (fp32 restatement of pva.py:97-109), same encoder output and CPU-RNG noise"}


def long_form(pg, dev, args, C, T=2400, nfe=256):
    """BASELINE configs[4]: 30 s utterances (2400 frames), nsteps-denoiser=256, B = 1 and 16, on the bench's
    handle (bf16) and on an fp8 handle (MX-fp8 conv_2/conv_3/mlp.0/mlp.2 on the large-M path, which B = 16
    (38,400 rows) takes and B = 1 (2,400 rows) does not: there the fp8 handle computes in bf16).  The fp8
    row also reports the rel-L2 between its solve and the bf16 one (same inputs)."""
    from flamed.models.synthesizer.prob_generator import DenoiserHIP
    hip = pg.denoiser.hip()
    hip8 = DenoiserHIP(pg.denoiser, "fp8")
    out = {"frames": T, "nfe": nfe, "dtype": args.dtype}
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    fp8 = {"dtype": "mx-fp8 e4m3 (pointwise H x H GEMMs, B*T >= 16384 rows) + bf16",
           "note": "OCP MX: e8m0 scale per 32 input channels of weights and activations, scale = 2^ceil(log2(amax/448))"}
    for B in (1, 16):
        g = torch.Generator().manual_seed(args.seed + 2)
        x0 = (torch.randn(B, T, C, generator=g) * 0.3 + torch.randn(B, T, C, generator=g)).to(dev)
        spk = torch.randn(B, C, generator=g).to(dev)
        sols = {}
        for name, h in (("bf16", hip), ("fp8", hip8)):
            with torch.inference_mode():
                h.solve(x0, ts, spk, nfe)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sols[name] = h.solve(x0, ts, spk, nfe)
                torch.cuda.synchronize()
                sec = time.perf_counter() - t0
            row = {"ms_per_solve": round(sec * 1e3, 3), "latent_frames_per_s": round(B * T / sec, 1),
                   "rtf_denoiser": round(sec / (B * T * 200 / 16000.0), 6)}
            if name == "bf16":
                out[f"B{B}"] = row
            else:
                row["fp8_active"] = B * T >= 16384
                row["rel_l2_vs_bf16"] = float((sols["fp8"] - sols["bf16"]).norm() / sols["bf16"].norm())
                fp8[f"B{B}"] = row
    out["fp8"] = fp8
    return out


def latest_mfma(workload, B, T, dtype, cls):
    """Per-class MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)), MFMA FLOPs (512 x
    SQ_INSTS_VALU_MFMA_MOPS_*) and HBM bytes of a rocprofv3 PMC run of this workload (tools/pmc_mfma.sh ->
    profiles/latest_mfma.json), or None when the recorded run is of another shape."""
    path = os.path.join(REPO, "profiles", "latest_mfma.json")
    if not os.path.exists(path):
        return None
    w = json.load(open(path)).get(workload)
    if not w or (w.get("batch"), w.get("frames"), w.get("dtype")) != (B, T, dtype):
        return None
    c = w["classes"]
    if cls is not None:
        return dict(c[cls], source=w["source"]) if cls in c else None
    return {"source": w["source"], "classes": {k: {f: v[f] for f in ("mfma_util", "mfma_TFs", "mean_us", "hbm_GBps") if f in v}
                                                for k, v in c.items() if v.get("mfma_util") or v.get("hbm_GBps", 0) > 500}}


def throughput_mode(pg, dev, nfe, args, H, C, NB, B=64, T=400):
    """BASELINE configs[2] on the same handle: B = 64 utterances x 400 frames, nfe-step graph solve (one
    timed solve after a warm one), with the in-graph per-class costs and the roofline of the dominant
    kernel class."""
    import ctypes
    from flamed import _native as nat
    hip = pg.denoiser.hip()
    g = torch.Generator().manual_seed(args.seed + 1)
    x0 = (torch.randn(B, T, C, generator=g) * 0.3 + torch.randn(B, T, C, generator=g)).to(dev)
    spk = torch.randn(B, C, generator=g).to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    with torch.inference_mode():
        hip.solve(x0, ts, spk, nfe)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hip.solve(x0, ts, spk, nfe)
        torch.cuda.synchronize()
        sec = time.perf_counter() - t0
        L = nat.lib()
        mods = hip.adaln(ts[:1], spk, torch.zeros(B, dtype=torch.int32, device=dev), torch.arange(B, dtype=torch.int32, device=dev))
        ws = nat.Workspace().get(L.flamed_den_workspace_size(hip.handle, B, T), dev)
        ms = (ctypes.c_float * (N_CLASSES + 1))()
        xs = x0.clone()
        nat.check(L.flamed_den_time_kernels_graph(hip.handle, nat.ptr(xs), nat.ptr(mods), B, T, nat.ptr(ws), ws.numel(), 4, ms,
                                                  nat.stream_ptr(dev)), "flamed_den_time_kernels_graph")
        torch.cuda.synchronize()
    es = 2 if args.dtype == "bf16" else 4
    fused = ms[N_CLASSES - 1] <= 0.0  # no combine launches: fused into proj_in (small M only)
    ks = []
    for cls in range(N_CLASSES):
        if (cls == 2 or cls == N_CLASSES - 1) and ms[cls] <= 0.0:
            continue
        nbytes, flops, per_step = kernel_costs(cls, B, T, H, C, NB, es, fused=fused)
        t = max(ms[cls], 1e-6) * 1e-3
        ks.append({"name": KERNEL_NAMES[cls], "us": round(ms[cls] * 1e3, 2), "per_step": per_step,
                   "GBps": round(nbytes / t / 1e9, 1), "TFLOPs": round(flops / t / 1e12, 2)})
    dom = max(ks, key=lambda k: k["us"] * k["per_step"])
    nbytes, flops, _ = kernel_costs(KERNEL_NAMES.index(dom["name"]), B, T, H, C, NB, es, fused=fused)
    ridge = MFMA_PEAK_TFS[args.dtype] * 1e12 / (HBM_PEAK_GBS * 1e9)
    if flops / nbytes > ridge:
        roof = {"bound": "mfma", "achieved": dom["TFLOPs"], "peak": MFMA_PEAK_TFS[args.dtype], "unit": "TFLOP/s"}
    else:
        roof = {"bound": "hbm", "achieved": dom["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roof.update({"frac": round(roof["achieved"] / roof["peak"], 4), "kernel": dom["name"], "launch_us": dom["us"],
                 "tflops": dom["TFLOPs"], "gbps": dom["GBps"]})
    # the MFMA side from rocprofv3 counters of this workload (tools/pmc_mfma.sh): every large-M class
    roof["mfma_pmc"] = latest_mfma("b64", B, T, args.dtype, None)
    # the same workload on an MX-fp8 handle (conv_2/conv_3/mlp.0/mlp.2 block-scaled e4m3 at 25,600 rows)
    fp8 = None
    if args.dtype == "bf16":
        from flamed.models.synthesizer.prob_generator import DenoiserHIP
        hip8 = DenoiserHIP(pg.denoiser, "fp8")
        with torch.inference_mode():
            ref = hip.solve(x0, ts, spk, nfe)
            hip8.solve(x0, ts, spk, nfe)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sol8 = hip8.solve(x0, ts, spk, nfe)
            torch.cuda.synchronize()
            sec8 = time.perf_counter() - t0
        fp8 = {"dtype": "mx-fp8 e4m3 (pointwise H x H GEMMs) + bf16", "value": round(B * T / sec8, 2),
               "ms_per_solve": round(sec8 * 1e3, 3), "rel_l2_vs_bf16": float((sol8 - ref).norm() / ref.norm())}
        del hip8
    return {"workload": f"BASELINE configs[2]: {B} utterances x {T} frames, nsteps-denoiser={nfe}, hipGraph solve",
            "value": round(B * T / sec, 2), "unit": "latent frames/s", "ms_per_solve": round(sec * 1e3, 3),
            "rtf_denoiser": round(sec / (B * T * 200 / 16000.0), 6), "step_us_graph": round(ms[N_CLASSES] * 1e3, 2),
            "roofline": roof,
            "kernels": ks, "fp8": fp8}


def configs3_leg(pg, dev, dist, world, rank, args, C):
    """BASELINE configs[3] on every rank at once: 64 utterances x 400 frames per GPU, nfe = 128, bf16, seed + rank
    (the scaling curve's own per-GPU workload), timed after warm-up as max over ranks, with every rank's
    frames/s and the efficiency against rank 0 running the same per-GPU workload alone."""
    cfg = CONFIGS[3]
    B, T, nfe = cfg["batch"], cfg["frames"], cfg["nfe"]
    hip = pg.denoiser.hip()
    g = torch.Generator().manual_seed(args.seed + 1000 + rank)
    x0 = (torch.randn(B, T, C, generator=g) * 0.3 + torch.randn(B, T, C, generator=g)).to(dev)
    spk = torch.randn(B, C, generator=g).to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    steps = 2

    def step():
        hip.solve(x0, ts, spk, nfe)

    def sync():
        torch.cuda.synchronize(dev)
    with torch.inference_mode():
        step()
        sync()
        dist.barrier()
        solo = _timed(step, steps, sync) if rank == 0 else None
        dist.barrier()
        sync()
        dist.barrier()
        sec = _timed(step, steps, sync)
        dist.barrier()
    sec, per_rank, eff = scaling_stats(dist, world, rank, B * T, sec, solo, dev)
    return {"workload": f"BASELINE configs[3]: {B} utterances x {T} frames per GPU, nsteps-denoiser={nfe}, bf16, "
                        f"utterance-sharded over {world} GPUs (global batch {B * world})",
            "value": round(world * B * T / sec, 2), "unit": "latent frames/s", "ms_per_step": round(sec * 1e3, 3),
            "steps": steps, "global_batch": B * world, "per_rank_frames_per_s": per_rank, "scaling_detail": eff}


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) outside a torchrun job: start N ranks of this same script under
    torch.distributed.run as a CHILD process (nothing here has touched the GPU: no exec from a process
    that initialised HIP) and return its exit code.  One rank per GPU, RCCL over xGMI only for the
    barrier and the max-over-ranks timing all-reduce (utterances shard with no data-path collective,
    reference synthesize.py:268-291 batches)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def scaling_stats(dist, world, rank, frames_per_rank, sec, solo_sec, dev=None):
    """Max-over-ranks step time (the contract's clock), every rank's own frames/s, and the efficiency of the
    whole job against N x the same per-GPU workload timed on rank 0 alone in the same process tree (the
    other ranks idle at a barrier meanwhile).  No process group: (sec, [frames/s], None); a group of one rank
    (--dist-single) takes the collective path below with world = 1."""
    if dist is None:
        return sec, [round(frames_per_rank / sec, 3)], None
    import torch.distributed  # noqa: F401
    tt = torch.tensor([sec], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    per = torch.zeros(world, dtype=torch.float64, device=dev)
    per[rank] = frames_per_rank / sec
    dist.all_reduce(per)
    smax = float(tt.item())
    solo = torch.tensor([solo_sec if rank == 0 else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(solo)
    solo_fps = frames_per_rank / float(solo.item())
    value = world * frames_per_rank / smax
    return smax, [round(float(v), 3) for v in per.cpu()], {
        "solo_rank0_frames_per_s": round(solo_fps, 3), "efficiency_vs_n1": round(value / (world * solo_fps), 4),
        "n1_reference": "the same per-GPU workload timed on rank 0 alone (other ranks idle), same process tree"}


def _timed(fn, steps, sync):
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    return (time.perf_counter() - t0) / steps


def plumbing(args, rank, world):
    """--plumbing: the launcher / timing / reporting harness on CPU over gloo (CI rehearsal of the
    multi-rank path; no GPU): each rank runs ProbGenerator.sample on its own tiny synthetic shard with
    the module's torch ops (the reference's --device cpu path, BASELINE configs[0]) and rank 0 prints
    the same JSON line shape as the GPU bench (label, global batch, per-rank frames/s, efficiency)."""
    import torch.distributed as dist
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    torch.set_num_threads(1)
    if world > 1:
        dist.init_process_group("gloo")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    B, T, nfe = args.batch, args.frames, args.nfe
    g = torch.Generator().manual_seed(args.seed + rank)
    cond = torch.randn(B, cfg["n_quantizers"], T, cfg["cond_dim"], generator=g)
    spk = torch.randn(B, cfg["target_dim"], generator=g)
    mask = torch.ones(B, T, 1, dtype=torch.bool)
    res = {}

    def step():
        res["out"] = pg.sample(cond, spk, mask, nfe=nfe, temperature=0.3)

    def nosync():
        pass
    with torch.inference_mode():
        for _ in range(max(1, args.warmup)):
            step()
        solo = None
        if world > 1:
            dist.barrier()
            if rank == 0:
                solo = _timed(step, args.steps, nosync)
            dist.barrier()
        sec = _timed(step, args.steps, nosync)
        if world > 1:
            dist.barrier()
        sec, per_rank, eff = scaling_stats(dist if world > 1 else None, world, rank, B * T, sec, solo)
    out = res["out"]
    _, label = workload_label(args, world)
    line = {"metric": "latent frames/s (plumbing: CPU torch path over gloo)", "value": round(world * B * T / sec, 3),
            "unit": "latent frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(sec * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic", "plumbing": True, "finite": bool(torch.isfinite(out).all()),
            "config": {"workload": "CPU plumbing of " + label, "batch_per_gpu": B,
                       "frames": T, "nfe": nfe, "global_batch": world * B,
                       "parallelism": f"utterance-sharded x{world} (no collectives)"},
            "per_rank_frames_per_s": per_rank, "scaling_detail": eff}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    global FOLD
    args = parse()
    FOLD = args.lnfold != 0  # flamed_tune lnfold (kernel_costs applies the size policy)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.plumbing:
        return plumbing(args, rank, world)
    dist = None
    if world > 1 or args.dist_single or args.config == 3:
        # one process per GPU over RCCL ("nccl" on ROCm); with one rank (--dist-single / --config 3) the same
        # branch runs as a group of one, so its device-tensor collectives have run before a multi-GPU job needs them
        import torch.distributed as dist  # noqa: F811
        torch.cuda.set_device(local)
        if world == 1:
            import socket
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            dist.init_process_group("nccl", rank=0, world_size=1)
        else:
            dist.init_process_group("nccl")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    from flamed import _native as nat

    for key in ("splitk_target", "splitk_max", "dup_class", "small_stages", "dma", "noctr", "bn32", "big", "big_ns", "dw_tc", "big_rows", "dw_cg32", "dw_cg", "dma_ns", "lnfold", "graph_steps", "xcd_strips", "x16", "g8p_rows", "dwgn", "dwgn_small", "fuse_euler", "persist", "persist_opt", "split_batch", "persist_capmode", "persist_multi", "coop"):
        v = getattr(args, key)
        if v is not None:
            nat.check(nat.lib().flamed_tune(key.encode(), v), "flamed_tune")

    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg.denoiser.hip_dtype = args.dtype
    pg.denoiser.hip_graph = True
    pg = pg.to(dev)
    den = pg.denoiser
    B, T, nfe, C, H, NB = args.batch, args.frames, args.nfe, cfg["target_dim"], cfg["hidden_dim"], cfg["n_layers"]

    g = torch.Generator().manual_seed(args.seed + rank)
    cond = torch.randn(B, T, C, generator=g)
    noise = torch.randn(B, T, C, generator=g)
    spk_cpu = torch.randn(B, C, generator=g)
    xt0 = (noise * 0.3 + cond).to(dev)
    spk = spk_cpu.to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    hip = den.hip()

    def step():
        return hip.solve(xt0, ts, spk, nfe)

    def sync():
        torch.cuda.synchronize(dev)

    with torch.inference_mode():
        for _ in range(max(1, args.warmup)):
            out = step()
        torch.cuda.synchronize()
        solo = None
        if dist:  # the N = 1 reference of the efficiency figure: rank 0 alone, the other ranks idle
            dist.barrier()
            if rank == 0:
                solo = _timed(step, args.steps, sync)
            dist.barrier()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        runs0 = hip.persist_info()[0] if args.dtype == "bf16" else 0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        persist_runs = (hip.persist_info()[0] - runs0) if args.dtype == "bf16" else 0
        # device time of each persistent launch of the timed region: HIP events around the kernel on its
        # launch stream, recorded by the library (flamed_den_persist_times), read after the region
        pms = hip.persist_times(args.steps) if persist_runs >= args.steps else []
        if dist:
            dist.barrier()
        sec = (t1 - t0) / args.steps
        sec, per_rank, eff = scaling_stats(dist, world, rank, B * T, sec, solo, dev)
        finite = bool(torch.isfinite(out).all().item())
        configs3 = None
        if dist and not args.no_configs3 and B != CONFIGS[3]["batch"]:
            configs3 = configs3_leg(pg, dev, dist, world, rank, args, C)

        # ---- live per-kernel timing, dominant kernel roofline: in-graph cost per launch of each kernel
        # class (graph of 4 Euler steps replayed as captured vs with that class doubled; HIP events on
        # the launch stream), so dispatch gaps count and per-launch event overhead does not
        L = nat.lib()
        xs = xt0.clone().contiguous()
        r = torch.arange(B, device=dev)
        mods = hip.adaln(ts[:1], spk, torch.zeros(B, dtype=torch.int32, device=dev), r.to(torch.int32))
        ws = nat.Workspace().get(L.flamed_den_workspace_size(hip.handle, B, T), dev)
        import ctypes
        ms = (ctypes.c_float * (N_CLASSES + 1))()
        nat.check(L.flamed_den_time_kernels_graph(hip.handle, nat.ptr(xs), nat.ptr(mods), B, T, nat.ptr(ws), ws.numel(),
                                                  args.kernel_iters, ms, nat.stream_ptr(dev)), "flamed_den_time_kernels_graph")
        torch.cuda.synchronize()
    es = 4 if args.dtype == "f32" else 2
    # small-M solve graphs fuse the conv_out combine + Euler update into the next proj_in (flamed_tune
    # fuse_euler; 25 launches per step): the timing graph then has no combine launches (class cost 0)
    fused = ms[N_CLASSES - 1] <= 0.0
    kernels = []
    for cls in range(N_CLASSES):
        nbytes, flops, per_step = kernel_costs(cls, B, T, H, C, NB, es, fused=fused)
        if cls == 2 and ms[cls] <= 0.0:  # GroupNorm finalize fused into class 1 (the last-arriving block)
            continue
        if cls == N_CLASSES - 1 and fused:  # combine + Euler update fused into the next step's proj_in
            continue
        t = max(ms[cls], 1e-6) * 1e-3
        kernels.append({"name": KERNEL_NAMES[cls], "us": round(ms[cls] * 1e3, 2), "per_step": per_step,
                        "GBps": round(nbytes / t / 1e9, 1), "TFLOPs": round(flops / t / 1e12, 2),
                        "bytes": nbytes, "flops": flops})
    dom = max(kernels, key=lambda k: k["us"] * k["per_step"])
    ridge = MFMA_PEAK_TFS[args.dtype] * 1e12 / (HBM_PEAK_GBS * 1e9)
    bound = "mfma" if dom["flops"] / dom["bytes"] > ridge else "hbm"
    if bound == "hbm":
        roof = {"bound": "hbm", "achieved": dom["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dom["GBps"] / HBM_PEAK_GBS, 4)}
    else:
        roof = {"bound": "mfma", "achieved": dom["TFLOPs"], "peak": MFMA_PEAK_TFS[args.dtype], "unit": "TFLOP/s",
                "frac": round(dom["TFLOPs"] / MFMA_PEAK_TFS[args.dtype], 4)}
    traffic = None
    tpath = os.path.join(REPO, "profiles", "latest_traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if (tj.get("batch"), tj.get("frames"), tj.get("dtype")) == (B, T, args.dtype):
            traffic = tj.get("bytes_per_launch", {}).get(dom["name"])
    roof.update({"kernel": dom["name"], "launch_us": dom["us"], "traffic": traffic,
                 "traffic_source": "rocprofv3 PMC 2*FETCH_SIZE+WRITE_SIZE per launch, profiles/latest_traffic.json"
                 if traffic is not None else None,
                 "algorithmic_bytes": dom["bytes"], "algorithmic_flops": dom["flops"]})

    # ---- step-level roofline: SURVEY.md §8(d) canonical bytes per step / one Euler step in the graph
    sbytes = step_bytes_canonical(pg, B, T)
    step_s = ms[N_CLASSES] * 1e-3
    roof["step"] = {"bytes_canonical": sbytes, "step_us": round(ms[N_CLASSES] * 1e3, 2),
                    "achieved_GBps": round(sbytes / step_s / 1e9, 1),
                    "frac": round(sbytes / step_s / 1e9 / HBM_PEAK_GBS, 4),
                    "bytes_model": "W (bf16 GEMM weights + fp32 vectors/taps) + 54,272 B per frame"}
    if persist_runs >= args.steps and pms:
        # B = 1 solves ran as ONE persistent launch each (persist.hip): that kernel is the dominant (only)
        # kernel of the timed region.  Algorithmic bytes per launch = nfe x the canonical step bytes;
        # duration = HIP events around the launch on its stream (median over the timed solves).
        pk_ms = sorted(pms)[len(pms) // 2]
        lbytes = sbytes * nfe
        lflops = nfe * (2 * 20081664 * B * T)  # 40.16 MFLOP per frame-step
        ach = lbytes / (pk_ms * 1e-3) / 1e9
        ptraffic = None
        if os.path.exists(tpath):
            tj = json.load(open(tpath))
            if (tj.get("batch"), tj.get("frames"), tj.get("dtype"), tj.get("nfe", nfe)) == (B, T, args.dtype, nfe):
                ptraffic = tj.get("bytes_per_launch", {}).get("den_persist_kernel")
        launch_path = dict(roof)
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "kernel": "den_persist_kernel", "launch_us": round(pk_ms * 1e3, 1),
                "launches_per_solve": 1, "traffic": ptraffic,
                "traffic_source": "rocprofv3 PMC 2*FETCH_SIZE+WRITE_SIZE per launch, profiles/latest_traffic.json"
                if ptraffic is not None else None,
                "algorithmic_bytes": lbytes, "algorithmic_flops": lflops, "tflops": round(lflops / (pk_ms * 1e-3) / 1e12, 2),
                "mfma_pmc": latest_mfma("b1", B, T, args.dtype, "den_persist_kernel"),
                "step": {"bytes_canonical": sbytes, "step_us": round(pk_ms * 1e3 / nfe, 2),
                         "achieved_GBps": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                         "bytes_model": "W (bf16 GEMM weights + fp32 vectors/taps) + 54,272 B per frame"},
                "launch_path": launch_path}
        sbytes_step_s = pk_ms * 1e-3 / nfe
    else:
        sbytes_step_s = step_s
    peaks = None
    if rank == 0 and world == 1 and not args.no_peaks:
        try:
            peaks = measured_peaks(dev)
            roof["peak_measured"] = peaks["hbm_stream_copy_GBps"] if roof["unit"] == "GB/s" else peaks["bf16_gemm_TFs"]
            roof["frac_of_measured"] = round(roof["achieved"] / roof["peak_measured"], 4)
            roof["step"]["frac_of_measured"] = round(sbytes / sbytes_step_s / 1e9 / peaks["hbm_stream_copy_GBps"], 4)
        except Exception as e:  # reported, never fatal
            peaks = {"error": f"{type(e).__name__}: {e}"}

    # ---- CPU baseline: oracle restatement on the host cores (rank 0, N=1 only), bounded sample
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import flamed_oracle as orc
        cpu_model, n_host, n_usable = host_cpu()
        # the CPU share this process is given: OMP_NUM_THREADS when the host sets it (16 per GPU on the GPU
        # pool, whose host shows 256 logical CPUs: 256 torch threads there measured 18.5 s per Euler step
        # against ~22 ms at 16 — oversubscribed), else every CPU in the affinity mask
        ncores = min(n_usable, int(os.environ.get("OMP_NUM_THREADS") or n_usable))
        torch.set_num_threads(ncores)
        sd = {"prob_generator." + k: v.detach().float().cpu() for k, v in pg.state_dict().items()}
        xc = (noise * 0.3 + cond).float()
        with torch.inference_mode():
            t_a = time.perf_counter()
            orc.euler_solve(sd, xc, spk_cpu, nfe, steps=1)
            one = time.perf_counter() - t_a
            k = int(max(1, min(nfe, math.ceil(args.cpu_seconds / max(one, 1e-3)))))
            t_a = time.perf_counter()
            orc.euler_solve(sd, xc, spk_cpu, nfe, steps=k)
            tk = time.perf_counter() - t_a
        solve_s = tk * nfe / k
        cpu = {"value": round(B * T / solve_s, 2), "unit": "latent frames/s", "cores": ncores, "kind": "port",
               "sample": f"oracle fp32 torch-CPU restatement, B={B} T={T}: {k} of {nfe} Euler steps timed "
                         f"({tk:.2f} s), extrapolated to the full solve ({solve_s:.2f} s)",
               "cpu": cpu_model, "host_logical_cpus": n_host, "threads": ncores}

    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary:
        try:
            secondary = secondary_measurements(dev, nfe)
        except Exception as e:  # reported, never fatal for the headline line
            secondary = {"error": f"{type(e).__name__}: {e}"}
        try:
            secondary["throughput_mode"] = throughput_mode(pg, dev, nfe, args, H, C, NB)
        except Exception as e:
            secondary["throughput_mode"] = {"error": f"{type(e).__name__}: {e}"}
        try:
            secondary["long_form"] = long_form(pg, dev, args, C)
        except Exception as e:
            secondary["long_form"] = {"error": f"{type(e).__name__}: {e}"}

    audio_s = T * 200 / 16000.0
    value = world * B * T / sec
    cfg_i, label = workload_label(args, world)
    label += " (one persistent launch per solve)" if persist_runs >= args.steps else " (hipGraph Euler solve)"
    line = {
        "metric": "latent frames/s (RTF at nsteps-denoiser=128)", "value": round(value, 2),
        "unit": "latent frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(sec * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (seeded random-init weights, N(0,1) condition/speaker)",
        "config": {"workload": label, "baseline_config": cfg_i,
                   "batch_per_gpu": B, "frames": T, "nfe": nfe, "global_batch": world * B,
                   "parallelism": f"utterance-sharded x{world} (no collectives)"},
        "per_rank_frames_per_s": per_rank, "scaling_detail": eff, "configs3": configs3,
        "rtf_denoiser": round(sec / audio_s, 6),
        "roofline": roof,
        "kernels": [{k: v for k, v in kk.items() if k not in ("bytes", "flops")} for kk in kernels],
        "kernel_timing": "graph-of-launches path (B > 1, and the B = 1 fallback): in-graph per-launch cost "
                         "(4-step graph with the class doubled minus as captured, HIP events)",
        "persistent": {"runs": persist_runs, "solves": args.steps,
                       "launch_ms": [round(x, 3) for x in pms] if pms else None},
        "step_us_graph": round(ms[N_CLASSES] * 1e3, 2),
        "cpu_baseline": cpu,
        "peaks": {"hbm_spec_GBps": HBM_PEAK_GBS, "bf16_dense_spec_TFs": MFMA_PEAK_TFS["bf16"], **(peaks or {})},
        "finite": finite,
        "secondary": secondary,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
