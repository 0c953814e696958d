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
MFMA_PEAK_TFS = {"bf16": 2500.0, "f32": 157.3}   # dense peaks


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=400, help="latent frames per utterance (80 Hz)")
    ap.add_argument("--nfe", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel-iters", type=int, default=10, help="eager steps timed in-context per kernel class")
    ap.add_argument("--splitk-target", type=int, default=None, help="flamed_tune splitk_target (1 disables split-K)")
    ap.add_argument("--splitk-max", type=int, default=None, help="flamed_tune splitk_max")
    ap.add_argument("--dup-class", type=int, default=None, help="ablation: flamed_tune dup_class")
    ap.add_argument("--small-stages", type=int, default=None, help="flamed_tune small_stages (3, 5, 7)")
    return ap.parse_args()


def kernel_costs(cls: int, B: int, T: int, H: int, C: int, NB: int, es: int):
    """Algorithmic (bytes, flops) per launch of each kernel class, and launches per Euler step.
    Bytes = every operand read once + every output written once."""
    M = B * T
    NT = H // 64
    TS = (T + 63) // 64
    stats = M * NT * 8
    if cls == 0:
        return M * C * 4 + H * C * es + M * H * 4 + stats, 2 * M * H * C, 1
    if cls == 1:
        return M * H * 4 + stats + M * H * 4 + B * TS * H * 12, 2 * 31 * M * H, NB + 1
    if cls == 2:
        return B * TS * H * 12 + B * H * 8, 10 * B * TS * H, NB + 1
    if cls == 3:
        return M * H * 4 + B * H * 8 + H * H * es + M * H * es, 2 * M * H * H, NB + 1
    if cls == 4:
        return M * H * es + H * H * es + 2 * M * H * 4 + 2 * stats, 2 * M * H * H, NB + 1
    if cls == 5:
        return M * H * 4 + stats + H * H * es + M * H * es, 2 * M * H * H, NB
    if cls == 6:
        return M * H * es + H * H * es + 2 * M * H * 4 + stats, 2 * M * H * H, NB
    if cls == 7:
        return M * H * 4 + stats + 3 * C * H * es + M * 3 * C * 4, 2 * M * 3 * C * H, 1
    return M * 3 * C * 4 + 2 * M * C * 4, 4 * M * C, 1


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    from flamed import _native as nat

    for key in ("splitk_target", "splitk_max", "dup_class", "small_stages"):
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

    with torch.inference_mode():
        for _ in range(max(1, args.warmup)):
            out = step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        sec = (t1 - t0) / args.steps
        if dist:
            tt = torch.tensor([sec], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            sec = float(tt.item())
        finite = bool(torch.isfinite(out).all().item())

        # ---- live per-kernel timing (HIP events on the launch stream), dominant kernel roofline
        L = nat.lib()
        xs = xt0.clone().contiguous()
        r = torch.arange(B, device=dev)
        mods = hip.adaln(ts[:1], spk, torch.zeros(B, dtype=torch.int32, device=dev), r.to(torch.int32))
        ws = nat.Workspace().get(L.flamed_den_workspace_size(hip.handle, B, T), dev)
        import ctypes
        ms = (ctypes.c_float * N_CLASSES)()
        nat.check(L.flamed_den_time_kernels(hip.handle, nat.ptr(xs), nat.ptr(mods), B, T, nat.ptr(ws), ws.numel(),
                                            args.kernel_iters, ms, nat.stream_ptr(dev)), "flamed_den_time_kernels")
        torch.cuda.synchronize()
    es = 2 if args.dtype == "bf16" else 4
    kernels = []
    for cls in range(N_CLASSES):
        nbytes, flops, per_step = kernel_costs(cls, B, T, H, C, NB, es)
        t = ms[cls] * 1e-3
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

    # ---- CPU baseline: oracle restatement on the host cores (rank 0, N=1 only), bounded sample
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import flamed_oracle as orc
        ncores = int(os.environ.get("OMP_NUM_THREADS", 0)) or min(16, os.cpu_count() or 1)
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
               "cpu": platform.processor() or platform.machine()}

    audio_s = T * 200 / 16000.0
    value = world * B * T / sec
    line = {
        "metric": "latent frames/s (RTF at nsteps-denoiser=128)", "value": round(value, 2),
        "unit": "latent frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(sec * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (seeded random-init weights, N(0,1) condition/speaker)",
        "config": {"workload": f"BASELINE configs[1]: {B} utterance(s) x {T} frames ({audio_s:.1f} s audio) per GPU, "
                               f"nsteps-denoiser={nfe}, hipGraph Euler solve",
                   "batch_per_gpu": B, "frames": T, "nfe": nfe, "global_batch": world * B,
                   "parallelism": f"utterance-sharded x{world} (no collectives)"},
        "rtf_denoiser": round(sec / audio_s, 6),
        "roofline": roof,
        "kernels": [{k: v for k, v in kk.items() if k not in ("bytes", "flops")} for kk in kernels],
        "cpu_baseline": cpu,
        "finite": finite,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
