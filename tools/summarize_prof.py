#!/usr/bin/env python3
"""Summarise a gpu_profile.sh run: rocprofv3 kernel stats per denoiser kernel class + PMC traffic.

  python tools/summarize_prof.py gpurun_out/<tag> profiles/<tag>   [--batch B --frames T --dtype bf16]

Writes <out>_kernels.md (table), <out>_kernel_stats.csv (raw rocprof stats) and <out>_traffic.json
(per-class mean HBM bytes per launch: 2*FETCH_SIZE + WRITE_SIZE, KiB units of rocprofv3 -> bytes;
the x2 is MI355X_MICROARCH.md §HBM's gfx950 correction for 16-B/lane streaming reads).  bench.py
reads the traffic file for its roofline.traffic field when the workload matches.
"""
import argparse
import csv
import json
import os
import re
import shutil
from collections import defaultdict

CLASSES = [
    ("proj_in_gemm", [r"LoadF32.*EpiBiasStatsT", r"LoadF32I.*EpiBiasStatsT", r"LoadEulerIn", r"gemm8p_kernel<fl::EpiBiasStatsT",
                      r"gemm8p_kernelINS_13EpiBiasStatsT"]),
    ("lnmod_dwconv_gnpartials", [r"dwconv_stats_kernel", r"dwgn_small_kernel", r"dwgn_kernel"]),
    ("gn_finalize", [r"gn_finalize_kernel"]),
    ("gnapply_conv2_gemm_gelu", [r"LoadGN", r"EpiBiasActIDF16bLi1E", r"EpiBiasAct<bf16, 1>",
                                 r"gemm8p_kernel<fl::EpiBiasAct<bool _Accum, int, E>", r"EpiBiasActF8ILi1E", r"EpiBiasActF8<1>"]),
    ("conv3_gemm_gated_resid", [r"EpiConvNeXtResid"]),
    ("lnmod_mlp0_gemm_silu", [r"LoadLNMod<[^>]*true>", r"LoadLNModI\w+Lb1E", r"EpiLNFold<[^>]*bf16", r"EpiLNFoldIDF16b"]),
    ("mlp2_gemm_gated_resid", [r"EpiGatedResid"]),
    ("lnmod_conv_out_gemm", [r"LoadLNMod<[^>]*false>", r"LoadLNModI\w+Lb0E", r"EpiLNFold<float", r"EpiLNFoldIf"]),
    ("conv_out_combine_euler", [r"conv3_combine_kernel", r"euler_cast_kernel"]),
    # B = 1 persistent solve (persist.hip): one launch per solve, every step inside
    ("den_persist_kernel", [r"den_persist_kernel"]),
]


def classify(name):
    for cls, pats in CLASSES:
        if any(re.search(p, name) for p in pats):
            return cls
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("out_prefix")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--nfe", type=int, default=128)
    a = ap.parse_args()
    stats = list(csv.DictReader(open(os.path.join(a.run_dir, "prof", "run_kernel_stats.csv"))))
    shutil.copy(os.path.join(a.run_dir, "prof", "run_kernel_stats.csv"), a.out_prefix + "_kernel_stats.csv")
    agg = defaultdict(lambda: [0, 0.0])
    for r in stats:
        c = classify(r["Name"])
        if c:
            agg[c][0] += int(r["Calls"])
            agg[c][1] += float(r["TotalDurationNs"])
    pmc = defaultdict(lambda: defaultdict(list))
    for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        path = os.path.join(a.run_dir, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per_dispatch = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != ctr:
                continue
            per_dispatch[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for d, v in per_dispatch.items():
            c = classify(names[d])
            if c:
                pmc[c][ctr].append(v)
    traffic = {}
    lines = ["| kernel class | calls | avg µs (rocprofv3) | FETCH_SIZE KiB/launch | WRITE_SIZE KiB/launch | HBM bytes/launch (2F+W) |",
             "|---|---|---|---|---|---|"]
    for cls, _ in CLASSES:
        if cls not in agg:
            continue
        calls, tot = agg[cls]
        f = pmc[cls].get("FETCH_SIZE", [])
        w = pmc[cls].get("WRITE_SIZE", [])
        fm = sum(f) / len(f) if f else None
        wm = sum(w) / len(w) if w else None
        hb = (2 * fm + wm) * 1024 if (fm is not None and wm is not None) else None
        if hb is not None:
            traffic[cls] = hb
        lines.append(f"| {cls} | {calls} | {tot / calls / 1e3:.2f} | {'' if fm is None else f'{fm:.1f}'} | "
                     f"{'' if wm is None else f'{wm:.1f}'} | {'' if hb is None else f'{hb:.0f}'} |")
    meta = {"batch": a.batch, "frames": a.frames, "dtype": a.dtype, "nfe": a.nfe, "source": os.path.basename(a.out_prefix),
            "bytes_per_launch": traffic}
    json.dump(meta, open(a.out_prefix + "_traffic.json", "w"), indent=1)
    bench = os.path.join(a.run_dir, "bench.json")
    with open(a.out_prefix + "_kernels.md", "w") as fo:
        fo.write(f"# rocprofv3 summary — {os.path.basename(a.out_prefix)} (B={a.batch}, T={a.frames}, {a.dtype})\n\n")
        fo.write("Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline --no-secondary --no-peaks"
                 " --coop 0 --steps 2 --warmup 1`; PMC: separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of the same"
                 " bench.  The profiled persistent launch is a plain launch (`--coop 0`: rocprofv3's teardown faults after"
                 " cooperative launches, README \"Known issues\"); the bench's own HIP-event timing of the shipped"
                 " cooperative launch agrees within ~1.5 %.\n\n")
        fo.write("\n".join(lines) + "\n")
        if os.path.exists(bench):
            fo.write("\nBench line of the same run:\n\n```json\n" + open(bench).read().strip() + "\n```\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
