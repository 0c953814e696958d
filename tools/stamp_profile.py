"""Per-block phase timeline of the denoiser kernels (diagnostic; needs libflamed_hip_stamps.so from
`make -C flamed-tts_amd/csrc stamps`).  For each kernel class, one eager Euler step is run with that
class's blocks recording s_memtime at their phase boundaries; prints the launch span, the spread of
block start times, and the mean per-phase time.
Usage: python tools/stamp_profile.py [--batch B] [--frames T] [--clock-ghz G]"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["FLAMED_HIP_LIB"] = os.path.join(REPO, "flamed-tts_amd", "flamed", "_native", "libflamed_hip_stamps.so")
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

from flamed import _native as nat  # noqa: E402

NAMES = {0: ("proj_in", ["prologue", "mainloop", "splitk", "epi+stats", ""]),
         1: ("dwconv+gn", ["X/partials loads+LN stats", "LN+mod->LDS", "conv", "GN sums (2 passes)", "normalise+store"]),
         3: ("conv2(GN)", ["prologue", "mainloop", "splitk", "epi+stats", ""]),
         4: ("conv3 resid", ["prologue", "mainloop", "splitk", "epi+stats", ""]),
         5: ("mlp0(LN)", ["prologue", "mainloop", "splitk", "epi+stats", ""]),
         6: ("mlp2 resid", ["prologue", "mainloop", "splitk", "epi+stats", ""]),
         7: ("conv_out", ["prologue", "mainloop", "splitk", "epi+stats", ""])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    ap.add_argument("--dma", type=int, default=1)
    ap.add_argument("--tune", nargs="*", default=[], help="extra flamed_tune key=value pairs")
    ap.add_argument("--classes", default="", help="comma-separated kernel classes (default: all)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg.denoiser.hip_dtype = "bf16"
    pg = pg.to(dev)
    hip = pg.denoiser.hip()
    B, T = a.batch, a.frames
    g = torch.Generator().manual_seed(0)
    xt = torch.randn(B, T, 256, generator=g).to(dev)
    spk = torch.randn(B, 256, generator=g).to(dev)
    ts = torch.linspace(0, 1, 129, device=dev)
    L = nat.lib()
    nat.check(L.flamed_tune(b"dma", a.dma), "tune")
    for kv in a.tune:
        k, v = kv.split("=")
        nat.check(L.flamed_tune(k.encode(), int(v)), "tune")
    only = [int(x) for x in a.classes.split(",") if x]
    with torch.inference_mode():
        hip.solve(xt, ts, spk, 128)  # loads the weights into the handle
        torch.cuda.synchronize()
        mods = hip.adaln(ts[:1], spk, torch.zeros(B, dtype=torch.int32, device=dev),
                         torch.arange(B, dtype=torch.int32, device=dev))
        ws = nat.Workspace().get(L.flamed_den_workspace_size(hip.handle, B, T), dev)
        buf = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
        nat.check(L.flamed_stamp_buffer(nat.ptr(buf)), "stamp_buffer")
        st = nat.stream_ptr(dev)
        for cls, (name, phases) in NAMES.items():
            if only and cls not in only:
                continue
            nat.check(L.flamed_tune(b"stamp_class", cls), "tune")
            for _ in range(2):
                buf.zero_()
                nat.check(L.flamed_den_step(hip.handle, nat.ptr(xt), nat.ptr(mods), T, B, T, ctypes.c_float(0.0),
                                            nat.ptr(ws), ws.numel(), st), "den_step")
            torch.cuda.synchronize()
            s = buf.view(-1, 8).cpu().numpy().astype(np.float64)
            s = s[s[:, 0] > 0]
            t0 = s[:, 0].min()
            last = np.where(s[:, 5] > 0, s[:, 5], s[:, 4])
            span = (last.max() - t0) / (a.clock_ghz * 1e3)
            starts = (s[:, 0] - t0) / (a.clock_ghz * 1e3)
            ph = []
            for i, pn in enumerate(phases):
                if not pn:
                    continue
                ok = (s[:, i + 1] > 0) & (s[:, i] > 0)
                if ok.any():
                    ph.append(f"{pn}={np.mean(s[ok, i + 1] - s[ok, i]) / (a.clock_ghz * 1e3):.2f}")
            print(f"class {cls} {name:12s} blocks={len(s):5d} span={span:6.2f}us start[p50/p90/max]="
                  f"{np.percentile(starts, 50):.2f}/{np.percentile(starts, 90):.2f}/{starts.max():.2f}us  "
                  + " ".join(ph))
        nat.check(L.flamed_tune(b"stamp_class", -1), "tune")


if __name__ == "__main__":
    main()
