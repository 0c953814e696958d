"""Timeline of one Euler step of the persistent B = 1 solve (diagnostic; needs libflamed_hip_stamps.so from
`make -C flamed-tts_amd/csrc stamps`).  Thread 0 of every workgroup stamps s_memrealtime (10 ns ticks,
chip-wide) at each wait begin / wait end / GEMM done / signal of the chosen step; the stamps are aligned
by index (every workgroup runs the same sequence) and printed as per-interval medians and maxima.
Usage: python tools/persist_timeline.py [--frames T] [--nfe N] [--step S]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["FLAMED_HIP_LIB"] = os.path.join(REPO, "flamed-tts_amd", "flamed", "_native", "libflamed_hip_stamps.so")
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

from flamed import _native as nat  # noqa: E402

SLOTS = 160


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--nfe", type=int, default=16)
    ap.add_argument("--step", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--opt", type=int, default=None, help="flamed_tune persist_opt")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg = pg.to(dev)
    hip = pg.denoiser.hip()
    T, nfe = a.frames, a.nfe
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(1, T, 256, generator=g).to(dev)
    spk = torch.randn(1, 256, generator=g).to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    buf = torch.zeros(256 * SLOTS, dtype=torch.int64, device=dev)
    L = nat.lib()
    if a.opt is not None:
        nat.check(L.flamed_tune(b"persist_opt", a.opt), "flamed_tune")
    with torch.inference_mode():
        hip.solve(x0, ts, spk, nfe)
        print("after warm solve: persist_info", hip.persist_info(), flush=True)
        nat.check(L.flamed_persist_stamps(nat.ptr(buf), a.step), "flamed_persist_stamps")
        hip.solve(x0, ts, spk, nfe)
        torch.cuda.synchronize()
        nat.check(L.flamed_persist_stamps(None, -1), "flamed_persist_stamps")
    runs, broken = hip.persist_info()
    st = buf.view(256, SLOTS).cpu().numpy().astype(np.int64)
    n = int((st[0] > 0).sum())
    if n == 0:
        print(f"no stamps recorded (runs={runs} broken={broken}, nonzero={(st != 0).sum()})")
        return
    st = st[:, :n]
    t0 = st[:, 0].min()
    rel = (st - t0) * 10e-3  # microseconds
    med = np.median(rel, axis=0)
    mx = rel.max(axis=0)
    mn = rel.min(axis=0)
    lines = [f"persistent solve T={T} nfe={nfe} step {a.step}: {n} stamps per workgroup, runs={runs} broken={broken}",
             f"step span (median WG): {med[-1] - med[0]:.2f} us",
             "  k   median_us   d_med   min_us   max_us  spread"]
    for k in range(n):
        d = med[k] - med[k - 1] if k else 0.0
        lines.append(f"{k:3d} {med[k]:10.2f} {d:7.2f} {mn[k]:8.2f} {mx[k]:8.2f} {mx[k] - mn[k]:7.2f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
