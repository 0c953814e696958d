"""Timeline of one Euler step of the persistent PVA flow (diagnostic; needs libflamed_hip_stamps.so from
`make -C flamed-tts_amd/csrc stamps`).  Thread 0 of every workgroup stamps s_memrealtime (10 ns ticks) at
fixed points of the chosen step (pvaflow.hip PVST): start, conv1 done, H1 signalled, H1 passed, LN1 stats,
conv2 done, H2 signalled, H2 passed, head done.  Printed as per-interval medians over the workgroups.
Usage: python tools/pva_timeline.py [--phonemes L] [--nfe N] [--step S]"""
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

SLOTS = 16
NAMES = ["start", "conv1", "h1.signal", "h1.wait", "ln1.stats", "conv2", "h2.signal", "h2.wait", "head"]
# staged conv2 (pva_stage, row groups of >= 2 tiles): four more stamps inside conv2
NAMES_ST = NAMES[:5] + ["c2.stage0", "c2.chunk1", "c2.chunk3", "c2.chunk5"] + NAMES[5:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--phonemes", type=int, default=60)
    ap.add_argument("--nfe", type=int, default=64)
    ap.add_argument("--step", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--knob", action="append", default=[], help="flamed_tune key=value before the flow")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from flamed.models.synthesizer.pva import PVA
    from flamed.utils.seeded_init import randomize_module
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prior.yaml")))["variance_adaptor"]
    pva = PVA(cfg).eval()
    randomize_module(pva, 20251205)
    pva = pva.to(dev)
    L = a.phonemes
    g = torch.Generator().manual_seed(0)
    enc = torch.randn(1, L, 192, generator=g).to(dev)
    mask = torch.zeros(1, L, dtype=torch.bool, device=dev)
    buf = torch.zeros(256 * SLOTS, dtype=torch.int64, device=dev)
    lib = nat.lib()
    for kv in a.knob:
        k, v = kv.split("=")
        nat.check(lib.flamed_tune(k.encode(), int(v)), "flamed_tune")
    with torch.inference_mode():
        pva.flow(enc, mask, a.nfe, 0.3)
        nat.check(lib.flamed_pva_stamps(nat.ptr(buf), a.step), "flamed_pva_stamps")
        pva.flow(enc, mask, a.nfe, 0.3)
        torch.cuda.synchronize()
        nat.check(lib.flamed_pva_stamps(None, -1), "flamed_pva_stamps")
    runs, broken, ms = pva.hip().persist_info()
    st = buf.view(256, SLOTS).cpu().numpy().astype(np.int64)
    wgs = st[:, 0] > 0
    n = int((st[wgs][0] > 0).sum()) if wgs.any() else 0
    if n == 0:
        print(f"no stamps (runs={runs} broken={broken})")
        return
    st = st[wgs, :n]
    rel = (st - st[:, :1].min()) * 10e-3
    med, mx = np.median(rel, axis=0), rel.max(axis=0)
    lines = [f"persistent PVA flow L={L} nfe={a.nfe} step {a.step}: {int(wgs.sum())} workgroups, flow {ms:.3f} ms "
             f"({ms * 1e3 / a.nfe:.2f} us/step), step span (median) {med[-1] - med[0]:.2f} us",
             "  k  point        median_us  d_med  max_us"]
    for k in range(n):
        lines.append(f"{k:3d}  {(NAMES_ST if n == len(NAMES_ST) else NAMES)[k] if k < max(len(NAMES), n) and k < len(NAMES_ST if n == len(NAMES_ST) else NAMES) else '?':12s} {med[k]:9.2f} {med[k] - (med[k - 1] if k else 0):6.2f} {mx[k]:7.2f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
