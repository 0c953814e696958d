"""Persistent solve vs the graph-of-launches solve (same handle, same inputs) for each persist_opt value given:
rel-L2, whether it ran persistently, and two persistent solves bitwise equal.  Diagnostic.
Usage: python tools/persist_check.py [--frames T] [--nfe N] OPT [OPT ...]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))

import torch  # noqa: E402
import yaml  # noqa: E402

from flamed import _native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--nfe", type=int, default=32)
    ap.add_argument("opts", type=int, nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg = pg.to(dev)
    hip = pg.denoiser.hip()
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(1, a.frames, 256, generator=g).to(dev)
    spk = torch.randn(1, 256, generator=g).to(dev)
    ts = torch.linspace(0, 1, a.nfe + 1, device=dev)
    L = nat.lib()
    with torch.inference_mode():
        nat.check(L.flamed_tune(b"persist", 0), "tune")
        ref = hip.solve(x0, ts, spk, a.nfe)
        nat.check(L.flamed_tune(b"persist", 1), "tune")
        for o in a.opts:
            nat.check(L.flamed_tune(b"persist_opt", o), "tune")
            r0 = hip.persist_info()[0]
            x1 = hip.solve(x0, ts, spk, a.nfe)
            x2 = hip.solve(x0, ts, spk, a.nfe)
            runs, broken = hip.persist_info()
            e = float((x1 - ref).norm() / ref.norm())
            print(f"opt {o}: rel-L2 vs launch path {e:.3e}, persistent runs {runs - r0}/2, broken {broken}, "
                  f"deterministic {bool(torch.equal(x1, x2))}", flush=True)
        nat.check(L.flamed_tune(b"persist_opt", 0), "tune")


if __name__ == "__main__":
    main()
