"""Capture + instantiate cost of the solve graph vs its steady-state replay, per graph_steps setting
(B=1, nfe=128, bf16): first solve of a new shape (captures) vs the mean of the next 5 solves.
Usage: python tools/graph_cost.py [graph_steps ...]"""
import os
import sys
import time

import torch
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
from flamed import _native as nat  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg.denoiser.hip_dtype = "bf16"
    pg = pg.to(dev)
    hip = pg.denoiser.hip()
    L = nat.lib()
    g = torch.Generator().manual_seed(0)
    for gs in [int(a) for a in sys.argv[1:]] or (16, 32, 64, 128):
        nat.check(L.flamed_tune(b"graph_steps", gs), "tune")
        for T in (400, 401):  # a new shape forces a new capture
            xt = torch.randn(1, T, 256, generator=g).to(dev)
            spk = torch.randn(1, 256, generator=g).to(dev)
            ts = torch.linspace(0, 1, 129, device=dev)
            with torch.inference_mode():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                hip.solve(xt, ts, spk, 128)
                torch.cuda.synchronize()
                first = time.perf_counter() - t0
                t0 = time.perf_counter()
                for _ in range(5):
                    hip.solve(xt, ts, spk, 128)
                torch.cuda.synchronize()
                steady = (time.perf_counter() - t0) / 5
            print(f"graph_steps={gs:4d} T={T}: first solve {first * 1e3:8.1f} ms, steady {steady * 1e3:6.2f} ms", flush=True)
    nat.check(L.flamed_tune(b"graph_steps", 16), "tune")


if __name__ == "__main__":
    main()
