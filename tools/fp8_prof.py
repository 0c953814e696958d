"""Per-kernel profile of one long-form solve (BASELINE configs[4]: B=16, T=2400) on a bf16 and an fp8
denoiser handle, for rocprofv3 --kernel-trace --stats.  Usage: python tools/fp8_prof.py [B] [T] [nfe]."""
import os
import sys
import time

import torch
import yaml

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "flamed-tts_amd"))
from flamed.models.synthesizer.prob_generator import ProbGenerator, DenoiserHIP  # noqa: E402
from flamed.utils.seeded_init import randomize_module  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 2400
    nfe = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    dev = torch.device("cuda:0")
    cfg = yaml.safe_load(open(os.path.join(ROOT, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 7)
    pg = pg.to(dev)
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(B, T, 256, generator=g).to(dev)
    spk = torch.randn(B, 256, generator=g).to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    for name in ("bf16", "fp8"):
        h = DenoiserHIP(pg.denoiser, name)
        with torch.inference_mode():
            h.solve(x0, ts, spk, nfe)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h.solve(x0, ts, spk, nfe)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        print(f"{name}: B={B} T={T} nfe={nfe}: {ms:.2f} ms/solve, {ms / nfe:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
