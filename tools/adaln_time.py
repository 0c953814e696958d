#!/usr/bin/env python3
"""Split the B=1 solve time into AdaLN precompute and the graph-replayed Euler steps."""
import os, sys, time
import torch, yaml
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
from flamed.models.synthesizer.prob_generator import ProbGenerator  # noqa: E402
from flamed.utils.seeded_init import randomize_module  # noqa: E402
dev = torch.device("cuda:0")
cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
pg = ProbGenerator(cfg).eval(); randomize_module(pg, 1); pg = pg.to(dev)
h = pg.denoiser.hip()
B, T, nfe = int(sys.argv[1]) if len(sys.argv) > 1 else 1, 400, 128
x = torch.randn(B, T, 256, device=dev); spk = torch.randn(B, 256, device=dev); ts = torch.linspace(0, 1, nfe + 1, device=dev)
r = torch.arange(nfe * B, device=dev); ti = (r // B).to(torch.int32); si = (r % B).to(torch.int32)
with torch.inference_mode():
    for _ in range(3): h.solve(x, ts, spk, nfe); h.adaln(ts[:nfe], spk, ti, si)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(10): h.adaln(ts[:nfe], spk, ti, si)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    for _ in range(10): h.solve(x, ts, spk, nfe)
    torch.cuda.synchronize(); t2 = time.perf_counter()
print(f"B={B} adaln {(t1 - t0) * 100:.3f} ms  solve (incl. adaln) {(t2 - t1) * 100:.3f} ms")
