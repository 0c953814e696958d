"""Diagnostic: configs[2]-shaped solve (B utterances x T frames, nfe steps) as split chains (split_batch S) vs
unsplit, graph vs eager: pairwise max |diff| of the results (bitwise equal expected within one structure)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--nfe", type=int, default=32)
    a = ap.parse_args()
    from flamed import _native as nat
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    L = nat.lib()
    dev = torch.device("cuda:0")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg = pg.to(dev)
    g = torch.Generator().manual_seed(2)
    B, T, nfe = a.B, a.T, a.nfe
    x0 = (torch.randn(B, T, 256, generator=g) * 0.3 + torch.randn(B, T, 256, generator=g)).to(dev)
    spk = torch.randn(B, 256, generator=g).to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    hip = pg.denoiser.hip()
    res = {}
    with torch.inference_mode():
        for S, serial in ((1, 0), (2, 0)):
            nat.check(L.flamed_tune(b"split_batch", S), "tune")
            for graph in (True, True, False):
                pg.denoiser.hip_graph = graph
                out = hip.solve(x0, ts, spk, nfe)
                torch.cuda.synchronize()
                key = f"S{S}{'s' if serial else ''}_{'graph' if graph else 'eager'}"
                key = key + "2" if key in res else key
                res[key] = out.clone()
        pg.denoiser.hip_graph = True
    ks = list(res)
    for i in range(len(ks)):
        for j in range(i + 1, len(ks)):
            d = float((res[ks[i]] - res[ks[j]]).abs().max())
            print(f"{ks[i]:>10} vs {ks[j]:<10} max|d| {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
