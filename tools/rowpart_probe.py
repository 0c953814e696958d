"""Diagnostic for persist_opt bit 2 (whole-16-row-tile row groups): is each GroupNorm exchange form deterministic,
and where do the granule and counter forms part?  python tools/rowpart_probe.py --shapes 4x100,2x200,1x400"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402

DEFAULT = 361032


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4x100,2x200,1x400")
    ap.add_argument("--nfe", type=int, default=8)
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
    hip = pg.denoiser.hip()
    for shape in a.shapes.split(","):
        B, T = (int(v) for v in shape.split("x"))
        g = torch.Generator().manual_seed(40 + B)
        x0 = torch.randn(B, T, 256, generator=g).to(dev)
        spk = torch.randn(B, 256, generator=g).to(dev)
        ts = torch.linspace(0, 1, a.nfe + 1, device=dev)
        outs = {}
        for name, opt in (("shares/gran", DEFAULT), ("shares/ctr", DEFAULT ^ 512),
                          ("tiles/gran", DEFAULT | 2), ("tiles/ctr", (DEFAULT | 2) ^ 512)):
            nat.check(L.flamed_tune(b"persist_opt", opt), "tune")
            with torch.inference_mode():
                r = [hip.solve(x0.clone(), ts, spk, a.nfe).float().cpu() for _ in range(3)]
            det = all(torch.equal(r[0], v) for v in r[1:])
            outs[name] = r[0]
            print(f"B={B} T={T} {name}: deterministic over 3 runs {det}", flush=True)
        nat.check(L.flamed_tune(b"persist_opt", DEFAULT), "tune")
        for p, q in (("shares/gran", "shares/ctr"), ("tiles/gran", "tiles/ctr"), ("shares/gran", "tiles/gran")):
            d = (outs[p] - outs[q]).abs()
            per_u = [f"{d[u].max().item():.2e}" for u in range(B)]
            rows = (d.amax(dim=2) > 0).nonzero().tolist()
            first = rows[0] if rows else None
            print(f"B={B} T={T} {p} vs {q}: equal {torch.equal(outs[p], outs[q])}, max |diff| per utterance {per_u}, "
                  f"first differing (utt, row) {first}, differing rows {len(rows)}", flush=True)


if __name__ == "__main__":
    main()
