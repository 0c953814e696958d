"""Diagnostic for persist_opt bit 2 (whole-16-row-tile row groups): is each GroupNorm exchange form deterministic,
and where do the granule and counter forms part?  python tools/rowpart_probe.py --shapes 4x100,2x200,1x400
--dump (needs libflamed_hip_stamps.so, `make -C flamed-tts_amd/csrc stamps`): the GroupNorm exchange of every step as
each form's combining lanes read it (flamed_persist_gndump), compared between the two forms step by step."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if "--dump" in sys.argv:
    os.environ["FLAMED_HIP_LIB"] = os.path.join(REPO, "flamed-tts_amd", "flamed", "_native", "libflamed_hip_stamps.so")
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402

DEFAULT = 361032  # round-5 default (equal shares); the probe flips bit 2 itself


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4x100,2x200,1x400")
    ap.add_argument("--nfe", type=int, default=8)
    ap.add_argument("--dump", action="store_true")
    ap.add_argument("--base", type=int, default=DEFAULT)
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
    if a.dump:
        return dump(a, L, nat, hip, dev)
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


NAMES = ["n", "mean", "M2"]


def dump(a, L, nat, hip, dev):
    nb = 5
    for shape in a.shapes.split(","):
        B, T = (int(v) for v in shape.split("x"))
        g = torch.Generator().manual_seed(40 + B)
        x0 = torch.randn(B, T, 256, generator=g).to(dev)
        spk = torch.randn(B, 256, generator=g).to(dev)
        ts = torch.linspace(0, 1, a.nfe + 1, device=dev)
        forms = (("tiles/gran", a.base | 2), ("tiles/ctr", (a.base | 2) ^ 512))
        for step in range(a.nfe):
            dumps = {}
            for name, opt in forms:
                nat.check(L.flamed_tune(b"persist_opt", opt), "tune")
                buf = torch.full((nb * 256 * 32 * 32,), float("nan"), dtype=torch.float32, device=dev)
                nat.check(L.flamed_persist_gndump(nat.ptr(buf), step), "gndump")
                with torch.inference_mode():
                    hip.solve(x0.clone(), ts, spk, a.nfe)
                torch.cuda.synchronize()
                nat.check(L.flamed_persist_gndump(None, -1), "gndump")
                dumps[name] = buf.view(nb, 8, 32, 32, 32).cpu()  # [blk][g][s][c][k]
            p, q = dumps["tiles/gran"], dumps["tiles/ctr"]
            same = (p == q) | (p.isnan() & q.isnan())
            print(f"B={B} T={T} step {step}: dumps equal {bool(same.all())}", flush=True)
            if not bool(same.all()):
                idx = (~same).nonzero().tolist()
                print(f"  {len(idx)} differing entries; first 12:")
                for blk, gg, ss, cc, k in idx[:12]:
                    what = (f"group {k // 3} {NAMES[k % 3]}" if k < 24 else
                            {24: "combined mean", 25: "scale", 26: "own mean", 27: "own M2", 28: "own n"}.get(k, str(k)))
                    print(f"  blk {blk} g {gg} s {ss} c {cc} {what}: gran {p[blk, gg, ss, cc, k].item()!r} "
                          f"ctr {q[blk, gg, ss, cc, k].item()!r}")
                # which slots of k differ overall
                ks = sorted(set(i[4] for i in idx))
                print(f"  differing fields {ks}; groups {sorted(set(i[1] for i in idx))}; blks {sorted(set(i[0] for i in idx))}")
                break
        nat.check(L.flamed_tune(b"persist_opt", DEFAULT), "tune")


if __name__ == "__main__":
    main()
