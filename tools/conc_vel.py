"""Diagnostic: one velocity evaluation (B utterances) on two handles at once vs one after another: where do
the results differ (frames, channels, utterances)?"""
import copy
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402


def main():
    from flamed import _native as nat
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    L = nat.lib()
    for kv in os.environ.get("KNOBS", "").split(","):
        if kv:
            k, v = kv.split("=")
            nat.check(L.flamed_tune(k.encode(), int(v)), "tune")
    dev = torch.device("cuda:0")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg2 = copy.deepcopy(pg)
    pg, pg2 = pg.to(dev), pg2.to(dev)
    g = torch.Generator().manual_seed(2)
    B, T = 32, 400
    xs = [(torch.randn(B, T, 256, generator=g)).to(dev) for _ in range(2)]
    spk = [torch.randn(B, 256, generator=g).to(dev) for _ in range(2)]
    t = torch.full((B, 1), 0.3, device=dev)
    hips = [pg.denoiser.hip(), pg2.denoiser.hip()]
    with torch.inference_mode():
        ser = [hips[i].velocity(xs[i], t, spk[i]).clone() for i in range(2)]
        torch.cuda.synchronize()
        for rep in range(6):
            s = [torch.cuda.Stream(), torch.cuda.Stream()]
            o = [None, None]
            torch.cuda.synchronize()
            for i in range(2):
                with torch.cuda.stream(s[i]):
                    o[i] = hips[i].velocity(xs[i], t, spk[i]).clone()
            torch.cuda.synchronize()
            for i in range(2):
                d = (o[i] - ser[i]).abs()
                nz = d > 0
                if not bool(nz.any()):
                    print(f"rep {rep} handle {i}: equal", flush=True)
                    continue
                idx = torch.nonzero(nz)
                utt = torch.unique(idx[:, 0]).tolist()
                fr = torch.unique(idx[:, 1]).tolist()
                ch = torch.unique(idx[:, 2]).tolist()
                print(f"rep {rep} handle {i}: max {float(d.max()):.3e} n {int(nz.sum())} utts {utt[:12]}({len(utt)}) "
                      f"frames {fr[:16]}({len(fr)}) ch {ch[:16]}({len(ch)})", flush=True)


if __name__ == "__main__":
    main()
