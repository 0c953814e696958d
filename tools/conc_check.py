"""Diagnostic: two independent denoiser handles solving B/2 utterances each, eager (no graph), on two
streams at once vs one after another; any difference means a kernel's result depends on what else runs."""
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
    nat.check(L.flamed_tune(b"split_batch", 1), "tune")
    dev = torch.device("cuda:0")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg2 = copy.deepcopy(pg)
    pg, pg2 = pg.to(dev), pg2.to(dev)
    g = torch.Generator().manual_seed(2)
    B, T, nfe = 32, 400, 32
    xs = [(torch.randn(B, T, 256, generator=g)).to(dev) for _ in range(2)]
    spk = [torch.randn(B, 256, generator=g).to(dev) for _ in range(2)]
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    hips = [pg.denoiser.hip(), pg2.denoiser.hip()]
    sets = [[], [("dwgn", 0)], [("x16", 1)]]
    for knobs in sets:
        for k_, v_ in knobs:
            nat.check(L.flamed_tune(k_.encode(), v_), "tune")
        for graph in (False, True):
            pg.denoiser.hip_graph = pg2.denoiser.hip_graph = graph
            with torch.inference_mode():
                ser = [hips[i].solve(xs[i], ts, spk[i], nfe).clone() for i in range(2)]
                torch.cuda.synchronize()
                outs = []
                for rep in range(3):
                    s = [torch.cuda.Stream(), torch.cuda.Stream()]
                    o = [None, None]
                    torch.cuda.synchronize()
                    for i in range(2):
                        with torch.cuda.stream(s[i]):
                            o[i] = hips[i].solve(xs[i], ts, spk[i], nfe).clone()
                    torch.cuda.synchronize()
                    outs.append(o)
            for rep, o in enumerate(outs):
                d = [float((o[i] - ser[i]).abs().max()) for i in range(2)]
                print(f"knobs {knobs} graph {graph} rep {rep}: concurrent vs serial max|d| {d[0]:.3e} {d[1]:.3e}", flush=True)
        for k_, v_ in knobs:
            L.flamed_tune(k_.encode(), {"dwgn": 1, "x16": 0}[k_])


if __name__ == "__main__":
    main()
