"""Diagnostic: which concurrent neighbour perturbs a dwgn velocity evaluation?  Handle A's velocity runs on
stream A while stream B runs (m1) a torch matmul loop, (m2) handle B's velocity without dwgn, (m3) handle
B's velocity with dwgn while A runs without it.  A's result is compared with A alone."""
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
    big = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)

    def tune(k, v):
        nat.check(L.flamed_tune(k.encode(), v), "tune")

    for kv in os.environ.get("KNOBS", "").split(","):
        if kv:
            k, v = kv.split("=")
            tune(k, int(v))

    with torch.inference_mode():
        ref = {}
        for dw in (0, 1):
            tune("dwgn", dw)
            ref[dw] = hips[0].velocity(xs[0], t, spk[0]).clone()
        torch.cuda.synchronize()
        for mode in ("m1", "m2", "m3", "m4"):
            nbad = 0
            for rep in range(8):
                sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
                torch.cuda.synchronize()
                a_dw = 0 if mode == "m3" else 1
                with torch.cuda.stream(sB):
                    if mode == "m1":
                        for _ in range(12):
                            big = (big @ big).clamp_(-1, 1)
                    elif mode == "m4":
                        for _ in range(20):
                            torch.cuda._sleep(1000000)
                    else:
                        tune("dwgn", 0 if mode == "m2" else 1)
                        hips[1].velocity(xs[1], t, spk[1])
                with torch.cuda.stream(sA):
                    tune("dwgn", a_dw)
                    oa = hips[0].velocity(xs[0], t, spk[0]).clone()
                torch.cuda.synchronize()
                d = float((oa - ref[a_dw]).abs().max())
                nbad += d > 0
                print(f"{mode} rep {rep}: A max|d| {d:.3e}", flush=True)
            print(f"{mode}: {nbad}/8 differ", flush=True)
    tune("dwgn", 1)


if __name__ == "__main__":
    main()
