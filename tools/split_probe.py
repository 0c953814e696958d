"""Diagnostic: configs[2] (B = 64, T = 400, nfe = 128) as one B = 64 solve vs k concurrent B = 64/k solves on k
streams (separate handles, so separate workspaces / graphs / step counters).  Usage: python tools/split_probe.py [--k 2 4]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--nfe", type=int, default=128)
    ap.add_argument("--x16", type=int, default=None)
    a = ap.parse_args()
    from flamed import _native as nat
    from flamed.models.synthesizer.prob_generator import ProbGenerator, DenoiserHIP
    from flamed.utils.seeded_init import randomize_module
    if a.x16 is not None:
        nat.check(nat.lib().flamed_tune(b"x16", a.x16), "tune")
    dev = torch.device("cuda:0")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg = pg.to(dev)
    g = torch.Generator().manual_seed(1)
    B, T, nfe = a.B, a.T, a.nfe
    x0 = (torch.randn(B, T, 256, generator=g) * 0.3 + torch.randn(B, T, 256, generator=g)).to(dev)
    spk = torch.randn(B, 256, generator=g).to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    with torch.inference_mode():
        h = pg.denoiser.hip()
        ref = h.solve(x0, ts, spk, nfe)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            ref = h.solve(x0, ts, spk, nfe)
        torch.cuda.synchronize()
        one = (time.perf_counter() - t0) / 2
        print(f"B={B} one solve: {one * 1e3:.1f} ms", flush=True)
        for k in a.k:
            Bk = B // k
            hs = [DenoiserHIP(pg.denoiser, "bf16") for _ in range(k)]
            ss = [torch.cuda.Stream() for _ in range(k)]
            outs = [None] * k

            def run():
                cur = torch.cuda.current_stream()
                for i in range(k):
                    ss[i].wait_stream(cur)
                    with torch.cuda.stream(ss[i]):
                        outs[i] = hs[i].solve(x0[i * Bk:(i + 1) * Bk], ts, spk[i * Bk:(i + 1) * Bk], nfe)
                for i in range(k):
                    cur.wait_stream(ss[i])
            run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            sec = (time.perf_counter() - t0) / 2
            out = torch.cat(outs, 0)
            print(f"B={B} as {k} concurrent B={Bk} solves: {sec * 1e3:.1f} ms (x{one / sec:.3f}); max|d| vs one {float((out - ref).abs().max()):.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
