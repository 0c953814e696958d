"""Diagnostic: the persistent B = 1 solve captured into a torch.cuda.graph and replayed several times
(persist_opt given), printing per replay whether the output is finite, equal to the eager solve, and the
device failure count.  Usage: python tools/capture_probe.py [--opt N] [--replays R] [--frames T]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402
from flamed import _native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", type=int, default=None)
    ap.add_argument("--replays", type=int, default=4)
    ap.add_argument("--frames", type=int, default=257)
    ap.add_argument("--nfe", type=int, default=16)
    ap.add_argument("--raw", action="store_true", help="capture only the library's solve call (no adaln/copies)")
    ap.add_argument("--capmode", type=int, default=None, help="flamed_tune persist_capmode")
    a = ap.parse_args()
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    dev = torch.device("cuda:0")
    if a.opt is not None:
        nat.check(nat.lib().flamed_tune(b"persist_opt", a.opt), "tune")
    if a.capmode is not None:
        nat.check(nat.lib().flamed_tune(b"persist_capmode", a.capmode), "tune")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 7)
    pg = pg.to(dev)
    hip = pg.denoiser.hip()
    g = torch.Generator().manual_seed(3)
    T, nfe = a.frames, a.nfe
    xd = torch.randn(1, T, 256, generator=g).to(dev)
    sd = torch.randn(1, 256, generator=g).to(dev)
    ts = torch.linspace(0, 1, nfe + 1, device=dev)
    L = nat.lib()
    with torch.inference_mode():
        eager = hip.solve(xd, ts, sd, nfe)
        torch.cuda.synchronize()
        print("eager finite", bool(torch.isfinite(eager).all()), "fails", hip.persist_fails(), flush=True)
        if a.raw:
            B = 1
            bufs = hip._solve_bufs[(1, T, nfe)]
            x = bufs["x"]
            ws = hip.ws.get(L.flamed_den_workspace_size(hip.handle, B, T), dev)
            s = torch.cuda.Stream()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                nat.check(L.flamed_den_solve(hip.handle, nat.ptr(x), nat.ptr(bufs["mods"]), nfe, B, T, nat.ptr(ws), ws.numel(), 1,
                                             nat.stream_ptr(dev)), "solve")
            import time
            for r in range(a.replays):
                x.copy_(xd)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                gr.replay()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3
                print("raw replay", r, "finite", bool(torch.isfinite(x).all()), "equal", bool(torch.equal(x, eager)),
                      "unchanged", bool(torch.equal(x, xd)), "rel_vs_eager", float((x - eager).norm() / eager.norm()),
                      f"{ms:.2f} ms", "fails", hip.persist_fails(), flush=True)
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hip.solve(xd, ts, sd, nfe)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            out = hip.solve(xd, ts, sd, nfe)
        inputs = [xd.clone()] + [torch.randn(1, T, 256, generator=g).to(dev) for _ in range(a.replays - 1)]
        refs = [eager] + [hip.solve(x_, ts, sd, nfe) for x_ in inputs[1:]]  # eager solves of every input
        torch.cuda.synchronize()
        for r in range(a.replays):
            xd.copy_(inputs[r])  # the captured input tensor, rewritten between replays
            gr.replay()
            torch.cuda.synchronize()
            print("replay", r, "finite", bool(torch.isfinite(out).all()), "equal", bool(torch.equal(out, refs[r])),
                  "fails", hip.persist_fails(), flush=True)


if __name__ == "__main__":
    main()
