"""Time ProbGenerator solves (the denoiser's Euler loop) for given shapes under knob settings, e.g.
    python tools/solve_time.py --shapes 1x2400x256,2x400x128 --knobs persist=1 persist=0
prints one line per (shape, knob set): median ms per solve over --reps timed solves after a warm one, whether
the persistent launch ran, and whether the output equals (bitwise) the shape's first knob set's."""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1x2400x256")
    ap.add_argument("--knobs", nargs="*", default=[""])
    ap.add_argument("--reps", type=int, default=5)
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
    defaults = {}
    for shape in a.shapes.split(","):
        B, T, nfe = (int(v) for v in shape.split("x"))
        g = torch.Generator().manual_seed(3)
        x0 = (torch.randn(B, T, 256, generator=g) * 0.3 + torch.randn(B, T, 256, generator=g)).to(dev)
        spk = torch.randn(B, 256, generator=g).to(dev)
        ts = torch.linspace(0, 1, nfe + 1, device=dev)
        first = None
        for kn in a.knobs:
            kv = [p.split("=") for p in kn.split(",") if p]
            for k, v in kv:
                nat.check(L.flamed_tune(k.encode(), int(v)), "tune")
            with torch.inference_mode():
                ref = hip.solve(x0, ts, spk, nfe)
                torch.cuda.synchronize()
                r0 = hip.persist_status()[0]
                times = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    hip.solve(x0, ts, spk, nfe)
                    torch.cuda.synchronize()
                    times.append((time.perf_counter() - t0) * 1e3)
                runs = hip.persist_status()[0] - r0
            if first is None:
                first = ref.clone()
            print(f"B={B} T={T} nfe={nfe} [{kn or 'defaults'}]: {statistics.median(times):.2f} ms/solve "
                  f"(min {min(times):.2f}), persistent launches {runs}/{a.reps}, finite {bool(torch.isfinite(ref).all())}, "
                  f"equal to the first knob set {bool(torch.equal(ref, first))}"
                  f"{chain_info(L, hip)}", flush=True)
            for k, _ in kv:  # back to the process defaults of the Tune struct
                nat.check(L.flamed_tune(k.encode(), defaults.setdefault(k, DEFAULTS.get(k, 0))), "tune")


def chain_info(L, hip):
    import ctypes
    if not hasattr(L, "flamed_den_chain_info"):
        return ""
    pk, rt = ctypes.c_int(), ctypes.c_int()
    L.flamed_den_chain_info(hip.handle, ctypes.byref(pk), ctypes.byref(rt))
    return f", chain streams parked {pk.value} (re-created {rt.value})"


DEFAULTS = {"persist": 1, "persist_ntw": 8, "persist_multi": 1, "persist_pad": 1, "split_batch": 2, "split_prio": 2, "dwgn": 1, "fuse_euler": 1,
            "persist_opt": 885322, "persist_multi_ntw": 8}

if __name__ == "__main__":
    main()
