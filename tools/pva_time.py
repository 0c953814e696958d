"""Time PVA.sample (duration + silence flows and the length regulator) at given phoneme counts under knob sets:
    python tools/pva_time.py --L 60,285 --knobs pva_stage=1 pva_stage=0
prints one line per (L, knob set): ms per sample (10 timed after 3 warm) and whether the persistent flow ran."""
import argparse
import os
import sys
import time

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", default="60,285")
    ap.add_argument("--knobs", nargs="*", default=[""])
    ap.add_argument("--nfe", type=int, default=64)
    a = ap.parse_args()
    from flamed import _native as nat
    from flamed.models.synthesizer.pva import PVA
    from flamed.utils.seeded_init import randomize_module
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prior.yaml")))
    dev = torch.device("cuda:0")
    pva = PVA(cfg["variance_adaptor"]).eval()
    randomize_module(pva, 20251205)
    pva = pva.to(dev)
    L_ = nat.lib()
    for L in (int(v) for v in a.L.split(",")):
        g = torch.Generator().manual_seed(L)
        enc = torch.randn(1, L, 192, generator=g).to(dev)
        sl = torch.tensor([L], device=dev)
        mask = torch.zeros(1, L, dtype=torch.bool, device=dev)
        for kn in a.knobs:
            kv = [p.split("=") for p in kn.split(",") if p]
            old = {}
            for k, v in kv:
                nat.check(L_.flamed_tune(k.encode(), int(v)), "tune")
            with torch.inference_mode():
                for _ in range(3):
                    pva.sample(enc, sl, mask, nfe=a.nfe, temperature=0.3)
                torch.cuda.synchronize()
                r0 = pva.hip().persist_info()[0] if hasattr(pva, "hip") else -1
                t0 = time.perf_counter()
                for _ in range(10):
                    pva.sample(enc, sl, mask, nfe=a.nfe, temperature=0.3)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 100
                r1 = pva.hip().persist_info()[0] if hasattr(pva, "hip") else -1
            print(f"L={L} nfe={a.nfe} [{kn or 'defaults'}]: {ms:.3f} ms per sample, persistent flows {r1 - r0}/10", flush=True)
            for k, _ in kv:
                nat.check(L_.flamed_tune(k.encode(), old.get(k, DEFAULTS.get(k, 0))), "tune")


DEFAULTS = {"pva_stage": 1, "pva_persist": 1, "pva_split": 0}

if __name__ == "__main__":
    main()
