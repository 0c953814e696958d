"""Diagnostic: which part of the library leaves the process crashing at exit under rocprofv3?
mode vel: one bf16 velocity; graph: a B=1 solve on the graph of launches (persist 0); persist: a B=1
persistent solve; pva: the persistent PVA flow."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402


def main(mode):
    from flamed import _native as nat
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    dev = torch.device("cuda:0")
    if mode == "pva":
        from flamed.models.synthesizer.pva import PVA
        cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prior.yaml")))
        pva = PVA(cfg["variance_adaptor"]).eval()
        randomize_module(pva, 1)
        pva = pva.to(dev)
        enc = torch.randn(1, 60, 192).to(dev)
        with torch.inference_mode():
            pva.sample(enc, torch.tensor([60], device=dev), torch.zeros(1, 60, dtype=torch.bool, device=dev), nfe=8,
                       temperature=0.3)
    else:
        cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
        pg = ProbGenerator(cfg).eval()
        randomize_module(pg, 7)
        pg = pg.to(dev)
        x = torch.randn(1, 48, 256, device=dev)
        c = torch.randn(1, 256, device=dev)
        with torch.inference_mode():
            pg.denoiser.hip_dtype = "bf16"
            if mode == "vel":
                pg.denoiser(x, torch.tensor([[0.3]], device=dev), c)
            else:
                nat.check(nat.lib().flamed_tune(b"persist", 1 if mode == "persist" else 0), "tune")
                pg.denoiser.hip().solve(x, torch.linspace(0, 1, 9, device=dev), c, 8)
    torch.cuda.synchronize()
    print(f"exit_probe {mode} done", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
