import os, sys, time, torch, yaml
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
from flamed.models.synthesizer.pva import PVA
from flamed.utils.seeded_init import randomize_module
from flamed import _native as nat
cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prior.yaml")))
dev = torch.device("cuda:0")
pva = PVA(cfg["variance_adaptor"]).eval(); randomize_module(pva, 20251205); pva = pva.to(dev)
for L in (60, 247):
    enc = torch.randn(1, L, 192).to(dev); sl = torch.tensor([L], device=dev); mask = torch.zeros(1, L, dtype=torch.bool, device=dev)
    for sp in (1, 0):
        nat.check(nat.lib().flamed_tune(b"pva_split", sp), "t")
        with torch.inference_mode():
            for _ in range(3): pva.sample(enc, sl, mask, nfe=64, temperature=0.3)
            torch.cuda.synchronize(); t0 = time.perf_counter()
            for _ in range(10): pva.sample(enc, sl, mask, nfe=64, temperature=0.3)
            torch.cuda.synchronize()
        print(f"L={L} pva_split={sp} {(time.perf_counter()-t0)*100:.3f} ms", flush=True)
