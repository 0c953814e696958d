"""Diagnostic, third pass: is the concurrent perturbation of the large-M depthwise conv + GroupNorm kernel (dwgn)
about its packed-fp32 math or its LDS traffic, and which foreign work triggers it?  A runs adaln + proj_in + dwgn
(stop_after 2) with dwgn_var 0 (as shipped), 1 (scalar fp32 math) or 2 (scalar LDS accesses) while stream B runs
handle B's AdaLN GEMMs, a torch fp32 matmul (fp32 MFMA), a torch bf16 matmul, or torch fp32 elementwise work."""
import copy
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402

NAMES = ["X", "S0", "S1", "D", "U", "GP", "GNS", "Y", "SL", "A16", "XA", "XP"]


def main():
    from flamed import _native as nat
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    L = nat.lib()
    dev = torch.device("cuda:0")
    torch.backends.cuda.matmul.allow_tf32 = False
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg2 = copy.deepcopy(pg)
    pg, pg2 = pg.to(dev), pg2.to(dev)
    B, T, H = 32, 400, 1024
    M = B * T
    g = torch.Generator().manual_seed(2)
    xs = [(torch.randn(B, T, 256, generator=g)).to(dev) for _ in range(2)]
    spk = [torch.randn(B, 256, generator=g).to(dev) for _ in range(2)]
    t = torch.full((B, 1), 0.3, device=dev)
    hA, hB = pg.denoiser.hip(), pg2.denoiser.hip()
    f32a = torch.randn(4096, 4096, device=dev)
    bfa = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    ew = torch.randn(64 << 20, device=dev)

    def dtune(h, k, v):
        nat.check(L.flamed_den_tune(h.handle, k.encode(), v), "den_tune")

    with torch.inference_mode():
        hA.velocity(xs[0], t, spk[0])
        hB.velocity(xs[1], t, spk[1])
        torch.cuda.synchronize()
        offs = (ctypes.c_size_t * 12)()
        nat.check(L.flamed_den_ws_offsets(hA.handle, B, T, offs), "ws_offsets")
        o = offs[NAMES.index("A16")]
        r = torch.arange(B, device=dev, dtype=torch.int32)
        tv = torch.full((B,), 0.3, device=dev)

        def a16():
            return hA.ws.buf[o: o + 2 * M * H].clone()

        modes = [("adaln", lambda: [hB.adaln(tv, spk[1], r, r) for _ in range(40)]),
                 ("mm_f32", lambda: [torch.mm(f32a, f32a) for _ in range(4)]),
                 ("mm_bf16", lambda: [torch.mm(bfa, bfa) for _ in range(3)]),
                 ("ew_f32", lambda: [ew.mul_(1.0001).add_(1e-6) for _ in range(20)]),
                 ("velB", lambda: [hB.velocity(xs[1], t, spk[1]) for _ in range(2)])]
        dtune(hA, "stop_after", 2)
        ref0 = var0 = None
        for var in [int(v) for v in os.environ.get("VARS", "0,1,2").split(",")]:
            dtune(hA, "dwgn_var", var)
            hA.velocity(xs[0], t, spk[0])
            torch.cuda.synchronize()
            ref = a16()
            if ref0 is None:
                ref0, var0 = ref, var
            print(f"var {var}: solo vs var {var0} bitwise equal: {bool(torch.equal(ref, ref0))}", flush=True)
            for name, fn in modes:
                nbad, tot = 0, 0
                for rep in range(8):
                    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
                    torch.cuda.synchronize()
                    hA.ws.buf[o: o + 2 * M * H].fill_(0x5A)
                    torch.cuda.synchronize()
                    with torch.cuda.stream(sB):
                        fn()
                    with torch.cuda.stream(sA):
                        torch.cuda._sleep(15000 * rep)
                        hA.velocity(xs[0], t, spk[0])
                    torch.cuda.synchronize()
                    d = int((a16() != ref).sum())
                    nbad += d > 0
                    tot += d
                print(f"var {var} B={name}: {nbad}/8 runs differ ({tot} bytes)", flush=True)


if __name__ == "__main__":
    main()
