"""Diagnostic, second pass: WHICH concurrent kernel of another handle perturbs handle A's large-M depthwise conv +
GroupNorm kernel (dwgn), and HOW (per channel: an affine error over all frames = the GroupNorm statistics; local
rows = the staged window).  A runs adaln + proj_in + dwgn (stop_after 2) on stream A while stream B runs one of:
adaln only, velocity prefixes (stop_after k), the full velocity; A's dwgn output (A16) is compared with a solo run."""
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

    def dtune(h, k, v):
        nat.check(L.flamed_den_tune(h.handle, k.encode(), v), "den_tune")

    with torch.inference_mode():
        hA.velocity(xs[0], t, spk[0])
        hB.velocity(xs[1], t, spk[1])
        torch.cuda.synchronize()
        offs = (ctypes.c_size_t * 12)()
        nat.check(L.flamed_den_ws_offsets(hA.handle, B, T, offs), "ws_offsets")
        o = offs[NAMES.index("A16")]

        def a16():
            return hA.ws.buf[o: o + 2 * M * H].clone().view(torch.bfloat16).view(B, T, H).float()

        dtune(hA, "stop_after", 2)
        hA.velocity(xs[0], t, spk[0])
        torch.cuda.synchronize()
        ref = a16()
        r = torch.arange(B, device=dev, dtype=torch.int32)
        tv = torch.full((B,), 0.3, device=dev)

        def analyse(got):
            d = (got != ref)
            if not bool(d.any()):
                return "equal"
            idx = d.nonzero()
            pairs = sorted(set(zip(idx[:, 0].tolist(), (idx[:, 2] // 32).tolist())))
            out = [f"{int(d.sum())} elems in {len(pairs)} (utt, 32-ch group) blocks"]
            for u, gg in pairs[:3]:
                chans = sorted(set(idx[(idx[:, 0] == u) & (idx[:, 2] // 32 == gg)][:, 2].tolist()))
                desc = []
                for c in chans[:6]:
                    y, x = got[u, :, c].double(), ref[u, :, c].double()
                    A = torch.stack([x, torch.ones_like(x)], 1)
                    sol = torch.linalg.lstsq(A, y.unsqueeze(1)).solution.squeeze(1)
                    res = float((A @ sol - y).abs().max())
                    ch = [float((y - x)[k:k + 64].abs().max()) for k in range(0, T, 64)]
                    desc.append(f"c{c}: affine a={sol[0]:.4f} b={sol[1]:+.4f} resid {res:.2e}; per-64-row max|d| "
                                + " ".join(f"{v:.2f}" for v in ch))
                out.append(f"  utt {u} grp {gg}: {len(chans)} channels {chans[:12]}\n    " + "\n    ".join(desc))
            return "\n".join(out)

        modes = [("adaln", lambda: [hB.adaln(tv, spk[1], r, r) for _ in range(40)]),
                 ("stop1", lambda: run_b(1, 12)), ("stop2", lambda: run_b(2, 8)), ("stop3", lambda: run_b(3, 6)),
                 ("stop5", lambda: run_b(5, 4)), ("stop7", lambda: run_b(7, 3)), ("full", lambda: run_b(-1, 2))]

        def run_b(k, n):
            dtune(hB, "stop_after", k)
            for _ in range(n):
                hB.velocity(xs[1], t, spk[1])

        for name, fn in modes:
            nbad = 0
            for rep in range(6):
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
                res = analyse(a16())
                nbad += res != "equal"
                print(f"{name} rep {rep}: {res}", flush=True)
            print(f"== {name}: {nbad}/6 differ", flush=True)


if __name__ == "__main__":
    main()
