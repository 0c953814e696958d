"""Diagnostic: does a concurrent evaluation on another stream change what the large-M depthwise conv +
GroupNorm kernel (dwgn) of handle A writes?  A runs proj_in + dwgn only (knob stop_after 2) and its
workspace buffers X, S0 (dwgn's inputs) and A16 (dwgn's output) are compared with a solo run, byte for byte,
while stream B runs: another handle's full velocity (dwgn 0 or 1), or a torch matmul loop (control).  The
pattern of the differing A16 elements (utterances, 32-channel groups, rows) is printed."""
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
    B, T, H = int(os.environ.get("CB", 32)), 400, 1024
    M = B * T
    g = torch.Generator().manual_seed(2)
    xs = [(torch.randn(B, T, 256, generator=g)).to(dev) for _ in range(2)]
    spk = [torch.randn(B, 256, generator=g).to(dev) for _ in range(2)]
    t = torch.full((B, 1), 0.3, device=dev)
    hA, hB = pg.denoiser.hip(), pg2.denoiser.hip()
    big = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    stop = int(os.environ.get("STOP", 2))

    def dtune(h, k, v):
        nat.check(L.flamed_den_tune(h.handle, k.encode(), v), "den_tune")

    with torch.inference_mode():
        hA.velocity(xs[0], t, spk[0])
        hB.velocity(xs[1], t, spk[1])
        torch.cuda.synchronize()
        offs = (ctypes.c_size_t * 12)()
        nat.check(L.flamed_den_ws_offsets(hA.handle, B, T, offs), "ws_offsets")
        size = {"X": 4 * M * H, "S0": 8 * M * 8, "A16": 2 * M * H, "U": 2 * M * H}

        def snap():
            ws = hA.ws.buf
            return {n: ws[offs[NAMES.index(n)]: offs[NAMES.index(n)] + size[n]].clone() for n in size}

        dtune(hA, "stop_after", stop)
        hA.velocity(xs[0], t, spk[0])
        torch.cuda.synchronize()
        ref = snap()
        for r in range(3):
            hA.ws.buf.fill_(0x5A)
            hA.velocity(xs[0], t, spk[0])
            torch.cuda.synchronize()
            s = snap()
            print("solo", r, {n: int((s[n] != ref[n]).sum()) for n in s}, flush=True)

        def pattern(a, b):
            av = a.view(torch.bfloat16).view(B, T, H).float()
            bv = b.view(torch.bfloat16).view(B, T, H).float()
            d = (av != bv)
            if not bool(d.any()):
                return "A16 equal"
            idx = d.nonzero()
            utt = sorted(set(idx[:, 0].tolist()))
            grp = sorted(set((idx[:, 2] // 32).tolist()))
            pairs = sorted(set(zip(idx[:, 0].tolist(), (idx[:, 2] // 32).tolist())))
            per = [(u, gg, int(d[u, :, gg * 32:(gg + 1) * 32].any(dim=1).sum()), int(d[u, :, gg * 32:(gg + 1) * 32].sum()))
                   for u, gg in pairs[:8]]
            mx = float((av - bv).abs().max())
            return (f"A16 differs: {int(d.sum())} elems, max|d| {mx:.3e}, utts {utt[:10]}{'...' if len(utt) > 10 else ''}, "
                    f"groups {grp[:12]}, (utt,grp) pairs {len(pairs)}; first pairs (utt, grp, rows hit, elems): {per}")

        for mode in ("velB_dw0", "velB_dw1", "velB_dw0_dup", "matmul"):
            nbad = 0
            for rep in range(8):
                sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
                torch.cuda.synchronize()
                hA.ws.buf.fill_(0x5A)
                torch.cuda.synchronize()
                with torch.cuda.stream(sB):
                    if mode == "matmul":
                        for _ in range(8):
                            big = (big @ big).clamp_(-1, 1)
                    else:
                        dtune(hB, "dwgn", 1 if mode == "velB_dw1" else 0)
                        for _ in range(2 if mode.endswith("dup") else 1):
                            hB.velocity(xs[1], t, spk[1])
                with torch.cuda.stream(sA):
                    torch.cuda._sleep(20000 * rep)
                    hA.velocity(xs[0], t, spk[0])
                torch.cuda.synchronize()
                s = snap()
                nd = {n: int((s[n] != ref[n]).sum()) for n in s}
                bad = any(nd.values())
                nbad += bad
                print(f"{mode} rep {rep}: byte diffs {nd}", flush=True)
                if nd["A16"]:
                    print("   ", pattern(s["A16"], ref["A16"]), flush=True)
            print(f"{mode}: {nbad}/8 differ", flush=True)


if __name__ == "__main__":
    main()
