"""Diagnostic: do two HIP streams still run kernels concurrently when they were created after a cooperative
launch in this process?  Measured on MI355X (round 5): a B = 64 split solve (two graph branches) is 6 % slower
when its capture streams were created after the first persistent (cooperative) solve.  This probe times two
`torch.cuda._sleep` kernels on a stream pair (concurrent: ~1x, serialised: ~2x one sleep) for pairs created
before and after a cooperative launch (the persistent B = 1 solve), and after a plain launch of it (coop 0)."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))
import torch  # noqa: E402
import yaml  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def new_stream(nonblocking=True, priority=None):
    s = ctypes.c_void_p()
    if priority is None:
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1 if nonblocking else 0)) == 0
    else:
        assert hip.hipStreamCreateWithPriority(ctypes.byref(s), ctypes.c_uint(1), ctypes.c_int(priority)) == 0
    return s.value


def pair_time(sa, sb, cycles=20_000_000):
    A, B = torch.cuda.ExternalStream(sa), torch.cuda.ExternalStream(sb)
    torch.cuda.synchronize()
    with torch.cuda.stream(A):
        torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(A):
        torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    one = time.perf_counter() - t0
    t0 = time.perf_counter()
    with torch.cuda.stream(A):
        torch.cuda._sleep(cycles)
    with torch.cuda.stream(B):
        torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    two = time.perf_counter() - t0
    return two / one


def mm_time(sx, a, n=20):
    S = torch.cuda.ExternalStream(sx)
    torch.cuda.synchronize()
    with torch.cuda.stream(S):
        for _ in range(3):
            a @ a
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(S):
        for _ in range(n):
            a @ a
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    coop = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    from flamed import _native as nat
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    from flamed.utils.seeded_init import randomize_module
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    before = [new_stream() for _ in range(4)]
    print(f"pairs created before any persistent launch: {pair_time(before[0], before[1]):.2f} "
          f"{pair_time(before[2], before[3]):.2f}  (1.0 = concurrent, 2.0 = serialised)", flush=True)
    a0 = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    print("bf16 8192^3 matmul ms before the persistent launch, on: " + " ".join(f"{mm_time(x, a0):.3f}" for x in before))
    nat.check(nat.lib().flamed_tune(b"coop", coop), "tune")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    randomize_module(pg, 20251205)
    pg = pg.to(dev)
    h = pg.denoiser.hip()
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(1, 400, 256, generator=g).to(dev)
    spk = torch.randn(1, 256, generator=g).to(dev)
    with torch.inference_mode():
        h.solve(x0, torch.linspace(0, 1, 9, device=dev), spk, 8)
    torch.cuda.synchronize()
    print(f"persistent solve ran ({'cooperative' if coop else 'plain'} launch), runs {h.persist_status()[0]}", flush=True)
    after = [new_stream() for _ in range(4)]
    print(f"pairs created before, timed after:  {pair_time(before[0], before[1]):.2f} {pair_time(before[2], before[3]):.2f}")
    print(f"pairs created after:                {pair_time(after[0], after[1]):.2f} {pair_time(after[2], after[3]):.2f}")
    print(f"mixed (before[0], after[k]):        " + " ".join(f"{pair_time(before[0], a):.2f}" for a in after))
    ts = torch.cuda.Stream(), torch.cuda.Stream()
    print(f"torch pool streams after:           {pair_time(ts[0].cuda_stream, ts[1].cuda_stream):.2f}")
    lo, hi = ctypes.c_int(), ctypes.c_int()
    hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
    hp = [new_stream(priority=hi.value) for _ in range(3)]
    null = torch.cuda.default_stream().cuda_stream
    print(f"priority range {lo.value}..{hi.value}; null stream with before / after / high-priority streams:")
    print("  before: " + " ".join(f"{pair_time(null, b):.2f}" for b in before))
    print("  after:  " + " ".join(f"{pair_time(null, a):.2f}" for a in after))
    print("  high:   " + " ".join(f"{pair_time(null, x):.2f}" for x in hp))
    print("  high x after: " + " ".join(f"{pair_time(x, a):.2f}" for x in hp for a in after))
    lp = [new_stream(priority=lo.value) for _ in range(3)]
    print("  high x high:  " + " ".join(f"{pair_time(hp[i], hp[j]):.2f}" for i in range(3) for j in range(i + 1, 3)))
    print("  low x low:    " + " ".join(f"{pair_time(lp[i], lp[j]):.2f}" for i in range(3) for j in range(i + 1, 3)))
    print("  low x high:   " + " ".join(f"{pair_time(a, b):.2f}" for a in lp for b in hp))
    print("  null x low:   " + " ".join(f"{pair_time(null, a):.2f}" for a in lp))
    print("bf16 8192^3 matmul ms after the persistent launch, alone on: null %.3f" % mm_time(null, a0))
    print("  before: " + " ".join(f"{mm_time(x, a0):.3f}" for x in before))
    print("  after:  " + " ".join(f"{mm_time(x, a0):.3f}" for x in after))
    print("  high:   " + " ".join(f"{mm_time(x, a0):.3f}" for x in hp))
    print("  low:    " + " ".join(f"{mm_time(x, a0):.3f}" for x in lp))
    # two matmuls at once on a stream pair: ~1x one matmul's time = no overlap gain possible (each fills the GPU);
    # what matters for the split chains is whether either pair slows down
    for name, (x, y) in {"after pair": (after[0], after[1]), "high pair": (hp[0], hp[1])}.items():
        X, Y = torch.cuda.ExternalStream(x), torch.cuda.ExternalStream(y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            with torch.cuda.stream(X):
                a0 @ a0
            with torch.cuda.stream(Y):
                a0 @ a0
        torch.cuda.synchronize()
        print(f"  {name}: 20 matmuls {((time.perf_counter() - t0) * 1e3):.2f} ms")


if __name__ == "__main__":
    main()
