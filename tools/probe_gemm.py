"""GEMM / graph-node latency probes on the GPU (flamed_probe_gemm / flamed_probe_empty).
Per-launch us inside a graph of back-to-back launches for tile/pipeline variants, with weights either
L2-hot (one buffer) or streamed (24 rotating 2 MB buffers, as the 21 GEMMs of a denoiser step)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flamed-tts_amd"))
from flamed import _native as nat  # noqa: E402

VARIANTS = {0: "32x64s3", 9: "32x32s3", 10: "32x64dma", 11: "32x32dma", 1: "64x64s3", 6: "32x64r4", 5: "128x64s3",
            3: "128x128s3", 12: "128x128dma3x", 13: "128x128dma2x", 16: "128x128dma3", 14: "256x128dma3x",
            15: "256x128dma2x", 18: "128x128k32dma4x", 19: "128x128k32dma3x", 21: "128x128k32dma2x", 20: "256x128k32dma4x",
            22: "wsk32x32w4", 23: "wsk32x32w8", 24: "wsk32x64w8", 25: "wsk64x32w8", 26: "wsk64x64w8",
            27: "wsk16x64w8", 28: "wsk32x32w16", 29: "wsk16x32w8",
            30: "64x64sk2", 31: "64x64sk4", 32: "128x64sk2", 33: "128x64sk4", 34: "32x64sk2", 35: "32x64sk4",
            36: "64x32dma", 37: "32x32dma4", 38: "32x32k32dma8", 39: "32x32k32dma16", 40: "32x32dma8x", 41: "64x32dma4",
            42: "32x32dma2", 43: "32x32dma8s", 44: "32x32dma4s", 45: "32x64dma4s", 46: "32x64dma4", 47: "32x32dma3", 50: "256x256x8p"}
WSK = (22, 23, 24, 25, 26, 27, 28, 29)
BIG = (3, 5, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 50)


VSEL = [int(x) for x in os.environ.get("PROBE_VARIANTS", "").split(",") if x]


def main():
    dev = torch.device("cuda:0")
    L = nat.diag_lib()
    st = nat.stream_ptr(dev)
    us = ctypes.c_float()
    nat.check(L.flamed_probe_empty(256, 64, ctypes.byref(us), st), "empty")
    print(f"empty kernel: {us.value:6.2f} us/launch")
    N = 1024
    for M in ([int(a) for a in sys.argv[1:]] or (131, 400, 1600, 25600)):
        for K in ((1024,) if M != 400 else (256, 1024)):
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
            nb = 24
            W = torch.randn(nb * N, K, device=dev).to(torch.bfloat16)
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ref = (A.float() @ W[:N].float().t())
            for wb in (1, nb):
                row = []
                for v, name in VARIANTS.items():
                    if (v in BIG and M < 1600) or (v not in BIG and M > 4000) or (v in WSK and K != 1024) or (VSEL and v not in VSEL):
                        continue
                    reps = 48 if M < 4000 else 24
                    rc = L.flamed_probe_gemm(v, M, N, K, reps, wb, nat.ptr(A), nat.ptr(W), nat.ptr(C), ctypes.byref(us), st)
                    if rc:
                        row.append(f"{name}=ERR({nat.diag_lib().flamed_last_error().decode()[:40]})")
                        continue
                    tf = 2 * M * N * K / (us.value * 1e-6) / 1e12
                    row.append(f"{name}={us.value:6.2f}({tf:4.0f}TF)")
                    if M <= 1600 or v in BIG:  # correctness of this variant (launch 0 reads buffer 0)
                        nat.check(L.flamed_probe_gemm(v, M, N, K, 1, 1, nat.ptr(A), nat.ptr(W), nat.ptr(C),
                                                      ctypes.byref(us), st), "chk")
                        torch.cuda.synchronize()
                        err = (C.float() - ref).abs().max().item() / ref.abs().max().item()
                        rel = ((C.float() - ref).norm() / ref.norm()).item()
                        if err >= 2e-2:
                            row.append(f"[{name} WRONG max {err:.2e} rel {rel:.2e}]")
                print(f"M={M:6d} K={K:5d} wbufs={wb:2d}: " + " ".join(row))


if __name__ == "__main__":
    main()
