"""Does warming the next GEMM's weights into L2 (concurrent graph branch) shorten a B=1-shaped GEMM chain?
flamed_probe_gemm_pf at M = 131 / 400, N = K = 1024, 24 rotating weight buffers (the step's weights stream
from MALL), for the default small-M DMA tile and a few warm-up grid sizes."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flamed-tts_amd"))
from flamed import _native as nat  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = nat.diag_lib()
    st = nat.stream_ptr(dev)
    us = ctypes.c_float()
    N = K = 1024
    for M in (131, 400):
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = torch.randn(24 * N, K, device=dev).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for v, name in ((11, "32x32dma"), (10, "32x64dma")):
            row = []
            for pf in (0, 64, 128, 256):
                for wb in (24, 1):
                    nat.check(L.flamed_probe_gemm_pf(v, M, N, K, 48, wb, pf, nat.ptr(A), nat.ptr(W), nat.ptr(C),
                                                     ctypes.byref(us), st), "probe_pf")
                    row.append(f"pf{pf}/wb{wb}={us.value:5.2f}")
            print(f"M={M:4d} {name}: " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
