"""Per-CU ingest probe (flamed_probe_stream): us per launch and GB/s per block / aggregate, for blocks x KB
slices read from a buffer larger than L2 (MALL/HBM-resident), by LDS-DMA ring vs register loads."""
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
    for blocks, kb in ((208, 192), (256, 192), (208, 64), (208, 768), (1024, 192), (256, 1024)):
        src = torch.empty(blocks * kb * 1024, dtype=torch.uint8, device=dev).random_(0, 255)
        row = []
        for mode in (1, 0):
            nat.check(L.flamed_probe_stream(blocks, kb, mode, 32, nat.ptr(src), ctypes.byref(us), st), "stream")
            per = kb * 1024 / (us.value * 1e-6) / 1e9
            row.append(f"{'dma' if mode else 'reg'}={us.value:7.2f}us ({per:6.1f} GB/s/blk, {per * blocks / 1e3:5.2f} TB/s)")
        print(f"blocks={blocks:5d} KB/blk={kb:5d}: " + "  ".join(row))


if __name__ == "__main__":
    main()
