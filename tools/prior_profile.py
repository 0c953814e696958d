#!/usr/bin/env python3
"""Time the HIP prior transformer (flamed_prior_encode / flamed_prior_decode) at the bench shape, for
rocprofv3 kernel stats:  rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/prior_profile.py"""
import os
import sys
import time

import torch
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flamed-tts_amd"))

from flamed.models.synthesizer.prior_generator import PriorGenerator  # noqa: E402
from flamed.utils.seeded_init import randomize_module  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cfg = yaml.safe_load(open(os.path.join(REPO, "flamed-tts_amd", "configs", "prior.yaml")))
    pg = PriorGenerator(cfg).eval()
    randomize_module(pg, 3)
    pg = pg.to(dev)
    g = torch.Generator().manual_seed(0)
    L, T, P = 247, 400, 240
    ids = torch.randint(1, 300, (1, L), generator=g).to(dev)
    smask = torch.zeros(1, L, dtype=torch.bool, device=dev)
    x = torch.randn(1, T, 192, generator=g).to(dev)
    tmask = torch.zeros(1, T, dtype=torch.bool, device=dev)
    codes = torch.randint(0, 1024, (1, 6, P), generator=g).to(dev)
    h = pg.hip()
    dts = sys.argv[1:] or ["bf16"]  # decoder-side GEMM operand types to time (bf16, f32)
    with torch.inference_mode():
        for dt in dts:
            pg.hip_dec_dtype = dt
            for graph in (False, True):
                pg.hip_graph = graph
                for _ in range(3):
                    h.encode(ids, smask)
                    h.decode(x, tmask, codes, P)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    h.encode(ids, smask)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(10):
                    h.decode(x, tmask, codes, P)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                print(f"decoders {dt} graph={graph} encode {(t1 - t0) * 100:.3f} ms decode {(t2 - t1) * 100:.3f} ms",
                      flush=True)


if __name__ == "__main__":
    main()
