"""Which K elements one lane's MX scale covers in v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3): run the probe
in both candidate lane layouts with random e4m3 data and random per-(row, block) scales and compare with
an fp64 reference in which scale block b = K [32 b, 32 b + 32) of the row in memory order.
Measured (gpurun_out/mx, tools/mx_dbg.py): lane group g holds instruction K [16 g, 16 g + 16) in VGPRs 0-3
and [64 + 16 g, ...) in VGPRs 4-7, and the scale of instruction K block b is the one lane group b passes.
So with mode 1 (chunks g and 4 + g: instruction K == memory K) block b is the contiguous memory bytes
[32 b, 32 b + 32), whose scale lane group b supplies — the layout gemm_8p.hpp's fp8 path uses; mode 0
fails.  GPU only (libflamed_diag.so)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flamed-tts_amd"))
from flamed import _native as nat  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    a = (torch.randn(16, 128, generator=g) * 4).to(torch.float8_e4m3fn)
    b = (torch.randn(16, 128, generator=g) * 4).to(torch.float8_e4m3fn)
    sa = torch.randint(120, 134, (16, 4), generator=g, dtype=torch.uint8)
    sb = torch.randint(120, 134, (16, 4), generator=g, dtype=torch.uint8)
    L = nat.diag_lib()
    ok = {}
    for mode in (0, 1):
        grp = torch.arange(128) // 32  # scale block of each memory K index
        fa = a.double() * torch.exp2(sa.double() - 127)[:, grp]
        fb = b.double() * torch.exp2(sb.double() - 127)[:, grp]
        ref = fa @ fb.T
        C = torch.zeros(16, 16, device=dev)
        ad, bd = a.view(torch.uint8).to(dev), b.view(torch.uint8).to(dev)
        sad, sbd = sa.to(dev), sb.to(dev)
        nat.check(L.flamed_probe_mx(nat.ptr(ad), nat.ptr(bd), nat.ptr(sad), nat.ptr(sbd), nat.ptr(C), mode,
                                    nat.stream_ptr(dev)), "flamed_probe_mx")
        torch.cuda.synchronize()
        err = float((C.double().cpu() - ref).norm() / ref.norm())
        ok[mode] = err < 1e-4  # the MFMA sums at fp32 accumulation accuracy (1.7e-5 measured)
        print(f"mode {mode}: rel err {err:.3e} {'PASS' if ok[mode] else 'FAIL'}")
    # the same data with unit scales: layout-independent sanity check of the e4m3 decode
    C = torch.zeros(16, 16, device=dev)
    one = torch.full((16, 4), 127, dtype=torch.uint8, device=dev)
    ad, bd = a.view(torch.uint8).to(dev), b.view(torch.uint8).to(dev)  # kept alive across the launch
    nat.check(L.flamed_probe_mx(nat.ptr(ad), nat.ptr(bd), nat.ptr(one), nat.ptr(one), nat.ptr(C), 0, nat.stream_ptr(dev)),
              "flamed_probe_mx")
    torch.cuda.synchronize()
    ref = a.double() @ b.double().T
    print(f"unit scales: rel err {float((C.double().cpu() - ref).norm() / ref.norm()):.3e}")


if __name__ == "__main__":
    main()
