"""Structured cases for the MX MFMA probe (diagnostic; see tools/probe_mx.py)."""
import os, sys, torch
sys.path.insert(0, "flamed-tts_amd")
from flamed import _native as nat
dev = torch.device("cuda:0")
L = nat.diag_lib()
def run(a, b, sa, sb, mode=0):
    C = torch.zeros(16, 16, device=dev)
    keep = [a.to(torch.float8_e4m3fn).view(torch.uint8).to(dev), b.to(torch.float8_e4m3fn).view(torch.uint8).to(dev),
            sa.to(dev), sb.to(dev)]
    nat.check(L.flamed_probe_mx(*[nat.ptr(t) for t in keep], nat.ptr(C), mode, nat.stream_ptr(dev)), "mx")
    torch.cuda.synchronize()
    return C.cpu()
one = torch.full((16, 4), 127, dtype=torch.uint8)
ones = torch.ones(16, 128)
g = torch.Generator().manual_seed(0)
ra = (torch.randn(16, 128, generator=g) * 4).to(torch.float8_e4m3fn).float()
rb = (torch.randn(16, 128, generator=g) * 4).to(torch.float8_e4m3fn).float()
ref = ra.double() @ rb.double().T
for mode in (0, 1):
    C = run(ra, rb, one, one, mode)
    print("random unit-scale mode", mode, float((C.double() - ref).norm() / ref.norm()))
for mode in (0, 1):
    for blk in range(4):
        s = one.clone(); s[:, blk] = 128
        print("mode", mode, "sa blk", blk, "x2 ->", run(ones, ones, s, one, mode)[0, 0].item(), "(128 + 32 expected)")
s = one.clone(); s[2, :] = 128
print("sa row2 x2", run(ones, ones, s, one)[:4, 0].tolist())
s = one.clone(); s[5, :] = 129
print("sb row5 x4", run(ones, ones, one, s)[0, :8].tolist())
for k in (0, 16, 32, 48, 64, 80, 96, 112):
    a = torch.zeros(16, 128); a[:, k] = 1
    res = []
    for blk in range(4):
        s = one.clone(); s[:, blk] = 128
        res.append(run(a, ones, s, one, 0)[0, 0].item())
    print("A elem k", k, "mode0 result with block-x2 per blk", res)
