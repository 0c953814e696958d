"""GPU: the MX-fp8 denoiser path (FLAMED_FP8 handles; BASELINE configs[4] "fp8 pointwise projections").

An fp8 handle runs conv_2 / conv_3 / mlp.0 / mlp.2 of every block as block-scaled MX-fp8 GEMMs (OCP e4m3
operands, one e8m0 scale per 32 input channels of weights AND activations, scale 2^ceil(log2(amax/448)))
on the large-M path; everything else is the bf16 path.  Two checks per case:

  * against the fp32 oracle, under a looser tolerance: velocity rel-L2 <= 8e-2
    (tests/fp8_sim.py "mxfp8c" on the same four GEMMs: 4.5e-2), solve rel-L2 <= 5e-2 (sim: 2.7e-2 at
    128 and 256 steps);
  * the MX-fp8 GEMM itself (producer quantization + weight packing + block-scaled 256x256 kernel, through
    flamed_probe_mx_gemm) against torch's e4m3 quantization of the same recipe followed by an fp64 matmul:
    rel-L2 <= 2e-4 (measured 4.7e-5: the scaled MFMA's internal summation, 1.7e-5 for one 128-K
    instruction in tools/probe_mx.py; the quantization itself is 3.8e-2), which pins layout, scales and
    rounding.  (A whole-network
    comparison against an emulated oracle cannot be tight: bf16-level input differences flip e4m3
    rounding decisions, ~6 % steps, and the flips compound through 20 GEMMs.)

Small cases force the fp8 path at 1,600 rows with the per-handle knob g8p_rows; the configs[4] case runs
at its real size (B = 16, T = 2400 = 38,400 rows) with the default knobs.
"""
import importlib
import os

import pytest
import torch

from _common import orc, rel_l2
from test_denoiser_gpu import _prob_gen

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
C = 256
FP8_VEL = 8e-2
FP8_SOLVE = 5e-2


def _sim():
    os.environ["FP8_SET"] = "big4"
    import fp8_sim
    return importlib.reload(fp8_sim)


@pytest.fixture(scope="module")
def pg8():
    from flamed import _native as nat
    pg, sd = _prob_gen("fp8")
    h = pg.denoiser.hip()
    h._ensure(torch.device(DEV))
    nat.check(nat.lib().flamed_den_tune(h.handle, b"g8p_rows", 1024), "flamed_den_tune")
    return pg, sd


def _inputs(seed, B, T):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, T, C, generator=g) * 0.3 + torch.randn(B, T, C, generator=g)
    t = torch.rand(B, 1, generator=g)
    c = torch.randn(B, C, generator=g)
    return x, t, c


@pytest.mark.parametrize("M", [512, 1000])
def test_mx_gemm_matches_recipe(M):
    from flamed import _native as nat
    sim = _sim()
    N, K = 1024, 1024
    g = torch.Generator().manual_seed(M)
    # rows of varied magnitude (the blocks' scales differ) and a few outliers per row
    A = torch.randn(M, K, generator=g) * torch.exp2(torch.randint(-6, 6, (M, 1), generator=g).float())
    A[:, ::97] *= 20
    W = torch.randn(N, K, generator=g) * 0.03
    ref = sim.mx_q(A.double(), 1, True) @ sim.mx_q(W.double(), 1, True).T
    Ad, Wd = A.to(DEV), W.to(DEV)
    Cd = torch.empty(M, N, device=DEV)
    nat.check(nat.diag_lib().flamed_probe_mx_gemm(nat.ptr(Ad), nat.ptr(Wd), M, N, K, nat.ptr(Cd), nat.stream_ptr(DEV)),
              "flamed_probe_mx_gemm")
    e = rel_l2(Cd.cpu().double(), ref)
    e_plain = rel_l2(Cd.cpu().double(), A.double() @ W.double().T)
    print(f"MX-fp8 GEMM M={M}: vs recipe {e:.3e}, vs unquantized {e_plain:.3e}")
    assert e < 2e-4, e
    assert e_plain > 1e-2  # it did quantize


def test_fp8_velocity_small(pg8):
    pg, sd = pg8
    x, t, c = _inputs(11, 2, 800)
    from flamed.models.synthesizer.prob_generator import DenoiserHIP
    with torch.inference_mode():
        v = pg.denoiser(x.to(DEV), t.to(DEV), c.to(DEV)).cpu()
        vb = DenoiserHIP(pg.denoiser, "bf16").velocity(x.to(DEV), t.to(DEV), c.to(DEV)).cpu()
    ref = orc.denoiser_forward(sd, x, t, c)
    e32, eb = rel_l2(v, ref), rel_l2(vb, ref)
    print(f"fp8 velocity B=2 T=800: vs fp32 {e32:.3e} (bf16 handle: {eb:.3e})")
    assert torch.isfinite(v).all()
    assert e32 < FP8_VEL, e32
    assert e32 > 3 * eb  # the fp8 GEMMs ran (an fp8 handle below g8p_rows computes exactly as bf16)


def test_fp8_solve_small(pg8):
    pg, sd = pg8
    x, _, c = _inputs(12, 2, 800)
    nfe = 32
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    with torch.inference_mode():
        xs = pg.denoiser.hip().solve(x.to(DEV), ts, c.to(DEV), nfe).cpu()
    e = rel_l2(xs, orc.euler_solve(sd, x, c, nfe))
    print(f"fp8 {nfe}-step solve B=2 T=800: vs fp32 oracle {e:.3e}")
    assert torch.isfinite(xs).all() and e < FP8_SOLVE, e


def test_fp8_configs4_long_form():
    """configs[4] at its size with default knobs: velocity vs the oracle, and the 256-step graph solve is
    finite and equal to the eager one bitwise."""
    pg, sd = _prob_gen("fp8")
    B, T = 16, 2400
    x, t, c = _inputs(13, B, T)
    with torch.inference_mode():
        v = pg.denoiser(x.to(DEV), t.to(DEV), c.to(DEV)).cpu()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref = orc.denoiser_forward(sd, x[:4], t[:4], c[:4])  # utterances are independent: a 4-utterance check
    e32 = rel_l2(v[:4], ref)
    print(f"fp8 velocity B=16 T=2400: vs fp32 (first 4 utterances) {e32:.3e}")
    assert e32 < FP8_VEL, e32
    nfe = 256
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    hip = pg.denoiser.hip()
    outs = []
    for graph in (True, False):
        pg.denoiser.hip_graph = graph
        with torch.inference_mode():
            outs.append(hip.solve(x.to(DEV), ts, c.to(DEV), nfe))
    pg.denoiser.hip_graph = True
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])


def test_fp8_configs4_solve_vs_oracle():
    """configs[4] as benchmarked: the 256-step B = 16, T = 2400 MX-fp8 graph solve (38,400 rows, fp8 GEMMs
    active), utterance 0 against a single-utterance fp32 oracle solve (equal lengths: no padding coupling,
    so a one-utterance reference is exact; reference prob_generator.py:439-447).  rel-L2 <= 5e-2."""
    pg, sd = _prob_gen("fp8")
    B, T, nfe = 16, 2400, 256
    x, _, c = _inputs(17, B, T)
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    with torch.inference_mode():
        sol = pg.denoiser.hip().solve(x.to(DEV), ts, c.to(DEV), nfe).cpu()
    assert torch.isfinite(sol).all()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref = orc.euler_solve(sd, x[:1], c[:1], nfe)
    e = rel_l2(sol[:1], ref)
    print(f"fp8 configs[4] 256-step solve, utterance 0 vs fp32 oracle: rel-L2 {e:.3e}")
    assert e < FP8_SOLVE, e
