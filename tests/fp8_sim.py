"""CPU estimate of what fp8 pointwise projections cost in accuracy (BASELINE configs[4]):
the oracle denoiser with every pointwise GEMM (proj_in, conv_2, conv_3, mlp.0, mlp.2, conv_out) computed
on quantized operands, against fp32.  Recipes:
  * bf16     — both operands rounded to bf16 (what the HIP path runs);
  * mxfp8    — OCP MX: e4m3 elements with one power-of-two (e8m0) scale per 32-element block along K, for
               BOTH the weights and the activations (the v_mfma_scale_f32_16x16x128_f8f6f4 recipe):
               scale = 2^(floor(log2(amax_block)) - 8), elements saturated to +-448;
  * fp8-chan — e4m3 weights per output channel (amax/448), activations at unit scale (round-1 strawman).
Reported: velocity rel-L2 at t in {0.1, 0.5, 0.9} and the rel-L2 of an nfe-step Euler solve (nfe = 128, and
256 as configs[4]) vs the fp32 oracle.
Usage: PYTHONPATH=flamed-tts_amd:. python tests/fp8_sim.py [T]   (CPU only; under tests/ because it runs the
oracle, which only test code may import)."""
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _common import seeded, orc  # noqa: E402  (checker only)

# FP8_SET=big4: only the four 1024x1024 GEMMs per block (conv_2, conv_3, mlp.0, mlp.2), what the HIP fp8
# path quantizes; proj_in (K = 256) and conv_out stay bf16
BIG4 = os.environ.get("FP8_SET", "") == "big4"
NAMES = ["conv_2", "conv_3", "mlp.0", "mlp.2"] if BIG4 else ["proj_in", "conv_2", "conv_3", "mlp.0", "mlp.2", "conv_out"]
E4M3 = torch.float8_e4m3fn


def mx_q(x: torch.Tensor, dim: int, ceil: bool = False) -> torch.Tensor:
    """MX-fp8 fake-quantisation of x along `dim` (blocks of 32; the dim must be a multiple of 32).
    floor (OCP MX spec): 2^(floor(log2 amax) - 8), the block maximum lands in [256, 512) and saturates at 448;
    ceil (what the HIP kernels use): 2^ceil(log2(amax / 448)), no element saturates."""
    xt = x.movedim(dim, -1)
    shp = xt.shape
    b = xt.reshape(*shp[:-1], shp[-1] // 32, 32)
    amax = b.abs().amax(-1, keepdim=True)
    if ceil:
        e = torch.ceil(torch.log2(amax.clamp_min(2.0 ** -126) / 448.0))
    else:
        e = torch.floor(torch.log2(amax.clamp_min(2.0 ** -126))) - 8
    s = torch.exp2(e)
    q = (b / s).clamp(-448, 448).to(E4M3).float() * s
    q = torch.where(amax > 0, q, torch.zeros_like(q))
    return q.reshape(shp).movedim(-1, dim)


def quant_w(w, recipe):
    if recipe == "bf16":
        return w.to(torch.bfloat16).float()
    if recipe.startswith("mxfp8"):
        return mx_q(w, 1, recipe.endswith("c"))  # (N, K[, taps]): blocks along the input-channel dim
    s = w.reshape(w.shape[0], -1).abs().amax(1).clamp_min(1e-12) / 448.0
    shp = (-1,) + (1,) * (w.dim() - 1)
    return (w / s.view(shp)).to(E4M3).float() * s.view(shp)


def quant_a(a, recipe, dim):
    if recipe == "bf16":
        return a.to(torch.bfloat16).float()
    if recipe.startswith("mxfp8"):
        return mx_q(a, dim, recipe.endswith("c"))
    return a.clamp(-448, 448).to(E4M3).float()


class Quantized:
    """Context: the oracle's pointwise GEMMs run on quantized operands (weights pre-quantized in sdq)."""

    def __init__(self, recipe):
        self.recipe = recipe

    def __enter__(self):
        self.conv0, self.lin0 = F.conv1d, orc._lin
        r = self.recipe

        def conv(x_, w, b=None, stride=1, padding=0, dilation=1, groups=1):
            q = groups == 1 and (w.shape[-1] == 1 or not BIG4)
            return self.conv0(quant_a(x_, r, 1) if q else x_, w, b, stride, padding, dilation, groups)

        def lin(sd_, p, x_):
            q = any(p.endswith(n) for n in (("mlp.0", "mlp.2") if BIG4 else ("proj_in", "mlp.0", "mlp.2")))
            return self.lin0(sd_, p, quant_a(x_, r, -1) if q else x_)
        orc.F.conv1d, orc._lin = conv, lin
        return self

    def __exit__(self, *a):
        orc.F.conv1d, orc._lin = self.conv0, self.lin0


def quantized_sd(sd, recipe):
    return {k: (quant_w(v, recipe) if (k.endswith(".weight") and "denoiser" in k and "adaLN" not in k
                                         and any(("." + n + ".") in k for n in NAMES)) else v) for k, v in sd.items()}


def rel(a, b):
    return float((a - b).norm() / b.norm())


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    torch.set_num_threads(8)
    sd = seeded("prob_generator")
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(1, T, 256, generator=g) * 0.3 + torch.randn(1, T, 256, generator=g)
    c = torch.randn(1, 256, generator=g)
    refs_v = {tv: orc.denoiser_forward(sd, x0, torch.tensor([[tv]]), c) for tv in (0.1, 0.5, 0.9)}
    refs_s = {n: orc.euler_solve(sd, x0, c, n) for n in (128, 256)}
    for recipe in os.environ.get("FP8_RECIPES", "bf16,mxfp8,mxfp8c,fp8-chan").split(","):
        sdq = quantized_sd(sd, recipe)
        with Quantized(recipe):
            ev = [rel(orc.denoiser_forward(sdq, x0, torch.tensor([[tv]]), c), r) for tv, r in refs_v.items()]
            es = {n: rel(orc.euler_solve(sdq, x0, c, n), r) for n, r in refs_s.items()}
        print(f"{recipe:9s} T={T}: velocity rel-L2 " + " ".join(f"{e:.3e}" for e in ev)
              + " | solve rel-L2 " + " ".join(f"nfe{n} {e:.3e}" for n, e in es.items()), flush=True)


if __name__ == "__main__":
    main()
