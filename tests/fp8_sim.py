"""CPU estimate of what fp8 (OCP e4m3) pointwise projections would cost in accuracy (BASELINE configs[4]):
the oracle denoiser forward with every GEMM's weights quantized per output channel (amax/448) and its
input activations quantized at unit scale (clamped to +-448), against fp32; the same with bf16 rounding.
Usage: PYTHONPATH=flamed-tts_amd:. python tests/fp8_sim.py   (CPU only; lives under tests/ because it runs the
oracle, which only test code may import)."""
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _common import seeded, orc  # noqa: E402  (checker only)

NAMES = ["proj_in", "conv_2", "conv_3", "mlp.0", "mlp.2", "conv_out"]


def qw(w, dt):
    if dt == torch.bfloat16:
        return w.to(dt).float()
    s = w.reshape(w.shape[0], -1).abs().amax(1).clamp_min(1e-12) / 448.0
    shp = (-1,) + (1,) * (w.dim() - 1)
    return (w / s.view(shp)).to(dt).float() * s.view(shp)


def qa(a, dt):
    return a.to(dt).float() if dt == torch.bfloat16 else a.clamp(-448, 448).to(dt).float()


def main():
    sd = seeded("prob_generator")
    g = torch.Generator().manual_seed(3)
    x, c, t = torch.randn(1, 200, 256, generator=g), torch.randn(1, 256, generator=g), torch.tensor([[0.4]])
    ref = orc.denoiser_forward(sd, x, t, c)
    for dt in (torch.bfloat16, torch.float8_e4m3fn):
        sdq = {k: (qw(v, dt) if (k.endswith(".weight") and "denoiser" in k and "adaLN" not in k
                                 and any(("." + n + ".") in k for n in NAMES)) else v) for k, v in sd.items()}
        conv0, lin0 = F.conv1d, orc._lin

        def conv(x_, w, b=None, stride=1, padding=0, dilation=1, groups=1):
            return conv0(qa(x_, dt) if groups == 1 else x_, w, b, stride, padding, dilation, groups)

        def lin(sd_, p, x_):
            return lin0(sd_, p, qa(x_, dt) if any(p.endswith(n) for n in ("proj_in", "mlp.0", "mlp.2")) else x_)

        orc.F.conv1d, orc._lin = conv, lin
        try:
            v = orc.denoiser_forward(sdq, x, t, c)
        finally:
            orc.F.conv1d, orc._lin = conv0, lin0
        print(f"{str(dt):22s} velocity rel-L2 vs fp32: {float((v - ref).norm() / ref.norm()):.3e}")


if __name__ == "__main__":
    main()
