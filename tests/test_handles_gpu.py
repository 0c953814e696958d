"""GPU tests of the C-ABI handle contract (include/flamed_hip.h): device pinning, owned weight copies,
re-pack on load_state_dict, per-handle knobs, concurrent handles on separate threads/streams, and the
autograd gate of the length regulator (reference pva.py:125-166 stays differentiable)."""
import ctypes
import threading

import pytest
import torch
import yaml

from _common import PKG, orc, rel_l2, seeded
from test_denoiser_gpu import BF16_VEL, _prob_gen

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _inputs(seed, B=1, T=200):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, T, 256, generator=g), torch.randn(B, 256, generator=g)


def _vel(pg, x, c, t=0.3):
    with torch.inference_mode():
        return pg.denoiser(x.to(DEV), torch.tensor([[t]], device=DEV), c.to(DEV)).cpu()


def test_handle_records_its_device():
    from flamed import _native as nat
    pg, _ = _prob_gen("bf16")
    x, c = _inputs(1)
    _vel(pg, x, c)
    assert nat.lib().flamed_den_device(pg.denoiser.hip().handle) == torch.device(DEV).index


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_handle_on_non_current_device():
    """Weights on cuda:1 while cuda:0 is current: the handle allocates and launches on cuda:1."""
    import os
    from flamed.models.synthesizer.prob_generator import ProbGenerator
    cfg = yaml.safe_load(open(os.path.join(PKG, "configs", "prob.yaml")))
    pg = ProbGenerator(cfg).eval()
    sd = seeded("prob_generator")
    pg.load_state_dict({k[len("prob_generator."):]: v for k, v in sd.items()})
    pg = pg.to("cuda:1")
    x, c = _inputs(2)
    torch.cuda.set_device(0)
    with torch.inference_mode():
        v = pg.denoiser(x.to("cuda:1"), torch.tensor([[0.3]], device="cuda:1"), c.to("cuda:1")).cpu()
    assert rel_l2(v, orc.denoiser_forward(sd, x, torch.tensor([[0.3]]), c)) < BF16_VEL


def test_weights_are_owned_by_the_handle():
    """After load the handle reads only its own arena: dropping and overwriting the fp32 copies the
    wrapper handed to flamed_den_load changes nothing (bitwise)."""
    pg, _ = _prob_gen("bf16")
    x, c = _inputs(3)
    v1 = _vel(pg, x, c)
    hip = pg.denoiser.hip()
    hip._keep = []
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    junk = [torch.full((1 << 22,), float("nan"), device=DEV) for _ in range(16)]
    v2 = _vel(pg, x, c)
    del junk
    assert torch.equal(v1, v2)


def test_load_state_dict_under_inference_mode_repacks():
    """load_state_dict copies in place (same pointers; inference tensors carry no version counter):
    the module's hook must make the next call re-pack, so the new weights are used."""
    pg, sd_a = _prob_gen("bf16")
    x, c = _inputs(4)
    t = torch.tensor([[0.3]])
    va = _vel(pg, x, c)
    sd_b = seeded("prob_generator", seed=77)
    with torch.inference_mode():
        pg.load_state_dict({k[len("prob_generator."):]: v.to(DEV) for k, v in sd_b.items()})
    vb = _vel(pg, x, c)
    assert rel_l2(va, orc.denoiser_forward(sd_a, x, t, c)) < BF16_VEL
    assert rel_l2(vb, orc.denoiser_forward(sd_b, x, t, c)) < BF16_VEL


def test_per_handle_tune_does_not_leak():
    """flamed_den_tune(h, "lnfold", 0) changes only that handle; it equals the process-wide knob."""
    from flamed import _native as nat
    L = nat.lib()
    pa, _ = _prob_gen("bf16")
    pb, _ = _prob_gen("bf16")
    x, c = _inputs(5, T=400)
    base = _vel(pb, x, c)
    assert torch.equal(_vel(pa, x, c), base)  # creates and loads pa's handle
    nat.check(L.flamed_den_tune(pa.denoiser.hip().handle, b"lnfold", 0), "flamed_den_tune")
    va = _vel(pa, x, c)
    vb = _vel(pb, x, c)
    assert torch.equal(vb, base)
    try:
        nat.check(L.flamed_tune(b"lnfold", 0), "flamed_tune")
        vg = _vel(pb, x, c)
    finally:
        nat.check(L.flamed_tune(b"lnfold", 1), "flamed_tune")
    assert torch.equal(va, vg) and not torch.equal(va, base)


def test_concurrent_handles_on_threads():
    """Two handles solved at once from two threads on their own streams give the sequential results
    bitwise (per-handle counters, graphs, knob snapshots; thread-local step state)."""
    pa, _ = _prob_gen("bf16")
    pb, _ = _prob_gen("bf16")
    xa, ca = _inputs(6, T=400)
    xb, cb = _inputs(7, T=300)
    ts = torch.linspace(0, 1, 33, device=DEV)

    def solve(pg, x, c):
        with torch.inference_mode():
            return pg.denoiser.hip().solve(x.to(DEV), ts, c.to(DEV), 32).cpu()
    ref_a, ref_b = solve(pa, xa, ca), solve(pb, xb, cb)
    out = {}

    def run(name, pg, x, c):
        s = torch.cuda.Stream(device=DEV)
        with torch.cuda.stream(s):
            for _ in range(3):
                out[name] = solve(pg, x, c)
        s.synchronize()
    th = [threading.Thread(target=run, args=("a", pa, xa, ca)), threading.Thread(target=run, args=("b", pb, xb, cb))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert torch.equal(out["a"], ref_a) and torch.equal(out["b"], ref_b)


def test_length_regulator_keeps_autograd_on_gpu():
    """Under autograd the CUDA length regulator takes the differentiable path: gradients reach x."""
    from flamed.models.synthesizer.pva import LengthRegulator
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 7, 16, generator=g).to(DEV).requires_grad_(True)
    pd = torch.tensor([[1, 2, 0, 3, 1, 1, 2], [2, 1, 1, 0, 0, 0, 0]], dtype=torch.float32, device=DEV)
    sd = torch.tensor([[0, 1, 0, 0, 2, 0, 1], [1, 0, 0, 0, 0, 0, 0]], dtype=torch.float32, device=DEV)
    sl = torch.tensor([7, 3], device=DEV)
    out, tl = LengthRegulator()(x, pd, sd, sl, None)
    assert out.requires_grad
    (out * torch.arange(out.numel(), device=DEV, dtype=torch.float32).view_as(out)).sum().backward()
    assert x.grad is not None and float(x.grad.abs().sum()) > 0
    with torch.no_grad():
        out_hip, tl_hip = LengthRegulator()(x.detach(), pd, sd, sl, None)
    assert torch.equal(out.detach(), out_hip) and torch.equal(tl, tl_hip)
