"""GPU: the torch.library ops (flamed/ops.py) are the path the modules take, they trace whole under
torch.compile (no graph break on the native call), and torch.library.opcheck accepts them."""
import pytest
import torch

from _common import rel_l2
from test_denoiser_gpu import _prob_gen, DEV

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    return _prob_gen("f32")[0]


def _inputs(B=2, T=48):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, T, 256, generator=g).to(DEV)
    t = torch.rand(B, 1, generator=g).to(DEV)
    c = torch.randn(B, 256, generator=g).to(DEV)
    return x, t, c


def test_forward_equals_op(pg):
    x, t, c = _inputs()
    with torch.inference_mode():
        v_mod = pg.denoiser(x, t, c)
        v_op = torch.ops.flamed_hip.den_velocity(pg.denoiser.hip().oid, x, t, c)
    assert torch.equal(v_mod, v_op)


def test_compile_traces_the_op_without_graph_break(pg):
    x, t, c = _inputs()
    oid = pg.denoiser.hip().oid
    with torch.inference_mode():
        ref = torch.ops.flamed_hip.den_velocity(oid, x, t, c) * 0.5 + x

    def f(x_, t_, c_):
        return torch.ops.flamed_hip.den_velocity(oid, x_, t_, c_) * 0.5 + x_

    torch._dynamo.reset()
    fc = torch.compile(f, fullgraph=True, backend="eager")  # fullgraph: a graph break raises
    with torch.inference_mode():
        out = fc(x, t, c)
    assert rel_l2(out, ref) == 0.0


def test_opcheck_den_velocity(pg):
    x, t, c = _inputs()
    torch.library.opcheck(torch.ops.flamed_hip.den_velocity.default, (pg.denoiser.hip().oid, x, t, c),
                          test_utils=("test_schema", "test_faketensor"))


def test_opcheck_length_regulate():
    x = torch.randn(2, 9, 16, device=DEV)
    pd = torch.randint(0, 4, (2, 9), device=DEV).float()
    sd = torch.randint(0, 2, (2, 9), device=DEV).float()
    sl = torch.tensor([9, 5], device=DEV)
    torch.library.opcheck(torch.ops.flamed_hip.length_regulate.default, (x, pd, sd, sl, 40, False),
                          test_utils=("test_schema", "test_faketensor"))
