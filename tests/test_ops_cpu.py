"""torch.library layer (flamed/ops.py): every HIP entry point the modules dispatch to is a
registered `flamed_hip::*` custom op with a schema and a fake (meta) implementation, so FakeTensor shape
propagation and torch.compile tracing see them.  CPU only: no op body runs here."""
import types

import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.symbolic_shapes import ShapeEnv

import _common  # noqa: F401  (sys.path)
from flamed import ops


def test_every_op_is_registered_with_a_schema():
    for name in ops.OPS:
        op = getattr(torch.ops.flamed_hip, name)
        schema = str(op.default._schema)
        assert schema.startswith(f"flamed_hip::{name}("), schema


def test_modules_dispatch_through_the_ops():
    import inspect
    from flamed.models.synthesizer import prob_generator, pva, prior_generator
    from flamed.models.facodec import facodec
    src = inspect.getsource(prob_generator) + inspect.getsource(pva) + inspect.getsource(facodec) + \
        inspect.getsource(prior_generator)
    for name in ops.OPS:
        assert f"ops.{name}(" in src, name


class _Owner:  # weak-referenceable stand-in for a HIP owner object
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _dummy_owner(**kw):
    o = _Owner(**kw)
    return o, ops.register(o)


def test_fake_shapes():
    pg, pid = _dummy_owner(pg=types.SimpleNamespace(target_dim=256))
    dec, did = _dummy_owner(dec=types.SimpleNamespace(hop_length=200))
    enc, eid = _dummy_owner(enc=types.SimpleNamespace(out_channels=256), out_len=lambda n: n // 200)
    with FakeTensorMode(shape_env=ShapeEnv()):
        x = torch.empty(2, 50, 256)
        v = torch.ops.flamed_hip.den_velocity(1, x, torch.empty(1, 1), torch.empty(2, 256))
        assert v.shape == (2, 50, 256) and v.dtype == torch.float32
        s = torch.ops.flamed_hip.den_solve(1, x, torch.empty(129), torch.empty(2, 256), 128)
        assert s.shape == (2, 50, 256)
        c = torch.ops.flamed_hip.cond_fold(pid, torch.empty(2, 4, 50, 64), torch.empty(2, 50, 1, dtype=torch.bool))
        assert c.shape == (2, 50, 256)
        d, si = torch.ops.flamed_hip.pva_flow(1, torch.empty(2, 9, 256), torch.empty(2, 9, dtype=torch.bool),
                                              torch.empty(2, 9), torch.empty(2, 9), torch.empty(33), 32)
        assert d.shape == (2, 9) and si.shape == (2, 9)
        out, tl = torch.ops.flamed_hip.length_regulate(torch.empty(2, 9, 256), torch.empty(2, 9), torch.empty(2, 9),
                                                       torch.empty(2, dtype=torch.int64), 40, False)
        assert out.shape == (2, 40, 256) and tl.shape == (2,) and tl.dtype == torch.int64
        out, _ = torch.ops.flamed_hip.length_regulate(torch.empty(2, 9, 256), torch.empty(2, 9), torch.empty(2, 9),
                                                      torch.empty(2, dtype=torch.int64), 0, True)
        assert isinstance(out.shape[1], torch.SymInt)  # data-dependent length (the reference's .tolist())
        w = torch.ops.flamed_hip.fac_decode(did, torch.empty(1, 256, 40), torch.empty(1, 256))
        assert w.shape == (1, 1, 8000)
        e = torch.ops.flamed_hip.enc_encode(eid, torch.empty(1, 1, 48000))
        assert e.shape == (1, 256, 240)
        vq = types.SimpleNamespace(quantizer=[types.SimpleNamespace(layers=[0] * n) for n in (1, 2, 3)])
        vo, void = _dummy_owner(dec=vq)
        outs, codes, qb, spk = torch.ops.flamed_hip.vq_encode(void, torch.empty(2, 256, 30))
        assert outs.shape == (2, 256, 30) and codes.shape == (6, 2, 30) and codes.dtype == torch.int64
        assert qb.shape == (3, 2, 256, 30) and spk.shape == (2, 256)
        ppg = types.SimpleNamespace(encoder=types.SimpleNamespace(d_model=192), prior_decoder=[None] * 6,
                                    shared_decoder=types.SimpleNamespace(d_model=384),
                                    head=types.SimpleNamespace(weight=torch.empty(1025, 384)))
        po, poid = _dummy_owner(pg=ppg)
        h = torch.ops.flamed_hip.prior_encode(poid, torch.empty(2, 17, dtype=torch.int64), torch.empty(2, 17, dtype=torch.bool))
        assert h.shape == (2, 17, 192) and h.dtype == torch.float32
        pe, pl = torch.ops.flamed_hip.prior_decode(poid, torch.empty(2, 40, 192), torch.empty(2, 40, dtype=torch.bool),
                                                   torch.empty(2, 6, 20, dtype=torch.int64), 20)
        assert pe.shape == (2, 6, 40, 384) and pl.shape == (2, 1025, 6, 40)


def test_dead_owner_raises():
    o, oid = _dummy_owner()
    del o
    with pytest.raises(RuntimeError, match="no live HIP owner"):
        ops.owner(oid)
