"""GPU parity: PVA duration / silence flow (HIP, exact-fp32 MFMA) and the HIP length regulator.

Tolerances: final log-durations rel-L2 <= 1e-5 vs the reference (fp32, summation order only);
frame counts / tgt_len / regulated frames BIT-EXACT (integer work); for random weights at larger
sizes any duration within 1e-4 of a .5 rounding boundary is excluded and counted as a possible flip.
"""
import numpy as np
import pytest
import torch
import yaml

from _common import golden, seeded, t32, rel_l2, orc, PKG

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def pva():
    import os
    from flamed.models.synthesizer.pva import PVA
    cfg = yaml.safe_load(open(os.path.join(PKG, "configs", "prior.yaml")))["variance_adaptor"]
    m = PVA(cfg).eval()
    sd = seeded("pva")
    m.load_state_dict({k[len("prior_generator.pva."):]: v for k, v in sd.items()})
    return m.to(DEV), sd


def test_pva_flow_and_sample_golden(pva):
    m, _ = pva
    g = golden("pva")
    src_len = t32(g["src_len"])
    L = g["enc"].shape[1]
    mask = torch.arange(L)[None, :] >= src_len[:, None]
    enc = t32(g["enc"]).to(DEV)
    with torch.inference_mode():
        torch.manual_seed(int(g["rng_seed"]))
        d, s = m.flow(enc, mask.to(DEV), int(g["nfe"]), float(g["temperature"]))
        assert rel_l2(d.cpu(), g["dur_final"]) < 1e-5 and rel_l2(s.cpu(), g["sil_final"]) < 1e-5
        torch.manual_seed(int(g["rng_seed"]))
        x_lr, tgt = m.sample(enc, src_len.to(DEV), mask.to(DEV), nfe=int(g["nfe"]), temperature=float(g["temperature"]))
    assert np.array_equal(tgt.cpu().numpy(), g["tgt_len"])
    assert x_lr.shape == g["x_lr"].shape and np.array_equal(x_lr.cpu().numpy(), g["x_lr"])


def _tune(key, v):
    from flamed import _native as nat
    nat.check(nat.lib().flamed_tune(key.encode(), v), "flamed_tune")


def test_pva_graph_equals_eager(pva):
    """The hipGraph of launches (persistent flow off) replays exactly the plain launches."""
    m, _ = pva
    gen = torch.Generator().manual_seed(3)
    B, L = 3, 41
    enc = torch.randn(B, L, 192, generator=gen).to(DEV)
    mask = (torch.arange(L)[None, :] >= torch.tensor([41, 30, 7])[:, None]).to(DEV)
    outs = []
    try:
        _tune("pva_persist", 0)
        with torch.inference_mode():
            for graph in (True, True, False):
                m.hip_graph = graph
                torch.manual_seed(5)
                outs.append(m.flow(enc, mask, 6, 0.3))
    finally:
        m.hip_graph = True
        _tune("pva_persist", 1)
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])


@pytest.mark.parametrize("B,L,nfe", [(1, 60, 64), (1, 285, 64), (3, 41, 6), (2, 247, 16), (1, 1, 8), (1, 17, 4),
                                     (5, 128, 8)])
def test_pva_persistent_flow(pva, B, L, nfe):
    """One persistent launch for every step of both nets (pvaflow.hip): it really ran (persist_info), two
    runs are bitwise equal (fixed combine orders), and against the oracle and the graph of launches the
    log-durations agree to rel-L2 <= 1e-5 with ZERO integer frame flips at positions not within 1e-4 of
    a .5 rounding boundary.  Covers one to eight 16-row tiles per row group, K split 4 / 2 / 1 ways over
    the waves, a single phoneme, ragged masks and utterance edges inside a row group."""
    m, sd = pva
    gen = torch.Generator().manual_seed(100 + B * L)
    enc = torch.randn(B, L, 192, generator=gen)
    lens = torch.tensor([L] + [max(1, L - 37 * i) for i in range(1, B)])
    mask = torch.arange(L)[None, :] >= lens[:, None]
    torch.manual_seed(7)
    dn, sn = torch.randn((B, L)), torch.randn((B, L))
    hp = m.hip()
    outs = []
    with torch.inference_mode():
        for persist in (1, 1, 0):
            _tune("pva_persist", persist)
            r0 = hp.persist_info()[0] if hp.handles[0] is not None else 0
            torch.manual_seed(7)
            outs.append(m.flow(enc.to(DEV), mask.to(DEV), nfe, 0.3))
            ran = hp.persist_info()[0] - r0
            assert ran == persist, (persist, ran, hp.persist_info())
    _tune("pva_persist", 1)
    assert not hp.persist_info()[1]
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    rd, rs = orc.pva_flow(sd, enc, mask, nfe, 0.3, noise=(dn, sn))
    flips = 0
    for got, graph, ref in ((outs[0][0].cpu(), outs[2][0].cpu(), rd), (outs[0][1].cpu(), outs[2][1].cpu(), rs)):
        assert rel_l2(got, ref) < 1e-5 and rel_l2(got, graph) < 1e-5
        e = torch.exp(ref) - 1
        safe = (e - e.floor() - 0.5).abs() > 1e-4
        flips += int((orc.log_to_frames(got)[safe] != orc.log_to_frames(ref)[safe]).sum())
    assert flips == 0


def test_pva_flow_vs_oracle_larger(pva):
    m, sd = pva
    gen = torch.Generator().manual_seed(11)
    B, L, nfe = 6, 97, 16
    enc = torch.randn(B, L, 192, generator=gen)
    lens = torch.tensor([97, 80, 64, 33, 12, 1])
    mask = torch.arange(L)[None, :] >= lens[:, None]
    torch.manual_seed(21)
    dn, sn = torch.randn((B, L)), torch.randn((B, L))
    with torch.inference_mode():
        torch.manual_seed(21)
        d, s = m.flow(enc.to(DEV), mask.to(DEV), nfe, 0.3)
    rd, rs = orc.pva_flow(sd, enc, mask, nfe, 0.3, noise=(dn, sn))
    assert rel_l2(d.cpu(), rd) < 1e-5 and rel_l2(s.cpu(), rs) < 1e-5
    for got, ref in ((d.cpu(), rd), (s.cpu(), rs)):
        e = torch.exp(ref) - 1
        safe = (e - e.floor() - 0.5).abs() > 1e-4
        gf, rf = orc.log_to_frames(got), orc.log_to_frames(ref)
        assert torch.equal(gf[safe], rf[safe])


def test_length_regulator_golden_cases_bit_exact():
    from flamed.models.synthesizer.pva import hip_length_regulate
    g = golden("lr_cases")
    for ci in range(int(g["n"])):
        mx = int(g[f"c{ci}_max"])
        out, tl = hip_length_regulate(t32(g[f"c{ci}_x"]).to(DEV), t32(g[f"c{ci}_pd"]).to(DEV),
                                      t32(g[f"c{ci}_sd"]).to(DEV), t32(g[f"c{ci}_sl"]).to(DEV),
                                      None if mx < 0 else mx)
        assert np.array_equal(tl.cpu().numpy(), g[f"c{ci}_tl"]), ci
        assert np.array_equal(out.cpu().numpy(), g[f"c{ci}_out"]), ci


@pytest.mark.parametrize("B,L,H,max_len", [(5, 37, 192, None), (2, 300, 64, 50), (7, 3, 8, None), (1, 1, 192, 3),
                                           (4, 513, 32, None)])
def test_length_regulator_random_bit_exact(B, L, H, max_len):
    from flamed.models.synthesizer.pva import hip_length_regulate
    rng = np.random.default_rng(B * 7919 + L)
    x = rng.standard_normal((B, L, H)).astype(np.float32)
    pd = rng.integers(0, 9, (B, L)).astype(np.float32)
    sdur = rng.integers(0, 4, (B, L)).astype(np.float32)
    sl = rng.integers(1, L + 1, (B,)).astype(np.int64)
    ref, rtl = orc.length_regulate(x, pd, sdur, sl, max_len)
    out, tl = hip_length_regulate(t32(x).to(DEV), t32(pd).to(DEV), t32(sdur).to(DEV), t32(sl).to(DEV), max_len)
    assert np.array_equal(tl.cpu().numpy(), rtl)
    assert np.array_equal(out.cpu().numpy(), ref)


def test_length_regulator_log_domain():
    from flamed.models.synthesizer.pva import hip_length_regulate
    rng = np.random.default_rng(3)
    B, L, H = 3, 50, 16
    x = rng.standard_normal((B, L, H)).astype(np.float32)
    d = rng.uniform(-1, 3, (B, L)).astype(np.float32)
    s = rng.uniform(-1, 1.5, (B, L)).astype(np.float32)
    sl = np.array([50, 20, 1], dtype=np.int64)
    pdf = orc.log_to_frames(t32(d)).numpy()
    sdf = orc.log_to_frames(t32(s)).numpy()
    ref, rtl = orc.length_regulate(x, pdf, sdf, sl)
    out, tl = hip_length_regulate(t32(x).to(DEV), t32(d).to(DEV), t32(s).to(DEV), t32(sl).to(DEV), None,
                                  log_domain=True)
    assert np.array_equal(tl.cpu().numpy(), rtl) and np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("B,L", [(1, 60), (2, 247)])
def test_pva_split_k_deterministic(pva, B, L):
    """The nets' small-M fp32 GEMMs split K over workgroups (flamed_tune pva_split, per-handle slabs and
    counters, slices summed in a fixed order): repeated graph solves are bitwise equal, and the flow
    differs from the one-chain form by fp32 reassociation only."""
    from flamed import _native as nat
    m, _ = pva
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(B, L, 192, generator=gen).to(DEV)
    mask = torch.zeros(B, L, dtype=torch.bool, device=DEV)
    d0 = torch.randn(B, L, generator=gen).to(DEV) * 0.3
    s0 = torch.randn(B, L, generator=gen).to(DEV) * 0.3
    ts = torch.linspace(0, 1, 65, device=DEV)
    L_ = nat.lib()
    outs = []
    try:
        nat.check(L_.flamed_tune(b"pva_persist", 0), "tune")  # the split applies to the graph of launches
        with torch.inference_mode():
            for sp in (1, 1, 0):
                nat.check(L_.flamed_tune(b"pva_split", sp), "tune")
                outs.append(m.hip().flow(x, mask, d0, s0, ts, 64))
    finally:
        nat.check(L_.flamed_tune(b"pva_split", 0), "tune")
        nat.check(L_.flamed_tune(b"pva_persist", 1), "tune")
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # the split really ran (the knob is part of the graph key): reassociated, so not bitwise equal
    assert not (torch.equal(outs[0][0], outs[2][0]) and torch.equal(outs[0][1], outs[2][1]))
    for a, b in zip(outs[0], outs[2]):
        assert rel_l2(a.cpu(), b.cpu()) < 1e-5


def test_pva_flow_default_nsteps_ragged(pva):
    """The reference CLI's default --nsteps-durgen 64 (synthesize.py:338; loop pva.py:97-112) at an
    end-to-end phoneme count (L = 285, the bench's 5 s utterance) on a ragged batch of 4: log-durations
    rel-L2 <= 1e-5 against the oracle, and ZERO integer frame flips at every position that is not within
    1e-4 of a .5 rounding boundary (positions near a boundary are counted and reported)."""
    m, sd = pva
    gen = torch.Generator().manual_seed(31)
    B, L, nfe = 4, 285, 64
    enc = torch.randn(B, L, 192, generator=gen)
    lens = torch.tensor([285, 240, 131, 17])
    mask = torch.arange(L)[None, :] >= lens[:, None]
    torch.manual_seed(41)
    dn, sn = torch.randn((B, L)), torch.randn((B, L))
    with torch.inference_mode():
        torch.manual_seed(41)
        d, s = m.flow(enc.to(DEV), mask.to(DEV), nfe, 0.3)
    rd, rs = orc.pva_flow(sd, enc, mask, nfe, 0.3, noise=(dn, sn))
    assert rel_l2(d.cpu(), rd) < 1e-5 and rel_l2(s.cpu(), rs) < 1e-5
    near, flips = 0, 0
    for got, ref in ((d.cpu(), rd), (s.cpu(), rs)):
        e = torch.exp(ref) - 1
        safe = (e - e.floor() - 0.5).abs() > 1e-4
        near += int((~safe).sum())
        gf, rf = orc.log_to_frames(got), orc.log_to_frames(ref)
        flips += int((gf[safe] != rf[safe]).sum())
    print(f"PVA nfe=64 L=285 B=4: non-boundary flips {flips}, positions near a .5 boundary {near}")
    assert flips == 0


def _flow_inputs(seed, B, L):
    gen = torch.Generator().manual_seed(seed)
    enc = torch.randn(B, L, 192, generator=gen).to(DEV)
    lens = torch.tensor([L] + [max(1, L - 29 * i) for i in range(1, B)])
    mask = (torch.arange(L)[None, :] >= lens[:, None]).to(DEV)
    d = (torch.randn(B, L, generator=gen) * 0.3).to(DEV)
    s = (torch.randn(B, L, generator=gen) * 0.3).to(DEV)
    return enc, mask, d, s


def test_pva_persist_graph_capture(pva):
    """the persistent PVA flow keeps the C-ABI contract -- only enqueued (no host sync) and
    capturable.  A torch.cuda.graph capture of the flow (after one uncaptured flow) takes the persistent launch
    (the cooperative node; the kernel resets its own counters), and replays with changed inputs equal the eager
    persistent flow bitwise."""
    m, _ = pva
    hp = m.hip()
    B, L, nfe = 2, 70, 16
    enc, mask, d0, s0 = _flow_inputs(61, B, L)
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    with torch.inference_mode():
        hp.flow(enc, mask, d0, s0, ts, nfe)  # warm: scratch, handles
        torch.cuda.synchronize()
        r0 = hp.persist_status()[0]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            hp.flow(enc, mask, d0, s0, ts, nfe)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            od, os_ = hp.flow(enc, mask, d0, s0, ts, nfe)
        assert hp.persist_status()[0] == r0 + 2, "the captured flow did not take the persistent launch"
        outs = []
        for rep in range(3):
            e2, _, d2, s2 = _flow_inputs(70 + rep, B, L)
            enc.copy_(e2), d0.copy_(d2), s0.copy_(s2)
            g.replay()
            torch.cuda.synchronize()
            outs.append((od.clone(), os_.clone()))
            ed, es = hp.flow(enc, mask, d0, s0, ts, nfe)
            torch.cuda.synchronize()
            assert torch.equal(outs[-1][0], ed) and torch.equal(outs[-1][1], es), rep
            assert torch.isfinite(ed).all()
    assert not torch.equal(outs[0][0], outs[1][0])


def test_pva_persist_failure_rerun_and_budget(pva):
    """A persistent flow that gives up (diagnostic knob pva_inject: every workgroup abandons at that step) leaves
    NaN in both states and is counted, without a host sync on the call path; the Python wrapper (check on, the
    default) waits, warns and re-runs it on the graph path, so the caller gets the graph path's exact result;
    after 3 failures the pair takes the graph path for good."""
    import warnings
    from flamed.models.synthesizer.pva import PvaHIP
    m, _ = pva
    hp = PvaHIP(m)  # a fresh pair: the module's own stays on the persistent path
    B, L, nfe = 1, 60, 8
    enc, mask, d0, s0 = _flow_inputs(81, B, L)
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    with torch.inference_mode():
        ref = hp._graph_flow(enc, mask, d0, s0, ts, nfe, 1 | 2)
        try:
            _tune("pva_inject", 3)
            hp.check_persist = False
            raw = hp.flow(enc, mask, d0, s0, ts, nfe)
            torch.cuda.synchronize()
            assert torch.isnan(raw[0]).all() and torch.isnan(raw[1]).all()
            assert hp.persist_status()[1] == 1
            hp.check_persist = True
            with warnings.catch_warnings(record=True) as wl:
                warnings.simplefilter("always")
                out = hp.flow(enc, mask, d0, s0, ts, nfe)
            assert any("persistent PVA flow failed" in str(w.message) for w in wl)
            assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
            hp.flow(enc, mask, d0, s0, ts, nfe)  # third failure: the pair gives up the persistent path
        finally:
            _tune("pva_inject", -1)
        runs, broken, _ = hp.persist_info()
        assert runs == 3 and broken
        after = hp.flow(enc, mask, d0, s0, ts, nfe)
        assert hp.persist_info()[0] == 3
    assert torch.equal(after[0], ref[0]) and torch.equal(after[1], ref[1])
