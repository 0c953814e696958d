"""GPU: the persistent B = 1 Euler solve (flamed-tts_amd/csrc/persist.hip) — every step of
ProbGenerator.sample's ODE loop (reference prob_generator.py:434-447, SimpleMLPAdaLN.forward :349-365) in
one launch of 256 workgroups with in-launch hand-offs.

Checks: the solve really ran persistently (flamed_den_persist_info), against the fp32 oracle under the
bf16 solve tolerance of the launch path (rel-L2 <= 6e-3 and max|d| < 0.05 at configs[1]), at edge lengths
(T = 16: most groups empty; 40 / 131 / 257: partial tiles; 512: every group full), against the launch path
(same bf16 operands, different fp32 reduction order: rel-L2 <= 4e-3), bitwise determinism, and parts
[0, G) + [G, nfe) equal to the whole (the fp32 state passes through xt exactly).
"""
import contextlib
import os

import pytest
import torch

from _common import orc, rel_l2
from test_denoiser_gpu import _prob_gen

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
C = 256
BF16_SOLVE = 6e-3


@contextlib.contextmanager
def knob(key, value, default):
    from flamed import _native as nat
    L = nat.lib()
    nat.check(L.flamed_tune(key.encode(), value), "flamed_tune")
    try:
        yield
    finally:
        nat.check(L.flamed_tune(key.encode(), default), "flamed_tune")


@pytest.fixture(scope="module")
def pgb():
    return _prob_gen("bf16")


def _inputs(seed, B, T, temp=0.3):
    g = torch.Generator().manual_seed(seed)
    cond = torch.randn(B, T, C, generator=g)
    noise = torch.randn(B, T, C, generator=g)
    spk = torch.randn(B, C, generator=g)
    return noise * temp + cond, spk


def _solve(pg, x0, spk, nfe):
    hip = pg.denoiser.hip()
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    with torch.inference_mode():
        return hip.solve(x0.to(DEV), ts, spk.to(DEV), nfe).cpu()


def _runs(pg):
    if pg.denoiser.hip().handle is None:  # no solve on this module yet (e.g. a -k selection)
        return 0
    runs, broken = pg.denoiser.hip().persist_info()
    assert not broken, "the handle gave up the persistent path (failed launches)"
    return runs


def test_persist_cfg1_vs_oracle_and_launch_path(pgb):
    pg, sd = pgb
    x0, spk = _inputs(1, 1, 400)
    r0 = _runs(pg) if pg.denoiser._hip is not None else 0
    out = _solve(pg, x0, spk, 128)
    assert _runs(pg) == r0 + 1, "the B = 1 solve did not take the persistent path"
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    ref = orc.euler_solve(sd, x0, spk, 128)
    e = rel_l2(out, ref)
    amax = float((out - ref).abs().max())
    with knob("persist", 0, 1):
        launch = _solve(pg, x0, spk, 128)
    el = rel_l2(out, launch)
    print(f"persistent configs[1] 128 steps: vs oracle rel-L2 {e:.3e} max|d| {amax:.3e}; vs launch path {el:.3e} "
          f"(launch path vs oracle {rel_l2(launch, ref):.3e})")
    assert torch.isfinite(out).all()
    assert e < BF16_SOLVE and amax < 0.05
    assert el < 4e-3


@pytest.mark.parametrize("T", [16, 40, 131, 257, 512])
def test_persist_lengths_vs_oracle(pgb, T):
    pg, sd = pgb
    x0, spk = _inputs(T, 1, T)
    r0 = _runs(pg) if pg.denoiser._hip is not None else 0
    out = _solve(pg, x0, spk, 8)
    assert _runs(pg) == r0 + 1
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    ref = orc.euler_solve(sd, x0, spk, 8)
    e = rel_l2(out, ref)
    print(f"persistent T={T} 8 steps: vs oracle rel-L2 {e:.3e}")
    assert e < BF16_SOLVE


def test_persist_deterministic_and_parts(pgb):
    from flamed import _native as nat
    pg, _ = pgb
    hip = pg.denoiser.hip()
    L = nat.lib()
    x0, spk = _inputs(5, 1, 300)
    nfe = 32
    a = _solve(pg, x0, spk, nfe)
    b = _solve(pg, x0, spk, nfe)
    assert torch.equal(a, b)
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    with torch.inference_mode():
        G = L.flamed_den_solve_chunk(hip.handle, nfe)
        r = torch.arange(nfe, device=DEV)
        mods = hip.adaln(ts[:nfe], spk.to(DEV), r.to(torch.int32), torch.zeros(nfe, dtype=torch.int32, device=DEV))
        x = x0.to(DEV).contiguous()
        ws = nat.Workspace().get(L.flamed_den_workspace_size(hip.handle, 1, 300), DEV)
        runs0 = _runs(pg)
        for s0, s1 in ((0, G), (G, nfe)):
            nat.check(L.flamed_den_solve_part(hip.handle, nat.ptr(x), nat.ptr(mods), nfe, 1, 300, nat.ptr(ws), ws.numel(),
                                              1, s0, s1, nat.stream_ptr(DEV)), "flamed_den_solve_part")
        torch.cuda.synchronize()
    assert _runs(pg) == runs0 + 2
    assert torch.equal(x.cpu(), a)


def test_persist_knob_off_uses_launch_path(pgb):
    pg, _ = pgb
    x0, spk = _inputs(7, 1, 64)
    _solve(pg, x0, spk, 4)
    r0 = _runs(pg)
    with knob("persist", 0, 1):
        _solve(pg, x0, spk, 4)
    assert _runs(pg) == r0
    x2, spk2 = _inputs(8, 2, 64)  # B = 2 with persist_multi off: the graph of launches
    with knob("persist_multi", 0, 1):
        _solve(pg, x2, spk2, 4)
    assert _runs(pg) == r0
    x3, spk3 = _inputs(9, 3, 64)  # B = 3 with persist_pad off (not 2 / 4 / 8): the graph of launches
    with knob("persist_pad", 0, 1):
        _solve(pg, x3, spk3, 4)
    assert _runs(pg) == r0
    x9, spk9 = _inputs(10, 9, 64)  # B = 9: beyond 8 row groups, never persistent
    _solve(pg, x9, spk9, 4)
    assert _runs(pg) == r0
    x5, spk5 = _inputs(11, 5, 500)  # B = 5 padded to 8 would need eight chunks (> persist_pad_ntw): graph of launches
    _solve(pg, x5, spk5, 4)
    assert _runs(pg) == r0
    x5, spk5 = _inputs(12, 5, 300)  # ... and five (> persist_pad_ntw 4): graph of launches too
    _solve(pg, x5, spk5, 4)
    assert _runs(pg) == r0
    x5, spk5 = _inputs(13, 5, 200)  # four chunks: persistent
    _solve(pg, x5, spk5, 4)
    assert _runs(pg) == r0 + 1


PERSIST_DEFAULT = 885322  # flamed_tune persist_opt default (csrc/common.hpp Tune::persist_opt)
NTW_DEFAULT, MULTI_NTW_DEFAULT = 8, 8  # flamed_tune persist_ntw / persist_multi_ntw defaults


@pytest.mark.parametrize("part", [0, 2])
@pytest.mark.parametrize("T", [400, 131, 16])
@pytest.mark.parametrize("flip", [64, 512, 64 | 512 | 1, 4096, 16384, 32768, 65536])
def test_persist_variants_bitwise(pgb, T, flip, part):
    """Hand-off variants change where and how data moves, never the arithmetic: the default equals, bitwise,
    the default with row-major instead of fragment-major A images (bit 64), counter-based instead of
    tagged-granule GroupNorm exchange (bit 512), both plus the other weight-DMA wave split (bit 1), the
    hand-off drain issued behind the next weight DMA (bit 4096), the seal verification modes (bit 16384:
    every group wait also checks the producers' hand-off seals; bit 65536: the same seals loaded with the
    phase's operands and checked a phase later), wave-local staging order (bit 32768), for full, partial-tile
    and nearly-empty
    row groups (rows past a group's end are stored as zeros; empty groups add nothing to the GroupNorm) -- under
    both row partitions (part: persist_opt bit 2 flipped from the default, equal shares vs whole 16-row tiles; the
    two partitions differ from each other at the rounding level, the variants within one must not)."""
    pg, _ = pgb
    x0, spk = _inputs(11, 1, T)
    base = PERSIST_DEFAULT ^ part
    r0 = _runs(pg)
    with knob("persist_opt", base, PERSIST_DEFAULT):
        a = _solve(pg, x0, spk, 8)
    with knob("persist_opt", base ^ flip, PERSIST_DEFAULT):
        b = _solve(pg, x0, spk, 8)
    assert _runs(pg) == r0 + 2
    assert torch.equal(a, b)


def test_persist_enqueue_is_async(pgb):
    """The C-ABI contract (include/flamed_hip.h conventions; SURVEY.md §8(b) threading row): the persistent solve
    is only enqueued.  Two back-to-back configs[1] solves return to the host while the device is still busy
    (no hipStreamSynchronize on the call path), and both give the same (deterministic) result -- with the Python
    wrapper's failure check ON: it records each launch and decides it later (settle), so the
    wrapper enqueues only, and a settle after the device is idle finds both launches succeeded (no re-run)."""
    from flamed.models.synthesizer.prob_generator import DenoiserHIP
    pg, _ = pgb
    hip = DenoiserHIP(pg.denoiser, "bf16")
    assert hip.check_persist
    x0, spk = _inputs(21, 1, 400)
    ts = torch.linspace(0, 1, 129, device=DEV)
    xd, sd_ = x0.to(DEV), spk.to(DEV)
    import time
    with torch.inference_mode():
        hip.solve(xd, ts, sd_, 128)  # warm: buffers, workspace, modulation table
        torch.cuda.synchronize()
        r0 = hip.persist_status()[0]
        t0 = time.perf_counter()
        a = hip.solve(xd, ts, sd_, 128)
        b = hip.solve(xd, ts, sd_, 128)
        host_ms = (time.perf_counter() - t0) * 1e3
        pending = not torch.cuda.current_stream().query()
        torch.cuda.synchronize()
    dev_ms = hip.persist_times(2)
    print(f"two persistent solves: host {host_ms:.2f} ms to enqueue, device {dev_ms} ms, pending after enqueue: {pending}")
    assert hip.persist_status()[0] == r0 + 2
    assert len(dev_ms) == 2 and host_ms < dev_ms[0]
    assert pending
    assert len(hip._pending) >= 1  # the second solve's check is still pending (the first may have been settled)
    assert hip.settle() == 0 and not hip._pending
    assert torch.equal(a, b) and torch.isfinite(a).all()


def test_persist_failure_poisons_and_retry_budget(pgb):
    """A persistent launch that gives up (forced by the diagnostic knob persist_inject: every workgroup abandons
    at that step) leaves NaN in x instead of a silently wrong result and is counted; the handle keeps the
    persistent path for 3 failures, then uses the graph of launches, whose result equals the launch path's.
    A fresh handle, so the module's shared handle stays on the persistent path."""
    from flamed.models.synthesizer.prob_generator import DenoiserHIP
    pg, _ = pgb
    h = DenoiserHIP(pg.denoiser, "bf16")
    h.check_persist = False  # the C-ABI behaviour itself (the wrapper's re-run: test_persist_failure_rerun_by_wrapper)
    x0, spk = _inputs(22, 1, 96)
    ts = torch.linspace(0, 1, 9, device=DEV)
    with torch.inference_mode():
        with knob("persist_inject", 3, -1):
            for k in range(1, 4):
                out = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)
                assert torch.isnan(out).all(), "a failed persistent solve must be NaN-poisoned"
                assert h.persist_fails() == k
        runs, broken = h.persist_info()
        assert runs == 3 and broken, (runs, broken)
        ok = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)
        assert h.persist_info()[0] == 3, "after the retry budget the handle must not launch persistently"
        with knob("persist", 0, 1):
            ref = pg.denoiser.hip().solve(x0.to(DEV), ts, spk.to(DEV), 8)
    assert torch.isfinite(ok).all() and torch.equal(ok, ref)


def test_persist_single_failure_then_recovers(pgb):
    """One failure is reported (fails = 1, not broken) and the next solve on the same handle is persistent and
    correct (it equals a solve on a handle that never failed)."""
    from flamed.models.synthesizer.prob_generator import DenoiserHIP
    pg, _ = pgb
    h = DenoiserHIP(pg.denoiser, "bf16")
    h.check_persist = False
    x0, spk = _inputs(23, 1, 131)
    ts = torch.linspace(0, 1, 9, device=DEV)
    with torch.inference_mode():
        with knob("persist_inject", 0, -1):
            bad = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)
        assert torch.isnan(bad).all()
        good = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)
        ref = pg.denoiser.hip().solve(x0.to(DEV), ts, spk.to(DEV), 8)
    runs, broken = h.persist_info()
    assert h.persist_fails() == 1 and not broken and runs == 2
    assert torch.equal(good, ref)


def test_persist_failure_rerun_by_wrapper(pgb):
    """ADVICE r4 / VERDICT r5 weak #7: the Python solve never lets a failed persistent launch reach the caller's
    sync point.  With the wrapper's check on (the default), a solve whose launch fails (persist_inject) is recorded
    without a wait; settle() (what Flamed.sample_batch calls at its own synchronisation, and what the handle's next
    call does without blocking) finds the launch's own error word set, warns, and re-runs it on the graph of
    launches (use_graph bit 2) into the tensor solve returned: the result is finite and equals the launch path
    bitwise, and the failure is still counted."""
    import warnings
    from flamed.models.synthesizer.prob_generator import DenoiserHIP
    pg, _ = pgb
    h = DenoiserHIP(pg.denoiser, "bf16")
    x0, spk = _inputs(27, 1, 120)
    ts = torch.linspace(0, 1, 9, device=DEV)
    with torch.inference_mode():
        with warnings.catch_warnings(record=True) as wl:
            warnings.simplefilter("always")
            with knob("persist_inject", 2, -1):
                out = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)
            assert len(h._pending) == 1
            assert h.settle() == 1 and not h._pending
        assert any("persistent solve failed" in str(w.message) for w in wl)
        assert h.persist_status()[1] == 1 and h.persist_fails() == 1
        with knob("persist", 0, 1):
            ref = pg.denoiser.hip().solve(x0.to(DEV), ts, spk.to(DEV), 8)
        again = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)  # the handle stays persistent (1 of 3 allowed)
        assert h.settle() == 0  # a later launch is judged on its own error word, not the handle's sticky count
    assert torch.isfinite(out).all() and torch.equal(out, ref)
    assert h.persist_status()[0] == 2 and torch.isfinite(again).all()


def test_persist_graph_capture(pgb):
    """The persistent solve inside a torch.cuda.graph capture (a caller capturing ProbGenerator.sample's solve):
    the cooperative launch is captured, the replay runs it, and the result equals the eager persistent solve
    bitwise."""
    pg, _ = pgb
    hip = pg.denoiser.hip()
    x0, spk = _inputs(24, 1, 257)
    ts = torch.linspace(0, 1, 17, device=DEV)
    xd, sd_ = x0.to(DEV), spk.to(DEV)
    with torch.inference_mode():
        eager = hip.solve(xd, ts, sd_, 16)
        torch.cuda.synchronize()
        r0 = _runs(pg)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hip.solve(xd, ts, sd_, 16)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = hip.solve(xd, ts, sd_, 16)
        assert _runs(pg) == r0 + 2, "the captured solve did not take the persistent path"
        g.replay()
        torch.cuda.synchronize()
        first = out.clone()
        g.replay()
        torch.cuda.synchronize()
    assert torch.equal(first, eager) and torch.equal(out, eager)


def test_solve_part_without_step0_rejected(pgb):
    """a later part of a solve whose step-0 part never ran on the handle (or ran for another shape)
    is rejected instead of reading a stale step counter / uninitialised state."""
    from flamed import _native as nat
    pg, _ = pgb
    hip = pg.denoiser.hip()
    L = nat.lib()
    nfe, T = 32, 77
    x0, spk = _inputs(25, 1, T)
    ts = torch.linspace(0, 1, nfe + 1, device=DEV)
    with torch.inference_mode():
        G = L.flamed_den_solve_chunk(hip.handle, nfe)
        r = torch.arange(nfe, device=DEV)
        mods = hip.adaln(ts[:nfe], spk.to(DEV), r.to(torch.int32), torch.zeros(nfe, dtype=torch.int32, device=DEV))
        x = x0.to(DEV).contiguous()
        ws = nat.Workspace().get(L.flamed_den_workspace_size(hip.handle, 1, T), DEV)
        rc = L.flamed_den_solve_part(hip.handle, nat.ptr(x), nat.ptr(mods), nfe, 1, T, nat.ptr(ws), ws.numel(), 1, G, nfe,
                                     nat.stream_ptr(DEV))
    assert rc == 1001


@pytest.mark.parametrize("bit", [16384, 65536])
def test_persist_seal_mode_cfg1(pgb, bit):
    """the configs[1] solve with every group hand-off sealed: each producer stores
    its hand-off number write-through ahead of the drain that precedes its counter add, and every consumer checks
    the seals of all the producers it reads -- after its counter wait, spinning on a lagging one (bit 16384), or
    loaded with the phase's operands and checked a phase later (bit 65536, no round trip on the chain).  No seal
    may lag its counter (a lag fails the launch with error 4 and NaN), and the result equals the unsealed solve
    bitwise."""
    pg, _ = pgb
    hip = pg.denoiser.hip()
    x0, spk = _inputs(26, 1, 400)
    hip._ensure(torch.device(DEV))  # (a -k selection may start here: load the handle before reading its count)
    f0 = hip.persist_fails()
    with knob("persist_opt", PERSIST_DEFAULT & ~(16384 | 65536), PERSIST_DEFAULT):
        a = _solve(pg, x0, spk, 128)
    with knob("persist_opt", (PERSIST_DEFAULT & ~(16384 | 65536)) | bit, PERSIST_DEFAULT):
        b = _solve(pg, x0, spk, 128)
    assert hip.persist_fails() == f0
    assert torch.isfinite(b).all() and torch.equal(a, b)


@pytest.mark.parametrize("bit", [16384, 65536])
def test_persist_seal_lag_detected(pgb, bit):
    """The seal modes catch a hand-off whose producer did not seal it (diagnostic knob persist_seal_skip: one
    workgroup skips its seal stores in step 3): the launch fails (NaN-poisoned x, failure counted) instead of
    returning a result; without a seal mode the same skip is invisible (the counters alone still complete)."""
    from flamed.models.synthesizer.prob_generator import DenoiserHIP
    pg, _ = pgb
    h = DenoiserHIP(pg.denoiser, "bf16")
    h.check_persist = False
    x0, spk = _inputs(27, 1, 200)
    ts = torch.linspace(0, 1, 9, device=DEV)
    base = PERSIST_DEFAULT & ~(16384 | 65536)
    with torch.inference_mode():
        with knob("persist_opt", base, PERSIST_DEFAULT), knob("persist_seal_skip", 3, -1):
            plain = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)
        assert torch.isfinite(plain).all() and h.persist_fails() == 0
        with knob("persist_opt", base | bit, PERSIST_DEFAULT), knob("persist_seal_skip", 3, -1):
            bad = h.solve(x0.to(DEV), ts, spk.to(DEV), 8)
        assert torch.isnan(bad).all(), "a seal lag must fail the launch"
        assert h.persist_fails() == 1


@pytest.mark.parametrize("part", [0, 2])
@pytest.mark.parametrize("B,T", [(2, 200), (4, 100), (8, 64), (4, 300)])
def test_persist_multi_counter_groupnorm(pgb, B, T, part):
    """ADVICE r4 / VERDICT r5 weak #1: several utterances with the counter-form GroupNorm exchange (persist_opt
    without bit 512): the other utterances' groups are masked entirely (count, mean and M2), so the result equals
    the granule form bitwise and each utterance meets the oracle bar -- under both row partitions (part = bit 2
    flipped).  Round 5 saw the forms part on utterance 0 of B = 4 T = 100 with whole-tile rows (groups of 48 and
    52 frames): each form inlined its own copy of the Chan combine and -ffp-contract=fast fused `mean + d (nb/nn)`
    in one copy only (an ulp at step 0, tools/rowpart_probe.py --dump); both now go through one uncontracted
    gn_finalize."""
    pg, sd = pgb
    x0, spk = _inputs(40 + B, B, T)
    base = PERSIST_DEFAULT ^ part
    with knob("persist_multi", 1, 1), knob("persist_multi_ntw", 5, MULTI_NTW_DEFAULT):
        with knob("persist_opt", base, PERSIST_DEFAULT):
            a = _solve(pg, x0, spk, 8)
        r0 = _runs(pg)
        with knob("persist_opt", base ^ 512, PERSIST_DEFAULT):
            b = _solve(pg, x0, spk, 8)
        assert _runs(pg) == r0 + 1
    errs = [rel_l2(b[u:u + 1], orc.euler_solve(sd, x0[u:u + 1], spk[u:u + 1], 8)) for u in range(B)]
    print(f"persistent B={B} T={T} counter GroupNorm: vs oracle per utterance max {max(errs):.3e}")
    assert torch.isfinite(b).all() and torch.equal(a, b) and max(errs) < BF16_SOLVE


@pytest.mark.parametrize("B,T", [(2, 200), (4, 100), (8, 64), (2, 37)])
def test_persist_multi_utterance(pgb, B, T):
    """the persistent solve for several equal-length utterances (knob persist_multi; each
    utterance's frames split over its 8 / B row groups, so its modulation row, GroupNorm statistics over T and
    zero padding stay its own).  Every utterance against a one-utterance oracle solve (equal lengths: no
    padding coupling; prob_generator.py:439-447) at the bf16 solve bar, and the batch against the graph of
    launches (same bf16 operands, other fp32 order) at 4e-3."""
    pg, sd = pgb
    x0, spk = _inputs(30 + B, B, T)
    with knob("persist_multi", 1, 1):  # the default since round 4 (1.55-1.6x the graph of launches)
        r0 = _runs(pg)
        out = _solve(pg, x0, spk, 8)
        assert _runs(pg) == r0 + 1, "the multi-utterance solve did not take the persistent path"
        with knob("persist", 0, 1):
            launch = _solve(pg, x0, spk, 8)
    assert torch.isfinite(out).all()
    el = rel_l2(out, launch)
    errs = [rel_l2(out[b:b + 1], orc.euler_solve(sd, x0[b:b + 1], spk[b:b + 1], 8)) for b in range(B)]
    print(f"persistent B={B} T={T} 8 steps: vs oracle per utterance max {max(errs):.3e}; vs launch path {el:.3e}")
    assert max(errs) < BF16_SOLVE and el < 4e-3


@pytest.mark.parametrize("B,T", [(3, 256), (3, 100), (5, 64), (6, 100), (7, 48)])
def test_persist_padded_batch(pgb, B, T):
    """VERDICT r5 missing #1: the reference's metadata mode batches 4 utterances and leaves a trailing batch of 1..3
    (synthesize.py:268-291, 344); B = 3 and 5..7 run as the persistent launch of B = 4 / 8 with idle zero utterances
    in the spare row groups (knob persist_pad).  It takes the persistent path; utterances are independent inside
    the kernel (own row groups, GroupNorm statistics, modulation row and zero padding), so the padded solve equals
    BITWISE the first B utterances of the unpadded B = 4 / 8 solve whatever the extra utterances hold; and every
    utterance matches the one-utterance oracle solve at the bf16 bar and the graph of launches at 4e-3."""
    pg, sd = pgb
    Bp = 4 if B == 3 else 8
    xp, spkp = _inputs(60 + B + T, Bp, T)
    x0, spk = xp[:B].clone(), spkp[:B].clone()
    r0 = _runs(pg)
    a = _solve(pg, x0, spk, 8)
    full = _solve(pg, xp, spkp, 8)
    assert _runs(pg) == r0 + 2, "the padded batch did not take the persistent path"
    with knob("persist", 0, 1):
        launch = _solve(pg, x0, spk, 8)
    assert torch.isfinite(a).all() and torch.equal(a, full[:B])
    el = rel_l2(a, launch)
    errs = [rel_l2(a[u:u + 1], orc.euler_solve(sd, x0[u:u + 1], spk[u:u + 1], 8)) for u in range(B)]
    print(f"persistent padded B={B} (as {Bp}) T={T}: vs launch path {el:.3e}, vs oracle per utterance max {max(errs):.3e}")
    assert el < 4e-3 and max(errs) < BF16_SOLVE


@pytest.mark.parametrize("B,T", [(1, 520), (1, 1000), (1, 2400), (2, 400), (4, 300), (2, 1111),
                                 (1, 3000), (4, 800), (3, 800), (4, 1024), (8, 500)])
def test_persist_multi_chunk(pgb, B, T):
    """the persistent solve beyond 64 frames per row group -- each group's rows as up
    to eight 64-frame chunks (one 16-row tile per wave per chunk; a kernel variant per chunk count), so long-form
    utterances (configs[4]: T = 2400), B = 2 at T = 400 and the reference's metadata batch of 4 (3) at T = 800 / 1024
    (six to eight chunks, B x T <= 4096) take one launch.  It must take the persistent path,
    be bitwise deterministic, match the graph of launches (same bf16 operands, other fp32 order) at 4e-3 and
    every utterance the one-utterance oracle solve at the bf16 solve bar (8 steps)."""
    pg, sd = pgb
    x0, spk = _inputs(50 + B + T, B, T)
    r0 = _runs(pg)
    with knob("persist_ntw", 8, NTW_DEFAULT), knob("persist_multi_ntw", 8, MULTI_NTW_DEFAULT):
        a = _solve(pg, x0, spk, 8)
        b = _solve(pg, x0, spk, 8)
    assert _runs(pg) == r0 + 2, "the multi-chunk solve did not take the persistent path"
    with knob("persist", 0, 1):
        launch = _solve(pg, x0, spk, 8)
    assert torch.isfinite(a).all() and torch.equal(a, b)
    el = rel_l2(a, launch)
    errs = [rel_l2(a[u:u + 1], orc.euler_solve(sd, x0[u:u + 1], spk[u:u + 1], 8)) for u in range(B)]
    print(f"persistent multi-chunk B={B} T={T}: vs launch path {el:.3e}, vs oracle per utterance max {max(errs):.3e}")
    assert el < 4e-3 and max(errs) < BF16_SOLVE


@pytest.mark.parametrize("B,T", [(1, 1000), (2, 1111), (4, 800)])
def test_persist_multi_chunk_variants_bitwise(pgb, B, T):
    """The multi-chunk kernel's hand-off variants change data movement only: bitwise equal to the default at
    T = 1000 (two chunks per group), B = 2 T = 1111 (five chunks) and B = 4 T = 800 (seven chunks: gemm_ko whatever
    524288 / 262144 say) for fragment-major off (64), counter-form
    GroupNorm (512), and -- ADVICE r5 -- the multi-chunk defaults against their alternatives: wave-local staging
    order (32768), the default K-outer gemm_ko (every tile per K-step) against the per-chunk gemm() sequence
    (524288 off) and the streamed gemm_multi (524288 and 262144 off) -- same products, same order per tile --,
    deferred seals (65536)."""
    pg, _ = pgb
    x0, spk = _inputs(61 + B, B, T)
    with knob("persist_ntw", 8, NTW_DEFAULT), knob("persist_multi_ntw", 8, MULTI_NTW_DEFAULT):
        a = _solve(pg, x0, spk, 8)
        for flip in (64, 512, 32768, 524288, 524288 | 262144, 65536):
            with knob("persist_opt", PERSIST_DEFAULT ^ flip, PERSIST_DEFAULT):
                r0 = _runs(pg)
                b = _solve(pg, x0, spk, 8)
                assert _runs(pg) == r0 + 1
            assert torch.equal(a, b), flip


@pytest.mark.parametrize("B,T", [(1, 400), (1, 131), (1, 16), (2, 37), (1, 1000), (2, 400)])
def test_persist_row_partition(pgb, B, T):
    """The two row partitions (persist_opt bit 2, an A/B variant measured 2-3 % faster: whole 16-row tiles per
    group; default: equal ceil(T / 8) shares) differ only in which group owns a row, i.e. in the GroupNorm partials' summation order:
    both take the persistent path, agree at 4e-3 and meet the one-utterance oracle solve at the bf16 solve bar."""
    pg, sd = pgb
    x0, spk = _inputs(70 + B + T, B, T)
    r0 = _runs(pg)
    a = _solve(pg, x0, spk, 8)
    with knob("persist_opt", PERSIST_DEFAULT ^ 2, PERSIST_DEFAULT):
        b = _solve(pg, x0, spk, 8)
    assert _runs(pg) == r0 + 2
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    d = rel_l2(a, b)
    errs = [rel_l2(a[u:u + 1], orc.euler_solve(sd, x0[u:u + 1], spk[u:u + 1], 8)) for u in range(B)]
    print(f"row partition B={B} T={T}: tiles vs shares {d:.3e}, vs oracle per utterance max {max(errs):.3e}")
    assert d < 4e-3 and max(errs) < BF16_SOLVE
