"""C-ABI library: loads without a GPU, exports every symbol include/flamed_hip.h declares, and its
host-side argument validation reports errors through flamed_last_error (no GPU work involved)."""
import ctypes
import os
import re

import pytest

from _common import PKG

HDR = os.path.join(os.path.dirname(PKG), "include", "flamed_hip.h")


def declared():
    src = open(HDR).read()
    return re.findall(r"FLAMED_API\s+[\w\s\*]+?\b(flamed_\w+)\s*\(", src)


@pytest.fixture(scope="module")
def lib():
    from flamed import _native
    return _native.lib()


def test_header_declares_entry_points():
    names = declared()
    assert len(names) >= 25
    for n in ("flamed_den_solve", "flamed_pva_flow", "flamed_lr_lengths", "flamed_lr_expand", "flamed_fac_decode"):
        assert n in names


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_bindings_cover_header():
    from flamed import _native
    assert set(declared()) == set(_native.SIGNATURES)


def test_host_side_validation_errors(lib):
    from flamed import _native
    h = ctypes.c_void_p()
    assert lib.flamed_den_create(256, 100, 4, 31, 256, 1, ctypes.byref(h)) == 1001
    assert b"unsupported dims" in lib.flamed_last_error()
    assert lib.flamed_den_create(256, 1024, 4, 7, 256, 1, ctypes.byref(h)) == 1001
    assert b"kernel_size=31" in lib.flamed_last_error()
    assert lib.flamed_den_create(256, 1024, 4, 31, 256, 1, ctypes.byref(h)) == 0
    assert lib.flamed_den_num_weights(h) == 8 + 18 * 4 + 12
    assert lib.flamed_den_destroy(h) == 0
    d = ctypes.c_void_p()
    assert lib.flamed_dur_create(192, 384, 5, ctypes.byref(d)) == 1001
    assert lib.flamed_dur_create(192, 384, 3, ctypes.byref(d)) == 0
    assert lib.flamed_dur_destroy(d) == 0
    f = ctypes.c_void_p()
    ups = (ctypes.c_int * 4)(5, 5, 4, 2)
    assert lib.flamed_fac_create(256, 1024, 4, ups, 1, ctypes.byref(f)) == 0
    assert lib.flamed_fac_num_weights(f) == 208
    assert lib.flamed_fac_destroy(f) == 0
    with pytest.raises(RuntimeError, match="status 1001"):
        _native.check(lib.flamed_den_create(256, 1024, 4, 31, 256, 9, ctypes.byref(h)), "create")
    # prior transformer handle (prior.yaml dims): 22 FFT layers x 16 + 2 + 3 + 1 + 3 + 6 + 2 weights
    pd = [361, 192, 4, 768, 9, 1, 6, 4096, 384, 12, 1536, 3, 1, 2, 8192, 1024, 6, 1, 2, 2, 3, 3, 3]
    pr = ctypes.c_void_p()
    assert lib.flamed_prior_create((ctypes.c_int * len(pd))(*pd), len(pd), ctypes.byref(pr)) == 0
    assert lib.flamed_prior_num_weights(pr) == 2 + 16 * 6 + 3 + 1 + 16 * 2 + 3 + sum(1 + 16 * n for n in pd[17:]) + 2
    assert lib.flamed_prior_encode(pr, None, None, 1, 10, None, None, None, 0, 0, None) == 1001  # not loaded
    assert b"not loaded" in lib.flamed_last_error()
    assert lib.flamed_prior_destroy(pr) == 0
    bad = list(pd)
    bad[2] = 5  # 192 / 5 heads
    assert lib.flamed_prior_create((ctypes.c_int * len(bad))(*bad), len(bad), ctypes.byref(pr)) == 1001
    assert lib.flamed_prior_create((ctypes.c_int * 17)(*pd[:17]), 17, ctypes.byref(pr)) == 1001
    # prompt quantizers + timbre encoder (codec.yaml dims)
    vd = [256, 8, 3, 1, 2, 3, 1024, 1024, 1024, 256, 4, 1024, 5, 4, 5000]
    vq = ctypes.c_void_p()
    assert lib.flamed_vq_create((ctypes.c_int * len(vd))(*vd), len(vd), ctypes.byref(vq)) == 0
    assert lib.flamed_vq_num_weights(vq) == 7 * 6 + 1 + 12 * 4 + 2
    assert lib.flamed_vq_destroy(vq) == 0
    bad = list(vd)
    bad[1] = 16  # codebook_dim
    assert lib.flamed_vq_create((ctypes.c_int * len(bad))(*bad), len(bad), ctypes.byref(vq)) == 1001


DIAG_HDR = os.path.join(os.path.dirname(PKG), "include", "flamed_diag.h")


def test_diag_header_bound_and_separate(lib):
    """Diagnostic probes live in libflamed_diag.so (include/flamed_diag.h, first section), not in the product
    library; the header's "libflamed_hip.so diagnostics" section is exported by the product library, bound in
    HIP_DIAG_SIGNATURES, and kept out of the product contract (flamed_hip.h)."""
    from flamed import _native
    src = open(DIAG_HDR).read()
    probe_src, hip_src = src.split("---- libflamed_hip.so diagnostics ----")
    pat = r"FLAMED_API\s+[\w\s\*]+?\b(flamed_\w+)\s*\("
    names, hip_names = re.findall(pat, probe_src), re.findall(pat, hip_src)
    assert set(names) | {"flamed_last_error"} == set(_native.DIAG_SIGNATURES)
    assert set(hip_names) == set(_native.HIP_DIAG_SIGNATURES)
    assert not (set(names) | set(hip_names)) & set(declared())
    for n in names:
        assert not hasattr(lib, n), f"{n} must not be exported by the product library"
    for n in hip_names:
        assert hasattr(lib, n), f"{n} must be exported by the product library"
    dl = _native.diag_lib()
    for n in names:
        if n not in ("flamed_stamp_buffer", "flamed_persist_stamps", "flamed_persist_gndump", "flamed_pva_stamps"):  # FL_STAMPS build only
            assert hasattr(dl, n), n


def test_tune_validation_and_per_handle_knobs(lib):
    assert lib.flamed_tune(b"no_such_knob", 1) == 1001
    assert b"unknown key" in lib.flamed_last_error()
    assert lib.flamed_tune(b"dma_ns", 5) == 1001
    assert lib.flamed_tune(b"dma_ns", 3) == 0
    h = ctypes.c_void_p()
    assert lib.flamed_den_create(256, 1024, 4, 31, 256, 1, ctypes.byref(h)) == 0
    try:
        assert lib.flamed_den_device(h) == -1  # not loaded yet
        assert lib.flamed_den_tune(h, b"lnfold", 0) == 0
        assert lib.flamed_den_tune(h, b"big_ns", 7) == 1001
        assert lib.flamed_den_tune(None, b"lnfold", 0) == 1001
    finally:
        assert lib.flamed_den_destroy(h) == 0


def test_tune_is_thread_safe(lib):
    """flamed_tune from many threads at once: every call succeeds (the defaults are mutex-guarded)."""
    import threading
    errs = []

    def worker(i):
        for k in range(200):
            rc = lib.flamed_tune(b"graph_steps", 1 + (i * 7 + k) % 64)
            if rc:
                errs.append(rc)
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs
    assert lib.flamed_tune(b"graph_steps", 16) == 0


def test_tracked_handles_released_once(lib):
    """flamed/_native.py track / destroy / the atexit hook: a tracked handle is destroyed exactly once (a later
    __del__ after the exit hook is a no-op), and the exit hook releases what is still alive."""
    from flamed import _native
    h = ctypes.c_void_p()
    assert lib.flamed_den_create(256, 1024, 4, 31, 256, 1, ctypes.byref(h)) == 0
    _native.track(h, "flamed_den_destroy")
    assert int(h.value) in _native._live
    _native.destroy(h, "flamed_den_destroy")
    assert int(h.value) not in _native._live
    _native.destroy(h, "flamed_den_destroy")  # second call: no-op (no double free)
    h2 = ctypes.c_void_p()
    assert lib.flamed_dur_create(192, 384, 3, ctypes.byref(h2)) == 0
    saved = dict(_native._live)  # other tests' live handles stay out of this hook run
    _native._live.clear()
    try:
        _native.track(h2, "flamed_dur_destroy")
        _native._release_all()
        assert not _native._live
        _native.destroy(h2, "flamed_dur_destroy")  # after the hook: no-op
    finally:
        _native._live.update(saved)


def test_persist_ticket_arithmetic_wraps(lib):
    """The persistent solve's reset-prologue tickets (persist.hpp arrive_target / arrive_reached): every launch
    adds 256 to each arrival counter, and the launch base and the reached test stay right across INT_MAX and
    the 32-bit wrap (a signed ticket divided by 256 broke after ~8.4M launches)."""
    tgt, ok = ctypes.c_uint(), ctypes.c_int()

    def q(ticket, cur):
        assert lib.flamed_persist_ticket(ticket % 2**32, cur % 2**32, ctypes.byref(tgt), ctypes.byref(ok)) == 0
        return tgt.value, bool(ok.value)

    for base in (0, 256 * 1000, 2**31 - 256, 2**31, 2**32 - 512, 2**32 - 256):
        for k in (0, 1, 128, 255):  # every workgroup of one launch computes the same target
            t, _ = q(base + k, 0)
            assert t == (base + 256) % 2**32
        assert q(base + 7, base + 255)[1] is False   # 255 of 256 arrived
        assert q(base + 7, base + 256)[1] is True    # all arrived (also when base + 256 wraps to 0)
        assert q(base + 7, base + 300)[1] is True    # the next launch has begun arriving
    # INT_MAX crossing: a launch whose tickets straddle 2^31 still agrees on one target
    assert q(2**31 - 1, 0)[0] == 2**31 and q(2**31 - 256, 0)[0] == 2**31
