"""ctypes binding of the gfx950 C-ABI library (include/flamed_hip.h -> flamed/_native/libflamed_hip.so).

The GPU path REQUIRES this library: every HIP entry point raises RuntimeError when it is missing or
a call fails — there is no silent fallback to PyTorch ops.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLAMED_HIP_LIB") or os.path.join(_HERE, "_native", "libflamed_hip.so")

_lock = threading.Lock()
_lib = None

c_int, c_float, c_size_t, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
P = c_void_p  # device pointers and opaque handles

# name -> (restype, argtypes); mirrors include/flamed_hip.h
SIGNATURES = {
    "flamed_last_error": (ctypes.c_char_p, []),
    "flamed_version": (c_int, []),
    "flamed_den_create": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(P)]),
    "flamed_den_destroy": (c_int, [P]),
    "flamed_den_num_weights": (c_int, [P]),
    "flamed_den_load": (c_int, [P, ctypes.POINTER(P), c_int, P]),
    "flamed_den_mods_stride": (c_int, [P]),
    "flamed_den_adaln_workspace_size": (c_size_t, [P, c_int, c_int]),
    "flamed_den_adaln": (c_int, [P, P, c_int, P, c_int, P, P, c_int, P, P, c_size_t, P]),
    "flamed_den_workspace_size": (c_size_t, [P, c_int, c_int]),
    "flamed_den_velocity": (c_int, [P, P, P, c_int, c_int, c_int, P, P, c_size_t, P]),
    "flamed_den_step": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P, c_size_t, P]),
    "flamed_den_solve": (c_int, [P, P, P, c_int, c_int, c_int, P, c_size_t, c_int, P]),
    "flamed_den_solve_chunk": (c_int, [P, c_int]),
    "flamed_den_persist_info": (c_int, [P, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_float)]),
    "flamed_den_persist_times": (c_int, [P, ctypes.POINTER(c_float), c_int]),
    "flamed_den_persist_status": (c_int, [P, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "flamed_den_persist_last": (c_int, [P, ctypes.POINTER(ctypes.c_longlong)]),
    "flamed_den_persist_query": (c_int, [P, ctypes.c_longlong, ctypes.POINTER(c_int)]),
    "flamed_den_solve_part": (c_int, [P, P, P, c_int, c_int, c_int, P, c_size_t, c_int, c_int, c_int, P]),
    "flamed_den_time_kernels_graph": (c_int, [P, P, P, c_int, c_int, P, c_size_t, c_int, ctypes.POINTER(c_float), P]),
    "flamed_tune": (c_int, [ctypes.c_char_p, c_int]),
    "flamed_den_tune": (c_int, [P, ctypes.c_char_p, c_int]),
    "flamed_den_device": (c_int, [P]),
    "flamed_cond_create": (c_int, [c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(P)]),
    "flamed_cond_destroy": (c_int, [P]),
    "flamed_cond_load": (c_int, [P, ctypes.POINTER(P), c_int, P]),
    "flamed_cond_workspace_size": (c_size_t, [P, c_int, c_int]),
    "flamed_cond_fold": (c_int, [P, P, P, c_int, c_int, P, P, c_size_t, P]),
    "flamed_dur_create": (c_int, [c_int, c_int, c_int, ctypes.POINTER(P)]),
    "flamed_dur_destroy": (c_int, [P]),
    "flamed_dur_load": (c_int, [P, ctypes.POINTER(P), c_int, P]),
    "flamed_pva_workspace_size": (c_size_t, [P, c_int, c_int, c_int]),
    "flamed_pva_flow": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, P, c_size_t, c_int, P]),
    "flamed_pva_persist_info": (c_int, [P, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_float)]),
    "flamed_pva_persist_ready": (c_int, [P, P, c_int, c_int, P]),
    "flamed_pva_persist_status": (c_int, [P, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "flamed_lr_lengths": (c_int, [P, P, P, c_int, c_int, c_int, P, P, P]),
    "flamed_lr_expand": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P]),
    "flamed_fac_create": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_int), c_int, ctypes.POINTER(P)]),
    "flamed_fac_destroy": (c_int, [P]),
    "flamed_fac_num_weights": (c_int, [P]),
    "flamed_fac_load": (c_int, [P, ctypes.POINTER(P), c_int, P]),
    "flamed_fac_workspace_size": (c_size_t, [P, c_int, c_int]),
    "flamed_fac_decode": (c_int, [P, P, P, c_int, c_int, P, P, c_size_t, c_int, P]),
    "flamed_enc_create": (c_int, [c_int, c_int, ctypes.POINTER(c_int), c_int, c_int, ctypes.POINTER(P)]),
    "flamed_enc_destroy": (c_int, [P]),
    "flamed_enc_num_weights": (c_int, [P]),
    "flamed_enc_load": (c_int, [P, ctypes.POINTER(P), c_int, P]),
    "flamed_enc_out_len": (c_int, [P, c_int]),
    "flamed_enc_workspace_size": (c_size_t, [P, c_int, c_int]),
    "flamed_enc_encode": (c_int, [P, P, c_int, c_int, P, P, c_size_t, c_int, P]),
    "flamed_vq_create": (c_int, [ctypes.POINTER(c_int), c_int, ctypes.POINTER(P)]),
    "flamed_vq_destroy": (c_int, [P]),
    "flamed_vq_num_weights": (c_int, [P]),
    "flamed_vq_load": (c_int, [P, ctypes.POINTER(P), c_int, P]),
    "flamed_vq_workspace_size": (c_size_t, [P, c_int, c_int]),
    "flamed_vq_encode": (c_int, [P, P, c_int, c_int, P, P, P, P, P, c_size_t, c_int, P]),
    "flamed_prior_create": (c_int, [ctypes.POINTER(c_int), c_int, ctypes.POINTER(P)]),
    "flamed_prior_destroy": (c_int, [P]),
    "flamed_prior_num_weights": (c_int, [P]),
    "flamed_prior_load": (c_int, [P, ctypes.POINTER(P), c_int, P]),
    "flamed_prior_workspace_size": (c_size_t, [P, c_int, c_int, c_int, c_int]),
    "flamed_prior_encode": (c_int, [P, P, P, c_int, c_int, P, P, P, c_size_t, c_int, P]),
    "flamed_prior_decode": (c_int, [P, P, P, P, c_int, c_int, c_int, P, P, P, P, c_size_t, c_int, P]),
    "flamed_prior_set_dtype": (c_int, [P, c_int]),
}

# include/flamed_diag.h: probes in libflamed_diag.so, phase stamps in libflamed_hip_stamps.so (tools only)
DIAG_LIB_PATH = os.path.join(_HERE, "_native", "libflamed_diag.so")
DIAG_SIGNATURES = {
    "flamed_last_error": (ctypes.c_char_p, []),
    "flamed_probe_gemm": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, ctypes.POINTER(c_float), P]),
    "flamed_probe_empty": (c_int, [c_int, c_int, ctypes.POINTER(c_float), P]),
    "flamed_probe_copy": (c_int, [P, P, c_size_t, c_int, c_int, c_int, ctypes.POINTER(c_float), P]),
    "flamed_probe_gemm_pf": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, ctypes.POINTER(c_float), P]),
    "flamed_probe_stream": (c_int, [c_int, c_int, c_int, c_int, P, ctypes.POINTER(c_float), P]),
    "flamed_probe_mx": (c_int, [P, P, P, P, P, c_int, P]),
    "flamed_probe_mx_gemm": (c_int, [P, P, c_int, c_int, c_int, P, P]),
    "flamed_stamp_buffer": (c_int, [P]),
    "flamed_persist_stamps": (c_int, [P, c_int]),
    "flamed_persist_gndump": (c_int, [P, c_int]),
    "flamed_pva_stamps": (c_int, [P, c_int]),
}
# include/flamed_diag.h, "libflamed_hip.so diagnostics" section: exported by the product library, used by
# tools and tests only
HIP_DIAG_SIGNATURES = {
    "flamed_den_persist_fails": (c_int, [P, ctypes.POINTER(c_int)]),
    "flamed_den_ws_offsets": (c_int, [P, c_int, c_int, ctypes.POINTER(c_size_t)]),
    "flamed_persist_ticket": (c_int, [ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(c_int)]),
    "flamed_den_chain_info": (c_int, [P, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "flamed_den_chain_busy": (c_int, [P, ctypes.POINTER(c_int)]),
}

FLAMED_F32, FLAMED_BF16, FLAMED_FP8 = 0, 1, 2
DTYPES = {"f32": FLAMED_F32, "fp32": FLAMED_F32, "float32": FLAMED_F32, "bf16": FLAMED_BF16, "bfloat16": FLAMED_BF16,
          "fp8": FLAMED_FP8}  # fp8: denoiser handles only (MX-fp8 pointwise GEMMs at large M, bf16 elsewhere)


_live = {}  # address of every handle this process created and has not destroyed -> its destroy function


def track(h, destroy_fn: str):
    """Record a created handle, so that an interpreter exit releases it while the HIP runtime (and any
    profiler attached to it) is still up, instead of leaving its streams / events / graphs / pinned words to
    the runtime's own teardown."""
    with _lock:
        _live[int(h.value)] = destroy_fn
    return h


def destroy(h, destroy_fn: str) -> None:
    """Destroy a tracked handle once (later calls, e.g. a __del__ after the exit hook, are no-ops)."""
    if h is None or not h.value:
        return
    with _lock:
        owned = _live.pop(int(h.value), None)
    if owned is not None:
        getattr(lib(), destroy_fn)(h)


@atexit.register
def _release_all() -> None:
    with _lock:
        items = list(_live.items())
        _live.clear()
    if not items:
        return
    try:
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:
        pass
    for addr, fn in items:
        try:
            getattr(lib(), fn)(ctypes.c_void_p(addr))
        except Exception:
            pass


def lib():
    """Load (once) and return the C-ABI library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"Flamed HIP extension not found at {LIB_PATH}. Build it with "
                    "`make -C flamed-tts_amd/csrc` (or `python -c 'import __graft_entry__ as g; g.build()'`).")
            _lib = _bind(ctypes.CDLL(LIB_PATH), {**DIAG_SIGNATURES, **HIP_DIAG_SIGNATURES, **SIGNATURES})
    return _lib


def _bind(so, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(so, name, None)
        if fn is None:  # e.g. flamed_stamp_buffer exists only in the FL_STAMPS build
            continue
        fn.restype = res
        fn.argtypes = args
    return so


_diag = None


def diag_lib():
    """The diagnostic probe library (tools only; never loaded by the product path)."""
    global _diag
    with _lock:
        if _diag is None:
            if not os.path.exists(DIAG_LIB_PATH):
                raise RuntimeError(f"diagnostic library not found at {DIAG_LIB_PATH} (make -C flamed-tts_amd/csrc diag)")
            _diag = _bind(ctypes.CDLL(DIAG_LIB_PATH), DIAG_SIGNATURES)
    return _diag


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().flamed_last_error()
        raise RuntimeError(f"{what} failed (status {rc}): {msg.decode() if msg else ''}")


_supported = {}


def supported(kind: str, *dims) -> bool:
    """Whether the library specialises a module's dims: runs flamed_<kind>_create (host-only: it
    validates the dims and allocates no device memory) and destroys the handle again.  Ints are passed
    as C ints, tuples as C int arrays.  The answer is cached per (kind, dims).  A module whose dims are
    not specialised keeps its own torch ops on ROCm (as before the HIP path existed); a MISSING library
    still raises (lib())."""
    key = (kind,) + tuple(tuple(d) if isinstance(d, (list, tuple)) else int(d) for d in dims)
    hit = _supported.get(key)
    if hit is not None:
        return hit
    L = lib()
    args = [(ctypes.c_int * len(d))(*d) if isinstance(d, tuple) else ctypes.c_int(d) for d in key[1:]]
    h = ctypes.c_void_p()
    ok = getattr(L, f"flamed_{kind}_create")(*args, ctypes.byref(h)) == 0
    if ok and h.value:
        getattr(L, f"flamed_{kind}_destroy")(h)
    if not ok:
        import warnings
        msg = L.flamed_last_error()
        warnings.warn(f"flamed HIP library does not specialise these {kind} dims ({msg.decode() if msg else ''}); "
                      "the module runs on its torch ops")
    _supported[key] = ok
    return ok


def ptr(t: torch.Tensor | None):
    if t is None:
        return None
    return c_void_p(t.data_ptr())


def stream_ptr(device: torch.device | None = None):
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def dtype_code(name: str) -> int:
    try:
        return DTYPES[name]
    except KeyError as e:
        raise ValueError(f"unknown HIP compute dtype {name!r}; use one of {sorted(DTYPES)}") from e


class Workspace:
    """Grow-only device scratch buffer (stable pointer between calls of the same size)."""

    def __init__(self):
        self.buf = None

    def get(self, nbytes: int, device) -> torch.Tensor:
        nbytes = max(int(nbytes), 256)
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != torch.device(device):
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        return self.buf


def tensor_version(t: torch.Tensor) -> int:
    """In-place version counter of a weight tensor, used to detect weight updates between calls.
    Inference tensors (created under torch.inference_mode) have no counter; they are reported as -1
    and identified by their data pointer alone."""
    try:
        return t._version
    except RuntimeError:
        return -1
