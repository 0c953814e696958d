"""ISA guard for the packed-fp32 hazard (DESIGN.md "packed fp32"): round 5 found a v_pk_fma_f32 fed by a 64-bit LDS
read returning a wrong low dword while fp32-MFMA waves of another kernel shared the CU (dwgn_kernel, two-stream
test).  Round 6 removes the pattern library-wide instead of kernel by kernel: the device code is built without the
packed-fp32 target feature (csrc/Makefile PKOFF), so no shipped code object may hold a v_pk_{fma,mul,add}_f32 at all --
in particular none fed by a wide LDS read (tools/isa_pk_lds_lint.py).  CPU only: disassembles the built libraries, no
GPU call."""
import importlib.util
import os
import shutil

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(REPO, "flamed-tts_amd", "flamed", "_native")
SO = os.path.join(NATIVE, "libflamed_hip.so")
LINT = os.path.join(REPO, "tools", "isa_pk_lds_lint.py")
needs_tools = pytest.mark.skipif(not os.path.exists(SO) or shutil.which("objcopy") is None
                                 or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                                 reason="needs the built library and the ROCm disassembler")


def _lint():
    spec = importlib.util.spec_from_file_location("isa_pk_lds_lint", LINT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _rows(so):
    lint = _lint()
    rows = []
    for dis in lint.code_objects(so):
        rows.extend(lint.scan(dis))
    return rows


@needs_tools
@pytest.mark.parametrize("name", ["libflamed_hip.so", "libflamed_hip_stamps.so"])
def test_no_packed_fp32_in_shipped_code_objects(name):
    so = os.path.join(NATIVE, name)
    if not os.path.exists(so):
        pytest.skip(f"{name} not built")
    rows = _rows(so)
    assert len(rows) > 100, "kernels not found in the code objects"
    kernels = {r[0] for r in rows}
    assert any("den_persist_kernel" in k for k in kernels) and any("dwgn_kernel" in k for k in kernels)
    packed = [(k, npk) for k, npk, hits, _ in rows if npk]
    assert not packed, f"{len(packed)} kernels carry packed-fp32 ops, e.g. {packed[:3]}"
