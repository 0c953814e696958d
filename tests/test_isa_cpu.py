"""ISA guard for the round-5 dwgn fix (DESIGN.md "dwgn concurrency"): in the shipped gfx950 code objects the default
(scalar pair math, VAR 1) depthwise conv + GroupNorm kernels carry (almost) no packed-fp32 instructions fed by 64-bit
LDS reads -- the pattern that was perturbed by co-resident fp32-MFMA waves -- while the diagnostic packed variant
(VAR 0) still shows it, so the screen (tools/isa_pk_lds_lint.py) is known to see it.  CPU only: disassembles
libflamed_hip.so, no GPU call."""
import importlib.util
import os
import re
import shutil

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "flamed-tts_amd", "flamed", "_native", "libflamed_hip.so")
LINT = os.path.join(REPO, "tools", "isa_pk_lds_lint.py")


def _lint():
    spec = importlib.util.spec_from_file_location("isa_pk_lds_lint", LINT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.skipif(not os.path.exists(SO) or shutil.which("objcopy") is None
                    or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built library and the ROCm disassembler")
def test_dwgn_default_has_no_packed_fp32_after_wide_lds_reads():
    lint = _lint()
    rows = []
    for dis in lint.code_objects(SO):
        rows.extend(lint.scan(dis))
    pat = re.compile(r"dwgn_kernelILb[01]ELi(\d)E(?:DF16b|f)Li(\d)EEEv")
    seen = {0: [], 1: [], 2: []}
    small = []
    for name, npk, hits, _ in rows:
        m = pat.search(name)
        if m:
            seen[int(m.group(2))].append((name, hits, npk))
        elif "dwgn_small_kernel" in name:
            small.append((name, hits, npk))
    assert seen[1] and seen[0] and small, "dwgn instantiations not found in the code objects"
    for name, hits, npk in seen[1] + small:
        assert hits <= 8, f"{name}: {hits} of {npk} packed-fp32 ops read wide-LDS-read VGPRs"
    for name, hits, npk in seen[0]:
        assert hits >= 100, f"diagnostic packed variant {name}: only {hits} flagged (the screen lost the pattern)"
