"""ISA lint for the gfx950 packed-fp32-after-wide-LDS-read pattern (DESIGN.md "dwgn concurrency").

On gfx950 a v_pk_{fma,mul,add}_f32 whose source VGPR pair was written by a 64/96/128-bit LDS read
(ds_read_b64 / ds_read2_b32 / ...) was measured to return a wrong low dword when waves of our fp32-MFMA
GEMMs were co-resident on the CU (tools/conc_dwgn3.py).  This tool disassembles every gfx950 code
object inside libflamed_hip.so and lists, per kernel, the packed-fp32 instructions that read a VGPR last
written by a wide LDS read.  It is a straight-line dataflow scan (a register's tag is its last writer
in program order, control flow ignored), so it is a screen, not a proof.

Result (round 5): the pattern is common in compiler output (attention, GEMM A-loaders, the
persistent solve ...), and every one of those kernels stayed bitwise under the same two-stream test
that broke the packed dwgn conv, so the pattern is necessary for the failure we saw but not sufficient;
the tool is kept to list where it occurs, and the two-stream bitwise tests are the gate.

  python tools/isa_pk_lds_lint.py [path/to/libflamed_hip.so] [--all] [--strict]

With --strict, exit status 1 when a product kernel (anything but the diagnostic dwgn_kernel<..., 0> /
<..., 2> instantiations) carries the pattern.
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
WIDE_LDS = re.compile(r"^ds_read(_b64|_b96|_b128|2_b32|2st64_b32|2_b64|2st64_b64)$")
PK_F32 = re.compile(r"^v_pk_(fma|mul|add)_f32$")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op):
    out = []
    for m in VREG.finditer(op):
        if m.group(3) is not None:
            out.append(int(m.group(3)))
        else:
            out.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def code_objects(so):
    # objcopy rewrites its input file when no output file is given: work on a private copy, never on the library
    # a process may have mapped
    work = tempfile.mkdtemp()
    cp, fb = os.path.join(work, "lib.so"), os.path.join(work, "fatbin")
    shutil.copyfile(so, cp)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", cp, os.path.join(work, "out.so")], check=True)
    data = open(fb, "rb").read()
    shutil.rmtree(work, ignore_errors=True)
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    for i, s in enumerate(starts):
        chunk = data[s:starts[i + 1] if i + 1 < len(starts) else len(data)]
        with tempfile.NamedTemporaryFile(suffix=".bundle", delete=False) as f:
            f.write(chunk)
            bpath = f.name
        opath = bpath + ".o"
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                            f"--input={bpath}", f"--output={opath}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(opath) > 0:
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", opath],
                                 capture_output=True, text=True, check=True).stdout
            yield dis
        for p in (bpath, opath):
            if os.path.exists(p):
                os.unlink(p)


def scan(dis):
    """Yields (kernel, n_pk, n_flagged, first flagged line)."""
    fn, tag, npk, hits, first = None, {}, 0, 0, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if fn is not None:
                yield fn, npk, hits, first
            fn, tag, npk, hits, first = m.group(1), {}, 0, 0, None
            continue
        s = line.strip()
        if fn is None or not s or s.startswith(";") or s.startswith("s_"):
            continue
        s = s.split("//")[0].strip()
        parts = s.split(None, 1)
        op, args = parts[0], (parts[1] if len(parts) > 1 else "")
        ops = [a.strip() for a in args.split(",")] if args else []
        if PK_F32.match(op) and ops:
            npk += 1
            src = [r for o in ops[1:] for r in regs(o)]
            if any(tag.get(r) == "lds" for r in src):
                hits += 1
                if first is None:
                    first = s
        if not ops or op.startswith(("ds_write", "global_store", "buffer_store", "scratch_store", "flat_store")):
            continue
        dst = regs(ops[0]) if ops[0].startswith("v") else []
        kind = "lds" if WIDE_LDS.match(op) else "other"
        for r in dst:
            tag[r] = kind


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    so = args[0] if args else os.path.join(os.path.dirname(__file__), "..", "flamed-tts_amd", "flamed", "_native",
                                             "libflamed_hip.so")
    rows = []
    for dis in code_objects(so):
        rows.extend(scan(dis))
    names = demangle([r[0] for r in rows])
    bad = 0
    for (raw, npk, hits, first), name in zip(rows, names):
        diag = name.startswith("void fl::dwgn_kernel<") and re.search(r", (0|2)>\(", name)
        if hits and not diag:
            bad += 1
        if hits or "--all" in sys.argv:
            print(f"{'DIAG ' if diag else ''}{hits:5d}/{npk:5d}  {name[:150]}")
            if hits and first:
                print(f"             first: {first}")
    print(f"{len(rows)} kernels scanned, {bad} product kernels with packed-fp32 reads of wide-LDS-read VGPRs")
    return 1 if bad and "--strict" in sys.argv else 0


if __name__ == "__main__":
    sys.exit(main())
