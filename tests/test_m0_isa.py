"""ISA check of the inline-asm LDS-DMA: two kernel files issue ``s_mov_b32 m0`` +
``buffer_load_dwordx4 ... lds`` from inline asm (csrc/dadmm_stream.hip dma16, and the A^T ring
of dadmm_fused.hip in both its builds). m0 is a register the compiler reserves, so the clobber is only safe while
no compiler-generated instruction relies on an m0 value set before one of those asm blocks.

The test compiles the device code of each file (the Makefile's flags, --cuda-device-only -S) and
checks, per function: every m0 write inside an asm block is followed in the same block by an LDS
DMA; every compiler-generated m0 reader (an LDS DMA from a builtin, movrel, sendmsg, GWS, ...) has
a compiler m0 write after the last asm m0 write and after the last branch target before it (a
loop back-edge could otherwise carry an asm-clobbered m0 into it). CPU only (hipcc cross-compile).
"""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "hyperparameter-gnn_unfolded-d-admm-main_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-slp-vectorize", "-mllvm", "-pragma-unroll-threshold=1000000"]
READERS = re.compile(r"\b(s_movrel|v_movrel|s_sendmsg|ds_gws|ds_ordered|v_interp|ds_\w+_addtid|"
                     r"global_load_lds|s_ttracedata)|\blds\s*$")


def _asm(src, tmp_path, defs=()):
    # the build's own assembly (csrc/Makefile ASMCHK) when it is up to date, else compile it here
    name = "dadmm_fused_rec.s" if defs else src.replace(".hip", ".s")
    built = os.path.join(CSRC, "build", name)
    if os.path.exists(built) and os.path.getmtime(built) >= os.path.getmtime(os.path.join(CSRC, src)):
        with open(built) as f:
            return f.read().splitlines()
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC, *FLAGS, *defs, "-x", "hip", "--cuda-device-only", "-S",
                    os.path.join(CSRC, src), "-o", str(out)], check=True,
                   capture_output=True, text=True, timeout=600)
    return out.read_text().splitlines()


def check_m0(lines):
    """[] when the invariant holds, else the violations (function, line, text)."""
    bad = []
    fn, in_asm, last, pending = None, False, None, None
    for i, raw in enumerate(lines):
        t = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            if pending is not None:
                bad.append((fn, pending, "asm m0 write without an LDS DMA in the same block"))
                pending = None
            in_asm = False
            continue
        if not t:
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:", t):
            if not t.startswith(".L") and not t.startswith("$"):
                fn, last = t[:-1], None
            else:
                last = None if last == "compiler" else last or None
                last = "label"
            continue
        if t.startswith("."):
            continue
        writes_m0 = re.match(r"^\S+\s+m0\s*,", t) is not None
        reads_m0 = READERS.search(t) is not None or (re.search(r"\bm0\b", t) is not None and not writes_m0)
        if in_asm:
            if writes_m0:
                pending = i
                last = "asm"
            elif reads_m0 and pending is not None and " lds" in t:
                pending = None
            continue
        if reads_m0 and last != "compiler":
            bad.append((fn, i + 1, t))
        if writes_m0:
            last = "compiler"
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,defs", [("dadmm_stream.hip", ()), ("dadmm_fused.hip", ()),
                                      ("dadmm_fused.hip", ("-DDADMM_FUSED_REC=1",))])
def test_inline_asm_m0_is_not_relied_on(tmp_path, src, defs):
    lines = _asm(src, tmp_path, defs)
    assert any("m0" in ln for ln in lines)
    assert check_m0(lines) == []


def test_checker_catches_a_reused_m0():
    """The checker itself: a compiler LDS DMA after an asm m0 write without a fresh compiler
    write is flagged; a fresh write makes it pass."""
    body = ["kern:", ";;#ASMSTART", "s_mov_b32 m0, s4", "buffer_load_dwordx4 v1, s[0:3], 0 offen lds",
            ";;#ASMEND", "buffer_load_dword v2, s[0:3], 0 offen lds"]
    assert check_m0(body) != []
    ok = body[:5] + ["s_mov_b32 m0, s5"] + body[5:]
    assert check_m0(ok) == []
    loop = ["kern:", "s_mov_b32 m0, s5", ".LBB0_1:", "buffer_load_dword v2, s[0:3], 0 offen lds",
            ";;#ASMSTART", "s_mov_b32 m0, s4", "buffer_load_dwordx4 v1, s[0:3], 0 offen lds",
            ";;#ASMEND", "s_cbranch_scc1 .LBB0_1"]
    assert check_m0(loop) != []
