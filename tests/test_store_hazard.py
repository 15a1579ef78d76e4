"""ISA check of a gfx950 store-data hazard, on the built libsng.so.

A vector-memory store of more than 8 B (buffer/global/flat _store_dwordx3/x4) reads its data VGPRs late, so a
VALU that writes one of them must wait 2 wait states (an s_nop k counts k + 1, any other instruction 1).
ROCm 7.2's LLVM inserts that wait for FLAT/global stores and for MUBUF stores whose soffset is an inline
constant, but not for MUBUF stores with an SGPR soffset, which it believes safe.  On gfx950 they are not:
round 4's first SoC-pair build lost the high dword of ~0.1 % of the stored SoC slots at 65,536 envs to a
v_cvt_f32_ubyte2 that overwrote the pair right after its store (134 such pairs in the library).  Every wide
raw-buffer store now passes a literal 0 soffset (bst2, sng_kernels.hip), and this test disassembles the
gfx950 code object the library ships -- compiler-emitted stores included -- and finds every wide store
followed, within its wait states and before any branch, by a VALU writing one of its data VGPRs.

`scan_library` also runs on any other build (tools/diag A/B libraries): on the pre-fix commit 12a6381^ it
reports the hazard pairs (profiles/r05_store_hazard_isa.txt)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "smart-nanogrid-gym_amd", "lib", "libsng.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
WAIT_STATES = 2   # gfx940+ (gfx950): a VALU write of a wide store's data VGPRs

_STORE = re.compile(r"^\s*(buffer|global|flat)_store_dwordx([34])\s+(.*?)\s*(//.*)?$")
_INSN = re.compile(r"^\s+([a-z_][a-z0-9_]*)\s*(.*?)\s*(//.*)?$")
_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def _vgprs(op):
    """VGPR numbers named by one operand text (v7, v[4:7])."""
    out = set()
    for m in _VREG.finditer(op):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _operands(text):
    return [x.strip() for x in text.split(",")] if text else []


def scan_listing(lines):
    """Hazards in an llvm-objdump listing: (store line, follower line) pairs.  A store's window ends after
    WAIT_STATES wait states, at a branch, or at the end of its function."""
    hazards, stores = [], 0
    for i, line in enumerate(lines):
        m = _STORE.match(line)
        if not m:
            continue
        stores += 1
        kind, ops = m.group(1), _operands(m.group(3))
        data = _vgprs(ops[1] if kind in ("global", "flat") else ops[0])   # global: vaddr, vdata, saddr
        waited = 0
        for nxt in lines[i + 1:i + 16]:
            mi = _INSN.match(nxt)
            if not mi or nxt.strip().endswith(":") or nxt.startswith("0"):   # a label or a function symbol
                break
            op, args = mi.group(1), _operands(mi.group(2))
            if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                break
            if op.startswith("v_") and args and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
                if _vgprs(args[0]) & data:
                    hazards.append((line.strip(), nxt.strip()))
            waited += int(args[0]) + 1 if op == "s_nop" else 1
            if waited >= WAIT_STATES:
                break
    return hazards, stores


def scan_library(path, workdir):
    """Extract the gfx950 code object of a HIP shared library and scan its disassembly."""
    lib = os.path.join(workdir, os.path.basename(path))
    shutil.copy(path, lib)
    subprocess.run([OBJDUMP, "--offloading", lib], check=True, capture_output=True, cwd=workdir)
    objs = [f for f in os.listdir(workdir) if "amdgcn-amd-amdhsa--gfx950" in f]
    assert objs, "no gfx950 code object in " + path
    hazards, stores = [], 0
    for f in objs:
        listing = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", os.path.join(workdir, f)], check=True,
                                 capture_output=True, text=True).stdout.splitlines()
        h, n = scan_listing(listing)
        hazards += h
        stores += n
    return hazards, stores


def test_scanner_finds_the_round4_pattern():
    """The faulting pair of round 4 (an SGPR soffset, then a VALU writing the pair's high dword) is found; the
    fixed form (literal 0 soffset, then the compiler's s_nop 1) and a write of the address VGPR are not."""
    bad = ["\tbuffer_store_dwordx4 v[44:47], v56, s[80:83], s12 offen nt   // 000000061D04: E07E1000",
           "\tv_cvt_f32_ubyte2_e32 v47, v20                                 // 000000061D0C: 7E5E2514"]
    good = ["\tbuffer_store_dwordx4 v[44:47], v56, s[80:83], 0 offen nt   // 000000061D04: E07E1000",
            "\ts_nop 1                                                    // 000000061D0C: BF800001",
            "\tv_mul_f32_e32 v44, 0x3d2aaaab, v43                         // 000000061D10: 0A5856FF"]
    addr = ["\tbuffer_store_dwordx4 v[48:51], v34, s[88:91], 0 offen nt   // 00000005BD74: E07E1000",
            "\tv_mul_f32_e32 v34, 0x3d2aaaab, v31                         // 00000005BD7C: 0A443EFF"]
    glob = ["\tglobal_store_dwordx3 v[0:1], v[6:8], off offset:-8         // 0000000546D0: DC789FF8",
            "\tv_mov_b32_e32 v7, 0                                        // 0000000546D8: 7E0E0280"]
    assert len(scan_listing(bad)[0]) == 1
    assert scan_listing(good)[0] == [] and scan_listing(addr)[0] == []
    assert len(scan_listing(glob)[0]) == 1


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="ROCm llvm-objdump not installed")
def test_no_wide_store_data_hazard_in_libsng(tmp_path):
    assert os.path.exists(LIB), "build libsng.so first (make -C smart-nanogrid-gym_amd/csrc)"
    hazards, stores = scan_library(LIB, str(tmp_path))
    assert stores > 100, f"only {stores} wide stores found: is the listing parsed?"
    assert not hazards, f"{len(hazards)} wide stores with a VALU write of their data inside the wait window: " + \
        "; ".join(f"{a} -> {b}" for a, b in hazards[:5])
