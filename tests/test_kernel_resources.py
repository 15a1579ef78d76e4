"""The product kernels' register, scratch and occupancy budgets, read from the gfx950 code object that
libsng.so ships (AMDHSA metadata: .vgpr_count, .agpr_count, .sgpr_count, .private_segment_fixed_size,
.vgpr_spill_count).

Several measured numbers depend on how many wavefronts of a kernel share a SIMD, and that is set by the
compiler's register allocation, not by the source alone:
  - ref_day2_kernel reserves v175 (`asm volatile("v_mov_b32 v175, 0" ::: "v175")`, sng_kernels.hip) so its
    VGPR count is above 512 / 3 and it runs at most two wavefronts per SIMD: 86.9 -> 77.5 us of span
    (profiles/r05_ab_refday_two_wavefronts.txt).  A toolchain that allocated differently, or dropped the
    clobber, would silently bring back the three-per-SIMD placement.
  - the headline step kernel (step_wide_kernel<10, 2, true, false, false>) and config 5's
    (step_wide_kernel<50, 2, true, false, true>) and the device generator (generate_kernel<24, false>) must
    not spill: a spill puts scratch traffic on the step's critical path (round 4's store hazard was the same
    class of silent compiler-dependent change).
A compiler upgrade that moves any of these fails here, on the CPU, before a GPU number moves.

`kernel_resources(path)` also reads any A/B library (tools/diag/variant.sh); profiles/r06_kernel_resources.txt
records this check failing on a build of the current source without the v175 clobber.
"""
import os
import shutil
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "smart-nanogrid-gym_amd", "lib", "libsng.so")
LLVM = "/opt/rocm/lib/llvm/bin"
VGPRS_PER_SIMD_LANE = 512   # gfx950: unified VGPR + AGPR file, 512 per lane of a SIMD
VGPR_GRANULE = 8
MAX_WAVES_PER_SIMD = 8


def waves_per_simd(vgprs, agprs=0):
    """Wavefronts of a kernel a SIMD can hold by registers (gfx950: VGPRs then AGPRs, each block a multiple of
    the allocation granule, out of 512 per lane)."""
    g = VGPR_GRANULE
    regs = (vgprs + g - 1) // g * g + (agprs + g - 1) // g * g
    return min(MAX_WAVES_PER_SIMD, VGPRS_PER_SIMD_LANE // max(regs, g))


def kernel_resources(path, workdir):
    """{mangled kernel name: its AMDHSA metadata dict} of the gfx950 code object inside a HIP shared library."""
    lib = os.path.join(workdir, os.path.basename(path))
    shutil.copy(path, lib)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", lib], check=True, capture_output=True,
                   cwd=workdir)
    objs = [f for f in os.listdir(workdir) if "amdgcn-amd-amdhsa--gfx950" in f]
    assert objs, "no gfx950 code object in " + path
    out = {}
    for f in objs:
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(workdir, f)],
                               check=True, capture_output=True, text=True).stdout.splitlines()
        start = next(i for i, line in enumerate(notes) if line.strip() == "---")
        end = next((i for i in range(start + 1, len(notes)) if notes[i].strip() == "..."), len(notes))
        meta = yaml.safe_load("\n".join(notes[start + 1:end]))
        for k in meta["amdhsa.kernels"]:
            out[k[".name"]] = k
    return out


# (readable name, mangled-name prefix, expected waves per SIMD by registers, SGPR spills at most).  SGPR spills
# go to VGPR lanes (v_writelane / v_readlane), not to scratch; the counts of this build are the ceilings.
def _mangled(kernel, *targs):
    enc = {"true": "Lb1E", "false": "Lb0E"}
    body = "".join(enc[a] if a in enc else f"Li{a}E" for a in targs)
    return f"_ZN3sng{len(kernel)}{kernel}I{body}E"


PINNED = [
    # the headline step (BASELINE config 3): 138 VGPRs today, three wavefronts' worth of registers per SIMD
    # (its 2,048 one-wavefront workgroups sit two per SIMD, tools/stamps.py); no spills
    ("step_wide_kernel<10, 2, true, false, false>", _mangled("step_wide_kernel", 10, 2, "true", "false", "false"), 3, 10),
    # config 5's step: 239 VGPRs, two per SIMD, no spills (the non-packed variants of N = 50 do spill; they
    # run only on injected or reference-RNG days of a 50-charger station)
    ("step_wide_kernel<50, 2, true, false, true>", _mangled("step_wide_kernel", 50, 2, "true", "false", "true"), 2, 26),
    # the device-RNG reset of the headline: 50 VGPRs, the hardware maximum of eight wavefronts per SIMD
    ("generate_kernel<24, false>", _mangled("generate_kernel", 24, "false"), 8, 0),
    ("generate_kernel<96, false>", _mangled("generate_kernel", 96, "false"), 8, 0),
    # the reference-RNG reset: held to two wavefronts per SIMD by the v175 reservation
    ("ref_day2_kernel<24, false, 64>", _mangled("ref_day2_kernel", 24, "false", 64), 2, 0),
]


@pytest.fixture(scope="module")
def resources(tmp_path_factory):
    if not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("ROCm llvm-readelf not installed")
    assert os.path.exists(LIB), "build libsng.so first (make -C smart-nanogrid-gym_amd/csrc)"
    return kernel_resources(LIB, str(tmp_path_factory.mktemp("co")))


def _find(resources, prefix):
    names = [n for n in resources if n.startswith(prefix)]
    assert len(names) == 1, f"{prefix}: {len(names)} kernels match ({names[:3]})"
    return resources[names[0]]


def check_pinned(resources):
    """The list of violations of PINNED in a library's resources (empty = every budget holds)."""
    bad = []
    for label, prefix, waves, sgpr_spills in PINNED:
        k = _find(resources, prefix)
        if k[".private_segment_fixed_size"] != 0 or k.get(".vgpr_spill_count", 0) != 0:
            bad.append(f"{label}: scratch {k['.private_segment_fixed_size']} B, "
                       f"{k.get('.vgpr_spill_count', 0)} VGPR spills")
        if k.get(".sgpr_spill_count", 0) > sgpr_spills:
            bad.append(f"{label}: {k['.sgpr_spill_count']} SGPR spills (into VGPR lanes), at most {sgpr_spills}")
        w = waves_per_simd(k[".vgpr_count"], k.get(".agpr_count", 0))
        if w != waves:
            bad.append(f"{label}: {k['.vgpr_count']} VGPRs -> {w} wavefronts per SIMD, expected {waves}")
    return bad


def test_waves_per_simd_arithmetic():
    assert waves_per_simd(50) == 8 and waves_per_simd(64) == 8 and waves_per_simd(65) == 7
    assert waves_per_simd(138) == 3 and waves_per_simd(168) == 3
    assert waves_per_simd(169) == 2 and waves_per_simd(176) == 2 and waves_per_simd(256) == 2
    assert waves_per_simd(128, 128) == 2


def test_pinned_kernels_budgets(resources):
    bad = check_pinned(resources)
    assert not bad, "; ".join(bad)


def test_ref_day2_reserves_v175(resources):
    """the reference-RNG day kernel's VGPR count stays above 512 / 3 (the v175 reservation),
    in every instantiation the library ships."""
    counts = {n: k[".vgpr_count"] for n, k in resources.items() if n.startswith("_ZN3sng15ref_day2_kernel")}
    assert len(counts) >= 8
    assert min(counts.values()) >= 169 and max(waves_per_simd(v) for v in counts.values()) == 2, counts


def test_every_product_kernel_is_listed(resources):
    """The kernels this test pins exist under exactly these names (a renamed template would skip a pin)."""
    for label, prefix, _, _ in PINNED:
        _find(resources, prefix)
