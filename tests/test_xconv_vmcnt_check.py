"""scripts/check_xconv_vmcnt.py (run by make) against a known-bad build.

xconv3_kernel's stage waits are exact vmcnt(N) counts of the vector-memory
instructions the template expects after a weight LDS-DMA.  Round 5's race
came from a count the emitted code contradicted (hipcc deleted counted
loads).  This builds one instantiation (48 -> 48, the
dominant layer) twice on the CPU -- as shipped, and with XCONV_DEAD_LOAD_PROBE,
which restores round 5's count -- and requires the check to pass the first
and fail the second at the stage whose loads it miscounts.  No GPU needed:
hipcc cross-compiles gfx950 and the schedule comes from host code.
"""
import glob
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
PROBE = ["-DXCONV_ISA_PROBE=48", "-DXCONV_PROBE_BN=48", "-DXCONV_PROBE_NRES=0", "-DXCONV_PROBE_RW=2",
         "-DXCONV_PROBE_KS=3"]


def _build(tmp, name, extra):
    """The probe's object and a library of it plus the other kernels' objects
    (the probe's host code calls into them)."""
    obj, lib = os.path.join(tmp, name + ".o"), os.path.join(tmp, name + ".so")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", *PROBE,
                    *extra, "-c", "-o", obj, os.path.join(REPO, "dcvc_amd/csrc/hip/xconv.hip")],
                   check=True, capture_output=True, timeout=600)
    others = [o for o in sorted(glob.glob(os.path.join(REPO, "build/hip/*.o"))) if not o.endswith("/xconv.o")]
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, obj, *others],
                   check=True, capture_output=True, timeout=600)
    return lib, obj


def _check(lib, obj):
    return subprocess.run([sys.executable, os.path.join(REPO, "scripts/check_xconv_vmcnt.py"), lib, obj],
                          capture_output=True, text=True, timeout=300)


@pytest.fixture(scope="module")
def toolchain():
    if not (os.path.exists(HIPCC) and shutil.which("python3")):
        pytest.skip("hipcc not present")
    if len(glob.glob(os.path.join(REPO, "build/hip/*.o"))) < 2:
        pytest.skip("build/hip objects not built (make hip)")


def test_shipped_probe_passes(toolchain, tmp_path):
    r = _check(*_build(str(tmp_path), "ok", []))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "1 xconv3_kernel instantiations match" in r.stdout


def test_dead_load_count_fails(toolchain, tmp_path):
    r = _check(*_build(str(tmp_path), "dead", ["-DXCONV_DEAD_LOAD_PROBE"]))
    assert r.returncode == 1, r.stdout + r.stderr
    # the tile's first stages load the 16-channel last chunk: 2 pieces (4
    # loads) emitted, round 5's count assumed 3 (6)
    assert "vector-memory instructions DLLLLD, the vmcnt schedule assumes DLLLLLLD" in r.stderr, r.stderr


def test_built_wconv_matches_its_schedule(toolchain):
    """wconv.hip's DMA wave (the only waves that issue LDS-DMAs and wait with
    exact vmcnt counts) in the built library: every instantiation's DMA loop
    issues exactly the schedule dcvc_internal_wconv_schedule reports."""
    lib = os.path.join(REPO, "dcvc_amd/lib/libdcvc_hip.so")
    obj = os.path.join(REPO, "build/hip/wconv.o")
    if not (os.path.exists(lib) and os.path.exists(obj)):
        pytest.skip("library not built (make hip)")
    r = _check(lib, obj)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "16 wconv3_kernel instantiations match" in r.stdout


def _sffn_listing():
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import check_xconv_vmcnt as c
    obj = os.path.join(REPO, "build/hip/sffn.o")
    if not os.path.exists(obj):
        pytest.skip("sffn.o not built (make hip)")
    return c.disassemble(obj)


def _check_listing(tmp_path, text):
    s = tmp_path / "sffn.s"
    s.write_text(text)
    return _check(os.path.join(REPO, "dcvc_amd/lib/libdcvc_hip.so"), str(s))


def test_built_sffn_waits_for_each_slice(toolchain, tmp_path):
    """sffn.hip's streamed kernels (C = 128: slices through four LDS buffers,
    exact vmcnt waits): on every path to each barrier, the DMA the barrier
    waits for has at least vmcnt(N) younger vector-memory instructions."""
    r = _check_listing(tmp_path, _sffn_listing())
    assert r.returncode == 0, r.stdout + r.stderr
    assert "3 streamed sffn_kernel instantiations wait for each slice's DMA" in r.stdout


def test_sffn_check_catches_a_lax_wait(toolchain, tmp_path):
    """B_1 / B_2 of sffn_kernel<128, 4, 1, 4> wait vmcnt(NDW + PFN) = 16; 17
    would let the slice's last DMA instruction still be in flight."""
    text = _sffn_listing().replace("s_waitcnt vmcnt(16) lgkmcnt(0)", "s_waitcnt vmcnt(17) lgkmcnt(0)")
    r = _check_listing(tmp_path, text)
    assert r.returncode == 1, r.stdout + r.stderr
    assert "sffn_kernel<128,4,1,4>" in r.stderr and "vmcnt(17)" in r.stderr, r.stderr


def test_sffn_check_catches_a_hoisted_prefetch(toolchain, tmp_path):
    """The next tile's input prefetch moved above B_0's slice DMA (what hipcc
    could do: the two are independent): B_2's vmcnt(NDW + PFN) then no longer
    covers slice 2's DMA, and the check says so."""
    lines = _sffn_listing().splitlines()
    start = next(i for i, ln in enumerate(lines) if "sffn_kernelILi128ELi4ELi1ELi4E" in ln and ln.endswith(">:"))
    b0 = next(i for i in range(start, len(lines)) if "s_barrier" in lines[i])
    b1 = next(i for i in range(b0 + 1, len(lines)) if "s_barrier" in lines[i])
    loads = [i for i in range(b0 + 1, b1) if "buffer_load" in lines[i] and " lds" not in lines[i].split("//")[0]]
    assert len(loads) == 8
    moved = [lines[i] for i in loads]
    rest = [ln for i, ln in enumerate(lines) if i not in set(loads)]
    text = "\n".join(rest[:b0 + 1] + moved + rest[b0 + 1:])
    r = _check_listing(tmp_path, text)
    assert r.returncode == 1, r.stdout + r.stderr
    assert "sffn_kernel<128,4,1,4>: barrier at" in r.stderr and "vmcnt(16), but only 8" in r.stderr, r.stderr
