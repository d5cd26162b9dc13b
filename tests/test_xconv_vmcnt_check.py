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
