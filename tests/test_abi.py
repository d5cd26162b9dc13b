"""The C-ABI libraries load (no GPU needed) and export every function the
public headers declare; the product package never imports the oracle."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = {"dcvc_rans.h": "libdcvc_rans.so", "dcvc_hip.h": "libdcvc_hip.so"}


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dcvc_[a-z0-9_]+)\s*\(", text)))


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_library_exports_every_declared_symbol(header):
    names = declared(header)
    assert len(names) >= 10
    lib = ctypes.CDLL(os.path.join(ROOT, "dcvc_amd", "lib", HEADERS[header]))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{HEADERS[header]} lacks {missing}"


def test_python_bindings_cover_the_headers():
    from dcvc_amd import hip, _native
    bound = {s[0] for s in hip.HIP_SYMBOLS} | {s[0] for s in _native.RANS_SYMBOLS}
    for header in HEADERS:
        assert set(declared(header)) <= bound, header


def test_product_package_does_not_import_the_oracle():
    pat = re.compile(r"^\s*(from|import)\s+oracle\b|^\s*from\s+\.\.+oracle", re.M)
    for d, _, files in os.walk(os.path.join(ROOT, "dcvc_amd")):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(d, f)).read()
                assert not pat.search(src), os.path.join(d, f)
