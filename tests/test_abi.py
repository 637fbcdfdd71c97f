"""The C ABI surface of libsrhip.so (CPU: no compute calls, no GPU needed)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "srhip.h")


def _header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(srhip_[a-z_0-9]+)\s*\(", src)))


def _header_enums():
    src = open(HEADER).read()
    return {k: int(v) for k, v in re.findall(r"\b(SRHIP_[A-Z0-9_]+)\s*=\s*(\d+)", src)}


def test_library_exports_every_declared_symbol():
    import srhip._lib as L

    lib = L.load()
    decl = _header_functions()
    assert len(decl) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (srhip_\w+)", out))
    missing = [f for f in decl if f not in exported]
    assert not missing, missing
    # and the Python binding declares a signature for every one of them
    assert set(decl) == set(L.SIGNATURES), set(decl) ^ set(L.SIGNATURES)
    for f in decl:
        assert getattr(lib, f) is not None


def test_constants_match_header():
    import srhip._lib as L

    en = _header_enums()
    for k, v in L.OP.items():
        assert en[f"SRHIP_OP_{k}"] == v, k
    for k, v in L.LOSS.items():
        assert en[f"SRHIP_LOSS_{k}"] == v, k
    assert en["SRHIP_F32"] == L.F32 and en["SRHIP_F64"] == L.F64 and en["SRHIP_I32"] == L.I32
    assert en["SRHIP_OK"] == 0 and en["SRHIP_ERR_DEVICE"] == L.ERR_DEVICE


def test_node_struct_layout():
    import srhip._lib as L

    assert L.NODE_DTYPE.itemsize == 24
    assert L.NODE_DTYPE.fields["l"][1] == 8 and L.NODE_DTYPE.fields["val"][1] == 16


def test_version_and_errors_without_device():
    import srhip._lib as L

    lib = L.load()
    assert lib.srhip_version().decode().startswith("srhip")
    n = lib.srhip_device_count()
    assert n >= 0
    if n == 0:
        h = ctypes.c_void_p()
        rc = lib.srhip_ctx_create(0, ctypes.byref(h))
        assert rc == L.ERR_DEVICE
        assert "device" in lib.srhip_last_error().decode()
        with pytest.raises(L.SrhipError):
            L.check(rc)


def test_product_does_not_reference_oracle():
    """The shipped path never links or imports the oracle."""
    pkg = os.path.join(ROOT, "symbolicregression.jl_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"import\s+oracle|from\s+oracle|liboracle|sr_oracle|oracle_eval", txt), f
    out = subprocess.run(["readelf", "-d", os.path.join(pkg, "build", "libsrhip.so")], capture_output=True, text=True).stdout
    assert "oracle" not in out
