"""librsc.so (the drop-in boundary) loads, exports every symbol include/rsc.h declares, and fails
loudly without a HIP device (no CPU fallback).  No compute calls here."""
import ctypes
import os
import re

import pytest

from rsc import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "rsc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rsc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = engine.load_library()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(engine.EXPORTED) == syms


def test_status_strings():
    L = engine.load_library()
    for code in (0, -1, -2, -3, -4, -5):
        assert L.rsc_status_string(code)


def test_no_device_fails_loudly():
    L = engine.load_library()
    h = ctypes.c_void_p()
    st = L.rsc_context_create(0, ctypes.byref(h))
    if st == 0:
        L.rsc_context_destroy(h)
        pytest.skip("a HIP device is present")
    assert st == -5
    with pytest.raises(RuntimeError):
        engine.Context(0)


def test_oracle_not_linked_into_product():
    """The product library must not contain oracle symbols (oracle = test infrastructure only)."""
    import subprocess
    out = subprocess.run(["nm", "-D", engine.LIB_PATH], capture_output=True, text=True).stdout
    assert "ora_" not in out and "rsc_oracle" not in out
