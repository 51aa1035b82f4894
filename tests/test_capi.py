"""The C-ABI library builds, loads and exports every entry point declared in include/bm2f.h (no GPU needed)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "bm2f.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\*|int)\s+(m2f_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_header_symbols():
    from bm2f_amd import _native
    lib = _native.load()
    names = _declared()
    assert len(names) >= 6
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native.exported_symbols())
    assert lib.m2f_abi_version() == _native.ABI_VERSION
    assert lib.m2f_last_error() == b""


def test_invalid_args_report_errors_without_gpu():
    from bm2f_amd import _native
    lib = _native.load()
    # null pointers are rejected before any HIP call
    rc = lib.m2f_msda_fwd_f32(None, None, None, None, None, 1, 1, 1, 32, 1, 1, 4, 64, None, None, None)
    assert rc == 1
    assert b"null" in lib.m2f_last_error()
