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


def test_shape_preconditions_rejected_without_gpu():
    """Shape preconditions the kernels rely on are checked in the C entry points themselves (not only by the Python
    callers), before any HIP call: fake aligned pointers never reach a kernel."""
    from bm2f_amd import _native
    lib = _native.load()
    p = ctypes.c_void_p(1 << 20)
    # the NHWC FPN merge stores float4s of 2w output columns: odd w is refused
    rc = lib.m2f_upsample2x_add_fwd_nhwc_f32(p, ctypes.c_int64(3 * 7 * 64), p, p, 1, 64, 3, 7, None)
    assert rc == 3 and b"even w" in lib.m2f_last_error()
    # the 16-bit NHWC input-gradient epilogue writes 8 channels per store: output channels % 16 != 0 is refused
    rc = lib.m2f_conv_x3_io(p, 0, 0, p, None, p, 1, 1, 1, 24, 32, 16, 16, 1, 1, p, ctypes.c_int64(1 << 30), None)
    assert rc == 3 and b"output channels" in lib.m2f_last_error()
