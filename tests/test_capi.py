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


def test_head_major_wb_rows():
    """msda.head_major_wb: the fused projection's rows regrouped per head -- head m's sampling offsets (L, P, 2)
    then its attention logits (L*P) -- from the two Linear layers (ms_deform_attn.py:59-60), gradients included."""
    import torch
    from bm2f_amd.msda import head_major_wb
    M, L, P, C = 8, 3, 4, 16
    g = torch.Generator().manual_seed(0)
    wo = torch.randn(M * L * P * 2, C, generator=g, requires_grad=True)
    bo = torch.randn(M * L * P * 2, generator=g, requires_grad=True)
    wa = torch.randn(M * L * P, C, generator=g, requires_grad=True)
    ba = torch.randn(M * L * P, generator=g, requires_grad=True)
    w, b = head_major_wb(wo, bo, wa, ba, M)
    LP = L * P
    for m in range(M):
        assert torch.equal(w[m * 3 * LP:m * 3 * LP + 2 * LP], wo[m * 2 * LP:(m + 1) * 2 * LP])
        assert torch.equal(w[m * 3 * LP + 2 * LP:(m + 1) * 3 * LP], wa[m * LP:(m + 1) * LP])
        assert torch.equal(b[m * 3 * LP:m * 3 * LP + 2 * LP], bo[m * 2 * LP:(m + 1) * 2 * LP])
        assert torch.equal(b[m * 3 * LP + 2 * LP:(m + 1) * 3 * LP], ba[m * LP:(m + 1) * LP])
    gw = torch.randn(w.shape, generator=g)
    (w * gw).sum().backward()
    for m in range(M):
        assert torch.equal(wo.grad[m * 2 * LP:(m + 1) * 2 * LP], gw[m * 3 * LP:m * 3 * LP + 2 * LP])
        assert torch.equal(wa.grad[m * LP:(m + 1) * LP], gw[m * 3 * LP + 2 * LP:(m + 1) * 3 * LP])
