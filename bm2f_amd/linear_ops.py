"""fp32 linear layers of the pixel decoder's encoder on the gfx950 f32-MFMA GEMMs (csrc/gemm.hip).

The encoder layer (reference msdeformattn.py:92-131 and ops/modules/ms_deform_attn.py:59-62) runs
value_proj, the sampling-offset / attention-weight projections, output_proj and the ReLU FFN on
(N*S, 256) fp32 rows with autocast off.  Here each is one autograd node whose forward is a GEMM with
the bias (and ReLU) in the epilogue and whose backward is:

  grad_input  = grad_out . W           (NT GEMM on W^T; for the FFN the ReLU mask rides in its epilogue)
  grad_weight = grad_out^T . input     (split-row TN GEMM, deterministic slab reduce)
  grad_bias   = sum_rows grad_out      (column sums taken inside the same TN GEMM)

All products are exact fp32 (no TF32-like mode exists on gfx950).  :func:`linear` / :func:`ffn`
take the reference's ``nn.Linear`` modules, so parameters and state-dict keys are unchanged.
CUDA fp32 inputs run on ``libbm2f`` (missing library -> error); anything else uses ``F.linear``.

Which GEMMs stay on hipBLASLt (measured on MI355X, tools/gemm_bench.py, M = 344064): the plain products
with a 1024-deep or 288-wide reduction, where the library kernel is 10-20 % faster than the
128x128-tile MFMA kernel here and there is no epilogue to fuse (linear2 forward, linear1 input
gradient, the sampling projection's input gradient).  Every weight/bias gradient (1.3-2x faster here),
every fused-epilogue product and the 256-wide products run on libbm2f.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd import Function

from . import _native


# Which fp32 GEMM engine the encoder linears use: "x3" (bf16 MFMA on exact three-way operand splits,
# csrc/gemm_x3.hip, fp32-accurate at 2.7x the f32 MFMA rate) or "exact" (f32-input MFMA, csrc/gemm.hip).
ENGINE = os.environ.get("M2F_F32_GEMM", "x3")


def _engine(engine):
    e = engine or ENGINE
    if e not in ("x3", "exact"):
        raise ValueError(f"fp32 GEMM engine {e!r}: expected 'x3' or 'exact'")
    return e


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _c64(v):
    return ctypes.c_int64(int(v))


def gemm_nt(a, b, bias=None, relu=False, mask=None, out=None, engine=None, b_kn=False):
    """C = a @ b.T (+ bias) (ReLU | * (mask > 0)); a (M, K), b (N, K) fp32 row-major (unit column stride).
    With ``b_kn`` b is (K, N) and C = a @ b (x3 engine: read in place; exact engine: transposed copy)."""
    M, K = a.shape
    N = b.shape[1] if b_kn else b.shape[0]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    msk = (mask.data_ptr() if mask is not None else None, _c64(mask.stride(0) if mask is not None else 0))
    if _engine(engine) == "x3":
        wsb = ctypes.c_int64(0)
        _native.call("m2f_gemm_f32x3_nt_workspace", N, K, ctypes.byref(wsb))
        ws = torch.empty(max(wsb.value, 16), device=a.device, dtype=torch.uint8)
        _native.call("m2f_gemm_f32x3_nt", a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)),
                     1 if b_kn else 0, bias.data_ptr() if bias is not None else None, 1 if relu else 0, *msk,
                     out.data_ptr(), _c64(out.stride(0)), M, N, K, ws.data_ptr(), _c64(ws.numel()), _stream(a))
        return out
    if b_kn:
        b = b.t().contiguous()
    _native.call("m2f_gemm_f32_nt", a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)),
                 bias.data_ptr() if bias is not None else None, 1 if relu else 0, *msk,
                 out.data_ptr(), _c64(out.stride(0)), M, N, K, _stream(a))
    return out


def gemm_tn(a, b, colsum=False, engine=None):
    """(a.T @ b, a.sum(0) if colsum) for a (M, N1), b (M, N2) fp32 row-major."""
    M, N1 = a.shape
    N2 = b.shape[1]
    out = torch.empty(N1, N2, device=a.device, dtype=torch.float32)
    cs = torch.empty(N1, device=a.device, dtype=torch.float32) if colsum else None
    fn = "m2f_gemm_f32x3_tn" if _engine(engine) == "x3" else "m2f_gemm_f32_tn"
    wsb = ctypes.c_int64(0)
    _native.call(fn + "_workspace", M, N1, N2, ctypes.byref(wsb))
    ws = torch.empty(max(wsb.value, 4), device=a.device, dtype=torch.uint8)
    _native.call(fn, a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)),
                 out.data_ptr(), _c64(N2), cs.data_ptr() if cs is not None else None, M, N1, N2, ws.data_ptr(),
                 _c64(ws.numel()), _stream(a))
    return out, cs


def _rows(x):
    return x.reshape(-1, x.shape[-1])


def _blas_preferred(k):
    """Plain (no-epilogue) NT product with reduction depth k: with the exact-f32 engine hipBLASLt wins at
    k >= 1024 or k % 128 != 0; the x3 engine wins everywhere."""
    return ENGINE == "exact" and (k >= 1024 or k % 128 != 0)


def _mm_nt(a, b, bias=None):
    """a @ b.T (+ bias) on whichever engine is faster for this depth (no fused epilogue)."""
    if _blas_preferred(a.shape[1]):
        return torch.addmm(bias, a, b.t()) if bias is not None else a @ b.t()
    return gemm_nt(a, b, bias)


def _mm_nn(a, w):
    """a @ w (an input gradient through weight w of shape (out, in))."""
    if _blas_preferred(a.shape[1]):
        return a @ w
    return gemm_nt(a, w, b_kn=True)


class LinearF32(Function):
    """y = x W^T + b (optionally ReLU) on the NT GEMM; backward as in the module docstring."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        x2 = _rows(x)
        if x2.stride(-1) != 1 or x2.stride(0) % 4:
            x2 = x2.contiguous()
        y = gemm_nt(x2, weight, bias, relu=True) if relu else _mm_nt(x2, weight, bias)
        ctx.save_for_backward(x2, weight, y if relu else None)
        ctx.relu = relu
        ctx.has_bias = bias is not None
        ctx.in_shape = x.shape
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, grad):
        x2, w, y = ctx.saved_tensors
        g = _rows(grad)
        if g.stride(-1) != 1 or g.stride(0) % 4:
            g = g.contiguous()
        if ctx.relu:
            g = torch.where(y > 0, g, torch.zeros((), device=g.device, dtype=g.dtype))
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _mm_nn(g, w).view(ctx.in_shape)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = gemm_tn(g, x2, colsum=ctx.has_bias and ctx.needs_input_grad[2])
        return dx, dw, db, None


class FFNF32(Function):
    """linear2(relu(linear1(x))) (msdeformattn.py:101-106 with dropout 0): the ReLU is the forward
    GEMM's epilogue and, in the backward, the mask applied in the epilogue of grad_h = grad_y . W2."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        x2 = _rows(x)
        if x2.stride(-1) != 1 or x2.stride(0) % 4:
            x2 = x2.contiguous()
        h = gemm_nt(x2, w1, b1, relu=True)
        y = _mm_nt(h, w2, b2)
        ctx.save_for_backward(x2, w1, w2, h)
        ctx.in_shape = x.shape
        ctx.biases = (b1 is not None, b2 is not None)
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, grad):
        x2, w1, w2, h = ctx.saved_tensors
        g = _rows(grad)
        if g.stride(-1) != 1 or g.stride(0) % 4:
            g = g.contiguous()
        nig = ctx.needs_input_grad
        dw2, db2 = gemm_tn(g, h, colsum=ctx.biases[1] and nig[4]) if (nig[3] or nig[4]) else (None, None)
        gh = gemm_nt(g, w2, mask=h, b_kn=True)                  # grad_h with the ReLU mask (h > 0)
        del h
        dw1, db1 = gemm_tn(gh, x2, colsum=ctx.biases[0] and nig[2]) if (nig[1] or nig[2]) else (None, None)
        dx = _mm_nn(gh, w1).view(ctx.in_shape) if nig[0] else None
        return dx, dw1, db1, dw2, db2


def _eligible_wb(x, weight, bias):
    return (x.is_cuda and x.dtype == torch.float32 and x.numel() > 0 and x.shape[-1] % 4 == 0
            and weight.dtype == torch.float32 and weight.dim() == 2 and weight.is_contiguous()
            and weight.shape[0] % 4 == 0 and weight.shape[1] % 4 == 0
            and (bias is None or bias.dtype == torch.float32))


def _eligible(x, *mods):
    return all(_eligible_wb(x, m.weight, m.bias) for m in mods)


def linear(x: torch.Tensor, mod: nn.Linear, relu: bool = False) -> torch.Tensor:
    """``mod(x)`` (then ReLU if ``relu``) on the fp32 MFMA GEMMs."""
    return linear_wb(x, mod.weight, mod.bias, relu)


def linear_wb(x: torch.Tensor, weight: torch.Tensor, bias, relu: bool = False) -> torch.Tensor:
    """``F.linear(x, weight, bias)`` (then ReLU) for a weight/bias not owned by one module (e.g. the
    concatenated sampling projections)."""
    if _eligible_wb(x, weight, bias):
        return LinearF32.apply(x, weight, bias, relu)
    y = F.linear(x, weight, bias)
    return F.relu(y) if relu else y


def ffn(x: torch.Tensor, lin1: nn.Linear, lin2: nn.Linear) -> torch.Tensor:
    """``lin2(relu(lin1(x)))`` with the ReLU fused into both passes."""
    if _eligible(x, lin1, lin2):
        return FFNF32.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias)
    return lin2(F.relu(lin1(x)))
