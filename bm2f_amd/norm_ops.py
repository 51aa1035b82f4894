"""Residual add + LayerNorm on the gfx950 kernel (csrc/norm.hip): the post-norm of the pixel decoder's
encoder layer, ``norm(src + dropout(src2))`` (reference msdeformattn.py:92-131; dropout is 0.0 in every
shipped config).

:func:`add_layernorm` takes the module's ``nn.LayerNorm`` so parameters and state-dict keys are those
of the reference.  CUDA fp32 tensors go to ``libbm2f`` (a missing library raises); other devices or
dtypes use the same math in PyTorch (the reference's own CPU behaviour).
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn
from torch.autograd import Function

from . import _native


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class AddLayerNorm(Function):
    @staticmethod
    def forward(ctx, a, b, weight, bias, eps):
        C = a.shape[-1]
        a2 = a.contiguous()
        b2 = b.contiguous() if b is not None else None
        rows = a2.numel() // C
        y = torch.empty_like(a2)
        mean = torch.empty(rows, device=a.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        w = weight.contiguous()
        _native.call("m2f_add_layernorm_fwd_f32", a2.data_ptr(), b2.data_ptr() if b2 is not None else None,
                     w.data_ptr(), bias.contiguous().data_ptr(), ctypes.c_int64(rows), C, ctypes.c_float(eps),
                     y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), _stream(a))
        ctx.save_for_backward(a2, b2, w, mean, rstd)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, grad):
        a, b, w, mean, rstd = ctx.saved_tensors
        C = a.shape[-1]
        rows = a.numel() // C
        g = grad.contiguous()
        dx = torch.empty_like(a)
        need_w, need_b = ctx.needs_input_grad[2], ctx.needs_input_grad[3]
        dw = torch.empty(C, device=a.device, dtype=torch.float32) if need_w else None
        db = torch.empty(C, device=a.device, dtype=torch.float32) if need_b else None
        wsb = ctypes.c_int64(0)
        _native.call("m2f_add_layernorm_workspace", ctypes.c_int64(rows), C, ctypes.byref(wsb))
        ws = torch.empty(max(wsb.value, 4), device=a.device, dtype=torch.uint8)
        _native.call("m2f_add_layernorm_bwd_f32", g.data_ptr(), a.data_ptr(), b.data_ptr() if b is not None else None,
                     w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), ctypes.c_int64(rows), C, dx.data_ptr(),
                     dw.data_ptr() if dw is not None else None, db.data_ptr() if db is not None else None,
                     ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(a))
        # one tensor for both summands, as AddBackward0 does (autograd only accumulates in place into a
        # buffer nothing else references)
        da = dx if ctx.needs_input_grad[0] else None
        dbb = dx if ctx.has_b and ctx.needs_input_grad[1] else None
        return da, dbb, dw, db, None


def _eligible(a, b, norm):
    return (a.is_cuda and a.dtype == torch.float32 and (b is None or (b.dtype == torch.float32 and b.shape == a.shape))
            and norm.elementwise_affine and norm.weight is not None and norm.bias is not None
            and len(norm.normalized_shape) == 1 and norm.weight.dtype == torch.float32
            and a.shape[-1] % 4 == 0 and a.shape[-1] <= 1024 and a.numel() > 0)


def add_layernorm(a: torch.Tensor, b: torch.Tensor | None, norm: nn.LayerNorm) -> torch.Tensor:
    """``norm(a + b)`` (or ``norm(a)`` when b is None) in one pass over HBM each way."""
    if _eligible(a, b, norm):
        return AddLayerNorm.apply(a, b, norm.weight, norm.bias, float(norm.eps))
    return norm(a if b is None else a + b)
