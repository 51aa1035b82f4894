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


def _gn_ws(N, C, G, HW, device):
    b = ctypes.c_int64(0)
    _native.call("m2f_group_norm_workspace", N, C, G, ctypes.c_int64(HW), ctypes.byref(b))
    return torch.empty(max(b.value, 16), device=device, dtype=torch.uint8)


class GroupNormAct(Function):
    """``relu?(F.group_norm(x, G, weight, bias, eps))`` for fp32 NCHW (csrc/gnorm.hip): statistics, the
    affine normalisation and the ReLU in two passes, the backward (ReLU mask recomputed from x) in two."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, relu):
        x = x.contiguous()
        N, C = x.shape[:2]
        HW = x.numel() // (N * C)
        y = torch.empty_like(x)
        mean = torch.empty(N * groups, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        ws = _gn_ws(N, C, groups, HW, x.device)
        _native.call("m2f_group_norm_fwd_f32", x.data_ptr(), weight.data_ptr() if weight is not None else None,
                     bias.data_ptr() if bias is not None else None, N, C, groups, ctypes.c_int64(HW),
                     ctypes.c_float(eps), 1 if relu else 0, y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                     ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(x))
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.meta = (groups, relu)
        return y

    @staticmethod
    def backward(ctx, grad):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        groups, relu = ctx.meta
        g = grad.contiguous()
        N, C = x.shape[:2]
        HW = x.numel() // (N * C)
        dx = torch.empty_like(x)
        nig = ctx.needs_input_grad
        dw = torch.empty(C, device=x.device, dtype=torch.float32) if weight is not None and nig[1] else None
        db = torch.empty(C, device=x.device, dtype=torch.float32) if bias is not None and nig[2] else None
        ws = _gn_ws(N, C, groups, HW, x.device)
        _native.call("m2f_group_norm_bwd_f32", g.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                     weight.data_ptr() if weight is not None else None, bias.data_ptr() if bias is not None else None,
                     N, C, groups, ctypes.c_int64(HW), 1 if relu else 0, dx.data_ptr(),
                     dw.data_ptr() if dw is not None else None, db.data_ptr() if db is not None else None,
                     ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(x))
        return dx, dw, db, None, None, None


def group_norm_act(x: torch.Tensor, norm: nn.GroupNorm, relu: bool = False) -> torch.Tensor:
    """``norm(x)`` (then ReLU) for an ``nn.GroupNorm``; fp32 CUDA NCHW on the gfx950 kernels."""
    if (x.is_cuda and x.dtype == torch.float32 and x.dim() >= 3 and isinstance(norm, nn.GroupNorm)
            and (not norm.affine or (norm.weight.dtype == torch.float32 and norm.bias.dtype == torch.float32))
            and (x.numel() // (x.shape[0] * x.shape[1])) % 4 == 0 and x.numel() > 0):
        w = norm.weight if norm.affine else None
        b = norm.bias if norm.affine else None
        return GroupNormAct.apply(x, w, b, norm.num_groups, float(norm.eps), relu)
    y = norm(x)
    return torch.relu(y) if relu else y
