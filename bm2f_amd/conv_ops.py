"""fp32 convolutions of the pixel decoder's dense tail on the x3 MFMA engine (csrc/conv_x3.hip).

The reference runs the pixel decoder with autocast off (msdeformattn.py:314,320), so its 1x1 input
projections / lateral conv / mask_features conv and the 3x3 output conv are fp32 convs on the vendor
library (reference: cuDNN, :213-292).  Here forward and input gradient are implicit GEMMs with the
weights split exactly into three bf16 planes and the activations split in registers (fp32-accurate, see
csrc/gemm_x3.hip), the weight gradient a split-over-pixels GEMM with its slabs summed in a fixed order.
CUDA fp32 NCHW inputs that meet the kernel's shape rules run here (a missing library raises); anything
else uses ``F.conv2d``.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import _native


# 3x3 weight-gradient engine (tools/conv_bench.py, bs16 256x256x256, wgrad share of the backward):
#   "tn"     nine x3 TN GEMMs over zero-bordered pixel-row copies of dO and I (_wgrad3_tn): ~9.4 ms
#   "miopen" fp32 igemm_wrw on its own NHWC transposes: ~10.1 ms
#   "x3"     the implicit-GEMM kernel of csrc/conv_x3.hip on NCHW (channel-strided operands): ~14 ms
WGRAD3 = "tn"   # 3x3 weight gradient: "tn" (x3 TN GEMMs per tap) or "miopen"; set by tools / tests


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _workspace(N, Ci, Co, H, W, k, device):
    b = ctypes.c_int64(0)
    _native.call("m2f_conv_f32x3_workspace", N, Ci, Co, H, W, k, ctypes.byref(b))
    return torch.empty(max(b.value, 16), device=device, dtype=torch.uint8)


def _ptr(t):
    return t.data_ptr() if t is not None else None


_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}   # M2F_F32 / M2F_F16 / M2F_BF16


def _act16(x):
    """A 16-bit activation as the 1x1 kernels read it: (tensor, nhwc) -- channels-last kept as it is, anything else
    made NCHW-contiguous."""
    if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        return x, 1
    return x.contiguous(), 0


class Conv2dX3(Function):
    """fp32 conv on the x3 kernels.  A 16-bit input (the backbone's autocast features feeding a 1x1 conv) is read
    as it is, NCHW or channels-last, instead of through the reference's ``.float()`` copy (exact: the same
    results), and its gradient is written back in its dtype and layout (the cast's backward rounding)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        weight = weight.contiguous()
        N, Ci, H, W = x.shape
        Co, k = weight.shape[0], weight.shape[-1]
        out = torch.empty(N, Co, H, W, device=x.device, dtype=torch.float32)
        ws = _workspace(N, Ci, Co, H, W, k, x.device)
        ctx.nhwc = 0
        if x.dtype == torch.float32:
            x = x.contiguous()
            _native.call("m2f_conv_f32x3", x.data_ptr(), weight.data_ptr(), _ptr(bias), out.data_ptr(), N, Ci, Co, H,
                         W, k, 0, ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(x))
        else:
            x, ctx.nhwc = _act16(x)
            _native.call("m2f_conv_x3_io", x.data_ptr(), _DT[x.dtype], ctx.nhwc, weight.data_ptr(), _ptr(bias),
                         out.data_ptr(), 0, 0, N, Ci, Co, H, W, k, 0, ws.data_ptr(), ctypes.c_int64(ws.numel()),
                         _stream(x))
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, grad):
        x, weight = ctx.saved_tensors
        g = grad.contiguous()
        N, Ci, H, W = x.shape
        Co, k = weight.shape[0], weight.shape[-1]
        ws = _workspace(N, Ci, Co, H, W, k, x.device)
        dx = dw = db = None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if x.dtype != torch.float32:   # 16-bit 1x1 input
            if ctx.needs_input_grad[0]:
                dx = (torch.empty(N, H, W, Ci, device=x.device, dtype=x.dtype).permute(0, 3, 1, 2) if ctx.nhwc
                      else torch.empty(N, Ci, H, W, device=x.device, dtype=x.dtype))
                _native.call("m2f_conv_x3_io", g.data_ptr(), 0, 0, weight.data_ptr(), None, dx.data_ptr(), _DT[x.dtype],
                             ctx.nhwc, N, Ci, Co, H, W, k, 1, ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(g))
            if ctx.needs_input_grad[1] or want_b:
                tck = torch.empty(k * k, Ci, Co, device=x.device, dtype=torch.float32)
                db = torch.empty(Co, device=x.device, dtype=torch.float32) if want_b else None
                _native.call("m2f_conv_x3_wgrad_io", g.data_ptr(), x.data_ptr(), _DT[x.dtype], ctx.nhwc, tck.data_ptr(),
                             _ptr(db), N, Ci, Co, H, W, k, ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(g))
                dw = tck.permute(2, 1, 0).reshape(Co, Ci, k, k) if ctx.needs_input_grad[1] else None
            return dx, dw, db
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _native.call("m2f_conv_f32x3", g.data_ptr(), weight.data_ptr(), None, dx.data_ptr(), N, Ci, Co, H, W, k, 1,
                         ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(g))
        if k == 3 and WGRAD3 == "tn" and ctx.needs_input_grad[1]:
            dw = _wgrad3_tn(g, x)
            db = g.sum((2, 3)).sum(0) if want_b else None   # two reductions with many outputs (graph-safe)
        elif k == 3 and WGRAD3 == "miopen" and (ctx.needs_input_grad[1] or want_b):
            # 3x3 weight gradient on the library (WGRAD3 = "miopen")
            _, dw, db = torch.ops.aten.convolution_backward(
                g, x, weight, [Co] if want_b else None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                [False, bool(ctx.needs_input_grad[1]), want_b])
        elif ctx.needs_input_grad[1] or want_b:
            tck = torch.empty(k * k, Ci, Co, device=x.device, dtype=torch.float32)
            db = torch.empty(Co, device=x.device, dtype=torch.float32) if want_b else None
            _native.call("m2f_conv_f32x3_wgrad", g.data_ptr(), x.data_ptr(), tck.data_ptr(), _ptr(db), N, Ci, Co, H, W,
                         k, ws.data_ptr(), ctypes.c_int64(ws.numel()), _stream(g))
            dw = tck.permute(2, 1, 0).reshape(Co, Ci, k, k) if ctx.needs_input_grad[1] else None
        return dx, dw, db


def _pad_nhwc(t):
    """(N, C, H, W) fp32 -> zero-bordered pixel rows (N*(H+2)*(W+2), C) inside a buffer with W+3 zero rows
    before and after (so a row shift by any 3x3 tap stays in the buffer); returns (buffer, margin)."""
    N, C, H, W = t.shape
    P = (H + 2) * (W + 2)
    margin = W + 3
    buf = torch.empty(2 * margin + N * P, C, device=t.device, dtype=torch.float32)
    buf[:margin].zero_()
    buf[margin + N * P:].zero_()
    img = buf[margin:margin + N * P].view(N, H + 2, W + 2, C)   # zero only the borders: the transposes
    img[:, 0].zero_()                                            # below write every interior row
    img[:, H + 1].zero_()
    img[:, 1:H + 1, 0].zero_()
    img[:, 1:H + 1, W + 1].zero_()
    t = t.contiguous()
    for n in range(N):   # per image: H row-batches of the (C x W) -> (W x C) transpose
        dst = buf.data_ptr() + ((margin + n * P + (W + 2) + 1) * C) * 4
        _transpose(t.data_ptr() + n * C * H * W * 4, W, H * W, dst, (W + 2) * C, C, H, C, W, t.device)
    return buf, margin


def _wgrad3_tn(g, x):
    """3x3 "same" conv weight gradient as nine x3 TN GEMMs over zero-bordered pixel-row layouts:
    dW[:, :, ky, kx] = sum_q dO_pad[q]^T I_pad[q + (ky-1)(W+2) + (kx-1)] (border rows of dO_pad are zero,
    so out-of-image taps contribute nothing)."""
    from . import linear_ops
    N, Ci, H, W = x.shape
    Co = g.shape[1]
    gb, m = _pad_nhwc(g)
    xb, _ = _pad_nhwc(x)
    M = N * (H + 2) * (W + 2)
    a = gb[m:m + M]
    dw = torch.empty(Co, Ci, 3, 3, device=x.device, dtype=torch.float32)
    for ky in range(3):
        for kx in range(3):
            off = (ky - 1) * (W + 2) + (kx - 1)
            out, _ = linear_ops.gemm_tn(a, xb[m + off:m + off + M])
            dw[:, :, ky, kx] = out
    return dw


def eligible(x, conv) -> bool:
    """Shapes and settings the x3 conv kernels cover (else F.conv2d): fp32 input, or a 16-bit one into a 1x1 conv."""
    if not (x.is_cuda and x.dtype in _DT and conv.weight.dtype == torch.float32 and x.dim() == 4):
        return False
    k = conv.weight.shape[-1]
    if x.dtype != torch.float32 and k != 1:
        return False
    if conv.weight.shape[-2] != k or k not in (1, 3) or conv.groups != 1:
        return False
    if tuple(conv.stride) != (1, 1) or tuple(conv.dilation) != (1, 1) or tuple(conv.padding) != (k // 2, k // 2):
        return False
    N, Ci, H, W = x.shape
    Co = conv.weight.shape[0]
    return Ci % 16 == 0 and Co % 16 == 0 and (H * W) % 128 == 0 and W % 8 == 0


def conv2d(x, conv):
    """``F.conv2d(x, conv.weight, conv.bias, ...)`` for an nn.Conv2d (no norm / activation applied)."""
    if eligible(x, conv):
        return Conv2dX3.apply(x, conv.weight, conv.bias)
    return F.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups)


def conv_norm_act(x, conv):
    """A detectron2-style Conv2d (conv -> norm -> activation) with the conv on the x3 kernels."""
    from .norm_ops import group_norm_act
    y = conv2d(x, conv)
    norm = getattr(conv, "norm", None)
    act = getattr(conv, "activation", None)
    if isinstance(norm, torch.nn.GroupNorm) and act in (None, F.relu, torch.relu):
        return group_norm_act(y, norm, relu=act is not None)   # GN (+ ReLU) fused (csrc/gnorm.hip)
    if norm is not None:
        y = norm(y)
    if act is not None:
        y = act(y)
    return y


class Upsample2xAdd(Function):
    """``lateral + F.interpolate(src, size=lateral.shape[-2:], mode="bilinear", align_corners=False)`` for
    the exact 2x case in one pass (csrc/upsample.hip); the FPN merge of msdeformattn.py:343-349."""

    @staticmethod
    def forward(ctx, src, lateral):
        lat = lateral.contiguous()
        N, C, h, w = src.shape
        out = torch.empty_like(lat)
        ctx.nhwc = _nhwc_view(src) and C % 64 == 0 and w <= 256 and w % 2 == 0
        if ctx.nhwc:
            # the encoder's (N, HW, C) map read channel-contiguous and transposed in LDS: no transposing copy, and
            # the gradient comes back channels-last like the decoder's gradient of the same map (one fast sum)
            sN = src.stride(0) if N > 1 else h * w * C   # a size-1 batch dimension's stride is arbitrary
            _native.call("m2f_upsample2x_add_fwd_nhwc_f32", src.data_ptr(), ctypes.c_int64(sN), lat.data_ptr(),
                         out.data_ptr(), N, C, h, w, _stream(lat))
        else:
            # the strided read of a transposed (N, HW, C) view costs a cache line per lane and tap (2.6 ms at
            # bs16 128->256); one transposing copy first makes every tap read coalesced (1.0 ms with the copy)
            src = src.contiguous()
            _native.call("m2f_upsample2x_add_fwd_f32", src.data_ptr(), *(ctypes.c_int64(s) for s in src.stride()),
                         lat.data_ptr(), out.data_ptr(), N, C, h, w, _stream(lat))
        ctx.src_shape = src.shape
        return out

    @staticmethod
    def backward(ctx, grad):
        g = grad.contiguous()
        N, C, h, w = ctx.src_shape
        gsrc = None
        if ctx.needs_input_grad[0]:
            if ctx.nhwc:
                gsrc = torch.empty(N, h, w, C, device=g.device, dtype=torch.float32).permute(0, 3, 1, 2)
                _native.call("m2f_upsample2x_bwd_nhwc_f32", g.data_ptr(), gsrc.data_ptr(), N, C, h, w, _stream(g))
            else:
                gsrc = torch.empty(N, C, h, w, device=g.device, dtype=torch.float32)
                _native.call("m2f_upsample2x_bwd_f32", g.data_ptr(), gsrc.data_ptr(), N, C, h, w, _stream(g))
        return gsrc, (g if ctx.needs_input_grad[1] else None)


def _nhwc_view(t):
    """t (N, C, h, w) is a channels-last view: (h, w, C) contiguous per image, the batch stride a multiple of 4 at
    least h*w*C (the encoder's level slices of (N, S, C))."""
    N, C, h, w = t.shape
    sN = t.stride(0)
    return (t.stride()[1:] == (1, w * C, C) and (N == 1 or (sN >= h * w * C and sN % 4 == 0))
            and t.data_ptr() % 16 == 0)


def upsample_add(src, lateral):
    """``lateral + F.interpolate(src, size=lateral.shape[-2:], mode="bilinear", align_corners=False)``."""
    ok = (src.is_cuda and src.dtype == torch.float32 and lateral.dtype == torch.float32 and src.dim() == 4
          and lateral.dim() == 4 and lateral.shape[:2] == src.shape[:2]
          and tuple(lateral.shape[-2:]) == (2 * src.shape[2], 2 * src.shape[3]) and (2 * src.shape[3]) % 4 == 0)
    if ok:
        return Upsample2xAdd.apply(src, lateral)
    return lateral + F.interpolate(src, size=lateral.shape[-2:], mode="bilinear", align_corners=False)


def _transpose(src, in_bs, in_ld, dst, out_bs, out_ld, B, R, Q, device):
    _native.call("m2f_transpose_f32", src, ctypes.c_int64(in_bs), ctypes.c_int64(in_ld), dst, ctypes.c_int64(out_bs),
                 ctypes.c_int64(out_ld), B, R, Q, torch.cuda.current_stream(device).cuda_stream)


class FlattenLevels(Function):
    """``torch.cat([x.flatten(2).transpose(1, 2) for x in xs], 1)`` for NCHW fp32 levels (msdeformattn.py:64-74)
    with LDS-tiled transposes each way (csrc/eltwise.hip) instead of a strided cat."""

    @staticmethod
    def forward(ctx, *xs):
        N, C = xs[0].shape[:2]
        sizes = [x.shape[2] * x.shape[3] for x in xs]
        S = sum(sizes)
        out = torch.empty(N, S, C, device=xs[0].device, dtype=torch.float32)
        start = 0
        for x, hw in zip(xs, sizes):
            x = x.contiguous()
            _transpose(x.data_ptr(), C * hw, hw, out.data_ptr() + start * C * 4, S * C, C, N, C, hw, x.device)
            start += hw
        ctx.shapes = [x.shape for x in xs]
        return out

    @staticmethod
    def backward(ctx, grad):
        g = grad.contiguous()
        N, S, C = g.shape
        grads, start = [], 0
        for shp in ctx.shapes:
            hw = shp[2] * shp[3]
            gx = torch.empty(shp, device=g.device, dtype=torch.float32)
            _transpose(g.data_ptr() + start * C * 4, S * C, C, gx.data_ptr(), C * hw, hw, N, hw, C, g.device)
            grads.append(gx)
            start += hw
        return tuple(grads)


def flatten_levels(xs):
    """``torch.cat([x.flatten(2).transpose(1, 2) for x in xs], 1)``: (N, C, H_l, W_l) levels -> (N, S, C)."""
    if all(x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[:2] == xs[0].shape[:2] for x in xs) \
            and xs[0].shape[0] <= 65535:
        return FlattenLevels.apply(*xs)
    return torch.cat([x.flatten(2).transpose(1, 2) for x in xs], 1)
