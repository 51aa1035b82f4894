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

import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd import Function

from . import _native


# Which fp32 GEMM engine the encoder linears use: "x3" (bf16 MFMA on exact three-way operand splits,
# csrc/gemm_x3.hip, fp32-accurate at 2.7x the f32 MFMA rate) or "exact" (f32-input MFMA, csrc/gemm.hip).
ENGINE = "x3"   # fp32 GEMM engine: "x3" (split-bf16 MFMA), "exact" (f32 MFMA) or the library; set by tools


def _engine(engine):
    e = engine or ENGINE
    if e not in ("x3", "exact"):
        raise ValueError(f"fp32 GEMM engine {e!r}: expected 'x3' or 'exact'")
    return e


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _c64(v):
    return ctypes.c_int64(int(v))


def gemm_nt(a, b, bias=None, relu=False, mask=None, out=None, engine=None, b_kn=False, add=()):
    """C = a @ b.T (+ bias) (ReLU | * (mask > 0)) (+ add[0] (+ add[1])); a (M, K), b (N, K) fp32 row-major
    (unit column stride).  With ``b_kn`` b is (K, N) and C = a @ b (x3 engine: read in place; exact engine:
    transposed copy).  ``add``: up to two (M, N) addends with one row stride (x3 engine; ``out`` may be one
    of them)."""
    M, K = a.shape
    N = b.shape[1] if b_kn else b.shape[0]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    msk = (mask.data_ptr() if mask is not None else None, _c64(mask.stride(0) if mask is not None else 0))
    add = [d for d in add if d is not None]
    if _engine(engine) == "x3":
        wsb = ctypes.c_int64(0)
        _native.call("m2f_gemm_f32x3_nt_workspace", N, K, ctypes.byref(wsb))
        ws = torch.empty(max(wsb.value, 16), device=a.device, dtype=torch.uint8)
        if add:
            if len(add) > 2 or any(d.shape != (M, N) or d.stride() != add[0].stride() or d.stride(1) != 1
                                   for d in add):
                raise RuntimeError("gemm_nt: addends must be (M, N) row-major tensors with one row stride")
            _native.call("m2f_gemm_f32x3_nt_add", a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)),
                         1 if b_kn else 0, bias.data_ptr() if bias is not None else None, 1 if relu else 0, *msk,
                         add[0].data_ptr(), add[1].data_ptr() if len(add) > 1 else None, _c64(add[0].stride(0)),
                         out.data_ptr(), _c64(out.stride(0)), M, N, K, ws.data_ptr(), _c64(ws.numel()), _stream(a))
            return out
        _native.call("m2f_gemm_f32x3_nt", a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)),
                     1 if b_kn else 0, bias.data_ptr() if bias is not None else None, 1 if relu else 0, *msk,
                     out.data_ptr(), _c64(out.stride(0)), M, N, K, ws.data_ptr(), _c64(ws.numel()), _stream(a))
        return out
    if add:
        raise RuntimeError("gemm_nt: addends need the x3 engine")
    if b_kn:
        b = b.t().contiguous()
    _native.call("m2f_gemm_f32_nt", a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)),
                 bias.data_ptr() if bias is not None else None, 1 if relu else 0, *msk,
                 out.data_ptr(), _c64(out.stride(0)), M, N, K, _stream(a))
    return out


def gemm_nt_rowadd(a, b, r, period):
    """C = a @ b.T + r[row % period] (x3 engine); a (M, K), b (N, K), r (period, N) fp32 row-major."""
    M, K = a.shape
    N = b.shape[0]
    out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    wsb = ctypes.c_int64(0)
    _native.call("m2f_gemm_f32x3_nt_workspace", N, K, ctypes.byref(wsb))
    ws = torch.empty(max(wsb.value, 16), device=a.device, dtype=torch.uint8)
    _native.call("m2f_gemm_f32x3_nt_rowadd", a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)), 0,
                 r.data_ptr(), _c64(r.stride(0)), period, out.data_ptr(), _c64(out.stride(0)), M, N, K, ws.data_ptr(),
                 _c64(ws.numel()), _stream(a))
    return out


def gemm_nt_bits(a, b, bias=None, bits_out=None, bits_in=None, b_kn=False):
    """x3 NT GEMM with the ReLU as a 1-bit mask: ``bits_out`` (M, N/32) int32 -> C = relu(a b^T + bias) and the
    mask of C > 0 written there; ``bits_in`` -> C = (a b^T + bias) where the mask bit is set, else 0."""
    M, K = a.shape
    N = b.shape[1] if b_kn else b.shape[0]
    out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    bits = bits_out if bits_out is not None else bits_in
    wsb = ctypes.c_int64(0)
    _native.call("m2f_gemm_f32x3_nt_workspace", N, K, ctypes.byref(wsb))
    ws = torch.empty(max(wsb.value, 16), device=a.device, dtype=torch.uint8)
    _native.call("m2f_gemm_f32x3_nt_bits", a.data_ptr(), _c64(a.stride(0)), b.data_ptr(), _c64(b.stride(0)),
                 1 if b_kn else 0, bias.data_ptr() if bias is not None else None, 1 if bits_out is not None else 0,
                 bits_out.data_ptr() if bits_out is not None else None,
                 bits_in.data_ptr() if bits_in is not None else None, _c64(bits.stride(0)),
                 out.data_ptr(), _c64(out.stride(0)), M, N, K, ws.data_ptr(), _c64(ws.numel()), _stream(a))
    return out


def _relu_bits(x2, w1, b1):
    """h = relu(x2 w1^T + b1) and its 1-bit mask (rows, N/32) when the x3 engine takes it, else (h, None)."""
    N = w1.shape[0]
    if ENGINE == "x3" and N % 32 == 0:
        bits = torch.empty(x2.shape[0], N // 32, device=x2.device, dtype=torch.int32)
        return gemm_nt_bits(x2, w1, b1, bits_out=bits), bits
    return gemm_nt(x2, w1, b1, relu=True), None


def _masked_dgrad(g, w2, h, bits):
    """grad_h = (g . w2) * (h > 0): from the 1-bit mask when there is one, else from h itself."""
    if bits is not None:
        return gemm_nt_bits(g, w2, bits_in=bits, b_kn=True)
    return gemm_nt(g, w2, mask=h, b_kn=True)


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
        h, bits = _relu_bits(x2, w1, b1)
        y = _mm_nt(h, w2, b2)
        ctx.save_for_backward(x2, w1, w2, h, bits)
        ctx.in_shape = x.shape
        ctx.biases = (b1 is not None, b2 is not None)
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, grad):
        x2, w1, w2, h, bits = ctx.saved_tensors
        g = _rows(grad)
        if g.stride(-1) != 1 or g.stride(0) % 4:
            g = g.contiguous()
        nig = ctx.needs_input_grad
        dw2, db2 = gemm_tn(g, h, colsum=ctx.biases[1] and nig[4]) if (nig[3] or nig[4]) else (None, None)
        gh = _masked_dgrad(g, w2, h, bits)                      # grad_h with the ReLU mask (h > 0)
        del h
        dw1, db1 = gemm_tn(gh, x2, colsum=ctx.biases[0] and nig[2]) if (nig[1] or nig[2]) else (None, None)
        dx = _mm_nn(gh, w1).view(ctx.in_shape) if nig[0] else None
        return dx, dw1, db1, dw2, db2


def _grad_rows(g, like):
    """A gradient as contiguous (rows, C) fp32 (zeros when autograd passes None)."""
    if g is None:
        return torch.zeros(like.shape, device=like.device, dtype=torch.float32)
    g = _rows(g)
    return g if g.is_contiguous() else g.contiguous()


class FFNResidualF32(Function):
    """(linear2(relu(linear1(x))), x): the FFN of :class:`FFNF32` that also hands ``x`` on for the residual
    add & norm that follows (msdeformattn.py:109-113), so the backward sums the residual gradient into
    grad_x inside the input-gradient GEMM's epilogue instead of autograd adding two (N*S, 256) tensors."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        x2 = _rows(x)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        h, bits = _relu_bits(x2, w1, b1)
        y = gemm_nt(h, w2, b2)
        ctx.save_for_backward(x2, w1, w2, h, bits)
        ctx.in_shape = x.shape
        ctx.biases = (b1 is not None, b2 is not None)
        return y.view(*x.shape[:-1], w2.shape[0]), x2.view(x.shape)

    @staticmethod
    def backward(ctx, grad, grad_pass):
        x2, w1, w2, h, bits = ctx.saved_tensors
        g = _grad_rows(grad, x2)
        nig = ctx.needs_input_grad
        dw2, db2 = gemm_tn(g, h, colsum=ctx.biases[1] and nig[4]) if (nig[3] or nig[4]) else (None, None)
        gh = _masked_dgrad(g, w2, h, bits)
        del h
        dw1, db1 = gemm_tn(gh, x2, colsum=ctx.biases[0] and nig[2]) if (nig[1] or nig[2]) else (None, None)
        dx = None
        if nig[0]:
            gp = _rows(grad_pass).contiguous() if grad_pass is not None else None
            dx = gemm_nt(gh, w1, b_kn=True, add=(gp,)).view(ctx.in_shape)
        return dx, dw1, db1, dw2, db2


class EncoderInProjF32(Function):
    """The two input projections of an encoder layer's MSDeformAttn, and ``src`` handed on for the residual
    (msdeformattn.py:115-119 with ms_deform_attn.py:97-103):

        value = src @ Wv^T + bv,   proj = (src + pos) @ Wq^T + bq,   src (for the residual add & norm)

    Wq / bq are the sampling-offset and attention-weight projections stacked.  ``src`` has three consumers,
    so autograd would add three (N*S, 256) gradients; here grad_src = grad_value . Wv + grad_proj . Wq +
    grad_residual leaves the two input-gradient GEMMs with the sums in their epilogues.

    A position embedding shared by the batch (pos (1, S, C), the encoder's case) is not added to src: by linearity
    proj = src Wq^T + R with R = pos Wq^T + bq formed once on the S rows of one image and added row-periodically in
    the GEMM epilogue (m2f_gemm_f32x3_nt_rowadd), so the (N*S, C) query is never materialised or saved.  The
    backward then forms d Wq = grad_proj^T src + (sum_n grad_proj[n])^T pos and d pos = (sum_n grad_proj[n]) Wq."""

    @staticmethod
    def forward(ctx, src, pos, wv, bv, wq, bq):
        s2 = _rows(src)
        if not s2.is_contiguous():
            s2 = s2.contiguous()
        value = gemm_nt(s2, wv, bv)
        S = src.shape[-2] if src.dim() >= 2 else 0
        ctx.shared_pos = (pos is not None and src.dim() == 3 and pos.dim() == 3 and pos.shape[0] == 1
                          and pos.shape[1:] == src.shape[1:] and src.shape[0] > 1)
        if ctx.shared_pos:
            p2 = pos.reshape(S, pos.shape[-1])
            if not p2.is_contiguous():
                p2 = p2.contiguous()
            r = gemm_nt(p2, wq, bq)                               # pos Wq^T + bq, once per layer (S rows)
            proj = gemm_nt_rowadd(s2, wq, r, S)
            ctx.save_for_backward(s2, p2, wv, wq)
        else:
            # pos may be one (1, S, C) embedding broadcast over a batch of 1, or a full tensor
            q2 = (s2.view(src.shape) + pos).view(s2.shape) if pos is not None else s2
            proj = gemm_nt(q2, wq, bq)
            ctx.save_for_backward(s2, q2, wv, wq)
        ctx.in_shape = src.shape
        ctx.has_pos = pos is not None
        ctx.pos_shape = pos.shape if pos is not None else None
        ctx.biases = (bv is not None, bq is not None)
        lead = src.shape[:-1]
        return value.view(*lead, wv.shape[0]), proj.view(*lead, wq.shape[0]), s2.view(src.shape)

    @staticmethod
    def backward(ctx, gvalue, gproj, gpass):
        s2, q2, wv, wq = ctx.saved_tensors
        nig = ctx.needs_input_grad
        gv = _grad_rows(gvalue, torch.empty(s2.shape[0], wv.shape[0], device=s2.device))
        gq = _grad_rows(gproj, torch.empty(s2.shape[0], wq.shape[0], device=s2.device))
        gr = _rows(gpass).contiguous() if gpass is not None else None
        dsrc = dpos = None
        dwq = dbq = None
        if ctx.shared_pos:
            p2 = q2                                               # the (S, C) embedding
            N, S = ctx.in_shape[0], ctx.in_shape[1]
            gqs = gq.view(N, S, -1).sum(0)                        # sum_n grad_proj[n]: (S, 3 M L P)
            if nig[1]:
                dpos = gemm_nt(gqs, wq, b_kn=True).view(ctx.pos_shape)
            if nig[0]:
                t = gemm_nt(gq, wq, b_kn=True, add=(gr,))
                dsrc = gemm_nt(gv, wv, b_kn=True, add=(t,), out=t).view(ctx.in_shape)
            if nig[4] or nig[5]:
                dwq, dbq = gemm_tn(gq, s2, colsum=ctx.biases[1] and nig[5])
                if nig[4]:
                    dwq = dwq + gemm_tn(gqs, p2)[0]
        else:
            if ctx.has_pos and nig[1]:
                dq = gemm_nt(gq, wq, b_kn=True)
                dpos = dq.view(ctx.in_shape)
                if ctx.pos_shape != ctx.in_shape:
                    dpos = dpos.sum(0, keepdim=True)
                if nig[0]:
                    dsrc = gemm_nt(gv, wv, b_kn=True, add=(dq, gr)).view(ctx.in_shape)
            elif nig[0]:
                t = gemm_nt(gq, wq, b_kn=True, add=(gr,))
                dsrc = gemm_nt(gv, wv, b_kn=True, add=(t,), out=t).view(ctx.in_shape)
            if nig[4] or nig[5]:
                dwq, dbq = gemm_tn(gq, q2, colsum=ctx.biases[1] and nig[5])
        dwv, dbv = gemm_tn(gv, s2, colsum=ctx.biases[0] and nig[3]) if (nig[2] or nig[3]) else (None, None)
        return dsrc, dpos, dwv, dbv, dwq, dbq


def residual_fusable(x, *mods) -> bool:
    """Whether the pass-through variants (:class:`FFNResidualF32`, :class:`EncoderInProjF32`) apply: CUDA fp32
    on the x3 engine (their gradient sums ride in the x3 GEMM epilogues)."""
    return ENGINE == "x3" and x.shape[-1] % 4 == 0 and _eligible(x, *mods) and all(
        m.weight.shape[0] % 4 == 0 for m in mods)


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


def ffn_residual(x: torch.Tensor, lin1: nn.Linear, lin2: nn.Linear):
    """``(lin2(relu(lin1(x))), x)``; use the second output as the residual (see :class:`FFNResidualF32`)."""
    if residual_fusable(x, lin1, lin2):
        return FFNResidualF32.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias)
    return ffn(x, lin1, lin2), x


def ffn(x: torch.Tensor, lin1: nn.Linear, lin2: nn.Linear) -> torch.Tensor:
    """``lin2(relu(lin1(x)))`` with the ReLU fused into both passes."""
    if _eligible(x, lin1, lin2):
        return FFNF32.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias)
    return lin2(F.relu(lin1(x)))
