"""Decoder ops on the gfx950 kernels: attention-mask bitmask, masked cross-attention, mask einsum.

* :func:`attn_mask_bits` — reference forward_prediction_heads resize + ``sigmoid() < 0.5``
  (mask2former_transformer_decoder.py:446-449) and the fully-masked-row fix (:400) in one kernel,
  emitting one bit per (b, q, pixel) for all heads.
* :class:`MaskedAttention` — the attention core of ``nn.MultiheadAttention(attn_mask=bool)`` as used by
  CrossAttentionLayer (:98-110), flash style, fwd + bwd.
* :class:`MaskEinsum` — ``einsum("bqc,bchw->bqhw")`` (:442) with the low-precision copy of the mask
  features cast once per decoder forward (the reference re-casts the 1 GB fp32 map on every one of its 10
  calls under AMP); its gradient is returned in the features' dtype, as the reference's cast would.
* :class:`MaskFeatureFold` — the same einsum for all of a decoder's heads, with the gradient w.r.t. the
  shared mask features summed by ONE batched GEMM over the stacked heads (K = heads x queries) in the
  backward, instead of one GEMM + cast + 1 GB fp32 accumulation per head.
"""
from __future__ import annotations

import contextlib
import ctypes
import math

import torch
from torch import nn
from torch.autograd import Function
from torch.nn import functional as F

from . import _native

_DTYPE_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def _code(dtype):
    try:
        return _DTYPE_CODE[dtype]
    except KeyError:
        raise RuntimeError(f"bm2f_amd decoder ops: unsupported dtype {dtype}") from None


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _require_device(*ts):
    for t in ts:
        if t.device.type != "cuda":
            raise RuntimeError("bm2f_amd decoder ops need HIP device tensors")


def num_words(hw: int) -> int:
    return (hw + 31) // 32


def attn_mask_bits(logits: torch.Tensor, size, row_fix: bool = True) -> torch.Tensor:
    """logits (B, Q, H, W) or (B, Q, T, H, W) -> int32 bits (B, Q, ceil(T*h*w/32)); set bit = blocked."""
    _require_device(logits)
    logits = logits.detach().contiguous()
    if logits.dim() == 4:
        B, Q, Hin, Win = logits.shape
        T = 1
    else:
        B, Q, T, Hin, Win = logits.shape
    Hout, Wout = int(size[0]), int(size[1])
    nw = num_words(T * Hout * Wout)
    bits = torch.empty((B, Q, nw), dtype=torch.int32, device=logits.device)
    _native.call("m2f_attn_mask_bits", logits.data_ptr(), _code(logits.dtype), B, Q, T, Hin, Win, Hout, Wout,
                 1 if row_fix else 0, bits.data_ptr(), nw, _stream(logits))
    return bits


def bits_to_bool(bits: torch.Tensor, hw: int, num_heads: int = 1) -> torch.Tensor:
    """Expand bits to the reference's bool layout (B*num_heads, Q, hw); for tests and interop only."""
    B, Q, nw = bits.shape
    shifts = torch.arange(32, device=bits.device, dtype=torch.int32)
    b = ((bits.unsqueeze(-1) >> shifts) & 1).bool().flatten(2)[..., :hw]
    return b.unsqueeze(1).expand(B, num_heads, Q, hw).flatten(0, 1)


def _plan(B, Lq, Lk, H):
    cl, nc = ctypes.c_int(), ctypes.c_int()
    fw, bw = ctypes.c_int64(), ctypes.c_int64()
    _native.call("m2f_masked_attn_plan", B, Lq, Lk, H, ctypes.byref(cl), ctypes.byref(nc), ctypes.byref(fw),
                 ctypes.byref(bw))
    return cl.value, nc.value, fw.value, bw.value


def _rows(t: torch.Tensor):
    """(B, L, H*32) view with unit inner stride -> (tensor, row_stride)."""
    if t.stride(-1) != 1 or t.stride(0) != t.shape[1] * t.stride(1):
        t = t.contiguous()
    return t, t.stride(1)


class MaskedAttention(Function):
    """softmax(q k^T * scale, blocked by bits) v; q (B, Lq, H*32), k/v (B, Lk, H*32) -> (B, Lq, H*32)."""

    @staticmethod
    def forward(ctx, q, k, v, bits, num_heads, scale):
        _require_device(q, k, v, bits)
        if not (q.dtype == k.dtype == v.dtype):
            raise RuntimeError("masked attention: q, k, v must share a dtype")
        q, qs = _rows(q)
        k, ks = _rows(k)
        v, vs = _rows(v)
        if ks != vs:
            k, v = k.contiguous(), v.contiguous()
            ks = k.stride(1)
        B, Lq, C = q.shape
        Lk = k.shape[1]
        if C != num_heads * 32:
            raise RuntimeError(f"masked attention: channels {C} != {num_heads} heads x 32")
        bits = bits.contiguous()
        _, _, fwb, _ = _plan(B, Lq, Lk, num_heads)
        out = torch.empty((B, Lq, C), dtype=q.dtype, device=q.device)
        lse = torch.empty((B, num_heads, Lq), dtype=torch.float32, device=q.device)
        ws = torch.empty((max(fwb, 4) // 4,), dtype=torch.float32, device=q.device)
        _native.call("m2f_masked_attn_fwd", _code(q.dtype), q.data_ptr(), k.data_ptr(), v.data_ptr(), bits.data_ptr(),
                     B, Lq, Lk, num_heads, 32, qs, ks, bits.shape[-1], ctypes.c_float(scale), out.data_ptr(),
                     lse.data_ptr(), ws.data_ptr(), ctypes.c_int64(fwb), _stream(q))
        ctx.save_for_backward(q, k, v, bits, out, lse)
        ctx.meta = (num_heads, scale, qs, ks)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        q, k, v, bits, out, lse = ctx.saved_tensors
        num_heads, scale, qs, ks = ctx.meta
        B, Lq, C = q.shape
        Lk = k.shape[1]
        grad_out = grad_out.to(q.dtype).contiguous()
        _, _, _, bwb = _plan(B, Lq, Lk, num_heads)
        dq = torch.empty((B, Lq, C), dtype=q.dtype, device=q.device)
        dk = torch.empty((B, Lk, C), dtype=q.dtype, device=q.device)
        dv = torch.empty((B, Lk, C), dtype=q.dtype, device=q.device)
        ws = torch.empty((max(bwb, 4) // 4,), dtype=torch.float32, device=q.device)
        _native.call("m2f_masked_attn_bwd", _code(q.dtype), q.data_ptr(), k.data_ptr(), v.data_ptr(), bits.data_ptr(),
                     out.data_ptr(), grad_out.data_ptr(), lse.data_ptr(), B, Lq, Lk, num_heads, 32, qs, ks,
                     bits.shape[-1], ctypes.c_float(scale), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                     ws.data_ptr(), ctypes.c_int64(bwb), _stream(q))
        return dq, dk, dv, None, None, None


def masked_attention(q, k, v, bits, num_heads, scale=None):
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1] // num_heads)
    return MaskedAttention.apply(q, k, v, bits, num_heads, float(scale))


class MaskEinsum(Function):
    """out[b,q,h,w] = sum_c e[b,q,c] f[b,c,h,w] on a precast copy ``f_lp`` of ``f``."""

    @staticmethod
    def forward(ctx, embed, feats, feats_lp):
        dt = feats_lp.dtype
        B, C, H, W = feats_lp.shape
        e = embed.to(dt)
        out = torch.bmm(e, feats_lp.view(B, C, H * W)).view(B, e.shape[1], H, W)
        ctx.save_for_backward(e, feats_lp)
        ctx.dtypes = (embed.dtype, feats.dtype)
        return out

    @staticmethod
    def backward(ctx, grad):
        e, f = ctx.saved_tensors
        B, C, H, W = f.shape
        g = grad.to(f.dtype).reshape(B, -1, H * W)
        de = de_f = None
        if ctx.needs_input_grad[0]:
            de = torch.bmm(g, f.view(B, C, H * W).transpose(1, 2)).to(ctx.dtypes[0])
        if ctx.needs_input_grad[1]:
            de_f = torch.bmm(e.transpose(1, 2), g).view(B, C, H, W).to(ctx.dtypes[1])
        return de, de_f, None


def mask_einsum(embed, feats, feats_lp=None):
    if feats_lp is None:
        feats_lp = feats
    return MaskEinsum.apply(embed, feats, feats_lp)


class _FoldGate(Function):
    """Identity gate between the mask features and every folded einsum.  Its output is an empty token
    the einsums take as an input, so autograd runs this backward only after every einsum's backward
    has run (each stashes its embed and incoming gradient on the fold); it then returns
    d feats = sum_i E_i^T G_i with fp32 accumulation over K = sum_i Q_i and one rounding: on the HIP kernel
    that reads the heads' gradients in place (bf16 / fp16), else as one GEMM over their concatenation."""

    @staticmethod
    def forward(ctx, feats, state):
        ctx.state = state          # not the fold itself: the fold holds this node's output (no cycle)
        ctx.feats_meta = (feats.shape, feats.dtype)
        return feats.new_empty(0)

    @staticmethod
    def backward(ctx, _token_grad):
        state = ctx.state
        items, state.items = state.items, []
        if not items:
            return None, None
        shape, dtype = ctx.feats_meta
        es, gs = [it[0] for it in items], [it[1] for it in items]
        del items
        if _fold_fusable(es, gs, dtype):
            return state.to_feats(mask_heads_bwd_feats(es, gs, dtype), shape), None
        e = es[0] if len(es) == 1 else torch.cat(es, dim=1)   # (B, K, C)
        g = gs[0] if len(gs) == 1 else torch.cat(gs, dim=1)   # (B, K, N)
        del es, gs
        et = e.transpose(1, 2)
        if g.is_cuda and g.dtype != dtype:
            df = torch.bmm(et, g, out_dtype=dtype)      # fp32 accumulate, one rounding to the feats' dtype
        else:
            df = torch.bmm(et, g).to(dtype)
        return state.to_feats(df, shape), None


class _FoldState:
    __slots__ = ("items", "to_feats")

    def __init__(self, to_feats):
        self.items = []
        self.to_feats = to_feats


def _bwd_fusable(f, g) -> bool:
    """Shapes / dtypes of the mask-head backward kernels (csrc/mask_heads.hip)."""
    B, C, N = f.shape
    return (f.is_cuda and f.dtype in (torch.bfloat16, torch.float16) and g.dtype == f.dtype and C == 256
            and N % 16 == 0 and g.shape[1] <= 256 and f.is_contiguous() and g.is_contiguous()
            and f.data_ptr() % 16 == 0 and g.data_ptr() % 16 == 0)


def _fold_fusable(es, gs, out_dtype) -> bool:
    g0 = gs[0]
    return (len(gs) <= 16 and g0.is_cuda and g0.dtype in (torch.bfloat16, torch.float16)
            and out_dtype in (torch.float32, g0.dtype) and es[0].shape[2] == 256 and g0.shape[2] % 8 == 0
            and all(g.shape == g0.shape and g.dtype == g0.dtype and g.is_contiguous() and g.data_ptr() % 16 == 0
                    for g in gs)
            and all(e.shape == es[0].shape and e.dtype == g0.dtype for e in es))


def mask_heads_bwd_embed(g, f):
    """d embed = g f^T: g (B, Q, N), f (B, 256, N) in bf16 / fp16 -> (B, Q, 256) in that dtype."""
    B, C, N = f.shape
    Q = g.shape[1]
    wb = ctypes.c_int64()
    _native.call("m2f_mask_heads_bwd_workspace", B, Q, ctypes.c_int64(N), ctypes.byref(wb))
    ws = torch.empty((max(wb.value, 4) // 4,), dtype=torch.float32, device=g.device)
    de = torch.empty((B, Q, C), dtype=g.dtype, device=g.device)
    _native.call("m2f_mask_heads_bwd_embed", _code(g.dtype), g.data_ptr(), f.data_ptr(), B, Q, C, ctypes.c_int64(N),
                 de.data_ptr(), ws.data_ptr(), ctypes.c_int64(wb.value), _stream(g))
    return de


def mask_heads_bwd_feats(es, gs, out_dtype):
    """sum_h e_h^T g_h over the heads: e_h (B, Q, 256), g_h (B, Q, N) -> (B, 256, N) in out_dtype, without
    concatenating the heads' gradients (the kernel takes their pointers)."""
    B, Q, C = es[0].shape
    N = gs[0].shape[2]
    H = len(es)
    QP = (Q + 15) // 16 * 16
    et = torch.zeros((B, H, QP, C), dtype=es[0].dtype, device=es[0].device)
    et[:, :, :Q] = torch.stack(es, 1)
    # (b, k = (step, half, e), c = (group, lane)) -> MFMA fragment order (b, group, step, half, lane, e) (bm2f.h)
    et = et.view(B, H * QP // 16, 2, 8, C // 32, 32).permute(0, 4, 1, 2, 5, 3).contiguous()
    ptrs = (ctypes.c_void_p * H)(*[g.data_ptr() for g in gs])
    df = torch.empty((B, C, N), dtype=out_dtype, device=gs[0].device)
    _native.call("m2f_mask_heads_bwd_feats", _code(gs[0].dtype), ctypes.cast(ptrs, ctypes.c_void_p), H, et.data_ptr(),
                 B, Q, QP, C, ctypes.c_int64(N), _code(out_dtype), df.data_ptr(), _stream(gs[0]))
    return df


def _folded_backward(ctx, grad):
    (e,) = ctx.saved_tensors
    fold = ctx.fold
    f = fold.feats_lp
    B, C, N = f.shape
    g = grad.to(f.dtype).reshape(B, -1, N).contiguous()
    de = None
    if ctx.needs_input_grad[0]:
        de = mask_heads_bwd_embed(g, f) if _bwd_fusable(f, g) else torch.bmm(g, f.transpose(1, 2))
        de = de.to(ctx.edtype)
    tok = None
    if ctx.needs_input_grad[1]:
        fold.state.items.append((e, g))
        tok = g.new_empty(0)
    return de, tok


class _FoldedMaskEinsum(Function):
    @staticmethod
    def forward(ctx, embed, token, fold):
        f = fold.feats_lp                                    # (B, C, N) low-precision copy
        e = embed.to(f.dtype)
        out = torch.bmm(e, f)
        ctx.fold = fold
        ctx.edtype = embed.dtype
        ctx.save_for_backward(e)
        return out.view(fold.out_shape(e.shape[1]))

    @staticmethod
    def backward(ctx, grad):
        return (*_folded_backward(ctx, grad), None)


class _FoldedMaskHeads(Function):
    """The einsum on the hand-written MFMA kernel (csrc/mask_heads.hip) with, when ``size`` is given, the
    next cross-attention's bitmask from the same launch (+ the row fix); backward as _FoldedMaskEinsum."""

    @staticmethod
    def forward(ctx, embed, token, fold, size):
        f = fold.feats_lp
        e = embed.to(f.dtype).contiguous()
        if e.data_ptr() % 16:
            e = e.clone()
        B, C, _ = f.shape
        T, H, W = fold.frames_hw
        Q = e.shape[1]
        out = torch.empty(fold.out_shape(Q), dtype=f.dtype, device=f.device)
        if size is not None:
            h, w = int(size[0]), int(size[1])
            keys = T * h * w
            nw = num_words(keys)
            bits = torch.zeros((B, Q, nw), dtype=torch.int32, device=f.device)
            bp = bits.data_ptr()
        else:
            h = w = nw = 0
            bits = torch.empty((0,), dtype=torch.int32, device=f.device)
            bp = None
        st = _stream(f)
        _native.call("m2f_mask_heads_fwd", _code(f.dtype), e.data_ptr(), f.data_ptr(), B, Q, C, T, H, W, h, w,
                     out.data_ptr(), bp, nw, st)
        if size is not None:
            _native.call("m2f_mask_row_fix", bp, B * Q, nw, keys, st)
        ctx.mark_non_differentiable(bits)
        ctx.fold = fold
        ctx.edtype = embed.dtype
        ctx.save_for_backward(e)
        return out, bits

    @staticmethod
    def backward(ctx, grad, _grad_bits):
        return (*_folded_backward(ctx, grad), None, None)


class MaskFeatureFold:
    """All mask einsums of one decoder forward against one mask-feature map.

    ``feats``     the features as the model holds them (e.g. fp32 (B, C, H, W)); gets the gradient.
    ``feats_lp``  (B, C, N) copy in the einsum's compute dtype (``feats`` itself when no autocast).
    ``out_tail``  trailing output dims after (B, Q): (H, W) for images, (T, H, W) for video.
    ``to_feats``  maps the (B, C, N) gradient back to ``feats``' shape.
    """

    def __init__(self, feats, feats_lp, out_tail, to_feats):
        self.feats_lp = feats_lp
        self.state = _FoldState(to_feats)
        self._tail = tuple(out_tail)
        track = feats.requires_grad and torch.is_grad_enabled()
        self.token = _FoldGate.apply(feats, self.state) if track else None

    def out_shape(self, q):
        return (self.feats_lp.shape[0], q) + self._tail

    @property
    def frames_hw(self):
        return self._tail if len(self._tail) == 3 else (1,) + self._tail

    def __call__(self, embed):
        return _FoldedMaskEinsum.apply(embed, self.token, self)

    def fused_ok(self, num_queries, size=None, channels=None) -> bool:
        """Shapes / dtypes the mask-heads kernel takes (m2f_mask_heads_fwd's constraints)."""
        f = self.feats_lp
        T, H, W = self.frames_hw
        if channels is not None and channels != f.shape[1]:
            return False     # the einsum path raises the reference's shape error
        if not (f.is_cuda and f.dtype in (torch.bfloat16, torch.float16) and f.is_contiguous()
                and f.shape[1] % 32 == 0 and W % 8 == 0 and num_queries <= 256 and f.data_ptr() % 16 == 0):
            return False
        if size is None:
            return True
        h, w = int(size[0]), int(size[1])
        s = H // h if h > 0 else 0
        return s >= 2 and s % 2 == 0 and s * h == H and s * w == W and 128 % s == 0


def mask_heads(fold: MaskFeatureFold, embed: torch.Tensor, size=None):
    """One prediction head's masks and (``size`` given) the next cross-attention's bitmask:
    ``fold(embed)`` + :func:`attn_mask_bits` (reference :442-449 and :400), in one kernel where the shapes
    allow (the pyramid's exact 2/4/8x reductions in bf16 / fp16), else as those two steps."""
    if embed.dim() != 3 or embed.shape[2] != fold.feats_lp.shape[1]:
        raise RuntimeError(f"einsum bqc,bchw->bqhw: embed {tuple(embed.shape)} does not match "
                           f"{fold.feats_lp.shape[1]} feature channels")
    if fold.fused_ok(embed.shape[1], size, embed.shape[2]):
        out, bits = _FoldedMaskHeads.apply(embed, fold.token, fold, size)
        return out, (bits if size is not None else None)
    out = fold(embed)
    return out, (attn_mask_bits(out, size) if size is not None else None)


def image_mask_fold(mask_features, mask_features_lp=None):
    """Fold for ``einsum("bqc,bchw->bqhw")`` (mask2former_transformer_decoder.py:442)."""
    lp = mask_features if mask_features_lp is None else mask_features_lp
    B, C, H, W = lp.shape
    return MaskFeatureFold(mask_features, lp.detach().reshape(B, C, H * W), (H, W), lambda df, shape: df.view(shape))


def colsum_f32(g2):
    """``g2.sum(0, dtype=float32)`` of a (R, C) matrix on the library's column-sum kernel (m2f_colsum: 1024-row
    fp32 partials added in a fixed order): torch reduces a long column to few outputs across workgroups with
    semaphores it zeroes by a memset, which the runtime's HIP graph packet capture replays wrongly
    (bench_model.GraphStep)."""
    if g2.dim() != 2:
        raise RuntimeError(f"colsum_f32 needs a matrix, got shape {tuple(g2.shape)}")
    g2 = g2.contiguous()
    R, C = g2.shape
    out = torch.empty(C, dtype=torch.float32, device=g2.device)
    if R == 0:
        return out.zero_()
    wf = ctypes.c_int64(0)
    _native.call("m2f_colsum_workspace", R, C, ctypes.byref(wf))
    ws = torch.empty(wf.value, dtype=torch.float32, device=g2.device)
    _native.call("m2f_colsum", _code(g2.dtype), g2.data_ptr(), R, C, ws.data_ptr(), wf, out.data_ptr(), _stream(g2))
    return out


class _RowBias(Function):
    """x + b with b (C,) broadcast over the leading dims of a channels-last x (..., C): the level-embedding adds
    (mask2former_transformer_decoder.py:376, msdeformattn.py:75).  Same forward (torch's add and its type
    promotion); d b is the column sum on m2f_colsum instead of autograd's reduction."""

    @staticmethod
    def forward(ctx, x, b):
        ctx.meta = (x.dtype, b.dtype, b.shape)
        return x + b

    @staticmethod
    def backward(ctx, g):
        xd, bd, bshape = ctx.meta
        gb = colsum_f32(g.reshape(-1, g.shape[-1])).to(bd).view(bshape) if ctx.needs_input_grad[1] else None
        return (g.to(xd) if ctx.needs_input_grad[0] else None), gb


class _ChanBias(Function):
    """x + b[None, :, None] for x (N, C, L) (the video decoder's level-embedding add,
    video_mask2former_transformer_decoder.py:388): d b sums L in two short stages (64-element pieces, then the
    pieces: every output of both reductions is one workgroup's, so torch zeroes no semaphore with a memset),
    then the N rows on m2f_colsum."""

    @staticmethod
    def forward(ctx, x, b):
        ctx.meta = (x.dtype, b.dtype, b.shape)
        return x + b[None, :, None]

    @staticmethod
    def backward(ctx, g):
        xd, bd, bshape = ctx.meta
        gb = None
        if ctx.needs_input_grad[1]:
            N, C, L = g.shape
            k = next((k for k in (64, 32, 16, 8, 4, 2) if L % k == 0), 1)
            gs = g
            if k == 1 and L > 64:   # odd L: zero-pad it to a multiple of 64 so the second stage stays short
                gs = F.pad(g, (0, (-L) % 64))
                k, L = 64, gs.shape[2]
            part = gs.reshape(N, C, L // k, k).sum(3, dtype=torch.float32).sum(2)
            gb = colsum_f32(part).to(bd).view(bshape)
        return (g.to(xd) if ctx.needs_input_grad[0] else None), gb


def chan_bias_add(x, b):
    """x (N, C, L) + b (C,) broadcast over N and L (:class:`_ChanBias`); plain add off the GPU."""
    if not x.is_cuda or b.dim() != 1 or x.dim() != 3 or x.shape[1] != b.shape[0]:
        return x + b[None, :, None]
    return _ChanBias.apply(x, b)


def row_bias_add(x, b):
    """x (..., C) + b (C,), b's gradient through m2f_colsum (:class:`_RowBias`); plain x + b off the GPU."""
    if not x.is_cuda or b.dim() != 1 or x.shape[-1] != b.shape[0]:
        return x + b
    return _RowBias.apply(x, b)


class _TokenLinear(Function):
    """y = x W^T + b for the cross-attention K/V projections over the memory tokens (B * HW_l rows, up to
    262,144 at 1024^2 bs16; reference: nn.MultiheadAttention's in_proj, mask2former_transformer_decoder.py
    :103-108).  Same forward; the weight gradient G^T X, a 256 x 256 output over that long reduction, runs
    as a split-K batched GEMM (2048-row chunks, fp32 chunk outputs summed in a fixed order) because the
    library's single-GEMM kernel for this shape reaches ~70 TF against ~500 TF batched
    (tools/wgrad_bf16_bench.py)."""

    CHUNK = 2048

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, grad):
        x, w = ctx.saved_tensors
        g2 = grad.reshape(-1, grad.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = (g2 @ w).view(x.shape)
        if ctx.needs_input_grad[1]:
            R, ch = g2.shape[0], _TokenLinear.CHUNK
            if g2.is_cuda and R % ch == 0 and R >= 2 * ch and g2.is_contiguous() and x2.is_contiguous():
                part = torch.bmm(g2.view(-1, ch, g2.shape[1]).transpose(1, 2), x2.view(-1, ch, x2.shape[1]),
                                 out_dtype=torch.float32)
                gw = part.sum(0).to(w.dtype)
            else:
                gw = g2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = colsum_f32(g2).to(w.dtype)
        return gx, gw, gb


class _TokenLinearCast(Function):
    """:class:`_TokenLinear` on a low-precision copy of x made once per forward (``x_lp``, shared by the
    decoder layers that read the same level) whose gradient returns to the fp32 x in fp32: the same
    values autocast's per-call cast gives (the bf16 input-gradient GEMM result, then its ToCopy back to
    fp32, summed over the layers in fp32), without casting the memory tokens again in every layer."""

    @staticmethod
    def forward(ctx, x, x_lp, weight, bias):
        ctx.save_for_backward(x_lp, weight)
        ctx.has_bias = bias is not None
        ctx.x_dtype = x.dtype
        return F.linear(x_lp, weight, bias)

    @staticmethod
    def backward(ctx, grad):
        x_lp, w = ctx.saved_tensors
        g = _TokenLinear.backward(_SavedLike(ctx, x_lp, w), grad)
        gx = g[0].to(ctx.x_dtype) if g[0] is not None else None
        return gx, None, g[1], g[2]


class _SavedLike:
    """The ctx view :meth:`_TokenLinear.backward` expects (saved x, w; needs_input_grad for x, w, b)."""

    def __init__(self, ctx, x, w):
        self.saved_tensors = (x, w)
        self.has_bias = ctx.has_bias
        n = ctx.needs_input_grad
        self.needs_input_grad = (n[0], n[2], n[3])


class GradSink:
    """The fp32 gradient of one memory-token tensor that several :func:`token_linear_sink` calls read (the K and V
    projections of the 3 decoder layers on one level): each call's input gradient -- the autocast-dtype GEMM result,
    as the reference's per-call cast backward sees it -- is kept, and the call whose backward completes the set sums
    them in fp32 in arrival order in one pass (m2f_sum_to_f32: the values of a cast of the first and an fp32 add of
    each further one, without re-reading and re-writing the fp32 sum per call) and hands the sum to autograd; the
    others return no input gradient.  Autograd's path casts every call's gradient to fp32 and adds the fp32 tensors.
    One sink per tensor and forward.

    ``count`` is the number of graph-recording calls, fixed by the forward and never consumed: every backward pass
    over the graph (a second ``backward(retain_graph=True)``, a second ``autograd.grad``) collects its own ``count``
    terms and gets its own complete sum.  Calls made without gradient recording (the no-grad first pass of a
    reentrant activation checkpoint) are not counted, so the recompute's calls are."""

    def __init__(self):
        self.terms = []
        self.count = 0

    def add(self, g):
        self.terms.append(g)
        if len(self.terms) < self.count:
            return None
        terms, self.terms = self.terms, []
        return sum_to_f32(terms)


def sum_to_f32(terms):
    """``terms[0].float() + terms[1] + ...`` in fp32, in order (each add an fp32 add of the converted term): one pass
    on m2f_sum_to_f32 for up to 8 same-shaped contiguous CUDA tensors, torch's adds otherwise."""
    t0 = terms[0]
    ok = (t0.is_cuda and 1 <= len(terms) <= 8 and t0.numel() % 8 == 0
          and all(t.shape == t0.shape and t.dtype == t0.dtype and t.is_contiguous() and t.data_ptr() % 16 == 0
                  for t in terms))
    if not ok:
        out = t0.to(torch.float32, copy=True)
        for t in terms[1:]:
            torch.add(out, t, out=out)
        return out
    out = torch.empty(t0.shape, dtype=torch.float32, device=t0.device)
    ptrs = (ctypes.c_void_p * len(terms))(*[t.data_ptr() for t in terms])
    _native.call("m2f_sum_to_f32", ptrs, len(terms), t0.numel(), _code(t0.dtype), out.data_ptr(), _stream(t0))
    return out


class _TokenLinearSink(Function):
    """y = x_lp W^T + b (x_lp: the autocast-dtype copy of the fp32 tensor x, or of x + a constant embedding) with
    x's gradient g W accumulated in the shared :class:`GradSink`: the same per-call terms as the reference's autocast
    path (an fp16 / bf16 GEMM result each, summed in fp32 over the calls) without a cast and an fp32 add per call."""

    @staticmethod
    def forward(ctx, x, x_lp, weight, bias, sink):
        ctx.save_for_backward(x_lp, weight)
        ctx.has_bias = bias is not None
        ctx.sink = sink
        ctx.x_shape = x.shape
        return F.linear(x_lp, weight, bias)

    @staticmethod
    def backward(ctx, grad):
        x_lp, w = ctx.saved_tensors
        sink = ctx.sink
        gx = None
        if ctx.needs_input_grad[0]:
            g2 = grad.reshape(-1, grad.shape[-1])
            if not g2.is_contiguous():
                g2 = g2.contiguous()
            gx_lp = g2 @ w                                   # the autocast-dtype input gradient of this call
            total = sink.add(gx_lp)
            if total is not None:
                gx = total.view(ctx.x_shape)
        sub = _SavedLike(ctx, x_lp, w)
        sub.needs_input_grad = (False, ctx.needs_input_grad[2], ctx.needs_input_grad[3])
        _, gw, gb = _TokenLinear.backward(sub, grad)
        return gx, None, gw, gb, None


def token_linear_sink(x, weight, bias, x_lp, sink):
    """``F.linear`` under autocast for a memory-token projection whose input's low-precision copy ``x_lp`` was made
    once (:func:`lowp_memory`) and whose fp32 input gradient goes to ``sink`` (:class:`GradSink`).  ``x`` is the
    fp32 tensor that receives the gradient (for a key ``memory + pos`` with a constant ``pos``: ``memory``)."""
    dt = x_lp.dtype
    weight = weight.to(dt)
    bias = bias.to(dt) if bias is not None else None
    if torch.is_grad_enabled() and x.requires_grad:
        sink.count += 1      # a call whose backward will deliver a term (see GradSink)
    with torch.autocast("cuda", enabled=False):
        return _TokenLinearSink.apply(x, x_lp, weight, bias, sink)


def lowp_memory(src, pos):
    """Per decoder level, ``(key_lp, memory_lp, sink)`` for the cross-attention K / V projections under CUDA autocast
    in fp16 / bf16: memory and memory + pos cast once per forward (the add and the cast in one kernel: the fp32 sum
    rounded to the autocast dtype, as autocast's cast of the fp32 sum), and one :class:`GradSink` for memory's
    gradient; None per level elsewhere (the caller then runs the plain per-call path)."""
    if not src or src[0].device.type != "cuda" or not torch.is_autocast_enabled("cuda"):
        return [None] * len(src)
    dt = torch.get_autocast_dtype("cuda")
    if dt not in (torch.float16, torch.bfloat16) or src[0].dtype != torch.float32:
        return [None] * len(src)
    out = []
    for s, p in zip(src, pos):
        sd = s.detach()
        shape = torch.broadcast_shapes(sd.shape, p.shape)
        # memory's own layout (a transposed view of the NCHW input): the K projection then runs the same GEMM as
        # on autocast's cast of memory + pos (a contiguous copy runs another kernel, another summation order)
        k_lp = (torch.empty_like(sd, dtype=dt) if shape == sd.shape
                else torch.empty(shape, device=sd.device, dtype=dt))
        torch.add(sd, p.detach(), out=k_lp)
        out.append((k_lp, sd.to(dt), GradSink()))
    return out


def token_linear(x, weight, bias=None, x_lp=None):
    """``F.linear`` for memory-token projections (autocast applied here as F.linear would).  ``x_lp``: an
    optional detached copy of x in the autocast dtype, made once and shared by several calls."""
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        if x_lp is not None and x_lp.dtype == dt and x.dtype != dt and dt in (torch.bfloat16, torch.float16):
            weight = weight.to(dt)
            bias = bias.to(dt) if bias is not None else None
            with torch.autocast("cuda", enabled=False):
                return _TokenLinearCast.apply(x, x_lp, weight, bias)
        x, weight = x.to(dt), weight.to(dt)
        bias = bias.to(dt) if bias is not None else None
    if x.dtype not in (torch.bfloat16, torch.float16) or not x.is_cuda:
        return F.linear(x, weight, bias)
    with torch.autocast("cuda", enabled=False):
        return _TokenLinear.apply(x, weight, bias)


# ------------------------------------------------------------------------------------------------------
# the decoder's GEMM weights cast to the autocast dtype once per forward, in a few kernels
# ------------------------------------------------------------------------------------------------------
class _FlatCast(Function):
    """Cast a list of parameters to ``dtype`` as views of one flat buffer (a cat and one cast, instead of one
    autocast copy kernel per weight and use), and their gradients back to the parameters' dtype the same way
    (instead of one ToCopyBackward per weight).  The values are those of autocast's per-call ``.to(dtype)``
    and of its backward cast."""

    @staticmethod
    def forward(ctx, dtype, *params):
        ctx.set_materialize_grads(False)  # an output no loss reached arrives as None, not zeros
        ctx.shapes = [p.shape for p in params]
        ctx.numels = [p.numel() for p in params]
        ctx.src_dtype = params[0].dtype
        flat = torch.cat([p.detach().reshape(-1) for p in params]).to(dtype)
        return tuple(o.view(sh) for o, sh in zip(flat.split(ctx.numels), ctx.shapes))

    @staticmethod
    def backward(ctx, *grads):
        # a parameter no output reached keeps grad None (as autocast's per-call casts leave it), so AdamW skips
        # it as the reference's optimizer does; the others are cast back in one cat + cast
        live = [i for i, g in enumerate(grads) if g is not None]
        if not live:
            return (None,) * (len(grads) + 1)
        flat = torch.cat([grads[i].reshape(-1) for i in live]).to(ctx.src_dtype)
        out = [None] * len(grads)
        for i, o in zip(live, flat.split([ctx.numels[i] for i in live])):
            out[i] = o.view(ctx.shapes[i])
        return (None,) + tuple(out)


_LOWP = [None]   # {id(param): low-precision view} of the decoder forward in progress (lowp_scope)


def _gemm_params(module):
    out = []
    for mod in module.modules():
        if isinstance(mod, nn.Linear):
            cand = (mod.weight, mod.bias)
        elif isinstance(mod, nn.MultiheadAttention) and mod._qkv_same_embed_dim:
            cand = (mod.in_proj_weight, mod.in_proj_bias)
        else:
            continue
        out.extend(p for p in cand if p is not None and p.is_cuda and p.dtype == torch.float32)
    return out


@contextlib.contextmanager
def lowp_scope(module):
    """Inside, :func:`lp` maps the GEMM parameters of ``module`` (nn.Linear weights / biases and
    nn.MultiheadAttention in-projections) to views of one low-precision copy made by :class:`_FlatCast`, when
    the forward runs under CUDA autocast in fp16 / bf16; elsewhere (or nested) it changes nothing.  LayerNorm,
    embedding and other parameters keep their fp32 tensors (autocast runs those ops in fp32)."""
    prev = _LOWP[0]
    m = None
    if prev is None and torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        if dt in (torch.float16, torch.bfloat16):
            params = _gemm_params(module)
            if params:
                m = {id(p): t for p, t in zip(params, _FlatCast.apply(dt, *params))}
    _LOWP[0] = m if m is not None else prev
    try:
        yield
    finally:
        _LOWP[0] = prev


def lp(p):
    """The low-precision view of parameter ``p`` inside :func:`lowp_scope`, else ``p``."""
    m = _LOWP[0]
    return m.get(id(p), p) if m is not None and p is not None else p


def linear(x, mod):
    """``mod(x)`` for an nn.Linear, with its parameters through :func:`lp`."""
    return F.linear(x, lp(mod.weight), lp(mod.bias))
