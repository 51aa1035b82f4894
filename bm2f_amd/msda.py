"""Multi-scale deformable attention: native op binding, autograd Function and nn.Module.

Drop-in for the reference's op stack (paths relative to the reference root,
``ops`` = ``mask2former/modeling/pixel_decoder/ops``):

* :func:`ms_deform_attn_forward` / :func:`ms_deform_attn_backward` replace the pybind functions of the
  compiled ``MultiScaleDeformableAttention`` module (``ops/src/vision.cpp:18-21``) with the same
  argument order, preconditions and error behaviour (``ops/src/cuda/ms_deform_attn_cuda.cu:33-57,
  98-124``: RuntimeError on non-contiguous / non-device inputs or a batch that ``im2col_step`` does not
  divide), backed by the HIP kernels in ``csrc/msda.hip`` through the C ABI.
* :class:`MSDeformAttnFunction` replaces ``ops/functions/ms_deform_attn_func.py:32-49``.
* :class:`MSDeformAttn` replaces ``ops/modules/ms_deform_attn.py:34-125`` (same parameters, init and
  forward), without the bare ``try/except`` that silently falls back to the CPU core (:116-121):
  here a failure raises.
"""
from __future__ import annotations

import ctypes
import math
import warnings
from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd import Function
from torch.autograd.function import once_differentiable
from torch.nn.init import constant_, xavier_uniform_

from . import _native, linear_ops

__all__ = [
    "ms_deform_attn_forward",
    "ms_deform_attn_backward",
    "MSDeformAttnFunction",
    "MSDeformAttnFusedFunction",
    "MSDeformAttn",
    "attach_host_shapes",
]

_HOST_ATTR = "_bm2f_host_shapes"


_LSI_ATTR = "_bm2f_level_starts"


def _prefix_starts(shapes):
    starts, acc = [], 0
    for h, w in shapes:
        starts.append(acc)
        acc += h * w
    return tuple(starts)


def attach_host_shapes(spatial_shapes: torch.Tensor, shapes: Sequence[Tuple[int, int]],
                       level_start_index: torch.Tensor = None) -> torch.Tensor:
    """Record the host-side (H, W) list on a device ``spatial_shapes`` tensor.

    The kernels only need the device tensor; the host copy lets the backward pick its spatially tiled
    grad_value accumulation without a device->host sync.  Results are identical either way.  The tiled and
    fused kernels take the level starts as the prefix sums of these shapes (include/bm2f.h), so the list is
    checked against the tensor here, once (one device->host copy), and ``level_start_index`` -- given here or
    met later by a backward -- must be those prefix sums; a mismatch raises instead of silently disagreeing
    with the untiled path, which reads the device level_start_index.
    """
    shapes = tuple((int(h), int(w)) for h, w in shapes)
    got = tuple(tuple(int(v) for v in row) for row in spatial_shapes.detach().cpu().tolist())
    if got != shapes:
        raise ValueError(f"attach_host_shapes: spatial_shapes holds {got}, not {shapes}")
    setattr(spatial_shapes, _HOST_ATTR, shapes)
    if level_start_index is not None:
        _check_level_starts(level_start_index, shapes)
    return spatial_shapes


def _check_level_starts(level_start_index: torch.Tensor, shapes) -> None:
    want = _prefix_starts(shapes)
    if getattr(level_start_index, _LSI_ATTR, None) == want:
        return
    got = tuple(int(v) for v in level_start_index.detach().cpu().tolist())
    if got != want:
        raise ValueError(f"level_start_index {got} is not the prefix sum {want} of the attached spatial shapes")
    setattr(level_start_index, _LSI_ATTR, want)   # checked once per tensor


def _derive_host_shapes(spatial_shapes: torch.Tensor, level_start_index: torch.Tensor):
    """Host shapes for a device ``spatial_shapes`` that arrived untagged -- the reference's unchanged
    ``MSDeformAttn.forward`` -> ``MSDeformAttnFunction.apply`` (ops/modules/ms_deform_attn.py:116-117) passes
    the encoder's device tensor as is.  One device->host copy per tensor object, cached on it (the encoder
    hands the same tensor to all six layers, msdeformattn.py:75-83, and autograd hands the same Python object
    back to the backward, tag included), so the op-level drop-in takes the tiled backward too.  Returns None (untiled kernels, same results) when
    the tensor cannot be read back here: during graph capture, or when ``level_start_index`` is not the
    prefix sum the tiled kernels assume."""
    if (spatial_shapes.dim() != 2 or spatial_shapes.shape[1] != 2 or spatial_shapes.dtype != torch.int64
            or level_start_index is None or spatial_shapes.device.type != "cuda"
            or torch.cuda.is_current_stream_capturing()):
        return None
    pair = torch.cat((spatial_shapes.reshape(-1), level_start_index.reshape(-1))).cpu().tolist()
    L = spatial_shapes.shape[0]
    shapes = tuple((int(pair[2 * i]), int(pair[2 * i + 1])) for i in range(L))
    if tuple(int(v) for v in pair[2 * L:]) != _prefix_starts(shapes):
        return None
    setattr(spatial_shapes, _HOST_ATTR, shapes)
    setattr(level_start_index, _LSI_ATTR, _prefix_starts(shapes))
    return shapes


def _host_shapes(spatial_shapes: torch.Tensor, level_start_index: torch.Tensor = None, derive: bool = False):
    hs = getattr(spatial_shapes, _HOST_ATTR, None)
    if hs is None:
        return _derive_host_shapes(spatial_shapes, level_start_index) if derive else None
    if level_start_index is not None:
        _check_level_starts(level_start_index, hs)
    return hs


def _check(t: torch.Tensor, name: str) -> None:
    if not t.is_contiguous():
        raise RuntimeError(f"{name} tensor has to be contiguous")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} must be a CUDA tensor")


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _host_shape_buffer(shapes):
    if shapes is None:
        return None
    flat = [v for hw in shapes for v in hw]
    return (ctypes.c_int64 * len(flat))(*flat)


def _dims(value, spatial_shapes, sampling_loc):
    if value.dim() != 4:
        raise RuntimeError(f"value must be (N, S, M, D), got shape {tuple(value.shape)}")
    if sampling_loc.dim() != 6 or sampling_loc.shape[-1] != 2:
        raise RuntimeError(f"sampling_loc must be (N, Lq, M, L, P, 2), got shape {tuple(sampling_loc.shape)}")
    N, S, M, D = value.shape
    L = spatial_shapes.shape[0]
    Lq, P = sampling_loc.shape[1], sampling_loc.shape[4]
    if sampling_loc.shape[0] != N or sampling_loc.shape[2] != M or sampling_loc.shape[3] != L:
        raise RuntimeError("sampling_loc shape does not match value / spatial_shapes")
    return N, S, M, D, L, Lq, P


def _suffix(dtype: torch.dtype) -> str:
    if dtype == torch.float32:
        return "f32"
    if dtype == torch.float64:
        return "f64"
    # the reference dispatches AT_DISPATCH_FLOATING_TYPES (ms_deform_attn_cuda.cu:69, :139)
    raise RuntimeError(f'"ms_deform_attn_forward_cuda" not implemented for \'{dtype}\'')


def ms_deform_attn_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step):
    """Native forward; returns (N, Lq, M*D).  Same contract as the reference binding."""
    for t, n in ((value, "value"), (spatial_shapes, "spatial_shapes"), (level_start_index, "level_start_index"),
                 (sampling_loc, "sampling_loc"), (attn_weight, "attn_weight")):
        _check(t, n)
    sfx = _suffix(value.dtype)
    if sampling_loc.dtype != value.dtype or attn_weight.dtype != value.dtype:
        raise RuntimeError("value, sampling_loc and attn_weight must share a dtype")
    if spatial_shapes.dtype != torch.int64 or level_start_index.dtype != torch.int64:
        raise RuntimeError("spatial_shapes and level_start_index must be int64")
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, sampling_loc)
    out = torch.empty((N, Lq, M * D), dtype=value.dtype, device=value.device)
    # an untagged device spatial_shapes is read back once and tagged (the reference's own MSDeformAttnFunction
    # saves this tensor object for its backward, where the tag then selects the tiled kernel)
    host = _host_shape_buffer(_host_shapes(spatial_shapes, level_start_index, derive=True))
    _native.call(f"m2f_msda_fwd_{sfx}", _ptr(value), _ptr(spatial_shapes), _ptr(level_start_index),
                 _ptr(sampling_loc), _ptr(attn_weight), N, S, M, D, L, Lq, P, int(im2col_step),
                 ctypes.cast(host, ctypes.c_void_p) if host is not None else None, _ptr(out), _stream(value.device))
    return out


def ms_deform_attn_backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output,
                            im2col_step):
    """Native backward; returns [grad_value, grad_sampling_loc, grad_attn_weight]."""
    for t, n in ((value, "value"), (spatial_shapes, "spatial_shapes"), (level_start_index, "level_start_index"),
                 (sampling_loc, "sampling_loc"), (attn_weight, "attn_weight"), (grad_output, "grad_output")):
        _check(t, n)
    sfx = _suffix(value.dtype)
    if grad_output.dtype != value.dtype:
        raise RuntimeError("grad_output must have the dtype of value")
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, sampling_loc)
    grad_value = torch.empty_like(value)
    grad_loc = torch.empty_like(sampling_loc)
    grad_attn = torch.empty_like(attn_weight)
    host = _host_shape_buffer(_host_shapes(spatial_shapes, level_start_index, derive=True))
    _native.call(f"m2f_msda_bwd_{sfx}", _ptr(value), _ptr(spatial_shapes), _ptr(level_start_index),
                 _ptr(sampling_loc), _ptr(attn_weight), _ptr(grad_output), N, S, M, D, L, Lq, P, int(im2col_step),
                 ctypes.cast(host, ctypes.c_void_p) if host is not None else None,
                 _ptr(grad_value), _ptr(grad_loc), _ptr(grad_attn), _stream(value.device))
    return [grad_value, grad_loc, grad_attn]


class MSDeformAttnFunction(Function):
    """Autograd wrapper, same ``apply`` signature as ops/functions/ms_deform_attn_func.py:32-49."""

    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations, attention_weights,
                im2col_step):
        ctx.im2col_step = im2col_step
        # derive=True: an untagged device spatial_shapes (the reference module's call) is read back once
        ctx.host_shapes = _host_shapes(value_spatial_shapes, value_level_start_index, derive=True)
        output = ms_deform_attn_forward(value, value_spatial_shapes, value_level_start_index, sampling_locations,
                                        attention_weights, ctx.im2col_step)
        ctx.save_for_backward(value, value_spatial_shapes, value_level_start_index, sampling_locations,
                              attention_weights)
        return output

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        value, shapes, lsi, loc, attn = ctx.saved_tensors
        if ctx.host_shapes is not None:
            # unpacked saved tensors are new objects: restore the tags the forward checked
            setattr(shapes, _HOST_ATTR, ctx.host_shapes)
            setattr(lsi, _LSI_ATTR, _prefix_starts(ctx.host_shapes))
        grad_value, grad_loc, grad_attn = ms_deform_attn_backward(
            value, shapes, lsi, loc, attn, grad_output.contiguous(), ctx.im2col_step)
        return grad_value, None, None, grad_loc, grad_attn, None


class MSDeformAttnFusedFunction(Function):
    """MSDA with the sampling front end fused into the kernels (encoder layout only).

    Inputs: value (N, S, M, 32) fp32; proj (N, S, M*L*P*3) = [sampling offsets (M, L, P, 2) | attention
    logits (M, L*P)], the raw output of the two projections of ms_deform_attn.py:102-103; ref (N, S, L, 2)
    reference points.  Computes softmax and loc = ref + offset / (W, H) in-kernel (ms_deform_attn.py:104-109)
    instead of materialising sampling_locations / attention_weights; the backward returns d value and
    d proj directly (reference points are constants of the encoder and get no gradient).  ``head_major``: proj
    rows hold one [offsets (L, P, 2) | logits (L*P)] record per head instead (:func:`head_major_wb`; the
    m2f_msda_fused_*_hm_f32 entry points), and d proj comes back in that layout.
    """

    @staticmethod
    def forward(ctx, value, proj, ref, host_shapes, n_points, head_major=False):
        N, S, M, D = value.shape
        L = len(host_shapes)
        if ref.stride(-1) != 1 or ref.stride(-2) != 2 or ref.stride(-3) != 2 * L:
            ref = ref.contiguous()
        if proj.stride(-1) != 1 or proj.stride(0) != proj.shape[1] * proj.stride(1):
            proj = proj.contiguous()
        hs = _host_shape_buffer(host_shapes)
        out = torch.empty((N, S, M * D), dtype=value.dtype, device=value.device)
        _native.call("m2f_msda_fused_fwd_hm_f32" if head_major else "m2f_msda_fused_fwd_f32", _ptr(value), _ptr(proj),
                     proj.stride(1), _ptr(ref), ref.stride(0), ctypes.cast(hs, ctypes.c_void_p), N, S, M, D, L, S,
                     n_points, _ptr(out), _stream(value.device))
        ctx.save_for_backward(value, proj, ref)
        ctx.meta = (tuple(host_shapes), n_points, bool(head_major))
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        value, proj, ref = ctx.saved_tensors
        host_shapes, n_points, head_major = ctx.meta
        N, S, M, D = value.shape
        L = len(host_shapes)
        grad_out = grad_out.contiguous()
        hs = _host_shape_buffer(host_shapes)
        grad_value = torch.empty_like(value)
        grad_proj = torch.empty((N, S, M * L * n_points * 3), dtype=proj.dtype, device=proj.device)
        # deterministic mode (native option msda_bwd_det, or torch.use_deterministic_algorithms(True)) needs an
        # int64 accumulator workspace; 0 bytes otherwise
        if torch.are_deterministic_algorithms_enabled() and _native.get_option("msda_bwd_det") < 0:
            with _native.options(msda_bwd_det=1):
                return MSDeformAttnFusedFunction.backward(ctx, grad_out)
        ws_bytes = ctypes.c_int64(0)
        _native.call("m2f_msda_fused_bwd_workspace", ctypes.cast(hs, ctypes.c_void_p), N, S, M, D, L, n_points,
                     ctypes.byref(ws_bytes))
        ws = torch.empty(ws_bytes.value, dtype=torch.uint8, device=value.device) if ws_bytes.value else None
        _native.call("m2f_msda_fused_bwd_hm_f32" if head_major else "m2f_msda_fused_bwd_f32", _ptr(value),
                     _ptr(proj), proj.stride(1), _ptr(ref), ref.stride(0), ctypes.cast(hs, ctypes.c_void_p),
                     _ptr(grad_out), N, S, M, D, L, S, n_points, _ptr(grad_value), _ptr(grad_proj),
                     None if ws is None else _ptr(ws), ctypes.c_int64(ws_bytes.value), _stream(value.device))
        return grad_value, grad_proj, None, None, None, None


def head_major_wb(w_off, b_off, w_attn, b_attn, n_heads):
    """The sampling-offset and attention-logit projections (ms_deform_attn.py:59-60) as one weight / bias whose
    output rows are head-major: per head m its offsets (L, P, 2) then its logits (L*P).  Built from views and a
    cat, so the parameters' gradients come back through slices (deterministic; no scatter)."""
    C = w_off.shape[1]
    w = torch.cat([w_off.view(n_heads, -1, C), w_attn.view(n_heads, -1, C)], 1).reshape(-1, C)
    b = torch.cat([b_off.view(n_heads, -1), b_attn.view(n_heads, -1)], 1).reshape(-1)
    return w, b


HEAD_MAJOR = True  # the module's fused path projects head-major (m2f_msda_fused_*_hm_f32); False: reference order


FUSED = True   # the encoder's fused MSDA front end; False: the reference's op chain (tests, A/B)


def _fused_enabled():
    return FUSED


def _is_power_of_2(n):
    if (not isinstance(n, int)) or (n < 0):
        raise ValueError("invalid input for _is_power_of_2: {} (type: {})".format(n, type(n)))
    return (n & (n - 1) == 0) and n != 0


class MSDeformAttn(nn.Module):
    """Multi-scale deformable attention layer (ops/modules/ms_deform_attn.py:34-125).

    Parameters and their initialisation match the reference so checkpoints load unchanged:
    ``sampling_offsets`` (M*L*P*2, C), ``attention_weights`` (M*L*P, C), ``value_proj``, ``output_proj``.
    """

    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError("d_model must be divisible by n_heads, but got {} and {}".format(d_model, n_heads))
        _d_per_head = d_model // n_heads
        if not _is_power_of_2(_d_per_head):
            warnings.warn("MSDeformAttn: a power-of-2 head dimension selects the vectorised gfx950 kernels; "
                          f"{_d_per_head} runs on the generic kernels.")
        self.im2col_step = 128
        self.d_model = d_model
        self.n_levels = n_levels
        self.n_heads = n_heads
        self.n_points = n_points
        self.sampling_offsets = nn.Linear(d_model, n_heads * n_levels * n_points * 2)
        self.attention_weights = nn.Linear(d_model, n_heads * n_levels * n_points)
        self.value_proj = nn.Linear(d_model, d_model)
        self.output_proj = nn.Linear(d_model, d_model)
        self._reset_parameters()

    def _reset_parameters(self):
        # ms_deform_attn.py:66-80: offsets start on 8 rays at distance 1..P, uniform attention
        constant_(self.sampling_offsets.weight.data, 0.0)
        thetas = torch.arange(self.n_heads, dtype=torch.float32) * (2.0 * math.pi / self.n_heads)
        grid = torch.stack([thetas.cos(), thetas.sin()], -1)
        grid = grid / grid.abs().max(-1, keepdim=True)[0]
        grid = grid.view(self.n_heads, 1, 1, 2).repeat(1, self.n_levels, self.n_points, 1)
        grid = grid * torch.arange(1, self.n_points + 1, dtype=torch.float32).view(1, 1, -1, 1)
        with torch.no_grad():
            self.sampling_offsets.bias = nn.Parameter(grid.reshape(-1))
        constant_(self.attention_weights.weight.data, 0.0)
        constant_(self.attention_weights.bias.data, 0.0)
        xavier_uniform_(self.value_proj.weight.data)
        constant_(self.value_proj.bias.data, 0.0)
        xavier_uniform_(self.output_proj.weight.data)
        constant_(self.output_proj.bias.data, 0.0)

    def sampling(self, query, reference_points, input_spatial_shapes):
        """Sampling locations (N, Lq, M, L, P, 2) and softmaxed weights (N, Lq, M, L, P)."""
        N, Len_q, _ = query.shape
        M, L, P = self.n_heads, self.n_levels, self.n_points
        offsets = self.sampling_offsets(query).view(N, Len_q, M, L, P, 2)
        attn = self.attention_weights(query).view(N, Len_q, M, L * P)
        attn = F.softmax(attn, -1).view(N, Len_q, M, L, P)
        if reference_points.shape[-1] == 2:
            normalizer = torch.stack([input_spatial_shapes[..., 1], input_spatial_shapes[..., 0]], -1)
            loc = reference_points[:, :, None, :, None, :] + offsets / normalizer[None, None, None, :, None, :]
        elif reference_points.shape[-1] == 4:
            loc = (reference_points[:, :, None, :, None, :2]
                   + offsets / P * reference_points[:, :, None, :, None, 2:] * 0.5)
        else:
            raise ValueError("Last dim of reference_points must be 2 or 4, but get {} instead.".format(
                reference_points.shape[-1]))
        return loc, attn

    def _fusable(self, query, reference_points, input_flatten, input_spatial_shapes, input_padding_mask,
                 input_level_start_index=None):
        hs = _host_shapes(input_spatial_shapes, input_level_start_index)
        return (_fused_enabled() and hs is not None and input_padding_mask is None and query.is_cuda
                and query.dtype == torch.float32 and input_flatten.dtype == torch.float32
                and self.d_model // self.n_heads == 32 and self.n_points == 4 and 1 <= self.n_levels <= 4
                and len(hs) == self.n_levels and query.shape[1] == input_flatten.shape[1]
                and reference_points.shape[-1] == 2 and not reference_points.requires_grad
                and not torch.is_autocast_enabled("cuda"))

    def _sampling_wb(self):
        """The fused path's projection weight / bias: both sampling projections in one GEMM, head-major rows
        (:func:`head_major_wb`) unless ``HEAD_MAJOR`` is off."""
        if HEAD_MAJOR:
            return head_major_wb(self.sampling_offsets.weight, self.sampling_offsets.bias,
                                 self.attention_weights.weight, self.attention_weights.bias, self.n_heads)
        return (torch.cat([self.sampling_offsets.weight, self.attention_weights.weight], 0),
                torch.cat([self.sampling_offsets.bias, self.attention_weights.bias], 0))

    def forward_src_pos(self, src, pos, reference_points, input_spatial_shapes, input_level_start_index,
                        input_padding_mask=None):
        """``(self.forward(src + pos, reference_points, src, ...), src)`` for an encoder layer whose query is
        ``src + pos`` and whose residual is ``src`` (msdeformattn.py:115-119).  On the fused path the two
        input projections are one autograd node (:class:`linear_ops.EncoderInProjF32`) and the returned
        ``src`` carries the residual's gradient into that node's GEMM epilogues."""
        if (self._fusable(src, reference_points, src, input_spatial_shapes, input_padding_mask,
                          input_level_start_index)
                and (pos is None or (pos.dtype == torch.float32 and pos.dim() == 3 and pos.shape[0] in (1, src.shape[0])
                                     and pos.shape[1:] == src.shape[1:]))
                and linear_ops.residual_fusable(src, self.value_proj)):
            N, Len_in, _ = src.shape
            w, b = self._sampling_wb()
            value, proj, src_res = linear_ops.EncoderInProjF32.apply(src, pos, self.value_proj.weight,
                                                                     self.value_proj.bias, w, b)
            value = value.view(N, Len_in, self.n_heads, self.d_model // self.n_heads)
            out = MSDeformAttnFusedFunction.apply(value, proj, reference_points,
                                                  _host_shapes(input_spatial_shapes), self.n_points, HEAD_MAJOR)
            return linear_ops.linear(out, self.output_proj), src_res
        query = src if pos is None else src + pos
        return self.forward(query, reference_points, src, input_spatial_shapes, input_level_start_index,
                            input_padding_mask), src

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes, input_level_start_index,
                input_padding_mask=None):
        N, Len_q, _ = query.shape
        N, Len_in, _ = input_flatten.shape
        if self._fusable(query, reference_points, input_flatten, input_spatial_shapes, input_padding_mask,
                         input_level_start_index):
            # one GEMM for both sampling projections; softmax + locations happen inside the MSDA kernels
            # fp32 linears on the MFMA GEMMs (linear_ops): bias in the epilogue, bias gradient in the
            # weight-gradient GEMM
            value = linear_ops.linear(input_flatten, self.value_proj).view(
                N, Len_in, self.n_heads, self.d_model // self.n_heads)
            w, b = self._sampling_wb()
            proj = linear_ops.linear_wb(query, w, b)
            out = MSDeformAttnFusedFunction.apply(value, proj, reference_points,
                                                  _host_shapes(input_spatial_shapes), self.n_points, HEAD_MAJOR)
            return linear_ops.linear(out, self.output_proj)
        value = self.value_proj(input_flatten)
        if input_padding_mask is not None:
            value = value.masked_fill(input_padding_mask[..., None], float(0))
        value = value.view(N, Len_in, self.n_heads, self.d_model // self.n_heads)
        loc, attn = self.sampling(query, reference_points, input_spatial_shapes)
        output = MSDeformAttnFunction.apply(value.contiguous(), input_spatial_shapes, input_level_start_index,
                                            loc.contiguous(), attn.contiguous(), self.im2col_step)
        return self.output_proj(output)
