"""Box-supervised (weak-supervision) ops on the gfx950 kernels of ``csrc/weaksup.hip`` and ``csrc/lsap.hip``:
batched Hungarian matching, the pairwise-affinity cost / loss, neighbour-similarity bits and the GPU target
preparation that replaces the reference's per-image host loop with skimage.

Every op takes CUDA tensors and raises on anything else: there is no CPU path (the CPU restatement lives in
``oracle/weaksup_ref.py`` and is test infrastructure only).
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import torch
from torch.autograd import Function

from . import _native


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("bm2f_amd.weaksup ops need CUDA (HIP) tensors; there is no CPU path")


def _ptr(t):
    return None if t is None else t.data_ptr()


def h2d(values: Sequence[int], device, dtype=torch.int32) -> torch.Tensor:
    """Small host list -> device tensor without a stream synchronisation (pinned, non-blocking)."""
    t = torch.tensor(list(values), dtype=dtype)
    return t.pin_memory().to(device, non_blocking=True)


# --------------------------------------------------------------------------------------------------------
# linear sum assignment
# --------------------------------------------------------------------------------------------------------
LSAP_STATUS = {1: "cost matrix is infeasible", 2: "problem too large for the GPU solver",
               3: "matrix contains invalid numeric entries"}


def lsap_batched(cost: torch.Tensor, cols: torch.Tensor | None = None, rows: torch.Tensor | None = None):
    """Solve ``cost[b, :rows[b], :cols[b]]`` for every b (scipy.optimize.linear_sum_assignment semantics).

    cost (B, R, C) fp32 (made contiguous); rows / cols int32 device tensors (default: full).  Returns
    ``match`` (B, R) int32 (column matched to row r, -1 if none) and ``status`` (B,) int32 (0 = ok, see
    LSAP_STATUS).  No host synchronisation.
    """
    _need_cuda(cost)
    if cost.dim() != 3:
        raise ValueError("cost must be (B, R, C)")
    B, R, C = cost.shape
    c = cost.float().contiguous()
    dev = c.device
    if rows is None:
        rows = torch.full((B,), R, dtype=torch.int32, device=dev)
    match = torch.empty((B, R), dtype=torch.int32, device=dev)
    status = torch.zeros((B,), dtype=torch.int32, device=dev)
    if B == 0 or R == 0:
        return match, status
    _native.call("m2f_lsap_batched", c.data_ptr(), B, R, C, ctypes.c_int64(R * C), rows.data_ptr(), _ptr(cols),
                 match.data_ptr(), status.data_ptr(), _stream(c))
    return match, status


def raise_on_lsap_status(status: torch.Tensor) -> None:
    """Raise ValueError like scipy for a failed problem (one host sync)."""
    s = status.max().item() if status.numel() else 0
    if s:
        raise ValueError(LSAP_STATUS.get(int(s), f"linear_sum_assignment failed ({s})"))


def indices_from_match(match: torch.Tensor, n_matched: Sequence[int]) -> List[tuple]:
    """(B, Q) match rows -> per image (query idx, target idx) int64, queries ascending (scipy's order).

    ``n_matched[b]`` (= min(Q, G_b), known on the host) sizes each slice, so nothing syncs.  Works on any
    device."""
    B, Q = match.shape
    if B == 0:
        return []
    ar = torch.arange(Q, device=match.device, dtype=torch.int64)
    key = torch.where(match >= 0, ar[None], torch.full_like(ar, Q)[None])
    src = key.sort(dim=1).values
    tgt = match.long().gather(1, src.clamp(max=Q - 1))
    return [(src[b, :n], tgt[b, :n]) for b, n in enumerate(n_matched)]


# --------------------------------------------------------------------------------------------------------
# pairwise affinity
# --------------------------------------------------------------------------------------------------------
def threshold_bits(sim: torch.Tensor, thr: float) -> torch.Tensor:
    """(N, 8, H, W) similarity -> (N, H, W) uint8 neighbour bits, bit k = sim[:, k] >= thr."""
    _need_cuda(sim)
    if sim.dim() != 4 or sim.shape[1] != 8:
        raise ValueError("similarity must be (N, 8, H, W) (pairwise_size 3)")
    s = sim.float().contiguous()
    N, _, H, W = s.shape
    bits = torch.empty((N, H, W), dtype=torch.uint8, device=s.device)
    _native.call("m2f_threshold_bits", s.data_ptr(), N, ctypes.c_int64(H * W), ctypes.c_float(thr), bits.data_ptr(),
                 _stream(s))
    return bits


def _rows_args(x, bits, t_row, box, box_row, dilation):
    _need_cuda(x, bits, t_row, box, box_row)
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 3:
        raise ValueError("x must be a contiguous fp32 (N, H, W) tensor")
    for t in (t_row, box_row):
        if t is not None and (t.dtype != torch.int32 or not t.is_contiguous()):
            raise ValueError("row index tensors must be contiguous int32")
    if box is not None and (box.dtype != torch.float32 or not box.is_contiguous()):
        raise ValueError("box must be contiguous fp32")
    if bits is not None and (bits.dtype != torch.uint8 or not bits.is_contiguous()):
        raise ValueError("bits must be contiguous uint8")
    if dilation < 1 or dilation > 4:
        raise ValueError("pairwise_dilation must be in [1, 4]")


def pairwise_map(x: torch.Tensor, bits: torch.Tensor, t_row: torch.Tensor, dilation: int) -> torch.Tensor:
    """out[r, p] = sum_k bit_k s_k(p) over rows of x (N, H, W); row r uses bits[t_row[r]]."""
    _rows_args(x, bits, t_row, None, None, dilation)
    N, H, W = x.shape
    out = torch.empty((N, H, W), dtype=torch.float32, device=x.device)
    _native.call("m2f_pairwise_rows", x.data_ptr(), None, N, H, W, dilation, bits.data_ptr(), t_row.data_ptr(), None,
                 None, 0, out.data_ptr(), None, _stream(x))
    return out


def pairwise_planes(x: torch.Tensor, dilation: int) -> torch.Tensor:
    """(N, H, W) logits -> (N, 8, H, W) s_k(p) = -log P(p and its k-th neighbour share a label)."""
    _rows_args(x, None, None, None, None, dilation)
    N, H, W = x.shape
    out = torch.empty((N, 8, H, W), dtype=torch.float32, device=x.device)
    _native.call("m2f_pairwise_rows", x.data_ptr(), None, N, H, W, dilation, None, None, None, None, 2, out.data_ptr(),
                 None, _stream(x))
    return out


def box_extents(box: torch.Tensor) -> torch.Tensor:
    """(B, G, H, W) masks -> (B, G, 4) int32 [y0, y1, x0, x1) bounding every nonzero pixel (empty: y0 = H)."""
    B, G, H, W = box.shape
    rows = box.ne(0).any(3)                                    # (B, G, H)
    cols = box.ne(0).any(2)                                    # (B, G, W)
    ar_h = torch.arange(H, device=box.device)
    ar_w = torch.arange(W, device=box.device)
    y0 = torch.where(rows, ar_h, H).amin(2)
    y1 = torch.where(rows, ar_h + 1, 0).amax(2)
    x0 = torch.where(cols, ar_w, W).amin(2)
    x1 = torch.where(cols, ar_w + 1, 0).amax(2)
    return torch.stack([y0, y1, x0, x1], -1).to(torch.int32).contiguous()


def match_cost(x: torch.Tensor, bits: torch.Tensor, box: torch.Tensor, gcount: torch.Tensor, dilation: int,
               extents: torch.Tensor | None = None):
    """The matcher's fused pass (``m2f_pairwise_match_cost``) over mask logits x (B, Q, H, W):

    returns num (B, Q, Gm) = sum_p box[b, g, p] sum_k bit_k(p) s_k(p) (0 for g >= gcount[b]), and the axis
    projections x.amax(3) (B, Q, H), x.amax(2) (B, Q, W) -- one read of x instead of three.  ``extents``
    (from :func:`box_extents`) lets the kernel skip tiles a target's mask does not touch."""
    _need_cuda(x, bits, box, gcount)
    if extents is None:
        extents = box_extents(box)
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 4:
        raise ValueError("x must be a contiguous fp32 (B, Q, H, W) tensor")
    if box.dtype != torch.float32 or not box.is_contiguous() or gcount.dtype != torch.int32:
        raise ValueError("box must be contiguous fp32 (B, Gm, H, W), gcount int32")
    B, Q, H, W = x.shape
    Gm = box.shape[1]
    lib = _native.load()
    tiles = lib.m2f_pairwise_tiles(H, W)
    ntx, nty = (W + 63) // 64, (H + 15) // 16
    part = torch.empty((B * Q, tiles, Gm), dtype=torch.float32, device=x.device)
    rmax = torch.empty((B * Q, H, ntx), dtype=torch.float32, device=x.device)
    cmax = torch.empty((B * Q, nty, W), dtype=torch.float32, device=x.device)
    _native.call("m2f_pairwise_match_cost", x.data_ptr(), B, Q, H, W, dilation, bits.data_ptr(), box.data_ptr(),
                 gcount.data_ptr(), extents.data_ptr(), Gm, part.data_ptr(), rmax.data_ptr(), cmax.data_ptr(),
                 _stream(x))
    return (part.sum(1).view(B, Q, Gm), rmax.amax(2).view(B, Q, H), cmax.amax(1).view(B, Q, W))


class PairwiseSums(Function):
    """Per-row ``num[r] = sum_{p,k} box(p) bit_k(p) s_k(p)`` and ``den[r] = sum_{p,k} box(p) bit_k(p)``;
    differentiable in the mask logits x (criterion.py:156-181 + 300-311, fused)."""

    @staticmethod
    def forward(ctx, x, bits, t_row, box, box_row, dilation):
        _rows_args(x, bits, t_row, box, box_row, dilation)
        N, H, W = x.shape
        lib = _native.load()
        tiles = lib.m2f_pairwise_tiles(H, W)
        num = torch.empty((N, max(tiles, 1)), dtype=torch.float32, device=x.device)
        den = torch.empty_like(num)
        if N and H and W:
            _native.call("m2f_pairwise_rows", x.data_ptr(), None, N, H, W, dilation, bits.data_ptr(), _ptr(t_row),
                         _ptr(box), _ptr(box_row), 1, num.data_ptr(), den.data_ptr(), _stream(x))
        else:
            num.zero_()
            den.zero_()
        ctx.save_for_backward(x, bits, t_row, box, box_row)
        ctx.dilation = dilation
        num_r, den_r = num.sum(1), den.sum(1)
        ctx.mark_non_differentiable(den_r)
        return num_r, den_r

    @staticmethod
    def backward(ctx, g_num, g_den):
        x, bits, t_row, box, box_row = ctx.saved_tensors
        N, H, W = x.shape
        grad = torch.empty_like(x)
        if N and H and W:
            g = g_num.float().contiguous()
            _native.call("m2f_pairwise_rows_bwd", x.data_ptr(), None, N, H, W, ctx.dilation, bits.data_ptr(),
                         _ptr(t_row), _ptr(box), _ptr(box_row), g.data_ptr(), grad.data_ptr(), _stream(x))
        return grad, None, None, None, None, None


def pairwise_sums(x, bits, t_row, box, box_row, dilation):
    return PairwiseSums.apply(x, bits, t_row, box, box_row, dilation)


# --------------------------------------------------------------------------------------------------------
# target preparation (maskformer_model.py:399-507)
# --------------------------------------------------------------------------------------------------------
def images_lab(images: torch.Tensor, stride: int) -> torch.Tensor:
    """(B, 3, Hp, Wp) 0..255 padded images -> (B, 3, Hp/stride, Wp/stride) Lab (avg-pool, .byte(), rgb2lab)."""
    _need_cuda(images)
    x = images.float().contiguous()
    B, C, Hp, Wp = x.shape
    if C != 3:
        raise ValueError("images must have 3 channels")
    lab = torch.empty((B, 3, Hp // stride, Wp // stride), dtype=torch.float32, device=x.device)
    _native.call("m2f_weaksup_lab", x.data_ptr(), B, Hp, Wp, stride, lab.data_ptr(), _stream(x))
    return lab


def color_similarity(lab: torch.Tensor, mask: torch.Tensor, dilation: int) -> torch.Tensor:
    """lab (B, 3, h, w), mask (B, h, w) -> (B, 8, h, w) neighbour colour similarity."""
    _need_cuda(lab, mask)
    lab = lab.float().contiguous()
    mask = mask.float().contiguous()
    B, _, h, w = lab.shape
    sim = torch.empty((B, 8, h, w), dtype=torch.float32, device=lab.device)
    _native.call("m2f_color_similarity", lab.data_ptr(), mask.data_ptr(), B, h, w, dilation, sim.data_ptr(),
                 _stream(lab))
    return sim


def _pad_stack(tensors, size_divisibility, pad_value):
    """detectron2 ImageList.from_tensors: pad bottom/right to the max size rounded up, then stack."""
    hs = max(t.shape[-2] for t in tensors)
    ws = max(t.shape[-1] for t in tensors)
    if size_divisibility > 1:
        s = size_divisibility
        hs, ws = (hs + s - 1) // s * s, (ws + s - 1) // s * s
    out = tensors[0].new_full((len(tensors),) + tuple(tensors[0].shape[:-2]) + (hs, ws), pad_value)
    for i, t in enumerate(tensors):
        out[i, ..., :t.shape[-2], :t.shape[-1]].copy_(t)
    return out


def _boxes_and_labels(t):
    if isinstance(t, dict):
        return t["boxes"], t["labels"]
    return t.gt_boxes.tensor, t.gt_classes        # detectron2 Instances


def prepare_weaksup_targets(targets, org_images, img_heights, *, size_divisibility=32, mask_out_stride=4,
                            bottom_pixels_removed=10, pairwise_size=3, pairwise_dilation=2):
    """GPU ``MaskFormer.prepare_weaksup_targets`` (maskformer_model.py:399-507).

    targets: per image a detectron2 ``Instances`` (``gt_boxes.tensor`` (G, 4) x0,y0,x1,y1 and
    ``gt_classes``) or a dict with "boxes" / "labels"; org_images: per image (3, H, W) 0..255 (uint8 or
    float) CUDA tensors; img_heights: the annotation heights (bottom-pixel removal scales with them).

    Returns the reference's per-image dicts: labels, box_masks (G, h, w), images_color_similarity
    (G, 8, h, w) -- a zero-copy ``expand`` of the image's one similarity map (the reference materialises
    G identical copies), and the four projection bounds.  Differences: an image without boxes yields
    empty tensors (the reference fails on ``torch.cat([])``, :498); boxes are taken as non-negative
    pixel coordinates (as detectron2 clips them).
    """
    if pairwise_size != 3:
        raise ValueError("only pairwise_size 3 is implemented")
    dev = org_images[0].device
    _need_cuda(*org_images)
    masks = []
    for i, img in enumerate(org_images):
        m = torch.ones(img.shape[-2:], dtype=torch.float32, device=dev)
        removed = int(bottom_pixels_removed * float(img.shape[-2]) / float(img_heights[i]))
        if removed > 0:
            m[-removed:, :] = 0
        masks.append(m)
    images = _pad_stack([x.float() for x in org_images], size_divisibility, 0.0)
    image_masks = _pad_stack(masks, size_divisibility, 0.0)
    stride = mask_out_stride
    start = stride // 2
    Hp, Wp = images.shape[-2:]
    if Hp % stride or Wp % stride:
        raise ValueError("padded image size must be a multiple of mask_out_stride")
    lab = images_lab(images, stride)
    ds_masks = image_masks[:, start::stride, start::stride]
    sim = color_similarity(lab, ds_masks, pairwise_dilation)        # (B, 8, h, w)
    h, w = Hp // stride, Wp // stride
    ys = start + stride * torch.arange(h, device=dev)
    xs = start + stride * torch.arange(w, device=dev)
    out = []
    for b, t in enumerate(targets):
        boxes, labels = _boxes_and_labels(t)
        boxes = boxes.to(dev).float()
        G = boxes.shape[0]
        # python int(): truncation toward zero; slices [y0, y1 + 1) clipped to the padded image
        ib = boxes.trunc().long()
        x0, y0 = ib[:, 0], ib[:, 1]
        x1 = ib[:, 2].clamp(max=Wp - 1)
        y1 = ib[:, 3].clamp(max=Hp - 1)
        in_y = (ys[None] >= y0[:, None]) & (ys[None] <= y1[:, None])        # (G, h)
        in_x = (xs[None] >= x0[:, None]) & (xs[None] <= x1[:, None])        # (G, w)
        box_masks = (in_y[:, :, None] & in_x[:, None, :]).float()
        nonempty_x = (x1 >= x0)[:, None]
        nonempty_y = (y1 >= y0)[:, None]
        # argmax of a box row = its first column (0 for an empty row); W - argmax(flipped) = last + 1 (or W)
        row_on = in_y & nonempty_x
        col_on = in_x & nonempty_y
        left = torch.where(row_on, x0[:, None].float(), 0.0) / stride
        right = torch.where(row_on, (x1 + 1)[:, None].float(), float(Wp)) / stride
        top = torch.where(col_on, y0[:, None].float(), 0.0) / stride
        bottom = torch.where(col_on, (y1 + 1)[:, None].float(), float(Hp)) / stride
        out.append({
            "labels": labels.to(dev),
            "box_masks": box_masks,
            "images_color_similarity": sim[b:b + 1].expand(G, 8, h, w),
            "left_bounds": left.float(), "right_bounds": right.float(),
            "top_bounds": top.float(), "bottom_bounds": bottom.float(),
        })
    return out
