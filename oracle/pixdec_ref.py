"""TEST INFRASTRUCTURE ONLY — a functional torch restatement of the reference pixel decoder's
``forward_features`` (mask2former/modeling/pixel_decoder/msdeformattn.py), used as the checker of the bm2f_amd
module at production size on the GPU (tests/test_scale_gpu.py).  Never imported by bm2f_amd.

It reads the parameters of a bm2f_amd ``MSDeformAttnPixelDecoder`` by their state-dict names (which are the
reference's) into fresh leaf tensors of the requested dtype, and evaluates the reference's math with plain torch
ops in that dtype: conv2d + GroupNorm, the sine position embedding, the deformable encoder with
``ms_deform_attn_core_pytorch`` (F.grid_sample; the reference's own CPU core) as the MSDA, the FPN top-down path
with bilinear upsampling, and the mask-feature conv.  In fp64 it is the yardstick of the fp32 HIP path; in fp32
it is the reference's own fp32 arithmetic, whose distance from fp64 is the fp32 noise floor.

Line citations are to msdeformattn.py unless noted.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def sine_pos(n, h, w, num_pos_feats, dtype, device, temperature=10000, scale=2 * math.pi):
    """PositionEmbeddingSine(normalize=True) without a mask (transformer_decoder/position_encoding.py:29-52),
    evaluated in ``dtype``."""
    y_embed = torch.arange(1, h + 1, dtype=dtype, device=device).view(1, h, 1).expand(n, h, w)
    x_embed = torch.arange(1, w + 1, dtype=dtype, device=device).view(1, 1, w).expand(n, h, w)
    eps = 1e-6
    y_embed = y_embed / (y_embed[:, -1:, :] + eps) * scale
    x_embed = x_embed / (x_embed[:, :, -1:] + eps) * scale
    dim_t = torch.arange(num_pos_feats, dtype=dtype, device=device)
    dim_t = temperature ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / num_pos_feats)
    pos_x = x_embed[:, :, :, None] / dim_t
    pos_y = y_embed[:, :, :, None] / dim_t
    pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
    pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2)


def core_grid_sample(value, shapes, loc, attn):
    """ms_deform_attn_core_pytorch (ops/functions/ms_deform_attn_func.py:52-72)."""
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = loc.shape
    vlist = value.split([h * w for h, w in shapes], dim=1)
    grids = 2 * loc - 1
    sampled = []
    for lid, (h, w) in enumerate(shapes):
        v = vlist[lid].flatten(2).transpose(1, 2).reshape(N * M, D, h, w)
        g = grids[:, :, :, lid].transpose(1, 2).flatten(0, 1)
        sampled.append(F.grid_sample(v, g, mode="bilinear", padding_mode="zeros", align_corners=False))
    a = attn.transpose(1, 2).reshape(N * M, 1, Lq, L * P)
    out = (torch.stack(sampled, dim=-2).flatten(-2) * a).sum(-1).view(N, M * D, Lq)
    return out.transpose(1, 2).contiguous()


def reference_points(shapes, dtype, device):
    """MSDeformAttnTransformerEncoder.get_reference_points with valid ratios 1 (:141-153): (1, S, L, 2)."""
    refs = []
    for h, w in shapes:
        ry, rx = torch.meshgrid(torch.linspace(0.5, h - 0.5, h, dtype=dtype, device=device),
                                torch.linspace(0.5, w - 0.5, w, dtype=dtype, device=device), indexing="ij")
        refs.append(torch.stack((rx.reshape(-1) / w, ry.reshape(-1) / h), -1))
    ref = torch.cat(refs, 0)[None]
    return ref[:, :, None].expand(1, ref.shape[1], len(shapes), 2)


def params_like(module, dtype):
    """{state-dict name: a fresh leaf copy of the parameter in ``dtype`` (requires_grad)}."""
    return {n: p.detach().to(dtype).clone().requires_grad_() for n, p in module.named_parameters()}


def _gn(x, P, pre, relu=False):
    y = F.group_norm(x, 32, P[pre + ".weight"], P[pre + ".bias"], 1e-5)
    return F.relu(y) if relu else y


def forward_features(dec, P, features, dtype, n_heads=8, n_points=4):
    """The reference's forward_features (:314-358) on parameters ``P`` (from :func:`params_like`) in ``dtype``.
    ``dec`` supplies only the configuration (feature names, levels, layer count).  Returns
    (mask_features, out[0], multi_scale_features)."""
    tin = dec.transformer_in_features[::-1]
    srcs, pos = [], []
    for idx, f in enumerate(tin):                                   # :319-322
        x = features[f].to(dtype)
        y = F.conv2d(x, P[f"input_proj.{idx}.0.weight"], P[f"input_proj.{idx}.0.bias"])
        srcs.append(_gn(y, P, f"input_proj.{idx}.1"))
        pos.append(sine_pos(x.shape[0], x.shape[2], x.shape[3], y.shape[1] // 2, dtype, x.device))
    # MSDeformAttnTransformerEncoderOnly.forward (:61-89), no padding
    shapes = [(s.shape[2], s.shape[3]) for s in srcs]
    src = torch.cat([s.flatten(2).transpose(1, 2) for s in srcs], 1)
    lvl_pos = torch.cat([p.flatten(2).transpose(1, 2) + P["transformer.level_embed"][lvl].view(1, 1, -1)
                         for lvl, p in enumerate(pos)], 1)
    N, S, C = src.shape
    L = len(shapes)
    ref = reference_points(shapes, dtype, src.device)
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=dtype, device=src.device)
    for k in range(len(dec.transformer.encoder.layers)):            # layer forward (:122-131)
        pre = f"transformer.encoder.layers.{k}."
        lin = lambda t, nm: F.linear(t, P[pre + nm + ".weight"], P[pre + nm + ".bias"])  # noqa: E731
        q = src + lvl_pos
        # MSDeformAttn.forward (ops/modules/ms_deform_attn.py:90-125)
        value = lin(src, "self_attn.value_proj").view(N, S, n_heads, C // n_heads)
        off = lin(q, "self_attn.sampling_offsets").view(N, S, n_heads, L, n_points, 2)
        aw = lin(q, "self_attn.attention_weights").view(N, S, n_heads, L * n_points)
        aw = F.softmax(aw, -1).view(N, S, n_heads, L, n_points)
        loc = ref[:, :, None, :, None, :] + off / norm[None, None, None, :, None, :]
        src2 = lin(core_grid_sample(value, shapes, loc, aw), "self_attn.output_proj")
        src = F.layer_norm(src + src2, (C,), P[pre + "norm1.weight"], P[pre + "norm1.bias"], 1e-5)
        src2 = lin(F.relu(lin(src, "linear1")), "linear2")           # forward_ffn (:116-120)
        src = F.layer_norm(src + src2, (C,), P[pre + "norm2.weight"], P[pre + "norm2.bias"], 1e-5)
    sizes = [h * w for h, w in shapes]                               # :320-335
    out = [z.transpose(1, 2).reshape(N, C, h, w) for z, (h, w) in zip(torch.split(src, sizes, 1), shapes)]
    nfpn = dec.num_fpn_levels
    for idx, f in enumerate(dec.in_features[:nfpn][::-1]):           # :337-349
        x = features[f].to(dtype)
        a = f"adapter_{nfpn - idx}"
        lo = f"layer_{nfpn - idx}"
        cur = _gn(F.conv2d(x, P[a + ".weight"], P.get(a + ".bias")), P, a + ".norm")
        y = cur + F.interpolate(out[-1], size=cur.shape[-2:], mode="bilinear", align_corners=False)
        y = _gn(F.conv2d(y, P[lo + ".weight"], P.get(lo + ".bias"), padding=1), P, lo + ".norm", relu=True)
        out.append(y)
    mf = F.conv2d(out[-1], P["mask_features.weight"], P["mask_features.bias"])
    return mf, out[0], out[:3]
